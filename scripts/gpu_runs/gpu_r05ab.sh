# Round 5, pass ab: fc1_bwd with its first dz chunk and first p / m / v issued before the a2 and
# routing operands (MIHVD_F32_F1R_ORD=1; 0 = the default order): the fused-Adam equivalence test,
# then the whole step alternating and the launch under rocprofv3 for both orders.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05ab; mkdir -p $O
MIHVD_F32_F1R_ORD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py -k "fused_adam or graph_replay or trajectory" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do for k in 0 1; do
  MIHVD_F32_F1R_ORD=$k timeout -k 10 200 python bench.py > $O/bench_o${k}_$i.log 2>&1 || { tail -20 $O/bench_o${k}_$i.log; exit 1; }
  python3 -c "import json; [print('ord=$k', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_o${k}_$i.log') if l.startswith('{')]"
done; done
for k in 0 1; do
  MIHVD_F32_F1R_ORD=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$k -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_bench$k.log 2>&1 || { tail -20 $O/prof_bench$k.log; exit 1; }
  python3 scripts/roofline_f32.py $O/prof$k/run_kernel_trace.csv $O/prof_bench$k.log > $O/roofline$k.md && grep "fc1_bwd" $O/roofline$k.md
done
echo ALLDONE
