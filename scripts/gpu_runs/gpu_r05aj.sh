# Round 5, pass aj: conv2_fwd with its image LDS-DMA issued by inline asm and an explicit vmcnt(25)
# before the staging barrier, so the 25 W2 loads stay in flight (MIHVD_F32_C2F_ADMA=1; 0 = builtin):
# fp32 tests, whole step alternating, the launch under rocprofv3 for both.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05aj; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/tests.log | head; exit $rc; }
for i in 1 2 3; do for k in 0 1; do
  MIHVD_F32_C2F_ADMA=$k timeout -k 10 200 python bench.py > $O/bench_w${k}_$i.log 2>&1 || { tail -20 $O/bench_w${k}_$i.log; exit 1; }
  python3 -c "import json; [print('adma=$k', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_w${k}_$i.log') if l.startswith('{')]"
done; done
for k in 0 1; do
  MIHVD_F32_C2F_ADMA=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$k -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_bench$k.log 2>&1 || { tail -20 $O/prof_bench$k.log; exit 1; }
  python3 scripts/roofline_f32.py $O/prof$k/run_kernel_trace.csv $O/prof_bench$k.log --stats $O/kernel_stats$k.txt > $O/roofline$k.md && grep -E "conv2_fwd|kernel sum" $O/roofline$k.md | head -2
done
echo ALLDONE
