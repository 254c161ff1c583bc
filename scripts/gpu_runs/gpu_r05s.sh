# Round 5, pass s: the conv1 launch's W2 fragment-copy blocks (MIHVD_F32_W2F_BLOCKS: 28 = the
# default, each thread ~4 dependent rounds; 100 = one float4 per thread): whole-step A/B at the
# default length, alternating, then a kernel trace with 100 for the per-kernel times.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py -k "conv1 or conv2_fwd or fragment or graph_replay" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for k in 28 100 56; do
  MIHVD_F32_W2F_BLOCKS=$k timeout -k 10 200 python bench.py > $O/bench_w${k}_$i.log 2>&1 || { tail -20 $O/bench_w${k}_$i.log; exit 1; }
  python3 -c "import json; [print('w2f blocks $k', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_w${k}_$i.log') if l.startswith('{')]"
done; done
MIHVD_F32_W2F_BLOCKS=100 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
python3 scripts/roofline_f32.py $O/prof/run_kernel_trace.csv $O/prof_bench.log --stats $O/kernel_stats.txt > $O/roofline.md && sed -n 5,16p $O/roofline.md
echo ALLDONE
