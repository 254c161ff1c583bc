# Round 4, pass t: HEAD evidence — fp32 tests, benches (driver form x2, 400 steps), rocprof trace of
# the bench (roofline), kbench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04t; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_gpu.py > $O/t_f32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t_f32.log | tail -5; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
for i in 1 2 3; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; tail -1 $O/bench_drv$i.log | cut -c1-200; done
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
tail -1 $O/prof_bench.log | cut -c1-200
timeout -k 10 300 python scripts/kbench_f32.py --json $O/kbench.json > $O/kbench.log 2>&1 || { tail -30 $O/kbench.log; exit 1; }
cat $O/kbench.log
echo ALLDONE
