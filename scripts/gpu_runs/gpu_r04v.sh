# Round 4, pass v: bench with the lead-graph replay schedule (driver form x4, 400 steps), and the
# bench-flow / rehearsal GPU tests that drive bench.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04v; mkdir -p $O
for i in 1 2 3 4; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; tail -1 $O/bench_drv$i.log | cut -c1-200; done
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --lead-steps 0 > $O/bench_drv_nolead.log 2>&1 || { tail -20 $O/bench_drv_nolead.log; exit 1; }
tail -1 $O/bench_drv_nolead.log | cut -c1-200
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log | cut -c1-200
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_fused_distributed_gpu.py -k "rehearsal or bench_flow" tests/test_examples_gpu.py > $O/t_bench.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t_bench.log | tail -14; [ $rc -ne 0 ] && { tail -40 $O/t_bench.log; exit $rc; }
echo ALLDONE
