# Round 4, pass m: conv2_fwd A reads two steps ahead, exact-batch fc1 wgrad chain, conflict-free fc1_fwd
# B reads, and the fp32 factor-gather plane (dgrad-only fc1_bwd, RCCL all-to-all, world-1 capture,
# 4/8-rank gloo equivalence); full kbench and benches.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04m; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_f32_gpu.py > $O/t_f32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t_f32.log | tail -5; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 200 $T tests/test_native_comm_gpu.py -k rccl_comm > $O/t_ncomm.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t_ncomm.log | tail -4; [ $rc -ne 0 ] && { tail -40 $O/t_ncomm.log; exit $rc; }
timeout -k 10 600 $T tests/test_fused_distributed_gpu.py -k "factor or (collectives_inside and fp32) or (equivalence_n_ranks and fp32 and factor)" > $O/t_dist.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t_dist.log | tail -10; [ $rc -ne 0 ] && { tail -60 $O/t_dist.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --json $O/kbench_f32.json > $O/kbench_f32.log 2>&1 || { tail -30 $O/kbench_f32.log; exit 1; }
cat $O/kbench_f32.log
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; tail -1 $O/bench_drv$i.log | cut -c1-200; done
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log | cut -c1-200
echo ALLDONE
