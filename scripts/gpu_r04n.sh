# Round 4, pass n: the fp32 factor-gather plane (dgrad-only fc1_bwd, RCCL all-to-all, world-1 capture,
# 4/8-rank gloo equivalence) and the exact-batch fc1 wgrad chain; kbench of the new launches.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04n; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_f32_gpu.py -k "fc1_bwd" > $O/t_f32_fc1.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t_f32_fc1.log | tail -8; [ $rc -ne 0 ] && { tail -40 $O/t_f32_fc1.log; exit $rc; }
timeout -k 10 300 $T tests/test_native_comm_gpu.py -k rccl_comm > $O/t_ncomm.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t_ncomm.log | tail -4; [ $rc -ne 0 ] && { tail -40 $O/t_ncomm.log; exit $rc; }
timeout -k 10 900 $T tests/test_fused_distributed_gpu.py -k "factor or (collectives_inside and fp32) or (equivalence_n_ranks and fp32)" > $O/t_dist.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t_dist.log | tail -14; [ $rc -ne 0 ] && { tail -60 $O/t_dist.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --match "fc1|factor|whole step (graph|padded" > $O/kbench.log 2>&1 || { tail -30 $O/kbench.log; exit 1; }
cat $O/kbench.log
echo ALLDONE
