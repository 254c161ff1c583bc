# Round 4, pass r: the 8-wave conv2_fwd (tests, kbench A/B, whole step) and the fp32 factor plane on
# the library GEMM (capture + 4/8-rank equivalence).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04r; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_gpu.py -k "conv2_fwd or conv12 or w2_frag or step_matches or conv2_bwd" > $O/t_f32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t_f32.log | tail -5; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 400 $T tests/test_fused_distributed_gpu.py -k "factor" > $O/t_dist.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t_dist.log | tail -6; [ $rc -ne 0 ] && { tail -60 $O/t_dist.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --match "conv2_fwd|whole step (graph|8 waves" > $O/kbench.log 2>&1 || { tail -30 $O/kbench.log; exit 1; }
cat $O/kbench.log
echo ALLDONE
