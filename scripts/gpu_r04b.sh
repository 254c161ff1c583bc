# Round 4, pass b: the fc1 row kernel (dgrad + dW3 + fused dense/kernel Adam from one read of W3):
# every fp32 kernel/step test, the fp32 multi-rank (gloo, one GPU) equivalence tests, per-kernel
# times, the headline bench and a kernel-trace profile.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04b; mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 500 $T tests/test_f32_gpu.py > $O/t_f32.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_f32.log | tail -40; [ $rc -ne 0 ] && { tail -60 $O/t_f32.log; exit $rc; }
timeout -k 10 200 python scripts/kbench_f32.py --json $O/kbench_f32.json > $O/kbench_f32.log 2>&1 || { tail -30 $O/kbench_f32.log; exit 1; }
cat $O/kbench_f32.log
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 300 bash scripts/profile_bench.sh $O/prof > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -16 $O/prof.log
timeout -k 10 900 $T tests/test_fused_distributed_gpu.py -k "fp32" > $O/t_dist_fp32.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_dist_fp32.log | tail -40; [ $rc -ne 0 ] && { tail -60 $O/t_dist_fp32.log; exit $rc; }
echo ALLDONE
