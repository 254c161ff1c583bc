# Round 4, pass b: the fc1 row kernel (dgrad + dW3 + fused dense/kernel Adam from one read of W3),
# conv1 fused into the conv2 forward, the W2 prefetch: every fp32 kernel/step test, per-kernel times,
# the headline bench, a kernel-trace profile, PMC passes, the BERT capture bisection, and the fp32
# multi-rank (gloo, one GPU) equivalence tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04b; mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_gpu.py > $O/t_f32.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_f32.log | tail -40; [ $rc -ne 0 ] && { tail -60 $O/t_f32.log; exit $rc; }
# fp16-operand kernel set (mixed_float16): a plain test failure (rc 1) does not stop the pass
timeout -k 10 300 $T tests/test_f16_gpu.py > $O/t_f16.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_f16.log | tail -20; [ $rc -ne 0 ] && tail -40 $O/t_f16.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python scripts/kbench_f32.py --json $O/kbench_f32.json > $O/kbench_f32.log 2>&1 || { tail -30 $O/kbench_f32.log; exit 1; }
cat $O/kbench_f32.log
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 300 bash scripts/profile_bench.sh $O/prof > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -16 $O/prof.log
timeout -k 10 400 bash scripts/pmc_r04.sh $O/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
tail -20 $O/pmc.log
# BERT-base capture bisection (round 4 variants): which op needs the held / synced warm-up
timeout -k 10 400 python -u scripts/bert_graph_bisect.py --variants C,H,C0,H0,S,P,N,L,M,Z --steps 6 --loss-only > $O/bert_bisect.log 2>&1
echo "bert bisect rc=$?"; grep "^{" $O/bert_bisect.log | cut -c1-200
timeout -k 10 600 $T tests/test_fused_distributed_gpu.py -k "fp32 and (4-fp32-0 or rehearsal_on_one_gpu\[2 or checkpoint)" > $O/t_dist_fp32.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_dist_fp32.log | tail -40; [ $rc -ne 0 ] && { tail -60 $O/t_dist_fp32.log; exit $rc; }
echo ALLDONE
