# Round 4, pass h: the one-round fp32 conv2 backward (tests over all forms, kernel A/B, bench,
# profile + roofline inputs), then its stamps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04h; mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 500 $T tests/test_f32_gpu.py > $O/t_f32.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_f32.log | tail -50; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --json $O/kbench_f32.json > $O/kbench_f32.log 2>&1 || { tail -30 $O/kbench_f32.log; exit 1; }
cat $O/kbench_f32.log
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log | cut -c1-200
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-200
timeout -k 10 300 bash scripts/profile_bench.sh $O/prof > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -v "^W2026\|^E2026" $O/prof.log | tail -12
timeout -k 10 600 $T tests/test_fused_distributed_gpu.py -k "fp32" > $O/t_dist.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_dist.log | tail -30; [ $rc -ne 0 ] && { tail -40 $O/t_dist.log; exit $rc; }
MIHVD_STRESS_TRACE=1 MIHVD_STRESS_SYNC_EACH=1 timeout -k 10 300 python -u benchmarks/stress_models.py --model bert-base --batch-size 16 --steps 8 --warmup 3 --graph > $O/stress_bert_graph.log 2>&1 || { tail -20 $O/stress_bert_graph.log; exit 1; }
echo "stream-mismatch warnings: $(grep -c "AccumulateGrad node's stream" $O/stress_bert_graph.log)"; grep "per-step loss" $O/stress_bert_graph.log | cut -c1-300
timeout -k 10 400 $T tests/test_stress_gpu.py tests/test_kernels_gpu.py -k "stress or captured_step" > $O/t_graphs.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_graphs.log | tail -20; [ $rc -ne 0 ] && { tail -30 $O/t_graphs.log; exit $rc; }
MIHVD_F32_STAMPS=1 timeout -k 10 400 python -m mihvd._build kernels --force > $O/stamps_build.log 2>&1 || { tail -20 $O/stamps_build.log; exit 1; }
timeout -k 10 200 python scripts/stamps_f32.py > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
echo ALLDONE
