# Round 4, pass d: wgrad software pipeline in f32_conv2_bwd, conv1 as its own launch by default,
# the fp16 tests at measured tolerances, kernel/whole-step studies, the headline bench + profile, and
# the BERT capture bisection's follow-ups (A0/T0/R0/B0 from the failing form C0).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04d; mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_f32_gpu.py -k "conv2_bwd or step_matches or dropout or trajectory" > $O/t_f32.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_f32.log | tail -20; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 300 $T -s tests/test_f16_gpu.py > $O/t_f16.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|rel err" $O/t_f16.log | tail -20; [ $rc -ne 0 ] && tail -30 $O/t_f16.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python scripts/kbench_f32.py --json $O/kbench_f32.json > $O/kbench_f32.log 2>&1 || { tail -30 $O/kbench_f32.log; exit 1; }
cat $O/kbench_f32.log
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 300 bash scripts/profile_bench.sh $O/prof > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -v "^W2026\|^E2026" $O/prof.log | tail -12
timeout -k 10 600 python -u scripts/bert_graph_bisect.py --variants A0,T0,R0,B0 --steps 5 --loss-only --diag > $O/bert_bisect.log 2>&1
echo "bert bisect rc=$?"; grep "^{" $O/bert_bisect.log | cut -c1-300
echo ALLDONE
