# Round 4, pass g: fc1_bwd row kernel with its LDS operands read ahead of the MFMAs (pinned order,
# four wgrad chains); CapturedStep back on torch's capture stream (A0 form); the BERT bisection's
# capture-time diagnostic (which gradients a capture changed = work that ran eagerly); stamps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04g; mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_gpu.py -k "fc1_bwd or step_matches or fused_optimizer or trajectory" > $O/t_f32.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_f32.log | tail -20; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --json $O/kbench_f32.json > $O/kbench_f32.log 2>&1 || { tail -30 $O/kbench_f32.log; exit 1; }
grep -E "^fc1_bwd|^conv2_bwd  |whole step" $O/kbench_f32.log
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log | cut -c1-200
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-200
timeout -k 10 500 python -u scripts/bert_graph_bisect.py --variants C0,A0,AR --steps 4 --loss-only --diag > $O/bert_bisect.log 2>&1
echo "bert bisect rc=$?"; grep "^{" $O/bert_bisect.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); k = list(d)[0]; v = d[k]
    print(k, 'loss', [round(x, 3) for x in v['loss']], 'changed by capture: grads', v.get('n_grads_changed_by_capture'), v.get('grads_changed_by_capture'), 'params', v.get('n_params_changed_by_capture'))
"
MIHVD_STRESS_TRACE=1 MIHVD_STRESS_SYNC_EACH=1 timeout -k 10 300 python -u benchmarks/stress_models.py --model bert-base --batch-size 16 --steps 8 --warmup 3 --graph > $O/stress_bert_graph.log 2>&1 || { tail -20 $O/stress_bert_graph.log; exit 1; }
grep -c "AccumulateGrad node's stream" $O/stress_bert_graph.log; grep "per-step loss" $O/stress_bert_graph.log | cut -c1-300; tail -1 $O/stress_bert_graph.log | cut -c1-200
timeout -k 10 400 $T tests/test_stress_gpu.py tests/test_kernels_gpu.py -k "stress or captured_step" > $O/t_graphs.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_graphs.log | tail -20; [ $rc -ne 0 ] && { tail -30 $O/t_graphs.log; exit $rc; }
MIHVD_F32_STAMPS=1 timeout -k 10 400 python -m mihvd._build kernels --force > $O/stamps_build.log 2>&1 || { tail -20 $O/stamps_build.log; exit 1; }
timeout -k 10 200 python scripts/stamps_f32.py > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
echo ALLDONE
