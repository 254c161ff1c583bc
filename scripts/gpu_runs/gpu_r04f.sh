# Round 4, pass f: CapturedStep holding the AccumulateGrad nodes (the BERT-base capture fix) —
# bisection variants C0/A0/AR/F0, the stress bench eager vs --graph (per-step losses, the autograd
# stream-mismatch warning), the CapturedStep GPU tests; fc1_bwd / conv2 stamps; fp32 tests + bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04f; mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 500 python -u scripts/bert_graph_bisect.py --variants C0,A0,AR,F0 --steps 5 --loss-only --diag > $O/bert_bisect.log 2>&1
echo "bert bisect rc=$?"; grep "^{" $O/bert_bisect.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); k = list(d)[0]; v = d[k]
    print(k, 'loss', [round(x, 3) for x in v['loss']], 'bad grads', [x['n_grad'] for x in v.get('diag', [])])
"
for mode in eager graph; do
  G=""; [ $mode = graph ] && G="--graph"
  MIHVD_STRESS_TRACE=1 MIHVD_STRESS_SYNC_EACH=1 timeout -k 10 300 python -u benchmarks/stress_models.py --model bert-base --batch-size 16 --steps 8 --warmup 3 $G > $O/stress_bert_$mode.log 2>&1 || { tail -20 $O/stress_bert_$mode.log; exit 1; }
  grep -c "AccumulateGrad node's stream" $O/stress_bert_$mode.log; grep "per-step loss" $O/stress_bert_$mode.log | cut -c1-400; tail -1 $O/stress_bert_$mode.log | cut -c1-200
done
timeout -k 10 400 $T tests/test_kernels_gpu.py -k "captured_step" > $O/t_graphs.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_graphs.log | tail -20; [ $rc -ne 0 ] && { tail -40 $O/t_graphs.log; exit $rc; }
timeout -k 10 400 $T tests/test_stress_gpu.py > $O/t_stress.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_stress.log | tail -20; [ $rc -ne 0 ] && { tail -40 $O/t_stress.log; exit $rc; }
timeout -k 10 400 $T tests/test_f32_gpu.py -k "fc1_bwd or step_matches or fused_optimizer" > $O/t_f32.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_f32.log | tail -20; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log | cut -c1-200
MIHVD_F32_STAMPS=1 timeout -k 10 400 python -m mihvd._build kernels --force > $O/stamps_build.log 2>&1 || { tail -20 $O/stamps_build.log; exit 1; }
timeout -k 10 200 python scripts/stamps_f32.py > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
echo ALLDONE
