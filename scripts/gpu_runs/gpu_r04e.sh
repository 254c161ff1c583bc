# Round 4, pass e: XCD-contiguous conv2 wgrad blocks, fc1_bwd p/m/v prefetch depth 4, conv1-wgrad
# epilogue back on VALU; tests, kernel/whole-step studies, bench + profile; the BERT capture
# bisection with the replaced .grad tensors named; last, a stamps build (in this box's copy only)
# for per-phase cycle counts of the conv2 backward roles.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04e; mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_gpu.py > $O/t_f32.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_f32.log | tail -40; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --json $O/kbench_f32.json > $O/kbench_f32.log 2>&1 || { tail -30 $O/kbench_f32.log; exit 1; }
cat $O/kbench_f32.log
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 300 bash scripts/profile_bench.sh $O/prof > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -v "^W2026\|^E2026" $O/prof.log | tail -12
timeout -k 10 400 python -u scripts/bert_graph_bisect.py --variants C0,A0,N --steps 4 --loss-only --diag > $O/bert_bisect.log 2>&1
echo "bert bisect rc=$?"; grep "^{" $O/bert_bisect.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); k = list(d)[0]; v = d[k]
    print(k, 'loss', [round(x, 3) for x in v['loss']], 'replaced', v.get('n_grad_replaced'), v.get('grad_replaced'), v.get('replaced_example'))
"
MIHVD_F32_STAMPS=1 timeout -k 10 400 python -m mihvd._build kernels --force > $O/stamps_build.log 2>&1 || { tail -20 $O/stamps_build.log; exit 1; }
timeout -k 10 200 python scripts/stamps_f32.py > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
echo ALLDONE
