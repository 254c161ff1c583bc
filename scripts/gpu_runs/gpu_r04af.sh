# Round 4, pass af: final HEAD evidence: whole GPU suite, driver-form benches, 400-step bench,
# rocprof trace (roofline), PMC of every step kernel.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04af; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  --durations=10 > $O/suite.log 2>&1
rc=$?
echo "suite rc=$rc"; grep -c PASSED $O/suite.log; grep -E "^FAILED|^ERROR" $O/suite.log | head -20; tail -2 $O/suite.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
python3 -c "import json; [print('400', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_400.log') if l.startswith('{')]"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
ONLY="conv1_fwd [+ W2 fragment copies],conv2_fwd [W2 fragment copy],conv2_bwd [W2 fragment copy],conv2_bwd [W2 fragment copy]:dg,fc1_fwd,head,fc1_bwd+W3 adam,conv_reduce+adam" timeout -k 10 300 bash scripts/pmc_r04.sh $O/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
echo ALLDONE
