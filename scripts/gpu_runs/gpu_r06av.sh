# Round 6, pass av: the whole GPU suite and smoke() with the final in-tree library (rebuilt after the reverted experiments
# ), the bench in the driver's form.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06av; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider --durations=15 > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -c PASSED $O/suite.log; grep -E "^FAILED|^ERROR" $O/suite.log | head -30; tail -1 $O/suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2 3; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('driver form', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
echo ALLDONE
