# Round 6, pass au: the rebuilt in-tree library (after the reverted factor experiments) at the final HEAD: factor / fp32 kernel tests, smoke().
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06au; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }; python3 -c "import json; [print('bench defaults', json.loads(l)['ms_per_step']*1000, json.loads(l)['steps'], json.loads(l)['warmup']) for l in open('$O/bench_default.log') if l.startswith('{')]"
echo ALLDONE
