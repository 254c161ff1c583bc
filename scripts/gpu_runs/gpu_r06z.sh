# Round 6, pass z: the next epoch order drawn ahead of the boundary (the driver form's timed region
# had a reshuffle between the lead graph and the long graph): fp32 tests, bench in the driver's form
# (4 fresh processes) and at 200 steps, kernel trace of the driver form.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py tests/test_f16_gpu.py > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3 4; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('driver form', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }; python3 -c "import json; [print('200 steps', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench.log') if l.startswith('{')]"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_drv -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_drv.log 2>&1 || { tail -30 $O/prof_drv.log; exit 1; }
echo ALLDONE
