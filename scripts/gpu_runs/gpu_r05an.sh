# Round 5, pass an (final HEAD check: the conv1 study knob reverted, tests added): the whole GPU suite, smoke, bench in the driver's form and at the
# default length, the forced-collectives (N > 1 step at world 1) bench, and a kernel trace of the
# default bench for the roofline / kernel-stats profiles.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05an; mkdir -p $O
t0=$(date +%s)
timeout -k 10 800 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu tests \
  --durations=15 > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc in $(( $(date +%s) - t0 )) s"; grep -c PASSED $O/suite.log; grep -E "^FAILED|^ERROR" $O/suite.log | head; tail -1 $O/suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
for i in 1 2 3; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
python3 -c "import json; [print('default', json.loads(l)['ms_per_step']*1000, json.loads(l)['value']) for l in open('$O/bench_default.log') if l.startswith('{')]"
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_fc.log 2>&1 || { tail -30 $O/bench_fc.log; exit 1; }
python3 -c "import json; [print('forced', json.loads(l)['ms_per_step']*1000, json.loads(l)['config'].get('data_plane')) for l in open('$O/bench_fc.log') if l.startswith('{')]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
python3 scripts/roofline_f32.py $O/prof/run_kernel_trace.csv $O/prof_bench.log --stats $O/kernel_stats.txt > $O/roofline.md && sed -n 5,16p $O/roofline.md
echo ALLDONE
