# Round 6, pass s: the whole GPU suite at HEAD (split-bf16 fp32 products by default), the forced
# collectives step at world 1, and a rocprofv3 kernel trace of the driver-form bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider --durations=15 > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -c PASSED $O/suite.log; grep -E "^FAILED|^ERROR" $O/suite.log | head -30; tail -3 $O/suite.log
[ $rc -ne 0 ] && exit $rc
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_fc.log 2>&1 || { tail -30 $O/bench_fc.log; exit 1; }
python3 -c "import json; [print('forced', json.loads(l)['ms_per_step']*1000, json.loads(l)['config'].get('data_plane')) for l in open('$O/bench_fc.log') if l.startswith('{')]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
echo ALLDONE
