# Round 5, pass q: bench with the communicator barrier (forced collectives at world 1), driver form,
# smoke, fp32 tests at HEAD.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_fc.log 2>&1 || { tail -30 $O/bench_fc.log; exit 1; }
python3 -c "import json; [print('forced', json.loads(l)['ms_per_step']*1000, json.loads(l)['config'].get('data_plane',{}).get('plane'), json.loads(l)['config'].get('rccl_nranks')) for l in open('$O/bench_fc.log') if l.startswith('{')]"
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
echo ALLDONE
