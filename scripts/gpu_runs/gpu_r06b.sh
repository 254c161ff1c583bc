# Round 6, pass b: the fp32 xGMI plane's row gather co-launched in the next step's conv1 (phase
# entry at world 1 too); the distributed GPU tests (split and co-launch forms), then the benches.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py tests/test_fused_distributed_gpu.py tests/test_xgmi_gpu.py tests/test_native_comm_gpu.py --durations=10 > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_fc.log 2>&1 || { tail -30 $O/bench_fc.log; exit 1; }
python3 -c "import json; [print('forced', json.loads(l)['ms_per_step']*1000, json.loads(l)['config'].get('data_plane')) for l in open('$O/bench_fc.log') if l.startswith('{')]"
echo ALLDONE
