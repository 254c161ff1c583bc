# Round 5, pass d: the split-form xGMI data launch with up to 4 blocks per CU and p/m/v loaded with
# the gradients. xGMI tests (one-GPU multi-rank), capture tests, the forced-collectives bench with
# plane selection and a kernel trace of the world-1 xGMI step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_xgmi_gpu.py tests/test_fused_distributed_gpu.py -k "xgmi or hip_graph" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -c PASSED $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head; tail -2 $O/tests.log
[ $rc -ne 0 ] && exit $rc
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_fc.log 2>&1 || { tail -30 $O/bench_fc.log; exit 1; }
python3 -c "import json; [print('forced', json.loads(l)['ms_per_step']*1000, json.loads(l)['config'].get('data_plane')) for l in open('$O/bench_fc.log') if l.startswith('{')]"
MIHVD_FORCE_COLLECTIVES=1 MIHVD_XGMI=on MIHVD_SHARD_W3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_xgmi -o run -- python3 bench.py --gpus 1 --steps 100 --warmup 10 > $O/prof_xgmi.log 2>&1 || { tail -30 $O/prof_xgmi.log; exit 1; }
python3 scripts/step_timeline.py $O/prof_xgmi
echo ALLDONE
