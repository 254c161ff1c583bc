# Round 5, pass b: the fp32 direct-xGMI plane + the pruned C++ forms. GPU tests of the changed paths,
# driver-form bench, forced-collectives (world-1) bench with plane selection, and kernel traces of the
# world-1 forced step on the xGMI plane and on the RCCL reduce-scatter plane.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1  # run the libraries built in the container, never a rebuild on the box
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  ${TESTS:-tests/test_f32_gpu.py tests/test_fused_distributed_gpu.py tests/test_native_comm_gpu.py tests/test_kernels_gpu.py} \
  > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -c PASSED $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head -20; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000, json.loads(l)['config'].get('rccl_nranks')) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_fc.log 2>&1 || { tail -30 $O/bench_fc.log; exit 1; }
python3 -c "import json; [print('forced', json.loads(l)['ms_per_step']*1000, json.loads(l)['config'].get('data_plane')) for l in open('$O/bench_fc.log') if l.startswith('{')]"
MIHVD_FORCE_COLLECTIVES=1 MIHVD_XGMI=on MIHVD_SHARD_W3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_xgmi -o run -- python3 bench.py --gpus 1 --steps 100 --warmup 10 > $O/prof_xgmi.log 2>&1 || { tail -30 $O/prof_xgmi.log; exit 1; }
MIHVD_FORCE_COLLECTIVES=1 MIHVD_XGMI=off MIHVD_F32_PLANE=rs MIHVD_SHARD_W3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rs -o run -- python3 bench.py --gpus 1 --steps 100 --warmup 10 > $O/prof_rs.log 2>&1 || { tail -30 $O/prof_rs.log; exit 1; }
echo ALLDONE
