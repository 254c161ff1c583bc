# fp32 iteration + the native RCCL communicator test
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_f32_iter.sh || exit $?
timeout -k 10 200 python -u -m pytest tests/test_native_comm_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/ncomm.log 2>&1
echo "ncomm rc=$?"; tail -30 gpurun_out/ncomm.log
