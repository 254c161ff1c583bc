# fp32 iteration + conv2_bwd phase stamps
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_f32_iter.sh || exit $?
timeout -k 10 120 python scripts/stamps_f32.py > gpurun_out/stamps.log 2>&1 || exit $?
cat gpurun_out/stamps.log
