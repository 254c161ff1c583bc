# Round 4, pass p: phase stamps (study build) of conv2_bwd with the W2 fragment copy, incl. the wgrad
# blocks' per-image ends, conv2_fwd and fc1_bwd.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04p; mkdir -p $O
MIHVD_F32_STAMPS=1 timeout -k 10 400 python -m mihvd._build kernels --force > $O/stamps_build.log 2>&1 || { tail -20 $O/stamps_build.log; exit 1; }
timeout -k 10 200 python scripts/stamps_f32.py > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
echo ALLDONE
