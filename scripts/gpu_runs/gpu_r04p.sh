# Round 4, pass p: kbench of fc1_bwd (dz swizzle) and the factor kernel, then phase stamps (study build) of conv2_bwd with the W2 fragment copy, incl. the wgrad
# blocks' per-image ends, conv2_fwd and fc1_bwd.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04p; mkdir -p $O
timeout -k 10 300 python scripts/kbench_f32.py --match "fc1_bwd|whole step (graph|factor" > $O/kbench.log 2>&1 || { tail -30 $O/kbench.log; exit 1; }
cat $O/kbench.log
MIHVD_F32_STAMPS=1 timeout -k 10 400 python -m mihvd._build kernels --force > $O/stamps_build.log 2>&1 || { tail -20 $O/stamps_build.log; exit 1; }
timeout -k 10 200 python scripts/stamps_f32.py > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
echo ALLDONE
