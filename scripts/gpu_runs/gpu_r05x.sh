# Round 5, pass x: in-kernel phase stamps (study build, MIHVD_F32_STAMPS=1) of conv2_bwd's two roles
# and of fc1_bwd at HEAD: where the non-MFMA time of the two largest launches goes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 200 python scripts/stamps_f32.py > $O/stamps.txt 2>&1 || { tail -30 $O/stamps.txt; exit 1; }
cat $O/stamps.txt
echo ALLDONE
