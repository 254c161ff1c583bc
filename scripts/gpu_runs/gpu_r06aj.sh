# Round 6, pass aj: fp32 plane switches through the replicated factor plane (2 ranks, gloo, one GPU),
# and the factor-plane tests at the final HEAD.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06aj; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_fused_distributed_gpu.py -k "factor or switches" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "^FAILED|Error|assert" $O/tests.log | head -20; [ $rc -ne 0 ] && exit $rc
echo ALLDONE
