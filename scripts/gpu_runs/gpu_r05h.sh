# Round 5, pass h: the whole GPU suite at HEAD with per-test durations (xGMI collectives in the
# split form when ranks share the GPU), then the fc1_bwd routing-prefetch A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05h; mkdir -p $O
t0=$(date +%s)
timeout -k 10 900 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu tests \
  --durations=40 > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc in $(( $(date +%s) - t0 )) s"; grep -c PASSED $O/suite.log; grep -E "^FAILED|^ERROR" $O/suite.log | head; tail -2 $O/suite.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python scripts/kbench_f32.py --match "fc1_bwd+W3 adam|whole step (graph|whole step [fc1_bwd routing" > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep -v "^#" $O/kbench.log | tail -12
echo ALLDONE
