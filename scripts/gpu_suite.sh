# the whole GPU test suite in one process (per-test timeout; no -x so every failure is listed)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1080 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  --durations=15 > gpurun_out/suite.log 2>&1
rc=$?
echo "suite rc=$rc"
grep -E "PASSED|FAILED|ERROR" gpurun_out/suite.log | grep -c PASSED
grep -E "FAILED|ERROR" gpurun_out/suite.log | head -30
tail -25 gpurun_out/suite.log
