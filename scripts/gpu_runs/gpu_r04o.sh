# Round 4, pass o: the whole GPU suite at HEAD (one process, per-test timeouts, every failure listed).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SUITE_OUT:-r04o}; mkdir -p $O
timeout -k 10 1080 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  --durations=20 > $O/suite.log 2>&1
rc=$?
echo "suite rc=$rc"
grep -c PASSED $O/suite.log
grep -E "FAILED|ERROR" $O/suite.log | head -30
tail -30 $O/suite.log
