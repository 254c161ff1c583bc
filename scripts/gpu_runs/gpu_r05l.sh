# Round 5, pass l: conv2 dgrad image by LDS-DMA (study form): fp32 tests and the A/B timings.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_f32_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -c PASSED $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head; tail -1 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/kbench_f32.py --match "conv2_bwd [W2 fragment copy]|dgrad image by LDS-DMA|dgrad role only, W2|dgrad role only, image|whole step (graph" > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep -v "^#" $O/kbench.log | tail -8
echo ALLDONE
