# Round 5, pass e: conv2_fwd W2 loads before the staging barrier, fc1_bwd LDS-only exchange barriers
# with the routing operands prefetched, conv2 wgrad store-spread start. fp32 kernel tests, A/B
# kernel timings, driver-form bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_f32_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -c PASSED $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head; tail -2 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python scripts/kbench_f32.py --match "conv2_fwd|conv2_bwd [W2|conv2_bwd [wgrad next|fc1_bwd+W3 adam|whole step" > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep -v "^#" $O/kbench.log | tail -30
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
echo ALLDONE
