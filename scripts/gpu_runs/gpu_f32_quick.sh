# fp32 kernel iteration: the fp32 kernel tests, per-kernel times, a short bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_f32_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/f32t.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/f32t.log | tail -30; tail -3 gpurun_out/f32t.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python scripts/kbench_f32.py --json gpurun_out/kbench_f32.json > gpurun_out/kbench_f32.log 2>&1 || exit $?
cat gpurun_out/kbench_f32.log
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > gpurun_out/f32b.log 2>&1 || exit $?
tail -1 gpurun_out/f32b.log
