# fp32 step on one MI355X: kernel numerics, a short bench, per-kernel times under rocprofv3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_f32_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/f32t.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > gpurun_out/f32b.log 2>&1 || exit $?
echo "bench ok"; tail -1 gpurun_out/f32b.log
timeout -k 10 200 python bench.py --steps 400 --warmup 40 --precision bf16 > gpurun_out/bf16b.log 2>&1 || exit $?
tail -1 gpurun_out/bf16b.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f32 -o run -- python bench.py --steps 200 --warmup 20 > gpurun_out/prof_f32.log 2>&1 || exit $?
echo "prof ok"
timeout -k 10 200 python scripts/kbench_f32.py --json gpurun_out/kbench_f32.json > gpurun_out/kbench_f32.log 2>&1 || exit $?
cat gpurun_out/kbench_f32.log
