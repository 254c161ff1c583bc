timeout -k 10 400 python -u -m pytest tests/test_f32_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/f32t.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/f32b.log 2>&1; echo "bench rc=$?"
fi
