# Round 6, pass r: both conv2_bwd roles on split-bf16 products (10-tile dgrad blocks): numerics, fp32
# suite, kernel times, bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_split_gpu.py > $O/tests_split.log 2>&1
rc=$?; tail -2 $O/tests_split.log; grep -E "^FAILED|Error" $O/tests_split.log | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py > $O/tests_f32.log 2>&1
rc=$?; tail -2 $O/tests_f32.log; grep -E "^FAILED|^ERROR" $O/tests_f32.log | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/kbench_f32.py > $O/kbench.txt 2>&1 || { tail -20 $O/kbench.txt; exit 1; }
cat $O/kbench.txt
for m in 6 0 6; do MIHVD_F32_PRODUCTS=$m timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_p$m.log 2>&1 || { tail -20 $O/bench_p$m.log; exit 1; }; python3 -c "import json; [print('products $m', json.loads(l)['ms_per_step']*1000, json.loads(l)['value']) for l in open('$O/bench_p$m.log') if l.startswith('{')]"; done
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv.log 2>&1 || { tail -20 $O/bench_drv.log; exit 1; }
python3 -c "import json; [print('driver form', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv.log') if l.startswith('{')]"
echo ALLDONE
