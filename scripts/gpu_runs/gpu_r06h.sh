# Round 6, pass h: split-bf16 x6 conv2_fwd in the fp32 step: fp32 suite + split numerics, then the
# bench (driver form, 200 steps) with x6 and with the fp32-input MFMA form.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v -s --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_split_gpu.py tests/test_f32_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head -20; [ $rc -ne 0 ] && exit $rc
for m in 6 0 6 0; do MIHVD_F32_PRODUCTS=$m timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_p$m.log 2>&1 || { tail -20 $O/bench_p$m.log; exit 1; }; python3 -c "import json; [print('products $m', json.loads(l)['ms_per_step']*1000, json.loads(l)['value'], json.loads(l)['config']['final_loss']) for l in open('$O/bench_p$m.log') if l.startswith('{')]"; done
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv.log 2>&1 || { tail -20 $O/bench_drv.log; exit 1; }
python3 -c "import json; [print('driver form', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv.log') if l.startswith('{')]"
echo ALLDONE
