# Round 6, pass l: kernel times with the split-bf16 conv2_bwd dgrad role, then the fp32 suite and
# the bench (conv2_fwd + conv2_bwd dgrad on split products).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 200 python scripts/kbench_f32.py --match "conv2_bwd|conv2_fwd|whole" > $O/kbench.txt 2>&1 || { tail -20 $O/kbench.txt; exit 1; }
cat $O/kbench.txt
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py > $O/tests_f32.log 2>&1
rc=$?; tail -2 $O/tests_f32.log; grep -E "^FAILED|^ERROR" $O/tests_f32.log | head -20; [ $rc -ne 0 ] && exit $rc
for m in 6 0; do MIHVD_F32_PRODUCTS=$m timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_p$m.log 2>&1 || { tail -20 $O/bench_p$m.log; exit 1; }; python3 -c "import json; [print('products $m', json.loads(l)['ms_per_step']*1000, json.loads(l)['value']) for l in open('$O/bench_p$m.log') if l.startswith('{')]"; done
echo ALLDONE
