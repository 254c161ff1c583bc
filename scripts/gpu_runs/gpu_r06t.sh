# Round 6, pass t: fc1_bwd dgrad on split-bf16 products over chunk pairs: numerics, the fp32 suite and
# the Keras example tests, kernel times, the bench (200 steps, driver form), the forced collectives
# step at world 1, and a rocprofv3 kernel trace (csv) of the bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 500 python -u -m pytest -v -s --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_f32_split_gpu.py tests/test_f32_gpu.py tests/test_examples_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "fc1_bwd d|fc1_bwd db|^FAILED|^ERROR" $O/tests.log | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/kbench_f32.py > $O/kbench.txt 2>&1 || { tail -20 $O/kbench.txt; exit 1; }
cat $O/kbench.txt | grep -E "fc1_bwd|whole"
for m in 6 6; do timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_p$m.log 2>&1 || { tail -20 $O/bench_p$m.log; exit 1; }; python3 -c "import json; [print('products $m', json.loads(l)['ms_per_step']*1000, json.loads(l)['value']) for l in open('$O/bench_p$m.log') if l.startswith('{')]"; done
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('driver form', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_fc.log 2>&1 || { tail -30 $O/bench_fc.log; exit 1; }
python3 -c "import json; [print('forced', json.loads(l)['ms_per_step']*1000, json.loads(l)['config'].get('data_plane')) for l in open('$O/bench_fc.log') if l.startswith('{')]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
echo ALLDONE
