# Round 4, pass x: XCD-aligned conv1 -> conv2_fwd block order: tests, kbench, benches (spin wait + lead graph).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04x; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_gpu.py > $O/t_f32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t_f32.log | tail -5; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --match "conv1|conv2_fwd|whole step (graph" > $O/kbench.log 2>&1 || { tail -30 $O/kbench.log; exit 1; }
cat $O/kbench.log
for i in 1 2 3 4; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
python3 -c "import json; [print('400', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_400.log') if l.startswith('{')]"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
echo ALLDONE
