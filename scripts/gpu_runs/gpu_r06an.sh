# Round 6, pass an: the next batch gathered by fc1_bwd's small-reduction blocks (on CUs the row
# blocks leave free) instead of the head: fp32 tests, the plane tests, kernel times, the bench
# (driver form x3, 200 steps), kernel trace (in-step head / fc1_bwd / conv1).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06an; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py tests/test_fused_distributed_gpu.py -k "f32 or factor or switches or gathered or epoch or collectives_inside" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/kbench_f32.py --match "conv1|head|fc1_bwd+W3|whole" > $O/kbench.txt 2>&1 || { tail -20 $O/kbench.txt; exit 1; }
grep -v amdgpu.ids $O/kbench.txt
for i in 1 2 3; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('driver form', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }; python3 -c "import json; [print('200 steps', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench.log') if l.startswith('{')]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
echo ALLDONE
