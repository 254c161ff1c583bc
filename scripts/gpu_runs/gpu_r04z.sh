# Round 4, pass z: the bench-driving GPU tests after the host-wait fix, then driver-form benches.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04z; mkdir -p $O
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_fused_distributed_gpu.py -k "rehearsal or bench_flow" tests/test_examples_gpu.py tests/test_native_comm_gpu.py > $O/t_bench.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t_bench.log | tail -20; [ $rc -ne 0 ] && { grep -B5 -A30 "Traceback" $O/t_bench.log | head -80; exit $rc; }
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
echo ALLDONE
