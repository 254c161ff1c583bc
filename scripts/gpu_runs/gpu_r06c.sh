# Round 6, pass c: the graph-replayed mixed_float16 step (fused fp16 trainer, device loss scaler),
# the API-routing test fix, then the benches (driver form, forced collectives, fp16) and a kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_f16_gpu.py "tests/test_native_comm_gpu.py::test_bucket_plane_carries_distributed_optimizer" --durations=10 > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000, json.loads(l)['value']) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_fc.log 2>&1 || { tail -30 $O/bench_fc.log; exit 1; }
python3 -c "import json; [print('forced', json.loads(l)['ms_per_step']*1000, json.loads(l)['config'].get('data_plane')) for l in open('$O/bench_fc.log') if l.startswith('{')]"
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 --precision fp16 > $O/bench_f16.log 2>&1 || { tail -30 $O/bench_f16.log; exit 1; }
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 --precision bf16 > $O/bench_bf16.log 2>&1 || { tail -30 $O/bench_bf16.log; exit 1; }
python3 -c "import json; [print(f, json.loads(l)['ms_per_step']*1000, json.loads(l)['value']) for f in ('$O/bench_f16.log','$O/bench_bf16.log') for l in open(f) if l.startswith('{')]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
echo ALLDONE
