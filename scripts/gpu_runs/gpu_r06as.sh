# Round 6, pass as: bench.py at the final HEAD in the driver's form (no event records) and with
# --device-span.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06as; mkdir -p $O
for i in 1 2 3 4; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('driver form', json.loads(l)['ms_per_step']*1000, json.loads(l)['config']['device_ms_per_step']) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --device-span > $O/bench_span.log 2>&1 || { tail -20 $O/bench_span.log; exit 1; }; python3 -c "import json; [print('with span', json.loads(l)['ms_per_step']*1000, json.loads(l)['config']['device_ms_per_step']*1000) for l in open('$O/bench_span.log') if l.startswith('{')]"
echo ALLDONE
