# Round 6, pass ap: the driver form's outliers: 8 fresh processes, host bracket against the device
# span of the timed steps (events), both per step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06ap; mkdir -p $O
for i in 1 2 3 4 5 6 7 8; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --device-span > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('driver form host', json.loads(l)['ms_per_step']*1000, 'device', json.loads(l)['config']['device_ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
echo ALLDONE
