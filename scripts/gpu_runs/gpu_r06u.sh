# Round 6, pass u: HEAD kernel traces: the headline bench (roofline input) and the forced-collectives
# step at world 1 (csv), plus the bench in the driver's form.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fc -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_fc.log 2>&1 || { tail -30 $O/prof_fc.log; exit 1; }
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('driver form', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }; python3 -c "import json; [print('200 steps', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench.log') if l.startswith('{')]"
echo ALLDONE
