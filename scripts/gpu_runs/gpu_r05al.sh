# Round 5, pass al: the driver's form (--steps 20 --warmup 5) with a lead graph of 1, 2 (default)
# or 3 steps, fresh processes, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05al; mkdir -p $O
for i in 1 2 3; do for k in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --lead-steps $k > $O/bench_l${k}_$i.log 2>&1 || { tail -20 $O/bench_l${k}_$i.log; exit 1; }
  python3 -c "import json; [print('lead=$k', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_l${k}_$i.log') if l.startswith('{')]"
done; done
echo ALLDONE
