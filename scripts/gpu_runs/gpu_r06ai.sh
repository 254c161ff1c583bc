# Round 6, pass ai: the driver form's run-to-run spread (one run in three or four ~3 us/step slower):
# Python GC off in the timed region (no collection in front of it), 6 fresh processes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06ai; mkdir -p $O
for rep in 1 2 3 4 5 6; do for lead in 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --lead-steps $lead > $O/bench_lead${lead}_$rep.log 2>&1 || { tail -20 $O/bench_lead${lead}_$rep.log; exit 1; }
  python3 -c "import json; [print('driver form lead $lead', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_lead${lead}_$rep.log') if l.startswith('{')]"
done; done
echo ALLDONE
