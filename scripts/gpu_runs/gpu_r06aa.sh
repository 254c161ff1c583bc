# Round 6, pass aa: the driver form's lead graph (2 steps left a ~30 us bubble before the long
# graph in the timed region): lead 2 / 3 / 4 / 6, fresh processes; the replicated factor plane with
# its all-gathers on the compute stream at forced world 1 (bench + kernel trace).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06aa; mkdir -p $O
for rep in 1 2; do for lead in 2 3 4 6; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --lead-steps $lead > $O/bench_lead${lead}_$rep.log 2>&1 || { tail -20 $O/bench_lead${lead}_$rep.log; exit 1; }
  python3 -c "import json; [print('driver form lead $lead', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_lead${lead}_$rep.log') if l.startswith('{')]"
done; done
MIHVD_FORCE_COLLECTIVES=1 MIHVD_F32_PLANE=factor_rep MIHVD_SHARD_W3=0 timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_frep.log 2>&1 || { tail -20 $O/bench_frep.log; exit 1; }
python3 -c "import json; [print('forced factor_rep (serial) 200 steps', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_frep.log') if l.startswith('{')]"
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_fused_distributed_gpu.py -k "factor_rep" > $O/tests_factor.log 2>&1
rc=$?; tail -1 $O/tests_factor.log; grep -E "^FAILED|Error" $O/tests_factor.log | head; [ $rc -ne 0 ] && exit $rc
MIHVD_FORCE_COLLECTIVES=1 MIHVD_F32_PLANE=factor_rep MIHVD_SHARD_W3=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_frep -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_frep.log 2>&1 || { tail -30 $O/prof_frep.log; exit 1; }
echo ALLDONE
