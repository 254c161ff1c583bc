# Round 5, pass aa: the bench's untimed setup replays before the driver's 20 timed steps
# (MIHVD_BENCH_SETUP_REPLAYS: 10 = default, 100, 400), fresh processes, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05aa; mkdir -p $O
for i in 1 2 3; do for k in 10 100 400; do
  MIHVD_BENCH_SETUP_REPLAYS=$k timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_s${k}_$i.log 2>&1 || { tail -20 $O/bench_s${k}_$i.log; exit 1; }
  python3 -c "import json; [print('setup=$k', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_s${k}_$i.log') if l.startswith('{')]"
done; done
echo ALLDONE
