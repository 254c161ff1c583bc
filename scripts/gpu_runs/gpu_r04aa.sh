# Round 4, pass aa: does the fresh-process timed region depend on how long the GPU has been busy
# before it (setup replays 1 vs 10), driver form, interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04aa; mkdir -p $O
for i in 1 2 3; do
  for r in 1 10; do
    MIHVD_BENCH_SETUP_REPLAYS=$r timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${r}_$i.log 2>&1 || { tail -20 $O/bench_${r}_$i.log; exit 1; }
    python3 -c "import json; [print('setup$r', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_${r}_$i.log') if l.startswith('{')]"
  done
done
echo ALLDONE
