# Round 4, pass w: host wait mode of the timed region's synchronize (HIP default vs spin), driver form,
# interleaved fresh processes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04w; mkdir -p $O
for i in 1 2 3 4; do
  for m in auto spin; do
    MIHVD_SYNC_WAIT=$m timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${m}_$i.log 2>&1 || { tail -20 $O/bench_${m}_$i.log; exit 1; }
    python3 -c "import json; [print('$m', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_${m}_$i.log') if l.startswith('{')]"
  done
done
echo ALLDONE
