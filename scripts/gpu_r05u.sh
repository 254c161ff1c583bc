# Round 5, pass u: where the head-inside-fc1_bwd launch loses its time (pass t: 46 us against
# 27 + 4.8): the device-scope fences of its grid wait. MIHVD_F32_HEAD_FENCE = 3 (release + acquire,
# the correct form), 1 (release only), 2 (acquire only), 0 (none) -- the last three are timing
# studies only (stale reads possible); MIHVD_F32_HEAD_IN_F1B=0 is the separate head launch.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 200 python bench.py > $O/bench_sep.log 2>&1 || { tail -20 $O/bench_sep.log; exit 1; }
for k in 3 1 2 0; do
  MIHVD_F32_HEAD_IN_F1B=1 MIHVD_F32_HEAD_FENCE=$k timeout -k 10 200 python bench.py > $O/bench_f$k.log 2>&1 || { tail -20 $O/bench_f$k.log; exit 1; }
done
MIHVD_F32_HEAD_IN_F1B=0 timeout -k 10 200 python bench.py > $O/bench_sep2.log 2>&1 || { tail -20 $O/bench_sep2.log; exit 1; }
for f in sep f3 f1 f2 f0 sep2; do python3 -c "import json; [print('$f', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_$f.log') if l.startswith('{')]"; done
echo ALLDONE
