# Round 5, pass ao (study): conv1's launch time with a one-thread spin kernel (torch.cuda._sleep) before it
# (MIHVD_STUDY_SLEEP = spin cycles; -1 = the normal step): compute-idle, not memory-bound, under rocprofv3: does the kernel conv1
# follows (conv_reduce right behind the MFMA-heavy conv2_bwd) set its 7.1 us?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05ao; mkdir -p $O
for g in -1 1 20000 200000; do
  MIHVD_STUDY_SLEEP=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$g -o run -- python3 bench.py --gpus 1 --steps 100 --warmup 10 > $O/prof_bench$g.log 2>&1 || { tail -20 $O/prof_bench$g.log; exit 1; }
  echo "sleep ${g}"; python3 scripts/step_timeline.py $O/prof$g > $O/timeline$g.txt 2>&1; head -14 $O/timeline$g.txt
done
echo ALLDONE
