# Round 5, pass ak: the N > 1 fp32 step at world 1 (every collective forced on, direct-xGMI plane)
# under rocprofv3 at closing HEAD: per-kernel medians of the graph-replayed steps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05ak; mkdir -p $O
MIHVD_FORCE_COLLECTIVES=1 MIHVD_XGMI=on MIHVD_SHARD_W3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_xgmi -o run -- python3 bench.py --gpus 1 --steps 100 --warmup 10 > $O/prof_xgmi.log 2>&1 || { tail -30 $O/prof_xgmi.log; exit 1; }
python3 scripts/step_timeline.py $O/prof_xgmi > $O/timeline_xgmi.txt 2>&1; cat $O/timeline_xgmi.txt | head -30
grep '^{' $O/prof_xgmi.log | python3 -c "import json,sys; [print('forced xgmi under rocprof', json.loads(l)['ms_per_step']*1000) for l in sys.stdin]"
echo ALLDONE
