# Round 4, pass u: the fixed cost of the driver's 20-step timed region (graph split schedules).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 400 python scripts/launch_probe.py > $O/launch_probe.log 2>&1 || { tail -30 $O/launch_probe.log; exit 1; }
cat $O/launch_probe.log
echo ALLDONE
