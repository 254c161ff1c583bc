# Sweep of the conv2_bwd optimizer tail: streamer waves per conv block x head fraction
# (scripts/kbench.py, one process per setting since the launcher reads the knobs once).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() {  # env assignments..., then the kbench --only list
  echo "$* :: $(env "$@" timeout -k 10 60 python scripts/kbench.py ${KB_ARGS:-} --only "$JOBS" 2>/dev/null | grep ' us' | tr '\n' ' ')" | tee -a gpurun_out/sweep.log
}
JOBS=${JOBS:-conv2_bwd_adam+reduce_adam}
for spec in ${SWEEP:-"4:0.0 4:0.4 4:1.0"}; do
  run MIHVD_TAIL_STREAMERS=${spec%%:*} MIHVD_TAIL_HEAD=${spec##*:}
done
