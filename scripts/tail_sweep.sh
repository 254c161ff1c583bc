# Sweep of the world-size-1 optimizer schedule (scripts/kbench.py, one process per setting since
# the launchers read the knobs once): each spec is "streamers:head[:reduce_w3]".
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() {  # env assignments..., then the kbench --only list
  echo "$* :: $(env "$@" timeout -k 10 60 python scripts/kbench.py ${KB_ARGS:-} --only "$JOBS" 2>/dev/null | grep ' us' | tr '\n' ' ')" | tee -a gpurun_out/sweep.log
}
JOBS=${JOBS:-conv2_bwd_adam+reduce_adam}
for spec in ${SWEEP:-"4:0.8:0.2"}; do
  IFS=: read -r sw hd rw <<< "$spec"
  run MIHVD_TAIL_STREAMERS=$sw MIHVD_TAIL_HEAD=$hd MIHVD_REDUCE_W3=${rw:-0} ${EXTRA:-}
done
# extra environment for every run: EXTRA="VAR=value ..."
