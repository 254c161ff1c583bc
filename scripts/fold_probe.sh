# Timing probe of the folded reduction (conv2_bwd_adam_fold): MIHVD_FOLD_DEBUG cuts it after the
# write-through stores (3), skips the wait (2) or the items (1); 0 = complete.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for d in 0 3 1 2; do
  echo "fold_debug=$d :: $(MIHVD_FOLD_DEBUG=$d timeout -k 10 60 python scripts/kbench.py --only 'conv2_bwd_adam_fold;conv2_bwd_adam' 2>/dev/null | grep ' us' | tr '\n' ' ')"
done
