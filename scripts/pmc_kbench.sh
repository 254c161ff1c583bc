#!/bin/bash
# LDS / wait-state PMC counters per fused-step kernel, one kernel per graph (scripts/kbench.py).
# Counters are collected in runs of their own (never combined with trace domains), each pass
# under its own time limit.
set -eu
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=${1:-gpurun_out/pmc_k}
rm -rf "$out"
only="conv1_fwd;conv2_fwd;fc1_fwd;head;fc1_wgrad;fc1_dgrad;conv2_bwd;conv2_wgrad_reduce;conv2_bwd_adam+reduce_adam;adam"
pass() {
  local dir=$1
  shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$out/$dir" -o run -- \
    python3 scripts/kbench.py --iters 20 --only "$only"
}
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
pass b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS
pass c SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE
python3 scripts/pmc_summary.py "$out" SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_INSTS_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE
