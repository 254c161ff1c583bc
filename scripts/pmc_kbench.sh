#!/bin/bash
# LDS / wait-state PMC counters per fused-step kernel, one kernel per graph (scripts/kbench.py).
# Counters are collected in runs of their own (never combined with trace domains).
set -eu
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=${1:-gpurun_out/pmc_k}
rm -rf "$out"
args="scripts/kbench.py --iters 20 --roles --only conv1_fwd,conv2_fwd,fc1_fwd,head,fc1_wgrad,fc1_dgrad,conv2_bwd,conv2_bwd[role0],conv2_bwd[role1],conv2_wgrad_reduce,adam"
rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d "$out/a" -o run -- python3 $args
rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS \
  --output-format csv -d "$out/b" -o run -- python3 $args
rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  --output-format csv -d "$out/c" -o run -- python3 $args
python3 scripts/pmc_summary.py "$out" SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_INSTS_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE
