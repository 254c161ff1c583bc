#!/bin/bash
# PMC counters per kernel of the fused step (own runs: --pmc never combined with trace domains).
set -eu
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=${1:-gpurun_out/pmc}
rm -rf "$out"
rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --output-format csv -d "$out/sq" -o run -- python3 bench.py --steps 20 --warmup 10
rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE --output-format csv -d "$out/tcc" -o run -- python3 bench.py --steps 20 --warmup 10
python3 scripts/pmc_summary.py "$out"
