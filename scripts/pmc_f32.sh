# PMC passes (one counter set per run) over selected fp32 kernels, eagerly dispatched
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ONLY="${ONLY:-conv2_fwd,conv2_bwd:dg,conv2_bwd:wg,fc1_bwd:fdg,fc1_bwd:fwg,fc1_fwd}"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcA -o run -- python scripts/kbench_f32.py --only "$ONLY" > gpurun_out/pmcA.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVES --output-format csv -d gpurun_out/pmcB -o run -- python scripts/kbench_f32.py --only "$ONLY" > gpurun_out/pmcB.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmcC -o run -- python scripts/kbench_f32.py --only "$ONLY" > gpurun_out/pmcC.log 2>&1 || exit $?
echo pmc ok
