# PMC passes over the fp32 step's kernels at round-5 HEAD (LDS-DMA staging in conv2_fwd and the conv2 wgrad role) (one counter set per run,
# eagerly dispatched by kbench_f32 --only), summarised into $1/pmc_summary.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=${1:-gpurun_out/pmc_r05}; mkdir -p $D
ONLY="${ONLY:-conv1_fwd [+ W2 fragment copies],conv2_fwd [W2 fragment copy],conv2_bwd [W2 fragment copy],conv2_bwd [W2 fragment copy]:dg,conv2_bwd [W2 fragment copy]:wg,fc1_bwd+W3 adam,fc1_fwd,head,conv_reduce+adam}"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES --output-format csv -d $D/A -o run -- python scripts/kbench_f32.py --only "$ONLY" > $D/A.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVES --output-format csv -d $D/B -o run -- python scripts/kbench_f32.py --only "$ONLY" > $D/B.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $D/C -o run -- python scripts/kbench_f32.py --only "$ONLY" > $D/C.log 2>&1 || exit $?
python scripts/pmc_summary.py $D/A $D/B $D/C > $D/pmc_summary.txt 2>&1
cat $D/pmc_summary.txt
