# Round 6, pass aq: PMC counters of the replicated factor plane's kernel (N = 2) beside fc1_bwd's
# fused wgrad + Adam (one counter set per run, eagerly dispatched).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06aq; mkdir -p $O
ONLY="factor full + Adam N=2 (HIP),fc1_bwd+W3 adam"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES --output-format csv -d $O/pmcA -o run -- python scripts/kbench_f32.py --only "$ONLY" > $O/pmcA.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVES --output-format csv -d $O/pmcB -o run -- python scripts/kbench_f32.py --only "$ONLY" > $O/pmcB.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmcC -o run -- python scripts/kbench_f32.py --only "$ONLY" > $O/pmcC.log 2>&1 || exit $?
python scripts/pmc_summary.py $O/pmcA $O/pmcB $O/pmcC > $O/pmc_summary.txt 2>&1
cat $O/pmc_summary.txt
echo ALLDONE
