# Round 4, pass ad: the swizzled unpadded LDS image of the 8-wave conv2_fwd: tests, kbench, PMC.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ad; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_gpu.py -k "conv2_fwd or w2_frag or step_matches or fused_optimizer or trajectory" > $O/t_f32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t_f32.log | tail -5; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --match "conv2_fwd|whole step (graph|4 waves" > $O/kbench.log 2>&1 || { tail -30 $O/kbench.log; exit 1; }
cat $O/kbench.log
ONLY="conv2_fwd [W2 fragment copy]" timeout -k 10 300 bash scripts/pmc_r04.sh $O/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
grep conv2_fwd $O/pmc/pmc_summary.txt | grep -o "grid *[0-9]*\|ACTIVE_INST_LDS=[^ ]*\|INSTS_LDS=[^ ]*\|LDS_BANK_CONFLICT=[^ ]*"
echo ALLDONE
