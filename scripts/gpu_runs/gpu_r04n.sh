# Round 4, pass n: W2 fragment copies on by default and the split fc1_fwd staging (tests + kbench
# A/B + whole step), rocprof of the bench for the roofline at HEAD, PMC of the conv / fc1 kernels.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04n; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_gpu.py > $O/t_f32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t_f32.log | tail -5; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 400 $T tests/test_fused_distributed_gpu.py -k "factor" > $O/t_dist.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t_dist.log | tail -6; [ $rc -ne 0 ] && { tail -60 $O/t_dist.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --match "conv2_fwd|conv2_bwd|fc1_fwd|whole step (graph|W2|K halves|factor" > $O/kbench.log 2>&1 || { tail -30 $O/kbench.log; exit 1; }
cat $O/kbench.log
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; tail -1 $O/bench_drv$i.log | cut -c1-200; done
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
tail -1 $O/prof_bench.log | cut -c1-200
ONLY="conv2_fwd [W2 fragment copy],conv2_bwd [W2 fragment copy],conv2_bwd [W2 fragment copy]:dg,fc1_fwd,fc1_bwd+W3 adam" timeout -k 10 300 bash scripts/pmc_r04.sh $O/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
cat $O/pmc/pmc_summary.txt
echo ALLDONE
