# Round 4, pass q: conv2 wgrad image loads one image ahead, factor kernel (5-stage ring, XCD-aware
# order): tests, kbench, benches, stamps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04q; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_gpu.py -k "conv2_bwd or factor or w2_frag or step_matches or fused_optimizer" > $O/t_f32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t_f32.log | tail -5; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 400 $T tests/test_fused_distributed_gpu.py -k "factor" > $O/t_dist.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t_dist.log | tail -6; [ $rc -ne 0 ] && { tail -60 $O/t_dist.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --match "conv2_bwd|factor|whole step (graph" > $O/kbench.log 2>&1 || { tail -30 $O/kbench.log; exit 1; }
cat $O/kbench.log
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; tail -1 $O/bench_drv$i.log | cut -c1-200; done
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log | cut -c1-200
MIHVD_F32_STAMPS=1 timeout -k 10 400 python -m mihvd._build kernels --force > $O/stamps_build.log 2>&1 || { tail -20 $O/stamps_build.log; exit 1; }
timeout -k 10 200 python scripts/stamps_f32.py > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
head -22 $O/stamps.log
echo ALLDONE
