# Round 4, pass ak: repeated A/B of the wgrad load placement (MIHVD_F32_C2B_WMID 2 vs 6): kbench of the
# conv2_bwd launch x3, alternating 400-step and driver-form benches.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ak; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 python scripts/kbench_f32.py --match "conv2_bwd [W2 fragment copy|whole step (graph" > $O/kbench$r.log 2>&1 || { tail -30 $O/kbench$r.log; exit 1; }
  grep -E "conv2_bwd|whole" $O/kbench$r.log
done
for r in 1 2 3 4; do
  for w in 2 6; do
    MIHVD_F32_C2B_WMID=$w timeout -k 10 120 python bench.py --steps 400 --warmup 20 > $O/b400_w${w}_$r.log 2>&1 || { tail -20 $O/b400_w${w}_$r.log; exit 1; }
    MIHVD_F32_C2B_WMID=$w timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bdrv_w${w}_$r.log 2>&1 || { tail -20 $O/bdrv_w${w}_$r.log; exit 1; }
    echo "WMID=$w 400: $(grep -o '"ms_per_step": [0-9.]*' $O/b400_w${w}_$r.log)  drv: $(grep -o '"ms_per_step": [0-9.]*' $O/bdrv_w${w}_$r.log)"
  done
done
echo ALLDONE
