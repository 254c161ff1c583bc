# Round 4, pass aj: conv2_bwd wgrad load offsets precomputed once; loads issued after step 0 (WMID=6) vs default 2:
# tests, kbench against the default, whole-step bench with and without it.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04aj; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_gpu.py -k "conv2_bwd" > $O/t_f32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t_f32.log | tail -5; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --match "conv2_bwd|whole step (graph" > $O/kbench.log 2>&1 || { tail -30 $O/kbench.log; exit 1; }
cat $O/kbench.log
for w in 2 6 2 6; do
  MIHVD_F32_C2B_WMID=$w timeout -k 10 120 python bench.py --steps 400 --warmup 20 > $O/bench_w$w.log 2>&1 || { tail -20 $O/bench_w$w.log; exit 1; }
  echo "WMID=$w $(grep -o '"ms_per_step": [0-9.]*' $O/bench_w$w.log)"
done
echo ALLDONE
