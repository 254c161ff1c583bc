# Round 4, pass s: conv2_fwd forms (4 / 8 waves x A reads one / two steps ahead, fragment W2): tests,
# kbench A/B, whole steps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04s; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_gpu.py -k "conv2_fwd or w2_frag" > $O/t_f32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t_f32.log | tail -5; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --match "conv2_fwd|whole step (graph|8 waves|step ahead" > $O/kbench.log 2>&1 || { tail -30 $O/kbench.log; exit 1; }
cat $O/kbench.log
echo ALLDONE
