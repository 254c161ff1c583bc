# Round 4, pass i: pipelined MFMA conv1-wgrad epilogue and the mid-loop wgrad image store in the
# one-round conv2 backward; tests, kernel A/B, bench, stamps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04i; mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 500 $T tests/test_f32_gpu.py -k "conv2_bwd or step_matches or dropout or trajectory" > $O/t_f32.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_f32.log | tail -30; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 300 python scripts/kbench_f32.py --json $O/kbench_f32.json > $O/kbench_f32.log 2>&1 || { tail -30 $O/kbench_f32.log; exit 1; }
grep -E "conv2_bwd|whole step" $O/kbench_f32.log
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log | cut -c1-200
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-200
MIHVD_F32_STAMPS=1 timeout -k 10 400 python -m mihvd._build kernels --force > $O/stamps_build.log 2>&1 || { tail -20 $O/stamps_build.log; exit 1; }
timeout -k 10 200 python scripts/stamps_f32.py > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
head -20 $O/stamps.log
MIHVD_F32_C2B_MEPI=1 timeout -k 10 200 python scripts/stamps_f32.py > $O/stamps_mepi.log 2>&1 || { tail -20 $O/stamps_mepi.log; exit 1; }
head -20 $O/stamps_mepi.log
echo ALLDONE
