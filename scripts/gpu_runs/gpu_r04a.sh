# Round 4, first GPU pass: the changed paths (fp32 default + dropout tests, native-comm capture of the
# fp32 sharded step, the rewritten native engine), the headline bench, the engine latency check,
# and a kernel-trace profile of the fp32 step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04a; mkdir -p $O
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_f32_gpu.py -k "dropout or default_precision or step_matches" > $O/t_f32.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_f32.log | tail -20; [ $rc -ne 0 ] && { tail -40 $O/t_f32.log; exit $rc; }
timeout -k 10 300 $T tests/test_native_comm_gpu.py > $O/t_ncomm.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_ncomm.log | tail -20; [ $rc -ne 0 ] && { tail -60 $O/t_ncomm.log; exit $rc; }
timeout -k 10 500 $T tests/test_fused_distributed_gpu.py -k "collectives_inside_hip_graph" > $O/t_capture.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_capture.log | tail -20; [ $rc -ne 0 ] && { tail -60 $O/t_capture.log; exit $rc; }
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/bench_400.log 2>&1 || { tail -20 $O/bench_400.log; exit 1; }
tail -1 $O/bench_400.log
for e in torch native; do
  MIHVD_ENGINE=$e timeout -k 10 200 python bench.py --impl torch --steps 200 --warmup 20 > $O/bench_torch_$e.log 2>&1 || { tail -20 $O/bench_torch_$e.log; exit 1; }
  echo "engine=$e"; tail -1 $O/bench_torch_$e.log
done
timeout -k 10 300 bash scripts/profile_bench.sh $O/prof > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -30 $O/prof.log
