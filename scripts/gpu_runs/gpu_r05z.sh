# Round 5, pass z: conv2_bwd's wgrad role with its next-image LDS-DMA issued by inline asm
# (MIHVD_F32_C2B_ADMA=1, default of this build) so LLVM's wait-count pass keeps the K-step operand
# reads in flight (lgkmcnt(4/5) instead of lgkmcnt(0)); builtin form = 0. Tests, per-role launch
# times, whole step alternating, driver form.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/tests.log | head; exit $rc; }
timeout -k 10 200 python scripts/c2b_epilogue_probe.py MIHVD_F32_C2B_ADMA > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep conv2_bwd $O/probe.txt
for i in 1 2; do for k in 0 1; do
  MIHVD_F32_C2B_ADMA=$k timeout -k 10 200 python bench.py > $O/bench_a${k}_$i.log 2>&1 || { tail -20 $O/bench_a${k}_$i.log; exit 1; }
  python3 -c "import json; [print('adma=$k', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_a${k}_$i.log') if l.startswith('{')]"
done; done
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
echo ALLDONE
