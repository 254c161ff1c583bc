# Round 5, pass y: the conv1 weight-gradient epilogue of conv2_bwd's dgrad role on MFMA
# (MIHVD_F32_C2B_MEPI=1, now with the W2 fragment copy too) against the VALU default: per-role
# launch times, and the whole step alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py -k "fragment or conv2_bwd_and_reduce" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/c2b_epilogue_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep conv2_bwd $O/probe.txt
for i in 1 2; do for k in 0 1; do
  MIHVD_F32_C2B_MEPI=$k timeout -k 10 200 python bench.py > $O/bench_m${k}_$i.log 2>&1 || { tail -20 $O/bench_m${k}_$i.log; exit 1; }
  python3 -c "import json; [print('mepi=$k', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_m${k}_$i.log') if l.startswith('{')]"
done; done
echo ALLDONE
