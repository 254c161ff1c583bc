# Round 5, pass v: fc1_bwd's streamed W3 / m / v as non-temporal accesses (MIHVD_F32_F1R_NT: bit 0
# loads, bit 1 stores; 0 = the default): whole-step A/B at the default length, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05v; mkdir -p $O
MIHVD_F32_F1R_NT=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py -k "fused_adam or graph_replay" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for k in 0 1 2 3; do
  MIHVD_F32_F1R_NT=$k timeout -k 10 200 python bench.py > $O/bench_nt${k}_$i.log 2>&1 || { tail -20 $O/bench_nt${k}_$i.log; exit 1; }
  python3 -c "import json; [print('nt=$k', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_nt${k}_$i.log') if l.startswith('{')]"
done; done
echo ALLDONE
