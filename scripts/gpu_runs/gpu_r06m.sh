# Round 6, pass m: split conv2_bwd dgrad phase study (dgrad blocks alone) + numerics.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -s --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_split_gpu.py > $O/tests_split.log 2>&1
rc=$?; tail -2 $O/tests_split.log; grep -E "x6 dW1|x6 db1|^FAILED|Error" $O/tests_split.log | head -20; [ $rc -ne 0 ] && exit $rc
for st in 0 1 3; do MIHVD_C2BX_ROLE=1 MIHVD_C2BX_STUDY=$st timeout -k 10 120 python scripts/kbench_f32.py --match "x6 dgrad" > $O/s$st.txt 2>&1 || { tail -20 $O/s$st.txt; exit 1; }; echo "study $st: $(grep x6 $O/s$st.txt)"; done
timeout -k 10 120 python scripts/kbench_f32.py --match "conv2_bwd|conv2_fwd" > $O/k.txt 2>&1; cat $O/k.txt
echo ALLDONE
