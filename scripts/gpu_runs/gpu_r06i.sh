# Round 6, pass i: split-bf16 dgrad role of conv2_bwd: numerics, kernel times, the fp32 suite, bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_split_gpu.py > $O/tests_split.log 2>&1
rc=$?; tail -2 $O/tests_split.log; grep -E "dW|db1|^FAILED|^ERROR|Error" $O/tests_split.log | head -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/kbench_f32.py --match "conv2_bwd|conv2_fwd [split" > $O/kbench.txt 2>&1 || { tail -20 $O/kbench.txt; exit 1; }
cat $O/kbench.txt
echo KDONE
