# Round 6, pass g: split-bf16 conv2_fwd (two co groups per wave, RNE split, x9 / x6) numerics + times.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_split_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "rel err|^FAILED|^ERROR|Error" $O/tests.log | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/kbench_f32.py --match "conv2_fwd" > $O/kbench.txt 2>&1 || { tail -20 $O/kbench.txt; exit 1; }
cat $O/kbench.txt
echo ALLDONE
