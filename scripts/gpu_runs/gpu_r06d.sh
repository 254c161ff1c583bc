# Round 6, pass d: split-bf16 conv2_fwd numerics + per-kernel times (fc1_bwd regression check).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_split_gpu.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "rel err|^FAILED|^ERROR" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/kbench_f32.py --json $O/kbench.json > $O/kbench.txt 2>&1 || { tail -20 $O/kbench.txt; exit 1; }
cat $O/kbench.txt
echo ALLDONE
