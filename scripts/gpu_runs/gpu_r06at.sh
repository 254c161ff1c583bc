# Round 6, pass at: f32_factor_full with the dz row offsets precomputed (32-bit) and only the last row
# group masked: kernel tests + times.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06at; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py -k "factor" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/kbench_f32.py --match "factor full|fc1_bwd" > $O/kbench.txt 2>&1 || { tail -20 $O/kbench.txt; exit 1; }
grep -v amdgpu.ids $O/kbench.txt
echo ALLDONE
