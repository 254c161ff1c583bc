# Round 5, pass k: LDS-DMA staging — conv2 wgrad (default now) and conv2_fwd (study); fp32 tests,
# A/B kernel timings, driver-form bench x3 and a kernel trace for the roofline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_f32_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -c PASSED $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head; tail -1 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/kbench_f32.py --match "conv2_fwd [W2 fragment copy|conv2_bwd [W2 fragment copy|register-staged|LDS-DMA|wgrad role only, W2|whole step (graph" > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep -v "^#" $O/kbench.log | tail -12
for i in 1 2 3; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
python3 scripts/roofline_f32.py $O/prof/run_kernel_trace.csv $O/prof_bench.log --stats $O/kernel_stats.txt > $O/roofline.md && sed -n 5,14p $O/roofline.md
echo ALLDONE
