# Round 5, pass ac: fc1_fwd with the a2 slice's loads, then the W3 loads, then the a2 LDS writes
# (masking moved to the store, tail chunk stored unconditionally into spare rows), so the MFMA
# chain consumes the W3 fragments as they arrive. fp32 tests, smoke, whole step, driver form,
# kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05ac; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2 3; do timeout -k 10 200 python bench.py > $O/bench_def$i.log 2>&1 || { tail -20 $O/bench_def$i.log; exit 1; }; python3 -c "import json; [print('default', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_def$i.log') if l.startswith('{')]"; done
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
python3 scripts/roofline_f32.py $O/prof/run_kernel_trace.csv $O/prof_bench.log --stats $O/kernel_stats.txt > $O/roofline.md && sed -n 5,16p $O/roofline.md
echo ALLDONE
