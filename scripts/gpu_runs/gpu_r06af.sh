# Round 6, pass af: f32_factor_full with its Adam as a tail stream (every p / m / v load of a lane at
# once) against the Adam under the last segment: kernel test, kernel times, forced world-1 bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06af; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py -k "factor" tests/test_fused_distributed_gpu.py -k "factor" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/kbench_f32.py --match "factor full|fc1_bwd" > $O/kbench.txt 2>&1 || { tail -20 $O/kbench.txt; exit 1; }
grep -v amdgpu.ids $O/kbench.txt
MIHVD_FORCE_COLLECTIVES=1 MIHVD_F32_PLANE=factor_rep MIHVD_SHARD_W3=0 timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_frep.log 2>&1 || { tail -20 $O/bench_frep.log; exit 1; }
python3 -c "import json; [print('forced factor_rep 200 steps', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_frep.log') if l.startswith('{')]"
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }; python3 -c "import json; [print('200 steps', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench.log') if l.startswith('{')]"
echo ALLDONE
