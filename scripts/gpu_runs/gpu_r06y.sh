# Round 6, pass y: f32_factor_full with operands two chunks / one segment ahead (a2 column in LDS):
# kernel tests + times; the forced world-1 step on the replicated factor plane (bench + kernel
# trace) and plane selection over every fp32 plane at forced world 1.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_f32_gpu.py -k "factor or gathered_ahead" > $O/tests_f32.log 2>&1
rc=$?; tail -1 $O/tests_f32.log; grep -E "^FAILED|Error" $O/tests_f32.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/kbench_f32.py --match "fc1_bwd|factor full" > $O/kbench.txt 2>&1 || { tail -20 $O/kbench.txt; exit 1; }
grep -v amdgpu.ids $O/kbench.txt
MIHVD_FORCE_COLLECTIVES=1 MIHVD_F32_PLANE=factor_rep MIHVD_SHARD_W3=0 timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_frep.log 2>&1 || { tail -20 $O/bench_frep.log; exit 1; }
python3 -c "import json; [print('forced factor_rep 200 steps', json.loads(l)['ms_per_step']*1000, json.loads(l)['config']['data_plane']) for l in open('$O/bench_frep.log') if l.startswith('{')]"
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_forced_auto.log 2>&1 || { tail -20 $O/bench_forced_auto.log; exit 1; }
python3 -c "import json; [print('forced auto 200 steps', json.loads(l)['ms_per_step']*1000, json.loads(l)['config']['data_plane']) for l in open('$O/bench_forced_auto.log') if l.startswith('{')]"
MIHVD_FORCE_COLLECTIVES=1 MIHVD_F32_PLANE=factor_rep MIHVD_SHARD_W3=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_frep -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_frep.log 2>&1 || { tail -30 $O/prof_frep.log; exit 1; }
echo ALLDONE
