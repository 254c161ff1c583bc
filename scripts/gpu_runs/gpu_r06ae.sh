# Round 6, pass ae: the replicated factor plane's all-gathers in place and grouped (one RCCL group
# after the head; conv2_fwd / the head write into the gather buffers): factor-plane tests, forced
# world-1 bench + kernel trace, plane selection at forced world 1.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06ae; mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_fused_distributed_gpu.py -k "factor or collectives_inside_hip_graph or bench_multirank" tests/test_native_comm_gpu.py > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head; [ $rc -ne 0 ] && exit $rc
MIHVD_FORCE_COLLECTIVES=1 MIHVD_F32_PLANE=factor_rep MIHVD_SHARD_W3=0 timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_frep.log 2>&1 || { tail -20 $O/bench_frep.log; exit 1; }
python3 -c "import json; [print('forced factor_rep 200 steps', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_frep.log') if l.startswith('{')]"
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_forced_auto.log 2>&1 || { tail -20 $O/bench_forced_auto.log; exit 1; }
python3 -c "import json; [print('forced auto 200 steps', json.loads(l)['ms_per_step']*1000, json.loads(l)['config']['data_plane']) for l in open('$O/bench_forced_auto.log') if l.startswith('{')]"
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }; python3 -c "import json; [print('200 steps', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench.log') if l.startswith('{')]"
MIHVD_FORCE_COLLECTIVES=1 MIHVD_F32_PLANE=factor_rep MIHVD_SHARD_W3=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_frep -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/prof_frep.log 2>&1 || { tail -30 $O/prof_frep.log; exit 1; }
echo ALLDONE
