# Round 6, pass al (after ak: no rescale kernel on the Adasum path): the reference's --use-adasum through bench.py at forced world 1 (the Adasum
# exchange on a 1-rank communicator, in the HIP graph), beside the average.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06al; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_fused_distributed_gpu.py -k adasum > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 --use-adasum > $O/bench_adasum.log 2>&1 || { tail -20 $O/bench_adasum.log; exit 1; }
python3 -c "import json; [print('forced adasum 200 steps', json.loads(l)['ms_per_step']*1000, json.loads(l)['config']['optimizer'], json.loads(l)['config']['data_plane']) for l in open('$O/bench_adasum.log') if l.startswith('{')]"
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_adasum -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 --use-adasum > $O/prof_adasum.log 2>&1 || { tail -30 $O/prof_adasum.log; exit 1; }
echo ALLDONE
