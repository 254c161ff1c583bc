# Round 5, pass c: the world-1 fp32 xGMI plane without the no-op collectives; the Keras fit path's
# images/sec (float32 and mixed_bfloat16, 3 epochs); forced-collectives bench with plane selection and
# a kernel trace of the world-1 xGMI step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_f32_gpu.py "tests/test_fused_distributed_gpu.py::test_collectives_inside_hip_graph" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -c PASSED $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head; tail -2 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/kbench_f32.py --match "head|fc1_bwd+W3 adam|whole step (graph|whole step [256|whole step [fc1_bwd waves" > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
cat $O/kbench.log | grep -v "^#" | tail -20
mkdir -p $O/keras && for pol in float32 mixed_bfloat16; do
  (cd $O/keras && timeout -k 10 300 python "$GRAFT_REPO_ROOT/examples/tensorflow_mnist_gpu.py" --num-steps 1800 --policy $pol \
     > keras_$pol.log 2>&1) || { tail -20 $O/keras/keras_$pol.log; exit 1; }
  grep -E "fit throughput|Test accuracy|Epoch" $O/keras/keras_$pol.log
done
MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_fc.log 2>&1 || { tail -30 $O/bench_fc.log; exit 1; }
python3 -c "import json; [print('forced', json.loads(l)['ms_per_step']*1000, json.loads(l)['config'].get('data_plane')) for l in open('$O/bench_fc.log') if l.startswith('{')]"
MIHVD_FORCE_COLLECTIVES=1 MIHVD_XGMI=on MIHVD_SHARD_W3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_xgmi -o run -- python3 bench.py --gpus 1 --steps 100 --warmup 10 > $O/prof_xgmi.log 2>&1 || { tail -30 $O/prof_xgmi.log; exit 1; }
python3 -c "import json; [print('xgmi forced traced', json.loads(l)['ms_per_step']*1000) for l in open('$O/prof_xgmi.log') if l.startswith('{')]"
echo ALLDONE
