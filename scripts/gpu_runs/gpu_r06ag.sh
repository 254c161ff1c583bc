# Round 6, pass ag: final-HEAD validation -- the whole GPU suite, smoke(), the bench (driver form x3,
# 200 steps), the bench's multi-rank rehearsal on one GPU, Keras fit throughput under every policy.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06ag; mkdir -p $O
for i in 1 2 3; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('driver form', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }; python3 -c "import json; [print('200 steps', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench.log') if l.startswith('{')]"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider --durations=15 > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -c PASSED $O/suite.log; grep -E "^FAILED|^ERROR" $O/suite.log | head -30; tail -1 $O/suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
mkdir -p $O/keras && for pol in float32 mixed_bfloat16 mixed_float16; do
  (cd $O/keras && timeout -k 10 300 python "$GRAFT_REPO_ROOT/examples/tensorflow_mnist_gpu.py" --num-steps 1800 --policy $pol --impl hip \
     > keras_$pol.log 2>&1) || { tail -20 $O/keras/keras_$pol.log; exit 1; }
  grep -E "fit throughput|Test accuracy" $O/keras/keras_$pol.log
done
echo ALLDONE
