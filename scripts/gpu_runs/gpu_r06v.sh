# Round 6, pass v: HEAD validation -- the whole GPU suite, smoke(), the Keras example's fit throughput
# under every policy (3 epochs x 600 steps; epochs 2-3 timed).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider --durations=15 > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -c PASSED $O/suite.log; grep -E "^FAILED|^ERROR" $O/suite.log | head -30; tail -3 $O/suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
mkdir -p $O/keras && for pol in float32 mixed_bfloat16 mixed_float16; do
  (cd $O/keras && timeout -k 10 300 python "$GRAFT_REPO_ROOT/examples/tensorflow_mnist_gpu.py" --num-steps 1800 --policy $pol --impl hip \
     > keras_$pol.log 2>&1) || { tail -20 $O/keras/keras_$pol.log; exit 1; }
  grep -E "fit throughput|Test accuracy" $O/keras/keras_$pol.log
done
echo ALLDONE
