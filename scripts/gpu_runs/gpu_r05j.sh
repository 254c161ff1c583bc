# Round 5, pass j: conv2 wgrad next image by LDS-DMA (tests + A/B); head kernels accumulate the Keras epoch metrics in place (no per-step reduction
# launches); head tests, Keras examples with their fit throughput, bench driver form, and the GPU
# suite's wall time after the round-5 trim.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_f32_gpu.py -k "conv2_bwd_and_reduce" > $O/dma_tests.log 2>&1 || { tail -30 $O/dma_tests.log; exit 1; }
tail -1 $O/dma_tests.log
timeout -k 10 300 python scripts/kbench_f32.py --match "conv2_bwd [W2 fragment copy]|LDS-DMA|wgrad role only, W2|whole step (graph" > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep -v "^#" $O/kbench.log | tail -8
mkdir -p $O/keras && for pol in float32 mixed_bfloat16; do
  (cd $O/keras && timeout -k 10 300 python "$GRAFT_REPO_ROOT/examples/tensorflow_mnist_gpu.py" --num-steps 1800 --policy $pol \
     > keras_$pol.log 2>&1) || { tail -20 $O/keras/keras_$pol.log; exit 1; }
  grep -E "fit throughput|Test accuracy" $O/keras/keras_$pol.log
done
t0=$(date +%s)
timeout -k 10 900 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu tests \
  --durations=15 > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc in $(( $(date +%s) - t0 )) s"; grep -c PASSED $O/suite.log; grep -E "^FAILED|^ERROR" $O/suite.log | head; tail -1 $O/suite.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv$i.log 2>&1 || { tail -20 $O/bench_drv$i.log; exit 1; }; python3 -c "import json; [print('drv', json.loads(l)['ms_per_step']*1000) for l in open('$O/bench_drv$i.log') if l.startswith('{')]"; done
echo ALLDONE
