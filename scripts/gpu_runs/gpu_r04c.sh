# Round 4, pass c: the fp16-operand kernel set (tests, the Keras mixed_float16 example on HIP kernels
# and its kernel profile), whole-step studies of the fp32 forward placement (conv1 fused or not, CU
# sharing, W2 prefetch) and of the conv1-wgrad epilogue, and the BERT capture bisection from the
# failing form (C0: the last warm-up loss freed before capture), with the non-finite tensors named.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04c; mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T -s tests/test_f16_gpu.py > $O/t_f16.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|rel err" $O/t_f16.log | tail -20; [ $rc -ne 0 ] && tail -40 $O/t_f16.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 $T tests/test_examples_gpu.py -k "keras and mixed_float16" > $O/t_keras_f16.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/t_keras_f16.log | tail -5; [ $rc -ne 0 ] && tail -30 $O/t_keras_f16.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_keras_f16 -o run -- python3 examples/tensorflow_mnist_gpu.py --impl hip --policy mixed_float16 --num-steps 30 > $O/keras_f16_prof.log 2>&1 || { tail -20 $O/keras_f16_prof.log; exit 1; }
python3 scripts/rocprof_summary.py $O/prof_keras_f16 > $O/keras_f16_kernels.txt 2>&1; head -20 $O/keras_f16_kernels.txt
timeout -k 10 300 python scripts/kbench_f32.py --json $O/kbench_f32.json > $O/kbench_f32.log 2>&1 || { tail -30 $O/kbench_f32.log; exit 1; }
grep "whole step\|conv2_bwd \|conv2_fwd\|conv12" $O/kbench_f32.log
timeout -k 10 600 python -u scripts/bert_graph_bisect.py --variants C0,S,P,N,L,M,Z --steps 5 --loss-only --diag > $O/bert_bisect.log 2>&1
echo "bert bisect rc=$?"; grep "^{" $O/bert_bisect.log | cut -c1-400
echo ALLDONE
