set -e
cd /tmp && rm -rf ckpt_tf1 && mkdir ckpt_tf1 && cd ckpt_tf1
timeout -k 10 240 python -u $GRAFT_REPO_ROOT/bin/mihvdrun -np 1 python -u $GRAFT_REPO_ROOT/examples/tensorflow_mnist.py --num-steps 300 --checkpoint-dir ./checkpoints 2>&1 | grep -v amdgpu.ids | tail -6
ls checkpoints | head
timeout -k 10 240 python -u $GRAFT_REPO_ROOT/bin/mihvdrun -np 1 python -u $GRAFT_REPO_ROOT/examples/tensorflow_mnist.py --num-steps 400 --checkpoint-dir ./checkpoints 2>&1 | grep -v amdgpu.ids | tail -3
timeout -k 10 300 python -u $GRAFT_REPO_ROOT/examples/tensorflow_mnist_gpu.py --num-steps 600 2>&1 | grep -v amdgpu.ids | tail -6
