#!/usr/bin/env python3
"""The reference's launched entrypoint (horovod/tensorflow_mnist.py), on mihvd.

Same flags (``--use-adasum``, ``--lr``, ``--num-steps``), same control flow and the same on-disk
layout: ``hvd.init()``; EEXIST-tolerant ``~/.keras/datasets`` mkdir; per-rank dataset name
``MNIST-data-<rank>``; LR × ``size()`` (× ``local_size()`` if RCCL for Adasum); TF1 Adam wrapped in
``hvd.DistributedOptimizer(op=Adasum|Average)``; hooks ``BroadcastGlobalVariablesHook(0)``,
``StopAtStepHook(last_step=num_steps // size())``, ``LoggingTensorHook({'step','loss'}, 10)``;
``./checkpoints`` on rank 0 only (``checkpoint`` index + ``model.ckpt-<step>``), restored and
broadcast on restart; batches of 100 from a per-epoch permutation.

On an MI355X the step runs the fused HIP kernels (``--impl fused``, default when a GPU is
present) at the reference's precision (``--precision fp32``: fp32 operands on the fp32-input
MFMAs; ``bf16`` optional), on the same path bench.py times: the training set is resident on the
device (a fresh permutation per epoch, batches gathered by index inside the first kernel — the
reference generator's semantics, :76-85), and each ``mon_sess.run`` replays a captured HIP graph of
``--steps-per-run`` (10) steps, so the hooks run between replays: ``LoggingTensorHook`` reads the
loss once per 10 steps (the reference's ``every_n_iter=10`` cadence) and the step counter logs
``global_step/sec`` and ``img_per_sec``. ``--impl torch`` runs stock PyTorch ops through the same
DistributedOptimizer, one host-fed step per run. Launch::

    mihvdrun -np 2 --allow-run-as-root -bind-to none -map-by slot -x LD_LIBRARY_PATH -x PATH \\
             -mca pml ob1 -mca btl ^openib python examples/tensorflow_mnist.py
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mihvd.tensorflow as hvd  # noqa: E402
from mihvd.utils.data import ensure_cache_dir, load_mnist, train_input_generator  # noqa: E402

# Training settings (module-level, like the reference: tensorflow_mnist.py:30-35)
parser = argparse.ArgumentParser(description="Tensorflow MNIST Example (mihvd / MI355X)")
parser.add_argument("--use-adasum", action="store_true", default=False, help="use adasum algorithm to do reduction")
parser.add_argument("--lr", default=0.001, type=float, help="Adam learning rate")
parser.add_argument("--num-steps", default=20000, type=int, help="Number of training steps")
parser.add_argument("--impl", choices=["auto", "fused", "torch"], default="auto", help="compute path")
parser.add_argument("--checkpoint-dir", default="./checkpoints")
parser.add_argument("--save-checkpoint-steps", type=int, default=None)
parser.add_argument("--log-step-count-steps", type=int, default=100)
parser.add_argument("--precision", choices=["fp32", "bf16"], default="fp32", help="fused: operand precision")
parser.add_argument("--steps-per-run", type=int, default=10, help="fused: steps per graph-replayed session run")
parser.add_argument("--shard-optimizer", action="store_true", help="fused bf16, size > 1: shard dense/kernel's Adam")
args = parser.parse_args()


def main():
    hvd.init()
    ensure_cache_dir()
    (x_train, y_train), (x_test, y_test) = load_mnist("MNIST-data-%d" % hvd.rank())[0]
    x_train = np.reshape(x_train, (-1, 784)).astype(np.float32) / 255.0
    x_test = np.reshape(x_test, (-1, 784)).astype(np.float32) / 255.0

    lr_scaler = hvd.size()
    if args.use_adasum:
        lr_scaler = hvd.local_size() if hvd.nccl_built() else 1
    op = hvd.Adasum if args.use_adasum else hvd.Average
    device = hvd.device()
    impl = args.impl
    if impl == "auto":
        impl = "fused" if device.type == "cuda" else "torch"

    last_step = args.num_steps // hvd.size()
    if impl == "fused":
        from mihvd.models.fused_mnist import FusedMNISTTrainer

        state = FusedMNISTTrainer(batch_size=100, lr=args.lr * lr_scaler, seed=0, device=device, op=op,
                                  precision=args.precision, shard_optimizer=args.shard_optimizer)
        # the reference generator (:76-85) on the device: per-rank independent permutations each epoch
        state.set_device_dataset(torch.from_numpy(x_train), torch.from_numpy(y_train.astype(np.int64)),
                                 seed=int(np.random.SeedSequence().entropy % (2 ** 31)) + hvd.rank())

        def train_op():
            # one run = up to steps_per_run steps replayed from a HIP graph (captured on the first
            # run, after restore + broadcast); never past StopAtStepHook's last step
            k = min(args.steps_per_run, last_step - state.global_step)
            state.run_steps(k, steps_per_replay=args.steps_per_run)
            return {"loss": state.loss_tensor()}
    else:
        from mihvd.models.mnist import MNISTConvNet, softmax_cross_entropy
        from mihvd.optim import TFAdam

        model = MNISTConvNet(impl="torch", seed=hvd.rank()).to(device)
        opt = hvd.DistributedOptimizer(TFAdam(model.parameters(), lr=args.lr * lr_scaler),
                                       named_parameters=model.named_parameters(), op=op)
        state = hvd.TorchTrainState(model, opt)

        def train_op(image, label):
            opt.zero_grad()
            loss = softmax_cross_entropy(model(image), label)
            loss.backward()
            opt.step()
            return {"loss": loss.detach()}

    hooks = [
        hvd.BroadcastGlobalVariablesHook(0),
        hvd.StopAtStepHook(last_step=last_step),
        hvd.LoggingTensorHook(tensors={"step": "global_step", "loss": "loss"}, every_n_iter=10),
    ]
    if args.log_step_count_steps:
        hooks.append(hvd.StepCounterHook(every_n_steps=args.log_step_count_steps, batch_size=100))
    checkpoint_dir = args.checkpoint_dir if hvd.rank() == 0 else None
    with hvd.MonitoredTrainingSession(checkpoint_dir=checkpoint_dir, hooks=hooks, state=state,
                                      save_checkpoint_steps=args.save_checkpoint_steps) as mon_sess:
        if impl == "fused":
            while not mon_sess.should_stop():
                mon_sess.run(train_op)
        else:
            gen = train_input_generator(x_train, y_train, batch_size=100)
            while not mon_sess.should_stop():
                image_, label_ = next(gen)
                image = torch.from_numpy(image_).to(device, non_blocking=True)
                label = torch.from_numpy(label_.astype(np.int64)).to(device, non_blocking=True)
                mon_sess.run(train_op, feed_dict={"image": image, "label": label})
    if impl == "fused":
        state.close()


if __name__ == "__main__":
    main()
