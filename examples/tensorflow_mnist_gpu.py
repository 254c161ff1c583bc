#!/usr/bin/env python3
"""The reference's Keras/GPU variant (horovod/tensorflow_mnist_gpu.py), on mihvd.

Flags ``--use-adasum --lr --num-steps --batch-size``; ``mixed_bfloat16`` policy by default (the
MI355X-native counterpart of the reference's ``mixed_float16``; ``--policy mixed_float16`` enables
fp16 with dynamic loss scaling); LR scaling as the reference; callbacks
``BroadcastGlobalVariablesCallback(0)``, ``MetricAverageCallback()`` and, on rank 0,
``TensorBoard('./logs')`` + ``ModelCheckpoint('./checkpoints/mnist-{epoch}.h5', save_best_only=True)``;
``steps_per_epoch = max(1, 60000 // (batch*size))``, ``validation_steps = max(1, 10000 // batch)``,
``epochs = max(1, num_steps // steps_per_epoch)``; rank 0 evaluates, prints Test loss/accuracy and
saves ``./final_model``.

On an MI355X the model trains through the hand-written CDNA4 kernels (``--impl hip``, the default
with a GPU): under ``mixed_bfloat16`` / ``float32`` ``fit`` drives the fused training step
(``FusedMNISTTrainer``: the dataset resident on the device, the whole step in seven launches, 20
steps per HIP-graph replay between the callback points; bf16 MFMA operands, or the exact-fp32
kernels under ``--policy float32``) and prints its images/sec; under ``mixed_float16`` every batch
is one fused forward+backward autograd node with the gradients through ``hvd.DistributedOptimizer``
and the HIP loss scaler. ``--impl torch`` runs stock PyTorch-ROCm layers instead.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mihvd.keras as hvd  # noqa: E402
from mihvd.models.mnist import MNISTConvNet  # noqa: E402
from mihvd.optim import TFAdam  # noqa: E402
from mihvd.utils.data import ensure_cache_dir, load_mnist  # noqa: E402

parser = argparse.ArgumentParser(description="Tensorflow MNIST Example (Keras-shaped, mihvd / MI355X)")
parser.add_argument("--use-adasum", action="store_true", default=False, help="use adasum algorithm to do reduction")
parser.add_argument("--lr", default=0.001, type=float, help="Adam learning rate")
parser.add_argument("--num-steps", default=20000, type=int, help="Number of training steps")
parser.add_argument("--batch-size", default=100, type=int, help="Batch size")
parser.add_argument("--policy", default="mixed_bfloat16", choices=["float32", "mixed_bfloat16", "mixed_float16"])
parser.add_argument("--impl", default="auto", choices=["auto", "hip", "torch"], help="compute path")
args = parser.parse_args()


def main():
    hvd.init()
    device = hvd.device()
    ensure_cache_dir()
    (x_train, y_train), (x_test, y_test) = load_mnist(f"MNIST-data-{hvd.rank()}")[0]
    x_train = np.reshape(x_train.astype(np.float32) / 255.0, (-1, 784))
    x_test = np.reshape(x_test.astype(np.float32) / 255.0, (-1, 784))

    policy = args.policy if device.type == "cuda" else "float32"
    impl = args.impl if args.impl != "auto" else ("hip" if device.type == "cuda" else "torch")
    model = hvd.Model(MNISTConvNet(impl=impl, seed=hvd.rank()).to(device), policy=policy)
    lr_scaler = hvd.size()
    if args.use_adasum:
        lr_scaler = hvd.local_size() if hvd.nccl_built() else 1
    opt = TFAdam(model.module.parameters(), lr=args.lr * lr_scaler, eps=1e-7)  # Keras Adam epsilon
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.module.named_parameters(),
                                   op=hvd.Adasum if args.use_adasum else hvd.Average)
    model.compile(optimizer=opt, loss=torch.nn.functional.cross_entropy, metrics=["accuracy"])

    callbacks = [hvd.callbacks.BroadcastGlobalVariablesCallback(0), hvd.callbacks.MetricAverageCallback()]
    if hvd.rank() == 0:
        callbacks.append(hvd.callbacks.TensorBoard(log_dir="./logs"))
        callbacks.append(hvd.callbacks.ModelCheckpoint("./checkpoints/mnist-{epoch}.h5", save_best_only=True))

    steps_per_epoch = max(1, len(x_train) // (args.batch_size * hvd.size()))
    validation_steps = max(1, len(x_test) // args.batch_size)
    epochs = max(1, args.num_steps // steps_per_epoch)
    model.fit(x_train, y_train, batch_size=args.batch_size, epochs=epochs, steps_per_epoch=steps_per_epoch,
              validation_data=(x_test, y_test), validation_steps=validation_steps, callbacks=callbacks,
              verbose=1 if hvd.rank() == 0 else 0, seed=hvd.rank())
    if hvd.rank() == 0 and getattr(model, "fit_throughput", None) is not None:
        print(f"fit throughput: {model.fit_throughput:.0f} images/sec (fused graph-replayed training steps, "
              f"policy {policy})", flush=True)
    if hvd.rank() == 0:
        score = model.evaluate(x_test, y_test, verbose=0)
        print("Test loss:", score[0])
        print("Test accuracy:", score[1])
        model.save("./final_model")


if __name__ == "__main__":
    main()
