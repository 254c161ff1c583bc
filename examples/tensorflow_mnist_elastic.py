#!/usr/bin/env python3
"""Elastic MNIST training on mihvd — the elastic variant the reference links to
(horovod/README.md:20-22: an external Horovod v1 elastic MPIJob) but does not ship.

Same model, batch 100, LR rule and Adam as examples/tensorflow_mnist.py; training is wrapped in
``hvd.elastic.run`` with a ``TorchState`` committed every ``--commit-every`` batches, so workers can
die, be replaced or be added while the job runs::

    mihvdrun -np 8 --min-np 4 --max-np 16 --respawn python examples/tensorflow_mnist_elastic.py

A failed worker rolls the survivors back to the last commit; an added worker receives the
committed state from rank 0. The LR follows the current world size after every re-formation.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mihvd.torch as hvd  # noqa: E402
from mihvd.models.mnist import MNISTConvNet, softmax_cross_entropy  # noqa: E402
from mihvd.optim import TFAdam  # noqa: E402
from mihvd.utils.data import load_mnist  # noqa: E402

parser = argparse.ArgumentParser(description="Elastic MNIST (mihvd / MI355X)")
parser.add_argument("--lr", default=0.001, type=float)
parser.add_argument("--epochs", default=2, type=int)
parser.add_argument("--batches-per-epoch", default=200, type=int)
parser.add_argument("--batch-size", default=100, type=int)
parser.add_argument("--commit-every", default=10, type=int)
args = parser.parse_args()


def main():
    hvd.init()
    device = hvd.device()
    (x_train, y_train), _ = load_mnist("MNIST-data-%d" % hvd.rank())[0]
    x_train = torch.from_numpy(np.reshape(x_train, (-1, 784)).astype(np.float32) / 255.0)
    y_train = torch.from_numpy(y_train.astype(np.int64))
    model = MNISTConvNet(impl="torch", seed=0).to(device)
    opt = hvd.DistributedOptimizer(TFAdam(model.parameters(), lr=args.lr * hvd.size()),
                                   named_parameters=model.named_parameters())
    state = hvd.elastic.TorchState(model, opt, epoch=0, batch=0)

    def on_reset():  # LR x size() follows the re-formed world (tensorflow_mnist.py:123)
        for g in opt.param_groups:
            g["lr"] = args.lr * hvd.size()

    state.register_reset_callbacks([on_reset])

    @hvd.elastic.run
    def train(state):
        while state.epoch < args.epochs:
            while state.batch < args.batches_per_epoch:
                g = torch.Generator().manual_seed(state.epoch * 100003 + state.batch * 101 + hvd.rank())
                idx = torch.randint(0, x_train.shape[0], (args.batch_size,), generator=g)
                opt.zero_grad()
                loss = softmax_cross_entropy(model(x_train[idx].to(device)), y_train[idx].to(device))
                loss.backward()
                opt.step()
                state.batch += 1
                if state.batch % args.commit_every == 0:
                    if hvd.rank() == 0:
                        print(f"epoch {state.epoch} batch {state.batch} size {hvd.size()} loss {loss.item():.4f}",
                              flush=True)
                    state.commit()
            state.epoch += 1
            state.batch = 0
            state.commit()

    train(state)
    if hvd.rank() == 0:
        print("done: epochs=%d world=%d" % (state.epoch, hvd.size()), flush=True)


if __name__ == "__main__":
    main()
