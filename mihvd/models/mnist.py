"""The reference MNIST CNN (horovod/tensorflow_mnist.py:38-73, tensorflow_mnist_gpu.py:40-88).

Architecture: reshape [-1,28,28,1] (NHWC) → conv 5×5×32 SAME + ReLU → max-pool 2×2/2 → conv
5×5×64 SAME + ReLU → max-pool 2×2/2 → flatten (NHWC order, 3136) → dense 1024 + ReLU → dropout
0.5 (training only) → dense 10 logits → mean softmax cross-entropy.

Parameters keep TensorFlow's names, layouts and shapes (HWIO kernels, [in, out] dense kernels)
so checkpoints carry over "in shape" (SURVEY.md §5.4):

    conv_layer1/conv2d/kernel [5,5,1,32]   conv_layer1/conv2d/bias [32]
    conv_layer2/conv2d/kernel [5,5,32,64]  conv_layer2/conv2d/bias [64]
    dense/kernel [3136,1024]               dense/bias [1024]
    dense_1/kernel [1024,10]               dense_1/bias [10]

``MNISTConvNet(impl="torch")`` runs stock PyTorch ops (the numerics oracle and the DDP
comparator); ``impl="hip"`` routes every layer through the hand-written CDNA4 kernels
(``mihvd.ops``), keeping autograd. The fully fused, graph-captured training step used by the
benchmark lives in ``mihvd.models.fused_mnist``.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

TF_PARAM_SHAPES = {
    "conv_layer1/conv2d/kernel": (5, 5, 1, 32),
    "conv_layer1/conv2d/bias": (32,),
    "conv_layer2/conv2d/kernel": (5, 5, 32, 64),
    "conv_layer2/conv2d/bias": (64,),
    "dense/kernel": (3136, 1024),
    "dense/bias": (1024,),
    "dense_1/kernel": (1024, 10),
    "dense_1/bias": (10,),
}
# Registration order == TF variable creation order (tensorflow_mnist.py:49-70).
TF_PARAM_ORDER = list(TF_PARAM_SHAPES)
NUM_PARAMS = sum(math.prod(s) for s in TF_PARAM_SHAPES.values())  # 3,274,634


def glorot_uniform_(t: torch.Tensor, fan_in: int, fan_out: int, generator=None):
    limit = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        return t.uniform_(-limit, limit, generator=generator)


class _Layer(nn.Module):
    def __init__(self, kshape, bshape):
        super().__init__()
        self.kernel = nn.Parameter(torch.empty(kshape))
        self.bias = nn.Parameter(torch.zeros(bshape))


class _Scope(nn.Module):
    def __init__(self, layer):
        super().__init__()
        self.conv2d = layer


def tf_name(torch_name: str) -> str:
    return torch_name.replace(".", "/")


def torch_name(tf: str) -> str:
    return tf.replace("/", ".")


class MNISTConvNet(nn.Module):
    def __init__(self, impl: str = "torch", dropout_rate: float = 0.5, seed: int | None = None,
                 compute_dtype: torch.dtype = torch.float32):
        super().__init__()
        if impl not in ("torch", "hip"):
            raise ValueError("impl must be 'torch' or 'hip'")
        self.impl = impl
        self.dropout_rate = dropout_rate
        self.compute_dtype = compute_dtype
        # impl="hip": operand precision of the HIP kernels ("bf16" MFMA operands or exact "fp32")
        self.hip_precision = "bf16"
        self.conv_layer1 = _Scope(_Layer((5, 5, 1, 32), (32,)))
        self.conv_layer2 = _Scope(_Layer((5, 5, 32, 64), (64,)))
        self.dense = _Layer((3136, 1024), (1024,))
        self.dense_1 = _Layer((1024, 10), (10,))
        self.reset_parameters(seed)

    def reset_parameters(self, seed: int | None = None):
        g = None
        if seed is not None:
            g = torch.Generator(device="cpu")
            g.manual_seed(seed)
        specs = [(self.conv_layer1.conv2d.kernel, 25 * 1, 25 * 32), (self.conv_layer2.conv2d.kernel, 25 * 32, 25 * 64),
                 (self.dense.kernel, 3136, 1024), (self.dense_1.kernel, 1024, 10)]
        for p, fi, fo in specs:
            if p.device.type == "cpu":
                glorot_uniform_(p, fi, fo, g)
            else:
                tmp = torch.empty(p.shape)
                glorot_uniform_(tmp, fi, fo, g)
                with torch.no_grad():
                    p.copy_(tmp)
        for b in (self.conv_layer1.conv2d.bias, self.conv_layer2.conv2d.bias, self.dense.bias, self.dense_1.bias):
            with torch.no_grad():
                b.zero_()

    def tf_state_dict(self) -> dict[str, torch.Tensor]:
        return {tf_name(k): v for k, v in self.state_dict().items()}

    def load_tf_state_dict(self, sd: dict[str, torch.Tensor]):
        self.load_state_dict({torch_name(k): v for k, v in sd.items()})

    def ordered_parameters(self):
        """Parameters in TF variable-creation order (the flat-buffer layout of the fused path)."""
        named = dict(self.named_parameters())
        return [(n, named[torch_name(n)]) for n in TF_PARAM_ORDER]

    # ---------------------------------------------------------------------------------------
    def forward(self, images: torch.Tensor) -> torch.Tensor:
        """images: [B, 784] or [B, 28, 28] floats in [0, 1]. Returns [B, 10] logits."""
        if self.impl == "hip":
            # inference through the HIP kernels; training goes through
            # mihvd.ops.functional.fused_mnist_loss (forward + backward in one fused node)
            from ..ops import functional as HF

            return HF.mnist_logits(self, images)
        x = images.reshape(-1, 28, 28, 1).permute(0, 3, 1, 2)  # NHWC view -> NCHW for torch conv
        cd = self.compute_dtype
        w1 = self.conv_layer1.conv2d.kernel.permute(3, 2, 0, 1)  # HWIO -> OIHW
        w2 = self.conv_layer2.conv2d.kernel.permute(3, 2, 0, 1)
        h = F.conv2d(x.to(cd), w1.to(cd), self.conv_layer1.conv2d.bias.to(cd), padding=2)
        h = F.max_pool2d(F.relu(h), 2, 2)
        h = F.conv2d(h, w2.to(cd), self.conv_layer2.conv2d.bias.to(cd), padding=2)
        h = F.max_pool2d(F.relu(h), 2, 2)
        h = h.permute(0, 2, 3, 1).reshape(-1, 7 * 7 * 64)  # NHWC flatten order (tensorflow_mnist.py:62)
        h = F.relu(h @ self.dense.kernel.to(cd) + self.dense.bias.to(cd))
        if self.training and self.dropout_rate > 0:
            h = F.dropout(h, self.dropout_rate, training=True)
        logits = h @ self.dense_1.kernel.to(cd) + self.dense_1.bias.to(cd)
        return logits.float()


def softmax_cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """``tf.losses.softmax_cross_entropy(one_hot(labels), logits)`` — mean over the batch."""
    return F.cross_entropy(logits.float(), labels.long())


def accuracy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    return (logits.argmax(1) == labels.long()).float().mean()

# fc1_fwd split-K slabs of the fused HIP step (csrc/kernels/fc.hip FC1_KS; the ops check the zpart shape)
FC1_KS = 7
