"""ResNet-50 (v1.5) for the "ResNet-50 synthetic ImageNet bf16 on 8×MI355X" stretch configuration of
BASELINE.json — an allreduce-bandwidth stress test of the DP engine (25.6 M parameters, 102 MB of
fp32 gradients per step, ~160 gradient tensors).

Compute uses stock PyTorch-ROCm ops (MIOpen convolutions, hipBLASLt GEMM) in channels-last bf16
autocast; the point of this model is the data-parallel layer (bucketed RCCL allreduce overlapped
with backward by ``mihvd.DistributedOptimizer``), not new kernels. Not part of the reference repo.
"""
from __future__ import annotations

import torch
import torch.nn as nn


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1):
        super().__init__()
        cout = width * self.expansion
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)  # v1.5: stride on the 3x3
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        nn.init.zeros_(self.bn3.weight)  # zero-init the last BN of each residual branch
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride, bias=False), nn.BatchNorm2d(cout))
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        idn = x if self.down is None else self.down(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return self.relu(y + idn)


class ResNet50(nn.Module):
    def __init__(self, num_classes: int = 1000, layers=(3, 4, 6, 3)):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False), nn.BatchNorm2d(64),
                                  nn.ReLU(inplace=True), nn.MaxPool2d(3, stride=2, padding=1))
        blocks = []
        cin = 64
        for i, (n, width) in enumerate(zip(layers, (64, 128, 256, 512))):
            for j in range(n):
                blocks.append(Bottleneck(cin, width, stride=2 if (j == 0 and i > 0) else 1))
                cin = width * Bottleneck.expansion
        self.blocks = nn.Sequential(*blocks)
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(cin, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x):
        x = self.blocks(self.stem(x))
        return self.fc(torch.flatten(self.pool(x), 1))


def num_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
