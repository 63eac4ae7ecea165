"""MobileNetV2 for 32x32 inputs (BASELINE config 4: CIFAR-100, on-device model).

Not in the reference (SURVEY §7.1 "Added").  CIFAR variant: 3x3/s1 stem and
the stride of the second stage set to 1 so the final feature map is 4x4.
Blocks are inverted residuals: 1x1 expand -> 3x3 depthwise -> 1x1 project,
BN after each conv, ReLU6 on the first two, identity skip when shapes match.
The native engine lowers the 1x1 convs to its MFMA GEMM and the depthwise
conv to a dedicated LDS-tiled HIP kernel.
"""
from __future__ import annotations

import torch.nn as nn
import torch.nn.functional as F

# (expansion, out_planes, num_blocks, stride)
CFG = [(1, 16, 1, 1), (6, 24, 2, 1), (6, 32, 3, 2), (6, 64, 4, 2),
       (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1)]


class InvertedResidual(nn.Module):
    def __init__(self, in_planes, out_planes, expansion, stride):
        super().__init__()
        self.stride = stride
        planes = expansion * in_planes
        self.conv1 = nn.Conv2d(in_planes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, groups=planes, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, out_planes, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(out_planes)
        self.shortcut = nn.Sequential()
        if stride == 1 and in_planes != out_planes:
            self.shortcut = nn.Sequential(nn.Conv2d(in_planes, out_planes, 1, bias=False),
                                          nn.BatchNorm2d(out_planes))

    def forward(self, x):
        out = F.relu6(self.bn1(self.conv1(x)))
        out = F.relu6(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.stride == 1:
            out = out + self.shortcut(x)
        return out


class MobileNetV2(nn.Module):
    def __init__(self, num_classes=100):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(32)
        layers = []
        in_planes = 32
        for expansion, out_planes, num_blocks, stride in CFG:
            for s in [stride] + [1] * (num_blocks - 1):
                layers.append(InvertedResidual(in_planes, out_planes, expansion, s))
                in_planes = out_planes
        self.layers = nn.Sequential(*layers)
        self.conv2 = nn.Conv2d(320, 1280, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(1280)
        self.linear = nn.Linear(1280, num_classes)

    def forward(self, x):
        out = F.relu6(self.bn1(self.conv1(x)))
        out = self.layers(out)
        out = F.relu6(self.bn2(self.conv2(out)))
        out = F.avg_pool2d(out, 4)
        return self.linear(out.flatten(1))
