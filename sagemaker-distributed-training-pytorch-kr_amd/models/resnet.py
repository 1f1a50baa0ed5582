"""ResNet family (18/34/50/101/152, ResNeXt-50/101) with torchvision-compatible parameter names.

The Oxford-Pet recipe builds its model through ``util.torch_model(name, num_classes,
pretrained)`` from the torchvision zoo (/root/reference/2_training_oxford-pet_ddp/util.py:34-66;
BASELINE config: ResNet-50 DDP bf16). torchvision is not part of this stack, so the
architectures are defined here with the same module names (``conv1``, ``bn1``, ``layer1..4``,
``downsample.0/1``, ``fc``) so torchvision state dicts load with ``load_state_dict`` when a local
checkpoint is available (no downloads).

MI355X notes: run with ``memory_format=torch.channels_last`` (NHWC) so MIOpen picks its
implicit-GEMM (MFMA) convolution kernels; bf16 autocast or bf16 parameters halve HBM traffic.
"""
from __future__ import annotations

from typing import List, Optional, Type, Union

import torch
import torch.nn as nn


def conv3x3(i, o, stride=1, groups=1, dilation=1):
    return nn.Conv2d(i, o, 3, stride=stride, padding=dilation, groups=groups, bias=False, dilation=dilation)


def conv1x1(i, o, stride=1):
    return nn.Conv2d(i, o, 1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        idt = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            idt = self.downsample(x)
        return self.relu(out + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = conv3x3(width, width, stride, groups, dilation)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            idt = self.downsample(x)
        return self.relu(out + idt)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes=1000,
                 zero_init_residual=False, groups=1, width_per_group=64):
        super().__init__()
        self.inplanes = 64
        self.groups, self.base_width = groups, width_per_group
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                 nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, down, self.groups, self.base_width)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


_SPECS = {
    "resnet18": (BasicBlock, [2, 2, 2, 2], {}),
    "resnet34": (BasicBlock, [3, 4, 6, 3], {}),
    "resnet50": (Bottleneck, [3, 4, 6, 3], {}),
    "resnet101": (Bottleneck, [3, 4, 23, 3], {}),
    "resnet152": (Bottleneck, [3, 8, 36, 3], {}),
    "resnext50_32x4d": (Bottleneck, [3, 4, 6, 3], {"groups": 32, "width_per_group": 4}),
    "resnext101_32x8d": (Bottleneck, [3, 4, 23, 3], {"groups": 32, "width_per_group": 8}),
    "wide_resnet50_2": (Bottleneck, [3, 4, 6, 3], {"width_per_group": 128}),
}


def resnet(name: str, num_classes: int = 1000, **kw) -> ResNet:
    block, layers, extra = _SPECS[name]
    return ResNet(block, layers, num_classes=num_classes, **{**extra, **kw})


def available():
    return sorted(_SPECS)
