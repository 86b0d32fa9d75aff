"""ResNet family (BASELINE.json config "ResNet-50 on synthetic ImageNet-shape, 8xMI355X
bucketed all-reduce + backward overlap" — an extension: the reference only has VGG,
SURVEY.md §0.1 item 3, §7.1 step 7).

Bottleneck ResNet (He et al. 2016, v1.5 placement of the stride on the 3x3 conv),
written from the architecture definition; parameter names follow the de-facto
layout of the widely used ImageNet implementation (``conv1``, ``bn1``,
``layer{1..4}.{i}.conv{1,2,3}``, ``.downsample.{0,1}``, ``fc``) so checkpoints are
interchangeable with it. ResNet-50 has 25,557,032 parameters (97.5 MiB of fp32
gradients per step — the all-reduce payload of the scaling benchmark).

MI355X notes: two layouts, one parameter set.

* ``layout="nhwc"`` (default on GPU): activations stay channels-last end to end and every
  layer is the framework's (``ops.cnn_nhwc``): each convolution one hipBLASLt GEMM on the
  matrix cores (1x1: the activation itself; k x k / strided: a gfx950 im2col gather, and the
  gather-style col2im in the backward), BatchNorm (+ residual) (+ ReLU) and the stem's max-pool
  gfx950 kernels (``csrc/kernels/cnn_nhwc.hip``) — no layout transposes in the step.
* ``layout="nchw"``: MIOpen convolutions, with every BatchNorm + ReLU (+ the bottleneck's
  residual add) one fused gfx950 pass forward and two backward (``ops.cnn.bn_act``,
  ``csrc/kernels/bn_nchw.hip``). CPU runs always take this layout.

fp32, or bf16 under autocast (fp32 master weights and BN statistics). Trained by
``parallel.ddp.DistributedDataParallel`` (flat bucketed gradients, RCCL all-reduce overlapped
with backward) and ``ops.optim.FusedSGD`` (one HIP launch per step).
"""
from __future__ import annotations

import os
from typing import List, Optional, Type, Union

import torch
import torch.nn as nn

from ..ops.cnn import bn_act, max_pool3s2
from ..ops.cnn_nhwc import (ResidualGradSink, act_dtype, bn_act_nhwc, bn_relu_maxpool_nhwc, conv_nhwc,
                            residual_sink_ok, to_nhwc)


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


def _downsample(ds: nn.Sequential, x: torch.Tensor) -> torch.Tensor:
    """the projection shortcut: conv1x1 + BN (no ReLU), the BN through the fused kernel"""
    return bn_act(ds[1], ds[0](x), relu=False)


def _downsample_nhwc(ds: nn.Sequential, x: torch.Tensor) -> torch.Tensor:
    return bn_act_nhwc(ds[1], conv_nhwc(x, ds[0]), relu=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, width: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = conv3x3(cin, width, stride)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = conv3x3(width, width)
        self.bn2 = nn.BatchNorm2d(width)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        idt = x if self.downsample is None else _downsample(self.downsample, x)
        y = bn_act(self.bn1, self.conv1(x))
        return bn_act(self.bn2, self.conv2(y), residual=idt)

    def forward_nhwc(self, x: torch.Tensor) -> torch.Tensor:
        idt = x if self.downsample is None else _downsample_nhwc(self.downsample, x)
        y = bn_act_nhwc(self.bn1, conv_nhwc(x, self.conv1))
        return bn_act_nhwc(self.bn2, conv_nhwc(y, self.conv2), residual=idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = conv1x1(cin, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = conv3x3(width, width, stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = conv1x1(width, width * 4)
        self.bn3 = nn.BatchNorm2d(width * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        idt = x if self.downsample is None else _downsample(self.downsample, x)
        y = bn_act(self.bn1, self.conv1(x))
        y = bn_act(self.bn2, self.conv2(y))
        return bn_act(self.bn3, self.conv3(y), residual=idt)

    def forward_nhwc(self, x: torch.Tensor) -> torch.Tensor:
        if residual_sink_ok(x, self.conv1):
            # the shortcut branch's gradient w.r.t. x joins conv1's data-gradient GEMM
            # (ops/cnn_nhwc.ResidualGradSink); the sink (and the downsample after it) is created after
            # conv1..conv3, so autograd runs that branch's backward first
            box: dict = {}
            y = bn_act_nhwc(self.bn1, conv_nhwc(x, self.conv1, grad_box=box))
            z = conv_nhwc(bn_act_nhwc(self.bn2, conv_nhwc(y, self.conv2)), self.conv3)
            xs = ResidualGradSink.apply(x, box)
            idt = xs if self.downsample is None else _downsample_nhwc(self.downsample, xs)
            return bn_act_nhwc(self.bn3, z, residual=idt)
        idt = x if self.downsample is None else _downsample_nhwc(self.downsample, x)
        y = bn_act_nhwc(self.bn1, conv_nhwc(x, self.conv1))
        y = bn_act_nhwc(self.bn2, conv_nhwc(y, self.conv2))
        return bn_act_nhwc(self.bn3, conv_nhwc(y, self.conv3), residual=idt)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = False, layout: str = "nhwc"):
        super().__init__()
        assert layout in ("nhwc", "nchw"), layout
        self.layout = layout
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                last = getattr(m, "bn3", None) if isinstance(m, Bottleneck) else getattr(m, "bn2", None)
                if isinstance(m, (Bottleneck, BasicBlock)) and last is not None:
                    nn.init.zeros_(last.weight)

    def _make_layer(self, block, width: int, blocks: int, stride: int = 1) -> nn.Sequential:
        down = None
        if stride != 1 or self.inplanes != width * block.expansion:
            down = nn.Sequential(conv1x1(self.inplanes, width * block.expansion, stride),
                                 nn.BatchNorm2d(width * block.expansion))
        layers = [block(self.inplanes, width, stride, down)]
        self.inplanes = width * block.expansion
        layers += [block(self.inplanes, width) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.layout == "nhwc" and x.is_cuda:
            return self.forward_nhwc(x)
        x = max_pool3s2(bn_act(self.bn1, self.conv1(x)))  # self.maxpool's op, on the gfx950 kernel
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))

    def forward_nhwc(self, x: torch.Tensor) -> torch.Tensor:
        """the same network on channels-last activations (input: [B, 3, H, W], any memory format)"""
        # the 3-channel image gets a zero 4th channel: the stem's im2col then moves 4-channel vectors
        x = to_nhwc(x, act_dtype(x), pad_c=1 if x.shape[1] == 3 else 0)
        x = bn_relu_maxpool_nhwc(self.bn1, conv_nhwc(x, self.conv1))
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                x = blk.forward_nhwc(x)
        return self.fc(x.mean(dim=(1, 2)))


def resnet18(num_classes: int = 1000, layout: str = "nhwc") -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, layout=layout)


def resnet34(num_classes: int = 1000, layout: str = "nhwc") -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes, layout=layout)


def resnet50(num_classes: int = 1000, layout: str = "nhwc") -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, layout=layout)


def resnet101(num_classes: int = 1000, layout: str = "nhwc") -> ResNet:
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes, layout=layout)
