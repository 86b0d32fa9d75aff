"""VGG family for 3x32x32 inputs / 10 classes.

Capability parity with the reference model (`master/part1/model.py:1-50`, copied
verbatim into every part directory):

* the same configuration table (VGG11/13/16/19, `model.py:3-8`),
* the same block structure: ``Conv2d(3x3, s1, p1, bias) -> BatchNorm2d -> ReLU``
  per integer entry and ``MaxPool2d(2, 2)`` per ``'M'`` (`model.py:11-27`),
* the same classifier ``fc1 = Linear(512, 10)`` after a flatten (`model.py:40-46`),
* therefore exactly the same ``state_dict`` key set / order (58 keys for VGG11,
  SURVEY.md §2.6) — the checkpoint layout this framework preserves.

Differences by design: all four factories are exported (the reference only
exposes ``VGG11``), and the module can execute through the MI355X-native fused
HIP path (``native=True``) — conv as MFMA implicit GEMM with BN statistics in the
epilogue, BN+ReLU+max-pool fused, linear+softmax-xent fused — while keeping the
PyTorch parameter objects (and thus `state_dict`, DDP hooks, optimizers) intact.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Union

import torch
import torch.nn as nn

CFG: Dict[str, List[Union[int, str]]] = {
    "VGG11": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "VGG13": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "VGG16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "VGG19": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
              512, 512, 512, 512, "M"],
}

NUM_CLASSES = 10
FLATTEN_FEATURES = 512


def make_layers(cfg: Sequence[Union[int, str]], in_channels: int = 3) -> nn.Sequential:
    """Build the feature extractor (reference `_make_layers`, `model.py:11-27`)."""
    layers: List[nn.Module] = []
    for entry in cfg:
        if entry == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers.append(nn.Conv2d(in_channels, int(entry), kernel_size=3, stride=1, padding=1, bias=True))
            layers.append(nn.BatchNorm2d(int(entry)))
            layers.append(nn.ReLU(inplace=True))
            in_channels = int(entry)
    return nn.Sequential(*layers)


class ConvBlockSpec:
    """Static description of one conv(+BN+ReLU)(+pool) block used by the fused paths."""

    __slots__ = ("conv_idx", "bn_idx", "cin", "cout", "pool", "hw")

    def __init__(self, conv_idx: int, bn_idx: int, cin: int, cout: int, pool: bool, hw: int):
        self.conv_idx, self.bn_idx, self.cin, self.cout, self.pool, self.hw = conv_idx, bn_idx, cin, cout, pool, hw

    def __repr__(self) -> str:  # pragma: no cover - debug helper
        return (f"ConvBlockSpec(conv=layers.{self.conv_idx}, cin={self.cin}, cout={self.cout}, "
                f"hw={self.hw}, pool={self.pool})")


def block_specs(cfg: Sequence[Union[int, str]], in_hw: int = 32) -> List[ConvBlockSpec]:
    """Group the Sequential indices into fused blocks (conv, bn, relu[, pool])."""
    specs: List[ConvBlockSpec] = []
    idx, cin, hw = 0, 3, in_hw
    for entry in cfg:
        if entry == "M":
            specs[-1].pool = True
            idx += 1
            hw //= 2
        else:
            specs.append(ConvBlockSpec(idx, idx + 1, cin, int(entry), False, hw))
            idx += 3
            cin = int(entry)
    return specs


class VGG(nn.Module):
    """VGG for 3x32x32 input, 10 classes (reference `_VGG`, `model.py:30-46`)."""

    def __init__(self, name: str = "VGG11", native: bool = False):
        super().__init__()
        if name not in CFG:
            raise ValueError(f"unknown VGG config {name!r}; choose from {sorted(CFG)}")
        self.name = name
        self.cfg = CFG[name]
        self.layers = make_layers(self.cfg)
        self.fc1 = nn.Linear(FLATTEN_FEATURES, NUM_CLASSES)
        self.native = native
        self._specs = block_specs(self.cfg)

    @property
    def specs(self) -> List[ConvBlockSpec]:
        return self._specs

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.native and x.is_cuda:
            from ..ops import functional as F_native
            return F_native.vgg_forward(self, x)
        y = self.layers(x)
        y = y.view(y.size(0), -1)
        return self.fc1(y)


def VGG11(native: bool = False) -> VGG:
    return VGG("VGG11", native=native)


def VGG13(native: bool = False) -> VGG:
    return VGG("VGG13", native=native)


def VGG16(native: bool = False) -> VGG:
    return VGG("VGG16", native=native)


def VGG19(native: bool = False) -> VGG:
    return VGG("VGG19", native=native)


def param_count(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
