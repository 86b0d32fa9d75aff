"""Autograd-path trainer for every model that is not VGG (ResNet family now; the
decoder LM of ``models.llama``): PyTorch-ROCm modules for the layer math, the
framework's own data-parallel runtime around them.

* DDP = ``parallel.ddp.DistributedDataParallel`` (flat gradient buffer, grads as
  bucket views, post-accumulate hooks launch bucketed all-reduce(AVG) while
  autograd is still producing earlier layers' gradients) over the native
  ``RcclComm`` (``comm="rccl"``) or ProcessGroupNCCL (``comm="torch"``);
  or any explicit strategy of ``parallel.sync`` (part2a / part2a_extra / part2b);
* optimizer = ``ops.optim.FusedSGD`` (one multi-tensor HIP launch per step);
* ResNets run the framework's channels-last path by default (``models.resnet`` ``layout="nhwc"``:
  hipBLASLt GEMM convolutions over gfx950 im2col / BatchNorm / pool kernels, no MIOpen);
  ``CS744_RESNET_LAYOUT=nchw`` selects MIOpen convolutions on NCHW with the fused NCHW
  BatchNorm kernels. MIOpen's own channels_last kernels (``CS744_CHANNELS_LAST=1`` with the
  NCHW layout) measured 10-18x SLOWER on MI355X (torch 2.10+rocm7.0: composable_kernel
  weight-gradient kernels up to 225 ms each). Optionally under bf16 autocast
  (``dtype="bf16"``; master weights and the optimizer stay fp32);
* data = device-resident synthetic batches of the named shape (no host traffic).
"""
from __future__ import annotations

from typing import Optional

import os

import torch
import torch.nn as nn

from ..parallel import DistributedDataParallel, make_comm, make_sync
from ..utils.metrics import roctx_range


def build_model(name: str) -> nn.Module:
    from ..models import resnet, vgg
    n = name.lower().replace("-", "")
    if n.startswith("vgg"):
        return vgg.VGG(n.upper())
    if n in ("resnet18", "resnet34", "resnet50", "resnet101"):
        return getattr(resnet, n)(layout=os.environ.get("CS744_RESNET_LAYOUT", "nhwc"))
    if n.startswith("llama") or n.startswith("decoder"):
        from ..models import llama
        return llama.build(name.lower())
    raise ValueError(f"unknown model {name!r}")


class SyntheticBatches:
    """A pool of random, fixed, device-resident samples; each step gathers a random batch.

    Images: uint8 NHWC pool -> fp32/bf16 normalised NCHW(channels_last) batch.
    Tokens: int64 [pool, seq+1] -> (input, target) shifted pair.
    """

    def __init__(self, kind: str, batch: int, device, shape=(3, 224, 224), classes: int = 1000, pool: int = 512,
                 seq: int = 0, vocab: int = 0, seed: int = 0, channels_last: bool = True):
        self.fmt = torch.channels_last if channels_last else torch.contiguous_format
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.kind, self.batch, self.device = kind, batch, device
        self.pool = max(pool, batch)
        if kind == "image":
            c, h, w = shape
            self.data = torch.randint(0, 256, (self.pool, h, w, c), generator=g, dtype=torch.uint8).to(device)
            self.labels = torch.randint(0, classes, (self.pool,), generator=g).to(device)
            self.mean = torch.tensor([0.485, 0.456, 0.406], device=device).view(1, 3, 1, 1) * 255
            self.std = torch.tensor([0.229, 0.224, 0.225], device=device).view(1, 3, 1, 1) * 255
        else:
            self.tokens = torch.randint(0, vocab, (self.pool, seq + 1), generator=g).to(device)
        self.gen = torch.Generator(device=device).manual_seed(seed + 1)

    def next(self):
        idx = torch.randint(0, self.pool, (self.batch,), device=self.device, generator=self.gen)
        if self.kind == "image":
            x = self.data.index_select(0, idx).permute(0, 3, 1, 2).float()
            x = ((x - self.mean) / self.std).contiguous(memory_format=self.fmt)
            return x, self.labels.index_select(0, idx)
        t = self.tokens.index_select(0, idx)
        return t[:, :-1].contiguous(), t[:, 1:].contiguous()


class TorchTrainer:
    def __init__(self, model: str, batch_size: int, device, rank: int = 0, world: int = 1, sync: str = "ddp",
                 comm: str = "rccl", bucket_mb: float = 25.0, bucket_policy: str = "layer", dtype: str = "fp32",
                 lr: float = 0.1, momentum: float = 0.9, weight_decay: float = 1e-4, seed: int = 5000,
                 seq_len: int = 0, fused_sgd: bool = True):
        from ..ops.optim import FusedSGD
        torch.manual_seed(seed)
        # MIOpen find mode for the CNN convolutions (CS744_CONV_BENCHMARK=1): time every solver
        # once per shape instead of taking the heuristic pick (opt-in: for ResNet-50 the search ran
        # for more than 3 minutes on MI355X before the first step finished)
        if os.environ.get("CS744_CONV_BENCHMARK", "0") == "1":
            torch.backends.cudnn.benchmark = True
        self.device, self.world, self.B = device, world, batch_size
        self.model_name = model
        self.module = build_model(model).to(device)
        self.is_lm = hasattr(self.module, "vocab_size")
        self.channels_last = not self.is_lm and os.environ.get("CS744_CHANNELS_LAST", "0") == "1"
        if self.channels_last:
            self.module = self.module.to(memory_format=torch.channels_last)
        self.dtype = dtype
        self.grad_comm_dtype = "fp32"
        if world > 1 and sync == "ddp":
            # gradients travel in fp32 like the reference's DDP; CS744_GRAD_COMM_DTYPE=bf16 halves the
            # all-reduce bytes for the decoder LMs (opt-in: RCCL then sums in bf16 over N ranks, a
            # rounding per hop that no reference fixture pins)
            gdt = os.environ.get("CS744_GRAD_COMM_DTYPE", "fp32")
            self.grad_comm_dtype = gdt
            self.net = DistributedDataParallel(self.module, comm=make_comm(comm), bucket_cap_mb=bucket_mb,
                                               bucket_policy=bucket_policy,
                                               grad_comm_dtype=torch.bfloat16 if gdt == "bf16" else None)
            self.sync = make_sync("none", [])
        else:
            self.net = self.module
            self.sync = make_sync(sync if world > 1 else "none", self.module.parameters())
        params = self.net.parameters()
        self.opt = FusedSGD(params, lr=lr, momentum=momentum, weight_decay=weight_decay) if fused_sgd and \
            torch.cuda.is_available() else torch.optim.SGD(params, lr=lr, momentum=momentum, weight_decay=weight_decay)
        self.crit = nn.CrossEntropyLoss()
        if self.is_lm:
            self.data = SyntheticBatches("tokens", batch_size, device, seq=seq_len or self.module.max_seq,
                                         vocab=self.module.vocab_size, seed=seed)
        else:
            shape = (3, 32, 32) if model.lower().startswith("vgg") else (3, 224, 224)
            classes = 10 if model.lower().startswith("vgg") else 1000
            # the NHWC ResNet reads the batch channels-last (its permute to [B, H, W, C] is then free)
            nhwc = getattr(self.module, "layout", "nchw") == "nhwc"
            self.data = SyntheticBatches("image", batch_size, device, shape=shape, classes=classes, seed=seed,
                                         channels_last=self.channels_last or nhwc)
        self.loss: Optional[torch.Tensor] = None

    def step(self) -> None:
        x, y = self.data.next()
        self.opt.zero_grad()  # DDP re-attaches its bucket views (and zeroes them) in forward
        with roctx_range("cs.forward"), torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.dtype == "bf16"):
            out = self.net(x)
            if self.is_lm:  # fused gfx950 softmax cross-entropy over the bf16 logits (ops.lm)
                from ..ops.lm import cross_entropy
                loss = cross_entropy(out.view(-1, out.shape[-1]), y.view(-1))
            else:
                loss = self.crit(out.float(), y)
        with roctx_range("cs.backward"):  # DDP's bucket all-reduces are enqueued from its hooks in here
            loss.backward()
        with roctx_range("cs.sync"):
            self.sync()
        with roctx_range("cs.sgd"):
            self.opt.step()
        self.loss = loss.detach()

    def last_loss(self) -> float:
        return float(self.loss.item()) if self.loss is not None else float("nan")

    def tokens_per_step(self) -> int:
        return self.B * (self.data.tokens.shape[1] - 1) if self.is_lm else self.B
