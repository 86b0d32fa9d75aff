"""CIFAR-10-shaped data pipeline.

The reference reads CIFAR-10 through torchvision with two DataLoader worker
processes (`master/part1/part1.py:66-93`) and shards it with
``DistributedSampler`` (`master/part2b/part2b.py:100`). torchvision is not
installed and there is no network, so this module provides:

* ``SyntheticCIFAR10`` — deterministic, *learnable* uint8 HWC images (class
  templates + noise) with CIFAR's sizes (50,000 train / 10,000 test) and layout;
* CPU transforms with torchvision semantics: ``RandomCrop(32, padding=4)``,
  ``RandomHorizontalFlip``, ``ToTensor``, ``Normalize(mean, std)`` using the
  reference's constants (`master/part1/part1.py:66-77`);
* ``DistributedSampler`` — index-for-index identical to
  ``torch.utils.data.DistributedSampler`` (shuffle by ``seed + epoch``, pad by
  wrap-around to a multiple of N, stride ``rank::N``);
* ``DeviceDataLoader`` — the MI355X path: the whole uint8 dataset resident in HBM
  (150 MB of 288 GB), per-epoch augmentation parameters drawn once on the host,
  and one fused HIP kernel (``ops.augment``) that gathers the batch by sampler
  indices and applies crop/flip/normalise, writing NCHW or NHWC fp32 directly.
  No worker processes, no pinned-memory copies, no H2D traffic per step.
"""
from __future__ import annotations

import math
from typing import Iterator, List, Optional, Sequence, Tuple

import torch

CIFAR_MEAN = [x / 255.0 for x in (125.3, 123.0, 113.9)]
CIFAR_STD = [x / 255.0 for x in (63.0, 62.1, 66.7)]
TRAIN_SIZE, TEST_SIZE = 50_000, 10_000
NUM_CLASSES = 10
PAD = 4


class SyntheticCIFAR10(torch.utils.data.Dataset):
    """Deterministic synthetic CIFAR-10 (uint8 [N, 32, 32, 3] + int64 labels).

    Each class owns a smooth random colour template; a sample is the template
    with a random brightness/contrast jitter and per-pixel noise, so a CNN can
    learn it (loss decreases) yet it is not trivially separable.
    """

    def __init__(self, train: bool = True, size: Optional[int] = None, seed: int = 0,
                 transform=None, materialize: bool = True):
        self.train = train
        self.size = size if size is not None else (TRAIN_SIZE if train else TEST_SIZE)
        self.seed = seed + (0 if train else 7919)
        self.transform = transform
        self._data: Optional[torch.Tensor] = None
        self._labels: Optional[torch.Tensor] = None
        if materialize:
            self._materialize()

    @staticmethod
    def templates(seed: int = 0) -> torch.Tensor:
        g = torch.Generator().manual_seed(1234 + seed)
        coarse = torch.rand(NUM_CLASSES, 3, 4, 4, generator=g)
        t = torch.nn.functional.interpolate(coarse, size=(32, 32), mode="bilinear", align_corners=False)
        return (t * 200 + 28).permute(0, 2, 3, 1).contiguous()  # [10, 32, 32, 3] float

    def _materialize(self) -> None:
        g = torch.Generator().manual_seed(self.seed)
        labels = torch.randint(0, NUM_CLASSES, (self.size,), generator=g)
        tmpl = self.templates(0)
        data = torch.empty(self.size, 32, 32, 3, dtype=torch.uint8)
        chunk = 4096
        for s in range(0, self.size, chunk):
            e = min(self.size, s + chunk)
            n = e - s
            scale = 0.7 + 0.6 * torch.rand(n, 1, 1, 1, generator=g)
            shift = 40 * (torch.rand(n, 1, 1, 1, generator=g) - 0.5)
            noise = 48 * torch.randn(n, 32, 32, 3, generator=g)
            img = tmpl[labels[s:e]] * scale + shift + noise
            data[s:e] = img.clamp_(0, 255).to(torch.uint8)
        self._data, self._labels = data, labels

    @property
    def data(self) -> torch.Tensor:
        if self._data is None:
            self._materialize()
        return self._data

    @property
    def targets(self) -> torch.Tensor:
        if self._labels is None:
            self._materialize()
        return self._labels

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, idx: int):
        img = self.data[idx]
        label = int(self.targets[idx])
        if self.transform is not None:
            img = self.transform(img)
        return img, label


# ----------------------------------------------------------- torchvision-equivalent transforms
class Compose:
    def __init__(self, ts):
        self.ts = list(ts)

    def __call__(self, x):
        for t in self.ts:
            x = t(x)
        return x


class ToTensor:
    """uint8 HWC -> float CHW in [0, 1] (torchvision ``ToTensor``)."""

    def __call__(self, img: torch.Tensor) -> torch.Tensor:
        return img.permute(2, 0, 1).float().div_(255.0)


class Normalize:
    def __init__(self, mean: Sequence[float], std: Sequence[float]):
        self.mean = torch.tensor(mean).view(-1, 1, 1)
        self.std = torch.tensor(std).view(-1, 1, 1)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        return (x - self.mean) / self.std


class RandomCrop:
    """``RandomCrop(size, padding)`` on a uint8 HWC image (zero padding)."""

    def __init__(self, size: int = 32, padding: int = PAD, generator: Optional[torch.Generator] = None):
        self.size, self.padding, self.g = size, padding, generator

    def __call__(self, img: torch.Tensor) -> torch.Tensor:
        p = self.padding
        h, w, c = img.shape
        padded = torch.zeros(h + 2 * p, w + 2 * p, c, dtype=img.dtype)
        padded[p:p + h, p:p + w] = img
        i = int(torch.randint(0, h + 2 * p - self.size + 1, (1,), generator=self.g))
        j = int(torch.randint(0, w + 2 * p - self.size + 1, (1,), generator=self.g))
        return padded[i:i + self.size, j:j + self.size]


class RandomHorizontalFlip:
    def __init__(self, p: float = 0.5, generator: Optional[torch.Generator] = None):
        self.p, self.g = p, generator

    def __call__(self, img: torch.Tensor) -> torch.Tensor:
        if float(torch.rand(1, generator=self.g)) < self.p:
            return img.flip(1)
        return img


def train_transform() -> Compose:
    return Compose([RandomCrop(32, PAD), RandomHorizontalFlip(), ToTensor(), Normalize(CIFAR_MEAN, CIFAR_STD)])


def test_transform() -> Compose:
    return Compose([ToTensor(), Normalize(CIFAR_MEAN, CIFAR_STD)])


# ----------------------------------------------------------------------- sampler
class DistributedSampler(torch.utils.data.Sampler):
    """Same index sequence as ``torch.utils.data.DistributedSampler``.

    ``set_epoch`` is provided (the reference never calls it, so every epoch
    repeats epoch 0's permutation there; callers here do call it).
    """

    def __init__(self, dataset_len: int, num_replicas: int = 1, rank: int = 0, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if not 0 <= rank < num_replicas:
            raise ValueError(f"invalid rank {rank} for {num_replicas} replicas")
        self.n, self.num_replicas, self.rank = dataset_len, num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        if drop_last and dataset_len % num_replicas != 0:
            self.num_samples = math.ceil((dataset_len - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(dataset_len / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def indices(self) -> List[int]:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad <= len(idx):
                idx += idx[:pad]
            else:
                idx += (idx * math.ceil(pad / len(idx)))[:pad]
        else:
            idx = idx[: self.total_size]
        return idx[self.rank: self.total_size: self.num_replicas]

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices())

    def __len__(self) -> int:
        return self.num_samples


def make_cpu_loader(dataset, batch_size: int, sampler=None, shuffle: bool = False, num_workers: int = 0):
    return torch.utils.data.DataLoader(dataset, batch_size=batch_size, sampler=sampler,
                                       shuffle=shuffle if sampler is None else False,
                                       num_workers=num_workers)


# ------------------------------------------------------------ device-resident path
def augment_params(n: int, seed: int, epoch: int, train: bool = True) -> torch.Tensor:
    """Per-sample (dy, dx, flip) int32 table for one epoch, keyed by dataset index."""
    if not train:
        p = torch.zeros(n, 3, dtype=torch.int32)
        p[:, 0] = PAD
        p[:, 1] = PAD
        return p
    g = torch.Generator().manual_seed(0x5EED + 1_000_003 * seed + epoch)
    off = torch.randint(0, 2 * PAD + 1, (n, 2), generator=g, dtype=torch.int64)
    flip = (torch.rand(n, generator=g) < 0.5).to(torch.int64)
    return torch.cat([off, flip[:, None]], 1).to(torch.int32)


def augment_reference(data_u8: torch.Tensor, idx: torch.Tensor, params: torch.Tensor,
                      channels_last: bool = False) -> torch.Tensor:
    """Pure-PyTorch fp32 reference of the fused augmentation kernel.

    data_u8: [N, 32, 32, 3] uint8; idx: [B] int64 dataset indices; params:
    [N, 3] (dy, dx, flip) -> normalised float [B, 3, 32, 32] (or NHWC).
    """
    imgs = data_u8[idx].float()  # [B, 32, 32, 3]
    B = imgs.shape[0]
    padded = torch.zeros(B, 32 + 2 * PAD, 32 + 2 * PAD, 3, dtype=imgs.dtype, device=imgs.device)
    padded[:, PAD:PAD + 32, PAD:PAD + 32] = imgs
    p = params[idx].long()
    ar = torch.arange(32, device=imgs.device)
    rows = (p[:, 0:1] + ar[None]).clamp_(0, 39)  # [B, 32]
    cols = (p[:, 1:2] + ar[None]).clamp_(0, 39)
    flip = p[:, 2].bool()
    cols = torch.where(flip[:, None], cols.flip(1), cols)
    out = padded[torch.arange(B, device=imgs.device)[:, None, None], rows[:, :, None], cols[:, None, :]]
    mean = torch.tensor(CIFAR_MEAN, device=imgs.device)
    std = torch.tensor(CIFAR_STD, device=imgs.device)
    out = (out / 255.0 - mean) / std  # [B, 32, 32, 3]
    return out.contiguous() if channels_last else out.permute(0, 3, 1, 2).contiguous()


class DeviceDataLoader:
    """Iterates batches of (images fp32, labels int64) produced on the device."""

    def __init__(self, dataset: SyntheticCIFAR10, batch_size: int, sampler: Optional[DistributedSampler] = None,
                 train: bool = True, device: Optional[torch.device] = None, layout: str = "nchw",
                 seed: int = 0, drop_last: bool = False, use_native: Optional[bool] = None):
        self.dataset, self.batch_size, self.sampler = dataset, batch_size, sampler
        self.train, self.layout, self.seed, self.drop_last = train, layout, seed, drop_last
        self.device = device or (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.data = dataset.data.to(self.device)
        self.labels = dataset.targets.to(self.device)
        self.epoch = 0
        if use_native is None:
            use_native = self.device.type == "cuda"
        self.use_native = use_native

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
        if self.sampler is not None:
            self.sampler.set_epoch(epoch)

    def _indices(self) -> List[int]:
        if self.sampler is not None:
            return self.sampler.indices()
        return list(range(len(self.dataset)))

    def __len__(self) -> int:
        n = len(self.sampler) if self.sampler is not None else len(self.dataset)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        idx_all = torch.tensor(self._indices(), dtype=torch.int64).to(self.device)
        params = augment_params(len(self.dataset), self.seed, self.epoch, self.train).to(self.device)
        nb = len(self)
        for b in range(nb):
            idx = idx_all[b * self.batch_size:(b + 1) * self.batch_size]
            yield self.make_batch(idx, params), self.labels[idx]

    def make_batch(self, idx: torch.Tensor, params: torch.Tensor) -> torch.Tensor:
        nhwc = self.layout == "nhwc"
        if self.use_native:
            from ..ops import native
            return native.augment(self.data, idx, params, nhwc)
        return augment_reference(self.data, idx, params, channels_last=nhwc)

    @property
    def n_samples(self) -> int:
        return len(self.sampler) if self.sampler is not None else len(self.dataset)
