"""Data pipeline parity: sampler == torch's DistributedSampler; augmentation semantics."""
import torch

from cs744_pytorch_distributed_tutorial_amd.utils import data as D


def test_sampler_matches_torch():
    import torch.utils.data.distributed as tdd

    class _DS(torch.utils.data.Dataset):
        def __init__(self, n):
            self.n = n

        def __len__(self):
            return self.n

        def __getitem__(self, i):
            return i

    for n, world in [(50000, 4), (50000, 8), (103, 4), (10, 3)]:
        for epoch in (0, 3):
            for rank in range(world):
                ours = D.DistributedSampler(n, world, rank, shuffle=True, seed=0)
                ref = tdd.DistributedSampler(_DS(n), num_replicas=world, rank=rank, shuffle=True, seed=0)
                ours.set_epoch(epoch)
                ref.set_epoch(epoch)
                assert list(ours) == list(ref)
                assert len(ours) == len(ref)


def test_iteration_counts_appendix_b():
    # 4 ranks x 12,500 samples, batch 64 -> 196 iterations, last batch 20
    s = D.DistributedSampler(50000, 4, 0)
    assert len(s) == 12500 and -(-12500 // 64) == 196 and 12500 - 195 * 64 == 20
    s8 = D.DistributedSampler(50000, 8, 0)
    assert len(s8) == 6250 and -(-6250 // 64) == 98


def test_synthetic_dataset_deterministic_and_shaped():
    a = D.SyntheticCIFAR10(train=True, size=256, seed=0)
    b = D.SyntheticCIFAR10(train=True, size=256, seed=0)
    assert a.data.shape == (256, 32, 32, 3) and a.data.dtype == torch.uint8
    assert torch.equal(a.data, b.data) and torch.equal(a.targets, b.targets)
    assert int(a.targets.min()) >= 0 and int(a.targets.max()) <= 9


def test_augment_reference_matches_per_sample_transforms():
    ds = D.SyntheticCIFAR10(train=True, size=32, seed=1)
    params = D.augment_params(32, seed=0, epoch=2, train=True)
    idx = torch.arange(32)
    out = D.augment_reference(ds.data, idx, params)
    norm = D.Normalize(D.CIFAR_MEAN, D.CIFAR_STD)
    for i in range(32):
        dy, dx, fl = params[i].tolist()
        img = ds.data[i]
        padded = torch.zeros(40, 40, 3, dtype=torch.uint8)
        padded[4:36, 4:36] = img
        crop = padded[dy:dy + 32, dx:dx + 32]
        if fl:
            crop = crop.flip(1)
        ref = norm(D.ToTensor()(crop))
        torch.testing.assert_close(out[i], ref, rtol=1e-5, atol=1e-5)


def test_test_params_are_identity():
    ds = D.SyntheticCIFAR10(train=False, size=8, seed=0)
    p = D.augment_params(8, 0, 0, train=False)
    out = D.augment_reference(ds.data, torch.arange(8), p)
    ref = torch.stack([D.test_transform()(ds.data[i]) for i in range(8)])
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
