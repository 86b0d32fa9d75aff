"""Bucket assignment (SURVEY.md §2.5 C-6 measured DDP buckets; §5.8 xGMI policy)."""
from cs744_pytorch_distributed_tutorial_amd.models import VGG11
from cs744_pytorch_distributed_tutorial_amd.parallel.buckets import MiB, assign_by_size, build_buckets


def _names_params():
    m = VGG11()
    names = [n for n, _ in m.named_parameters()]
    return names, list(m.parameters())


def test_ddp_size_policy_matches_reference_buckets():
    names, params = _names_params()
    bs = build_buckets(params, "size", 25.0, 1.0, names)
    assert [round(b.nbytes / MiB, 2) for b in bs] == [9.03, 25.9, 0.29]
    assert [names[i] for i in bs[0].param_indices] == ["fc1.bias", "fc1.weight", "layers.26.bias",
                                                       "layers.26.weight", "layers.25.bias", "layers.25.weight"]
    assert names[bs[1].param_indices[0]] == "layers.23.bias" and names[bs[1].param_indices[-1]] == "layers.8.weight"
    assert names[bs[2].param_indices[-1]] == "layers.0.weight"


def test_layer_policy_aligned_to_layers():
    names, params = _names_params()
    bs = build_buckets(params, "layer", 4.0, 1.0, names)
    assert len(bs) == 5
    for b in bs:
        first = names[b.param_indices[0]]
        assert first.endswith(".bias") and (first.startswith("fc1") or names.index(first) % 4 == 3)
    # contiguous, covering everything exactly once
    assert sorted(i for b in bs for i in b.param_indices) == list(range(len(params)))
    off = 0
    for b in bs:
        assert b.offset == off
        off += b.numel
    assert off == sum(p.numel() for p in params)


def test_assign_by_size_closes_on_reaching_cap():
    assert assign_by_size([1, 1, 1, 1], cap_bytes=2, first_cap_bytes=1) == [[3], [2, 1], [0]]
