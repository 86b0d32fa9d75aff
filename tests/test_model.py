"""Model layout parity with the reference (`master/part1/model.py`)."""
import torch

from cs744_pytorch_distributed_tutorial_amd.models import CFG, VGG, VGG11, VGG13, VGG16, VGG19, block_specs

# 34 parameters of VGG-11 in model.parameters() order
EXPECTED_PARAMS = [
    ("layers.0.weight", (64, 3, 3, 3)), ("layers.0.bias", (64,)), ("layers.1.weight", (64,)), ("layers.1.bias", (64,)),
    ("layers.4.weight", (128, 64, 3, 3)), ("layers.4.bias", (128,)), ("layers.5.weight", (128,)),
    ("layers.5.bias", (128,)), ("layers.8.weight", (256, 128, 3, 3)), ("layers.8.bias", (256,)),
    ("layers.9.weight", (256,)), ("layers.9.bias", (256,)), ("layers.11.weight", (256, 256, 3, 3)),
    ("layers.11.bias", (256,)), ("layers.12.weight", (256,)), ("layers.12.bias", (256,)),
    ("layers.15.weight", (512, 256, 3, 3)), ("layers.15.bias", (512,)), ("layers.16.weight", (512,)),
    ("layers.16.bias", (512,)), ("layers.18.weight", (512, 512, 3, 3)), ("layers.18.bias", (512,)),
    ("layers.19.weight", (512,)), ("layers.19.bias", (512,)), ("layers.22.weight", (512, 512, 3, 3)),
    ("layers.22.bias", (512,)), ("layers.23.weight", (512,)), ("layers.23.bias", (512,)),
    ("layers.25.weight", (512, 512, 3, 3)), ("layers.25.bias", (512,)), ("layers.26.weight", (512,)),
    ("layers.26.bias", (512,)), ("fc1.weight", (10, 512)), ("fc1.bias", (10,)),
]


def test_vgg11_parameter_layout():
    m = VGG11()
    got = [(n, tuple(p.shape)) for n, p in m.named_parameters()]
    assert got == EXPECTED_PARAMS
    assert sum(p.numel() for p in m.parameters()) == 9_231_114


def test_vgg11_state_dict_58_keys():
    sd = VGG11().state_dict()
    assert len(sd) == 58
    keys = list(sd)
    assert keys[:7] == ["layers.0.weight", "layers.0.bias", "layers.1.weight", "layers.1.bias",
                        "layers.1.running_mean", "layers.1.running_var", "layers.1.num_batches_tracked"]
    assert keys[-2:] == ["fc1.weight", "fc1.bias"]


def test_all_configs_forward_shape():
    for name, ctor in [("VGG11", VGG11), ("VGG13", VGG13), ("VGG16", VGG16), ("VGG19", VGG19)]:
        m = ctor().eval()
        y = m(torch.randn(2, 3, 32, 32))
        assert y.shape == (2, 10), name
        specs = block_specs(CFG[name])
        assert sum(1 for e in CFG[name] if e != "M") == len(specs)
        assert specs[-1].pool and specs[-1].cout == 512


def test_unknown_config_rejected():
    import pytest
    with pytest.raises(ValueError):
        VGG("VGG7")


def test_block_specs_vgg11():
    s = block_specs(CFG["VGG11"])
    assert [(b.conv_idx, b.cin, b.cout, b.hw, b.pool) for b in s] == [
        (0, 3, 64, 32, True), (4, 64, 128, 16, True), (8, 128, 256, 8, False), (11, 256, 256, 8, True),
        (15, 256, 512, 4, False), (18, 512, 512, 4, True), (22, 512, 512, 2, False), (25, 512, 512, 2, True)]
