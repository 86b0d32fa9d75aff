"""BASELINE.json extension models on CPU: ResNet family shapes / parameter
counts / key layout, Llama-3 configs (8.03 B parameters for llama3-8b), the LM
reference ops, and the autograd-path trainer's DDP keeping replicas identical
over a real 2-rank gloo world."""
import pytest
import torch

from mp_util import run_world


def test_resnet_counts_and_keys():
    from cs744_pytorch_distributed_tutorial_amd.models import resnet
    m = resnet.resnet50()
    assert sum(p.numel() for p in m.parameters()) == 25_557_032
    sd = m.state_dict()
    assert len(sd) == 320 and "layer4.2.conv3.weight" in sd and "layer1.0.downsample.1.running_var" in sd
    assert sum(p.numel() for p in resnet.resnet18().parameters()) == 11_689_512
    y = m.eval()(torch.randn(1, 3, 64, 64))
    assert y.shape == (1, 1000)


def test_llama_configs_and_forward():
    from cs744_pytorch_distributed_tutorial_amd.models import llama
    assert abs(llama.param_count(llama.CONFIGS["llama3-8b"]) - 8.03e9) < 0.01e9
    m = llama.build("llama-tiny")
    assert sum(p.numel() for p in m.parameters()) == llama.param_count(m.cfg)
    t = torch.randint(0, m.vocab_size, (2, 12))
    out = m(t)
    assert out.shape == (2, 12, m.vocab_size)
    # causal: position 3's logits do not depend on later tokens
    t2 = t.clone()
    t2[:, 5:] = (t2[:, 5:] + 1) % m.vocab_size
    torch.testing.assert_close(m(t2)[:, :5], out[:, :5])


def test_lm_reference_ops():
    from cs744_pytorch_distributed_tutorial_amd.models.llama import rope_tables
    from cs744_pytorch_distributed_tutorial_amd.ops import lm
    x = torch.randn(2, 6, 3, 8)
    cos, sin = rope_tables(6, 8, 10000.0, "cpu")
    y = lm.rope_ref(x, cos, sin)
    # rotation preserves pair norms; position 0 is the identity
    torch.testing.assert_close(y.view(2, 6, 3, 4, 2).norm(dim=-1), x.view(2, 6, 3, 4, 2).norm(dim=-1))
    torch.testing.assert_close(y[:, 0], x[:, 0])
    w = torch.rand(8) + 0.5
    r = lm.rms_norm_ref(x, w, 1e-5)
    torch.testing.assert_close((r / w).pow(2).mean(-1), torch.ones(2, 6, 3), rtol=1e-3, atol=1e-3)


def _lm_ddp(rank, world, sync):
    from cs744_pytorch_distributed_tutorial_amd.runtime.torch_trainer import TorchTrainer
    torch.set_num_threads(1)
    tr = TorchTrainer("llama-tiny", 4, torch.device("cpu"), rank, world, sync=sync, comm="torch", bucket_mb=0.5,
                      lr=0.05, weight_decay=0.0, seq_len=32, fused_sgd=False)
    for _ in range(3):
        tr.step()
    return torch.cat([p.detach().reshape(-1) for p in tr.module.parameters()])


def _lm_ddp_transport(rank, world, gdt):
    import os
    os.environ["CS744_GRAD_COMM_DTYPE"] = gdt
    from cs744_pytorch_distributed_tutorial_amd.runtime.torch_trainer import TorchTrainer
    torch.set_num_threads(1)
    tr = TorchTrainer("llama-tiny", 4, torch.device("cpu"), rank, world, sync="ddp", comm="torch", bucket_mb=0.5,
                      lr=0.05, weight_decay=0.0, seq_len=32, fused_sgd=False)
    p0 = torch.cat([p.detach().reshape(-1) for p in tr.module.parameters()]).clone()
    for _ in range(3):
        tr.step()
    return {"p": torch.cat([p.detach().reshape(-1) for p in tr.module.parameters()]), "p0": p0,
            "wire": str(tr.net.grad_comm_dtype)}


@pytest.mark.slow
def test_lm_ddp_bf16_gradient_transport_matches_fp32():
    """bf16 gradient transport (the LM default: half the xGMI bytes) vs fp32 transport, 2-rank gloo:
    replicas stay identical and the trained weights agree to bf16 rounding of the gradients."""
    bf = run_world(_lm_ddp_transport, 2, "bf16")
    fp = run_world(_lm_ddp_transport, 2, "fp32")
    assert bf[0]["wire"] == "torch.bfloat16" and fp[0]["wire"] == "None"
    assert torch.equal(torch.as_tensor(bf[0]["p"]), torch.as_tensor(bf[1]["p"]))
    pb, pf, p0 = (torch.as_tensor(t) for t in (bf[0]["p"], fp[0]["p"], fp[0]["p0"]))
    step = (pf - p0).abs().max()
    assert step > 0
    # each gradient element is rounded to 8 significant bits once (+ the average): the weight
    # difference stays a small fraction of the 3-step update, and not zero (the wire is bf16)
    assert 0 < (pb - pf).abs().max() <= 2e-2 * step


@pytest.mark.slow
@pytest.mark.parametrize("sync", ["ddp", "allreduce"])
def test_lm_data_parallel_replicas_identical(sync):
    outs = run_world(_lm_ddp, 2, sync)
    assert torch.equal(outs[0], outs[1])
