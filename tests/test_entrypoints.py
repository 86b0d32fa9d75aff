"""Integration: the reference-style entrypoints run end to end on CPU/gloo
(SURVEY.md §4.2 "Integration"): part1 single-process training, the part1
send/recv ping-pong, and part2a / part2a_extra / part2b / part3 as a real
multi-process world launched through the entrypoints' own ``main``. Small
synthetic datasets keep them fast; losses must be finite, the replicas must
end bit-identical (checked through the engine's ``final_params``), and the
printed lines keep the reference formats."""
import os
import subprocess
import sys

import pytest
import torch

from mp_util import run_world

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--device", "cpu", "--train-size", "96", "--test-size", "32", "--steps", "3", "--threads", "1",
          "--log-every", "1"]


def test_part1_single_process(capsys):
    from cs744_pytorch_distributed_tutorial_amd.config import config_from_args
    from cs744_pytorch_distributed_tutorial_amd.train import run
    cfg = config_from_args("part1", COMMON + ["--batch-size", "32"])
    res = run(cfg)
    out = capsys.readouterr().out
    assert "0 loss: " in out and "Test set: Average loss:" in out
    ep = res["epochs"][0]
    assert ep["train"]["images"] == 96 and ep["test"]["total"] == 32
    assert all(v == v for _, v in ep["train"]["losses"])


def _part(rank, world, part, extra):
    from cs744_pytorch_distributed_tutorial_amd.config import config_from_args
    from cs744_pytorch_distributed_tutorial_amd.train import run
    cfg = config_from_args(part, COMMON + ["--batch-size", "16", "--num-nodes", str(world), "--rank", str(rank)]
                           + extra)
    res = run(cfg)
    return torch.cat([p.reshape(-1) for p in res["final_params"]])


@pytest.mark.slow
@pytest.mark.parametrize("part", ["part2a", "part2a_extra", "part2b", "part3"])
def test_distributed_parts_keep_replicas_identical(part):
    outs = run_world(_part, 2, part, [])
    assert torch.equal(outs[0], outs[1]), part


@pytest.mark.slow
def test_distributed_parts_agree_with_each_other():
    # equivalence oracle: every sync strategy yields the same weights
    ref = run_world(_part, 2, "part2b", [])[0]
    for part in ("part2a", "part2a_extra", "part3"):
        out = run_world(_part, 2, part, [])[0]
        torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-6, msg=part)


@pytest.mark.slow
def test_pingpong_entrypoint_cli(tmp_path):
    from conftest import HostedStore
    hosted = HostedStore(2)
    port = str(hosted.port)
    env = hosted.env(dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1"))
    cmd = [sys.executable, "-m", "cs744_pytorch_distributed_tutorial_amd.entrypoints.part1_pingpong",
           "--master-ip", "127.0.0.1", "--num-nodes", "2"]
    procs = [subprocess.Popen(cmd + ["--rank", str(r), "--port", port], env=env, cwd=ROOT, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=180) for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert "round_trip_us" in outs[0][0] or "rtt" in outs[0][0].lower(), outs[0][0]
