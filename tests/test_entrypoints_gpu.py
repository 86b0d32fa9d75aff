"""Tutorial entrypoints on an MI355X: with no engine flags they run the native HIP engine
(reference loops: `master/part1/part1.py:20-44`, `master/part3/part3.py:114-123`), the
loss goes down, and a mid-epoch checkpoint/resume is bitwise the uninterrupted run."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = [pytest.mark.gpu]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--train-size", "8192", "--test-size", "512", "--log-every", "5"]


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(scope="module")
def tune_cache(tmp_path_factory):
    # one conv tile table for every run of this module: identical kernels -> bitwise comparable
    path = str(tmp_path_factory.mktemp("tune") / "tiles.json")
    old = os.environ.get("CS744_TUNE_CACHE")
    os.environ["CS744_TUNE_CACHE"] = path
    yield path
    if old is None:
        os.environ.pop("CS744_TUNE_CACHE", None)
    else:
        os.environ["CS744_TUNE_CACHE"] = old


def _run(part, args):
    from cs744_pytorch_distributed_tutorial_amd.config import config_from_args
    from cs744_pytorch_distributed_tutorial_amd.train import run
    return run(config_from_args(part, args))


def test_part1_defaults_to_native_and_learns(gpu, tune_cache, capsys):
    res = _run("part1", SMALL + ["--steps", "30"])
    out = capsys.readouterr().out
    assert res["engine"] == "native" and "[engine] native" in out
    assert "0 loss: " in out and "Test set: Average loss:" in out
    losses = [l for _, _, l in res["losses"]]
    # lr 0.1 from random init spikes the loss over the first steps; which logged step then sits
    # lowest is chaotic (bit-level changes in any kernel move it): the run must come back below its
    # starting loss, not at one fixed step (as test_part3_torchrun_world1_native)
    assert len(losses) == 6 and min(losses[-3:]) < losses[0], losses


def test_part1_resume_mid_epoch_is_bitwise(gpu, tune_cache, tmp_path):
    ck = str(tmp_path / "ck.pt")
    full = _run("part1", SMALL + ["--steps", "12", "--no-eval"])
    half = _run("part1", SMALL + ["--steps", "6", "--no-eval", "--checkpoint", ck])
    assert half["resume_point"] == (0, 6)
    st = torch.load(ck, weights_only=True)
    assert (st["epoch"], st["iter"]) == (0, 6) and len(st["model"]) == 58
    rest = _run("part1", SMALL + ["--steps", "12", "--no-eval", "--resume", ck])
    for k, v in full["final_state"].items():
        assert torch.equal(v, rest["final_state"][k]), k


@pytest.mark.slow
def test_part3_torchrun_world1_native(gpu, tune_cache):
    from conftest import torchrun_cmd
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = torchrun_cmd(1) + ["-m",
           "cs744_pytorch_distributed_tutorial_amd.entrypoints.part3", "--steps", "30"] + SMALL[:-1] + ["1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-1500:]
    assert "[engine] native" in r.stdout, r.stdout[-800:]
    losses = [float(l.split()[-1]) for l in r.stdout.splitlines() if l[:1].isdigit() and " loss: " in l]
    # lr 0.1 from random init spikes the loss over the first ~10 steps (to 15-20 at batch 64); which
    # logged step then sits lowest is chaotic (bit-level changes in any kernel move it), so the check
    # is that the run comes back below its starting loss, not the value at one fixed step
    assert len(losses) == 30 and all(l == l and l < 1e3 for l in losses), losses
    assert min(losses[-10:]) < losses[0], losses
