"""The auxiliary benchmarks run end to end as real torchrun worlds on CPU/gloo:
the collective bus-bandwidth sweep (BASELINE.json's "all-reduce bus BW") and the
per-sync-mode training sweep (the tutorial's part2a/2a_extra/2b/3 ordering)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import torchrun_cmd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torchrun(module, args, nproc=2, timeout=240):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    cmd = torchrun_cmd(nproc) + ["-m", module] + args
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    return [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]


def test_busbw_factors():
    from cs744_pytorch_distributed_tutorial_amd.bench.busbw import FACTORS, parse_size
    assert FACTORS["all_reduce"](8) == pytest.approx(1.75)
    assert FACTORS["all_gather"](4) == pytest.approx(0.75)
    assert FACTORS["broadcast"](8) == 1.0
    assert parse_size("4K") == 4096 and parse_size("35.21M") == int(35.21 * (1 << 20))


def test_vgg_bucket_plan_covers_whole_gradient():
    from cs744_pytorch_distributed_tutorial_amd.bench.busbw import bucket_plan_sizes, VGG11_GRAD_FLOATS
    sizes = bucket_plan_sizes(4.0)
    assert len(sizes) > 1
    # buckets are the flat buffer incl. 256-B alignment padding: >= the reference's 36,924,456 B
    assert VGG11_GRAD_FLOATS * 4 <= sum(sizes) < VGG11_GRAD_FLOATS * 4 * 1.01


@pytest.mark.slow
@pytest.mark.parametrize("op", ["all_reduce", "all_gather", "reduce_scatter", "broadcast"])
def test_busbw_sweep_gloo(op):
    rows = _torchrun("cs744_pytorch_distributed_tutorial_amd.bench.busbw",
                     ["--device", "cpu", "--op", op, "--sizes", "4K,256K", "--iters", "2", "--warmup", "1"])
    assert [r["bytes"] for r in rows] == [4096, 262144]
    for r in rows:
        assert r["n"] == 2 and r["busbw_GBps"] > 0 and r["op"] == op


@pytest.mark.slow
def test_busbw_vgg_buckets_gloo():
    rows = _torchrun("cs744_pytorch_distributed_tutorial_amd.bench.busbw",
                     ["--device", "cpu", "--vgg-buckets", "9", "--iters", "1", "--warmup", "1"])
    assert rows[0]["bench"] == "vgg11_ddp_buckets" and rows[0]["buckets"] >= 2


@pytest.mark.slow
def test_sync_modes_gloo():
    rows = _torchrun("cs744_pytorch_distributed_tutorial_amd.bench.sync_modes",
                     ["--device", "cpu", "--batch-size", "8", "--steps", "2", "--warmup", "1",
                      "--modes", "gather_scatter,p2p,allreduce,ddp"], timeout=400)
    assert [r["mode"] for r in rows] == ["gather_scatter", "p2p", "allreduce", "ddp"]
    assert all(r["images_per_s"] > 0 and r["final_loss"] == r["final_loss"] for r in rows)
