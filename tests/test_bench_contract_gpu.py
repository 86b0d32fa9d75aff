"""bench.py's one-line JSON contract on an MI355X: the metric/config BASELINE.json names, the
whole-job value consistent with ms_per_step, exactly the requested steps/warmup."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = [pytest.mark.gpu]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_line():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = subprocess.run([sys.executable, "bench.py", "--steps", "7", "--warmup", "3"], cwd=ROOT, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-1500:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert d["metric"].startswith("images/sec (whole node) VGG-11 CIFAR-shape")
    assert base["metric"].startswith(d["metric"])
    assert d["unit"] == "images/s" and d["n_gpus"] == 1 and d["steps"] == 7 and d["warmup"] == 3
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "fp32"
    assert "synthetic" in d["data"]
    c = d["config"]
    assert c["model"] == "VGG11" and c["global_batch"] == 64 and c["parallelism"] == "dp1" and c["seq_len"] is None
    assert d["value"] > 0 and abs(d["value"] - 64 * 1e3 / d["ms_per_step"]) / d["value"] < 1e-3
    assert d["vs_baseline"] == pytest.approx(d["value"] / 554.0, rel=1e-2)


def test_bench_two_ranks_staged_json_line():
    """The N > 1 branch of bench.py, exactly as the driver launches it (torch.distributed.run, one
    process per rank), with the staged transport so both ranks fit on the 1-GPU box: process-group
    init, the C++ data-parallel step (bucket all-reduces forked from the backward), the barrier +
    sync bracket, max-over-ranks time, the busBW report after the window, and ONE JSON line."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from conftest import torchrun_cmd
    cmd = torchrun_cmd(2) + ["bench.py", "--gpus", "2",
           "--comm", "staged", "--steps", "5", "--warmup", "2", "--busbw-iters", "3"]
    env = dict(os.environ, CS744_BENCH_CALIBRATE="0")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 5 and d["warmup"] == 2
    c = d["config"]
    assert c["comm"] == "staged" and c["parallelism"] == "dp2" and c["global_batch"] == 128
    assert c["sync"] == "ddp" and c["engine"] == "native"
    assert d["value"] > 0 and abs(d["value"] - 128 * 1e3 / d["ms_per_step"]) / d["value"] < 1e-3
    bw = d["busbw_GBps"]
    assert bw and all(v > 0 for v in bw.values()), bw
    assert "9.00MiB" in bw or any(k.endswith("MiB") for k in bw)


def test_bench_one_rank_rccl_probe_fields():
    """World 1 with a one-rank native RCCL communicator (--comm-probe 1): the data-parallel step's
    collectives run on the real RcclComm, and the JSON names the RCCL runtime actually loaded next
    to the header the communicator was built against, and its CTA budget."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = subprocess.run([sys.executable, "bench.py", "--steps", "4", "--warmup", "2", "--comm-probe", "1"], cwd=ROOT,
                       capture_output=True, text=True, timeout=240, env=dict(os.environ, CS744_BENCH_CALIBRATE="0"))
    assert r.returncode == 0, r.stderr[-1500:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    c = d["config"]
    assert c["comm"] == "probe:1" and d["comm_fallback"] is False
    v = c["rccl_version"]
    assert v["runtime"] >= 21700 and v["header"] >= 21700 and v["runtime"] // 10000 == v["header"] // 10000 == 2, v
    assert c["comm_ctas"] is not None


def test_bench_two_ranks_rccl_gloo_control_plane_fallback():
    """`--comm rccl` at N = 2 exactly as the driver launches it, on the 1-GPU box: the control plane
    is a gloo process group (no ProcessGroupNCCL next to the native communicator), both ranks build
    the native RcclComm on the same device, RCCL refuses the duplicate GPU on every rank, the agreed
    fallback takes both ranks to the staged communicator (the same C++ step over the gloo group), and
    the line says so at the top level."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from conftest import torchrun_cmd
    cmd = torchrun_cmd(2) + ["bench.py", "--gpus", "2", "--comm", "rccl", "--steps", "3", "--warmup", "2",
                             "--busbw-iters", "0"]
    # both ranks on cuda:0 (LOCAL_RANK 1 has no device of its own here)
    env = dict(os.environ, CS744_BENCH_CALIBRATE="0", HIP_VISIBLE_DEVICES="0")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    c = d["config"]
    assert c["control_plane"] == "gloo" and c["parallelism"] == "dp2"
    assert "runtime" in c["rccl_version"]
    if c["comm"] == "rccl":  # a stack that lets two ranks share a device
        assert d["comm_fallback"] is False
    else:
        assert d["comm_fallback"] is True and c["comm"] == "staged", c
