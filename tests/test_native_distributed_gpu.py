"""Multi-rank native engine on ONE MI355X.

RCCL refuses two ranks on one device ("Duplicate GPU detected", measured on the 1-GPU
box), so N processes share cuda:0 and talk over gloo:

* ``comm="staged"``: the native C++ ``StagedComm`` (csrc/runtime/staged_comm.h) drives the
  EXACT C++ data-parallel step the N-GPU benchmark runs (``VggEngine::step``: per-bucket
  all-reduce forked from the backward, BN-buffer broadcast behind bucket 0, join before
  SGD) — only the wire differs from RcclComm. Replicas must be bitwise identical and
  equal to the Python-orchestrated segment-graph path.
* ``comm="torch"``: the segment-graph path with collectives from Python (the reference's
  part3 loop shape, `master/part3/part3.py:116-123`).
* ``probe="order"`` (world 1): every collective is a scramble + spin + unscramble on the
  comm stream; the step must stay bitwise equal to a no-comm run, and skipping the join
  (negative control) must not.
"""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

from mp_util import run_world

pytestmark = [pytest.mark.gpu]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _train(rank, world, sync, graph, steps, comm="torch", B=16, autotune=False, env=None):
    os.environ.update(env or {})
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = NativeTrainer(batch_size=B, device=dev, rank=rank, world=world, sync=sync, comm=comm, bucket_mb=2.0,
                       graph=graph, train_size=max(512, 8 * B * world), test_size=64, autotune=autotune,
                       check_every=1)
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    ev = tr.evaluate(max_batches=2)
    maths = sorted({t["math"] for t in tr.tile_table()}) if autotune else []
    out = {"params": tr.params.cpu(), "mom": tr.mom.cpu(), "bufs": tr.bufs.cpu(), "nbt": tr.nbt.cpu(),
           "tiles": tr.tile_source, "maths": maths,
           "loss": tr.last_loss(), "buckets": len(tr.bucket_lows), "graph": tr.graph_mode,
           "calls": tr.native_comm.calls() if tr.native_comm is not None else -1,
           "kind": tr.native_comm.kind if tr.native_comm is not None else "none", "eval": ev}
    tr.close()
    return out


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.slow
def test_ddp_segments_replicas_identical_and_match_eager(gpu):
    seg = run_world(_train, 2, "ddp", "segments", 4)
    eag = run_world(_train, 2, "ddp", "none", 4)
    assert seg[0]["graph"] == "segments" and seg[0]["buckets"] > 1
    for r in range(2):
        assert torch.equal(seg[r]["params"], seg[0]["params"])
        assert torch.equal(eag[r]["params"], eag[0]["params"])
    # graphs replay the same kernels in the same order as eager: bitwise equal
    assert torch.equal(seg[0]["params"], eag[0]["params"]), (seg[0]["params"] - eag[0]["params"]).abs().max()
    # DDP broadcast_buffers: rank 0's running stats win on every rank
    assert torch.equal(seg[1]["nbt"], seg[0]["nbt"])


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 4])
def test_cpp_ddp_step_multi_rank_staged(gpu, world):
    """The N>1 benchmark's C++ step (not _step_eager) with `world` ranks on one GPU."""
    steps = 8
    ref = run_world(_train, world, "ddp", "segments", steps, "torch")
    # (each bucket's SGD runs on the comm stream right behind its all-reduce)
    nat = run_world(_train, world, "ddp", "none", steps, "staged", 16, False)
    nb = nat[0]["buckets"]
    assert nb > 1 and nat[0]["kind"] == "staged"
    # construction: 4 broadcasts; per step: one all-reduce per bucket + 2 buffer broadcasts
    assert nat[0]["calls"] == steps * (nb + 2), nat[0]["calls"]
    for r in range(world):
        for k in ("params", "mom", "bufs", "nbt"):
            assert torch.equal(nat[r][k], nat[0][k]), (r, k)
        assert nat[r]["eval"]["global_correct"] == world * nat[r]["eval"]["correct"]
    # same gradients, same averaging bytes, same SGD: the C++ step equals the Python-orchestrated one
    assert torch.equal(nat[0]["params"], ref[0]["params"])
    assert torch.equal(nat[0]["mom"], ref[0]["mom"])
    assert nat[0]["loss"] == ref[0]["loss"]


@pytest.mark.slow
def test_cpp_ddp_step_multi_rank_staged_bench_config(gpu):
    """The same multi-rank C++ step at the benchmark's configuration: B = 64 per rank and the
    shipped gfx950 N>1 tile table (split-bf16 X6S conv kernels, split-K), not the small default tiles."""
    steps = 4
    nat = run_world(_train, 2, "ddp", "none", steps, "staged", 64, True)
    ref = run_world(_train, 2, "ddp", "segments", steps, "torch", 64, True)
    assert nat[0]["tiles"] == "shipped" and "f3" in nat[0]["maths"], (nat[0]["tiles"], nat[0]["maths"])
    assert nat[0]["kind"] == "staged"
    for k in ("params", "mom", "bufs", "nbt"):
        assert torch.equal(nat[1][k], nat[0][k]), k
    assert torch.equal(nat[0]["params"], ref[0]["params"])
    assert torch.equal(nat[0]["mom"], ref[0]["mom"])


def _ragged(rank, world):
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = NativeTrainer(batch_size=16, device=dev, rank=rank, world=world, comm="staged", graph="none",
                       train_size=80, test_size=16, autotune=False, drop_last=False)
    assert tr.steps_per_epoch() == 3
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    out = {"params": tr.params.cpu(), "loss": tr.last_loss()}
    tr.close()
    return out


@pytest.mark.slow
def test_staged_ragged_last_batch(gpu):
    """drop_last=False ragged batch through the multi-rank C++ step: 2 ranks x 40 samples at
    B=16 -> batches 16, 16, 8."""
    out = run_world(_ragged, 2)
    assert torch.equal(out[0]["params"], out[1]["params"])
    assert torch.isfinite(out[0]["params"]).all()


@pytest.mark.slow
def test_sync_modes_agree(gpu):
    ref = run_world(_train, 2, "ddp", "none", 2)[0]["params"]
    for mode in ("allreduce", "flat"):
        out = run_world(_train, 2, mode, "segments", 2)
        assert torch.equal(out[0]["params"], out[1]["params"]), mode
        torch.testing.assert_close(out[0]["params"], ref, rtol=1e-5, atol=1e-6, msg=mode)


def _probe_run(probe, steps=6, skip=0, spin_us=40.0, defer=None, graph="none"):
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    old = os.environ.get("CS_COMM_DEFER")
    if defer is not None:
        os.environ["CS_COMM_DEFER"] = defer
    try:
        tr = NativeTrainer(batch_size=32, device=dev, bucket_mb=1.0, graph=graph, train_size=512, test_size=32,
                           autotune=False, probe=probe, probe_spin_us=spin_us)
    finally:
        if old is None:
            os.environ.pop("CS_COMM_DEFER", None)
        else:
            os.environ["CS_COMM_DEFER"] = old
    if defer not in (None, "none"):
        assert tr.comm_defer, defer
    tr.engine.set_debug_skip(skip)
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    out = {k: getattr(tr, k).clone() for k in ("params", "mom", "bufs", "nbt")}
    calls = tr.native_comm.calls() if tr.native_comm is not None else 0
    tr.close()
    return out, calls


def test_probe_comm_ordering_bitwise(gpu):
    """One-rank probe communicator (each collective = a spin + an exact scramble / unscramble on the
    comm stream): the data-parallel step — bucket all-reduces forked from the compute stream, each
    bucket's SGD behind its all-reduce on the comm stream, the closing join — equals the world-1
    step (SGD in the weight-gradient tails) bit for bit."""
    base, _ = _probe_run("0")
    probed, calls = _probe_run("order")
    assert calls > 6
    for k in base:
        assert torch.equal(base[k], probed[k]), k


def test_probe_comm_detects_missing_join(gpu):
    """Negative controls: without the closing join (the next forward reads parameters the comm
    stream's SGD has not written yet), or without the fork before the collectives (which the
    per-bucket SGD then follows on the comm stream), the results differ."""
    base, _ = _probe_run("0")
    bad, _ = _probe_run("order", skip=1)
    assert not torch.equal(base["params"], bad["params"])
    bad, _ = _probe_run("order", skip=2)
    assert not torch.equal(base["params"], bad["params"])


@pytest.mark.parametrize("probe,defer", [("order", "-2"), ("order", "-4,-2"), ("order", "0"), ("1", "-2")])
def test_probe_comm_deferred_buckets_bitwise(gpu, probe, defer):
    """Deferred buckets (VggEngine::set_comm_defer): their all-reduce + SGD go behind the last
    bucket on the comm stream and the NEXT forward waits for them before their lowest block. With
    scrambling probe collectives (and over a one-rank RCCL communicator) the steps stay bitwise
    equal to the world-1 run."""
    base, _ = _probe_run("0")
    probed, calls = _probe_run(probe, defer=defer)  # "1": a one-rank RCCL communicator
    assert calls > 6
    for k in base:
        assert torch.equal(base[k], probed[k]), (probe, defer, k)


def test_full_graph_after_deferred_eager_steps_bitwise(gpu):
    """graph='full' with a communicator and deferred buckets: steps 0-1 run eagerly and step 1 leaves
    a deferred all-reduce + SGD on the comm stream; the capture at step 2 must wait for it first
    (NativeTrainer._capture -> join_lag; VggEngine::step refuses a pending deferral inside a
    capture). Bitwise equal to the world-1 run over the one-rank RCCL communicator."""
    base, _ = _probe_run("0")
    graphed, calls = _probe_run("1", defer="-2", graph="full")
    assert calls > 6
    for k in base:
        assert torch.equal(base[k], graphed[k]), k


def test_probe_comm_deferred_buckets_negative_control(gpu):
    """Without the next forward's wait for the deferred buckets (debug bit 64; long probe
    collectives so the forward reaches the deferred block first) the results differ."""
    base, _ = _probe_run("0")
    bad, _ = _probe_run("order", skip=64, spin_us=3000.0, defer="-2")
    assert not torch.equal(base["params"], bad["params"])


def test_link_timeout_fails_loudly(gpu):
    """A link wait released by its timeout (here shorter than the probe collective it waits
    for) must surface: the next communicator check raises instead of training on."""
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = NativeTrainer(batch_size=32, device=dev, bucket_mb=1.0, graph="none", train_size=256, test_size=32,
                       autotune=False, probe="order", probe_spin_us=50000.0, timeout_s=0.002)
    try:
        tr.step()
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError, match="stream link"):
            tr.check_comm()
    finally:
        tr.close()


def test_link_default_timeout_waits_for_slow_collective(gpu):
    """The link timeout is the communicator timeout (1800 s default, was a fixed 10 s): slow
    collectives (60 ms each here) are waited for and the probe run stays bitwise equal to the
    no-comm run."""
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    base, _ = _probe_run("0", steps=2)
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    dev = torch.device("cuda", 0)
    tr = NativeTrainer(batch_size=32, device=dev, bucket_mb=1.0, graph="none", train_size=512, test_size=32,
                       autotune=False, probe="order", probe_spin_us=60000.0)
    if "CS_COMM_LINK_TIMEOUT_S" not in os.environ:
        assert native.C().link_timeout() == 1800.0
    for _ in range(2):
        tr.step()
    torch.cuda.synchronize()
    tr.check_comm()
    for k in ("params", "mom", "bufs", "nbt"):
        assert torch.equal(base[k], getattr(tr, k)), k
    tr.close()


def test_link_abort_releases_waits(gpu):
    """abort() (the watchdog path) releases a waiting link kernel; the error is reported."""
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    dev = torch.device("cuda", 0)
    tr = NativeTrainer(batch_size=32, device=dev, bucket_mb=1.0, graph="none", train_size=256, test_size=32,
                       autotune=False, probe="order", probe_spin_us=80000.0)
    try:
        tr.abort()
        tr.step()
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError, match="aborted"):
            tr.check_comm()
    finally:
        native.C().reset_link_abort()
        tr.close()


def test_rccl_one_rank_abort_path(gpu):
    """World-1 RCCL: async-error poll is clean, abort() makes the next collective raise
    instead of touching a freed communicator."""
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = NativeTrainer(batch_size=16, device=dev, graph="none", train_size=128, test_size=16, autotune=False,
                       probe="1", check_every=1)
    tr.step()
    tr.step()
    torch.cuda.synchronize()
    assert tr.native_comm.kind == "rccl" and tr.native_comm.async_error() == ""
    tr.abort()
    assert tr.native_comm.async_error() == "aborted"
    with pytest.raises(RuntimeError, match="aborted"):
        tr.step()
    tr.native_comm = None  # aborted: nothing to join
    tr.close()


@pytest.mark.slow
def test_killed_rank_fails_peer_promptly(gpu):
    """CS744_FAULT kills rank 1 inside the native all-reduce of step 3: rank 0 must exit
    non-zero within seconds (gloo sees the closed connection), not hang."""
    from conftest import HostedStore
    hosted = HostedStore(2)
    port = hosted.port
    code = textwrap.dedent(f"""
        import os, sys
        sys.path.insert(0, {ROOT!r})
        import torch
        from cs744_pytorch_distributed_tutorial_amd import distributed as D
        rank = int(sys.argv[1])
        if rank == 1:
            os.environ["CS744_FAULT"] = "all_reduce@7:1:kill"
        D.init_process_group("gloo", rank=rank, world_size=2, master_addr="127.0.0.1", master_port={port},
                             timeout_s=60)
        from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
        torch.cuda.set_device(0)
        tr = NativeTrainer(batch_size=16, rank=rank, world=2, comm="staged", graph="none", train_size=256,
                           test_size=16, autotune=False, check_every=1)
        for _ in range(10):
            tr.step()
        torch.cuda.synchronize()
        print("finished", flush=True)
    """)
    procs = [subprocess.Popen([sys.executable, "-c", code, str(r)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True, env=hosted.env()) for r in range(2)]
    try:
        outs = [p.communicate(timeout=100) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert procs[1].returncode == 17, outs[1][1][-800:]
    assert procs[0].returncode != 0 and "finished" not in outs[0][0], outs[0][1][-800:]
