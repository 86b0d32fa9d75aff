"""Aux subsystems: fault injection through the facade's
collectives, the step watchdog, the cross-rank replica checksum, NaN guard,
and checkpoint save -> resume with the reference's 58-key state_dict layout."""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

from mp_util import run_world

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fault_spec_raise_and_nth(monkeypatch):
    from cs744_pytorch_distributed_tutorial_amd.utils import faults
    faults._calls.clear()
    monkeypatch.setenv("CS744_FAULT", "all_reduce@2:0:raise")
    faults.maybe_inject("all_reduce", 0)  # 1st call: no fault
    with pytest.raises(RuntimeError, match="injected failure"):
        faults.maybe_inject("all_reduce", 0)
    faults.maybe_inject("all_reduce", 1)  # other rank unaffected
    faults.maybe_inject("broadcast", 0)   # other op unaffected
    monkeypatch.setenv("CS744_FAULT", "bogus")
    with pytest.raises(ValueError):
        faults.maybe_inject("x", 0)


def test_check_finite():
    from cs744_pytorch_distributed_tutorial_amd.utils import faults
    faults.check_finite([torch.ones(3)])
    with pytest.raises(FloatingPointError):
        faults.check_finite([torch.ones(2), torch.tensor([1.0, float("nan")])])


def _kill_child(port, spec):
    code = textwrap.dedent(f"""
        import os, sys
        sys.path.insert(0, {ROOT!r})
        os.environ["CS744_FAULT"] = {spec!r}
        import torch
        from cs744_pytorch_distributed_tutorial_amd import distributed as D
        D.init_process_group("gloo", rank=0, world_size=1, master_addr="127.0.0.1", master_port={port})
        t = torch.ones(4)
        D.all_reduce(t)
        D.all_reduce(t)
        print("survived", flush=True)
    """)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)


def test_fault_kill_exits_rank_with_code_17(hosted_store):
    r = _kill_child(hosted_store.port, "all_reduce@2:0:kill")
    assert r.returncode == 17, (r.returncode, r.stderr[-500:])
    assert "survived" not in r.stdout and "[fault]" in r.stderr


def test_watchdog_aborts_stalled_step():
    code = textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        from cs744_pytorch_distributed_tutorial_amd.utils.faults import Watchdog
        w = Watchdog(0.5, "step").start()
        time.sleep(5)
        print("not aborted")
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 18 and "[watchdog]" in r.stderr


def _replicas(rank, world, diverge):
    from cs744_pytorch_distributed_tutorial_amd.utils import faults
    ts = [torch.arange(10.0), torch.ones(3)]
    if diverge and rank == 1:
        ts[1] = ts[1] * 2
    try:
        return {"spread": faults.assert_replicas_in_sync(ts), "err": ""}
    except RuntimeError as e:
        return {"spread": -1.0, "err": str(e)}


@pytest.mark.slow
def test_replica_checksum_detects_divergence():
    ok = run_world(_replicas, 2, False)
    assert all(o["spread"] == 0.0 for o in ok)
    bad = run_world(_replicas, 2, True)
    assert all("replicas diverged" in o["err"] for o in bad)


def test_checkpoint_roundtrip_resume_matches_uninterrupted(tmp_path):
    """train 2 steps -> save -> load into fresh model+optimizer -> 2 more steps ==
    4 uninterrupted steps (bitwise, CPU)."""
    from cs744_pytorch_distributed_tutorial_amd.models import VGG11
    from cs744_pytorch_distributed_tutorial_amd.utils.checkpoint import (load_training_state,
                                                                         save_training_state)
    torch.set_num_threads(2)
    g = torch.Generator().manual_seed(0)
    batches = [(torch.randn(8, 3, 32, 32, generator=g), torch.randint(0, 10, (8,), generator=g)) for _ in range(4)]

    def make():
        torch.manual_seed(5000)
        m = VGG11()
        return m, torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)

    def run(m, opt, bs):
        m.train()
        for x, y in bs:
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            opt.step()

    m_ref, o_ref = make()
    run(m_ref, o_ref, batches)
    m1, o1 = make()
    run(m1, o1, batches[:2])
    path = str(tmp_path / "ck.pt")
    save_training_state(path, m1, o1, epoch=0, iteration=2)
    st = torch.load(path, weights_only=True)
    assert len(st["model"]) == 58 and st["iter"] == 2 and st["format"] == "cs744-amd/1"
    m2, o2 = make()
    load_training_state(path, m2, o2)
    run(m2, o2, batches[2:])
    for a, b in zip(m_ref.state_dict().values(), m2.state_dict().values()):
        assert torch.equal(a, b)


def _native_comm_fallback_worker(rank, world):
    import torch
    from cs744_pytorch_distributed_tutorial_amd.parallel import comm as cm
    # rank 1 cannot build the native communicator; rank 0 (pretend) can: all must agree on torch
    built = []

    def build():
        if rank == 1:
            raise RuntimeError("no RCCL on this rank")
        built.append(rank)
        return cm.TorchComm()

    c = cm._agreed(build, None, "rccl")
    t = torch.full((4,), float(rank + 1))
    c.all_reduce(t, "sum")
    return {"kind": type(c).__name__, "sum": t, "built": len(built)}


def _two_phase_fallback_worker(rank, world, fail_at):
    import torch
    import torch.distributed as dist
    from cs744_pytorch_distributed_tutorial_amd.parallel import comm as cm
    log = []

    def prepare():
        if fail_at == "prepare" and rank == 1:
            raise RuntimeError("cannot load the extension on this rank")
        log.append("prepare")
        return b"uid" if rank == 0 else None

    def share(uid):
        log.append("share")
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)  # the real path's collective exchange
        return obj[0]

    def build(uid):
        if fail_at == "build" and rank == 1:
            raise RuntimeError("ncclCommInitRankConfig failed on this rank")
        log.append("build:" + uid.decode())
        return cm.TorchComm()

    c = cm._agreed(build, None, "rccl", prepare=prepare, share=share)
    t = torch.full((4,), float(rank + 1))
    c.all_reduce(t, "sum")  # every rank reaches the same collectives: no hang, no mismatch
    return {"kind": type(c).__name__, "sum": t, "log": log}


@pytest.mark.parametrize("fail_at", ["prepare", "build", "none"])
def test_native_comm_two_phase_agreement(fail_at):
    """a rank failing BEFORE the unique-id broadcast must not leave its peers inside
    broadcast_object_list — phase 1 agrees first; a failure in ncclCommInitRankConfig is agreed
    after it. Both end with every rank on torch.distributed."""
    from mp_util import run_world
    out = run_world(_two_phase_fallback_worker, 2, fail_at)
    for r in range(2):
        assert out[r]["kind"] == "TorchComm"
        assert list(out[r]["sum"]) == [3.0] * 4
    if fail_at == "prepare":  # nobody entered the collective exchange
        assert all("share" not in out[r]["log"] for r in range(2))
    else:
        assert all("share" in out[r]["log"] for r in range(2))
    if fail_at == "none":
        assert out[0]["log"][-1] == "build:uid" and out[1]["log"][-1] == "build:uid"


def test_native_comm_failure_on_one_rank_falls_back_on_all():
    """a rank that cannot build the native RCCL communicator takes every rank to torch.distributed
    (agreed by one all-reduce) instead of leaving its peers inside the first native collective"""
    from mp_util import run_world
    out = run_world(_native_comm_fallback_worker, 2)
    for r in range(2):
        assert out[r]["kind"] == "TorchComm"
        assert list(out[r]["sum"]) == [3.0] * 4
