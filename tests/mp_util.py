"""Spawn a gloo world on 127.0.0.1 and collect per-rank results."""
import os
import traceback

import torch.multiprocessing as mp

from conftest import HostedStore


def _to_host(obj):
    """Tensors -> numpy (a torch.multiprocessing queue would share fds that die with the child)."""
    import torch
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu().numpy()
    if isinstance(obj, dict):
        return {k: _to_host(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_host(v) for v in obj)
    return obj


def _entry(rank, world, port, fn, args, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # the parent hosts the store (HostedStore): every rank, rank 0 included, is a client
    os.environ["TORCHELASTIC_USE_AGENT_STORE"] = "True"
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import torch
    torch.set_num_threads(1)
    try:
        # each rank is an entry point: raise HIP's hardware queues before anything initialises HIP,
        # as bench.py / train.py do (the side-stream weight-gradient path needs >= 8 with a comm)
        import cs744_pytorch_distributed_tutorial_amd as pkg
        pkg.ensure_hw_queues()
        from cs744_pytorch_distributed_tutorial_amd import distributed as D
        D.init_process_group(backend="gloo", rank=rank, world_size=world, master_addr="127.0.0.1",
                             master_port=port, timeout_s=120)
        out = _to_host(fn(rank, world, *args))
        q.put((rank, "ok", out))
        D.barrier()
        D.destroy_process_group()
    except Exception:  # pragma: no cover - reported to parent
        q.put((rank, "err", traceback.format_exc()))


def run_world(fn, world: int, *args, timeout: float = 240.0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    hosted = HostedStore(world)
    procs = [ctx.Process(target=_entry, args=(r, world, hosted.port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    import numpy as np
    import torch
    try:
        for _ in range(world):
            rank, status, out = q.get(timeout=timeout)
            if status != "ok":
                raise RuntimeError(f"rank {rank} failed:\n{out}")
            results[rank] = out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        del hosted
    def back(o):
        if isinstance(o, np.ndarray):
            return torch.from_numpy(o)
        if isinstance(o, dict):
            return {k: back(v) for k, v in o.items()}
        if isinstance(o, (list, tuple)):
            return type(o)(back(v) for v in o)
        return o
    return [back(results[r]) for r in range(world)]
