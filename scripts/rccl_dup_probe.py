"""Probe: can two RCCL ranks share ONE GPU on this stack? (NCCL refuses duplicate devices.)

Two processes on cuda:0 exchange an RCCL unique id over a gloo group and build the
native RcclComm; each all-reduces a small tensor. Prints one JSON line per rank.
Usage (GPU box): timeout -k 5 90 python3 scripts/rccl_dup_probe.py
"""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    torch.cuda.set_device(0)
    obj = [native.C().rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    out = {"rank": rank}
    try:
        c = native.C().RcclComm(obj[0], rank, world, 0)
        t = torch.full((1024,), float(rank + 1), device="cuda")
        c.all_reduce(t, "sum")
        c.join()
        torch.cuda.synchronize()
        out.update(ok=True, value=float(t[0].item()))
        del c
    except Exception as e:  # noqa: BLE001
        out.update(ok=False, err=str(e)[:300])
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_worker, args=(2, port), nprocs=2, start_method="spawn")
