"""One dataclass config whose defaults equal the reference's constants
(SURVEY.md §5.6): batch 256 (part1, `master/part1/part1.py:17`) / 64 per rank
(part2/3, `master/part2b/part2b.py:20`), SGD lr 0.1 / momentum 0.9 / wd 1e-4
(`:120-121`), 1 epoch (`:123`), seed 5000 (`:82`), log every 20 iterations,
ports 29501 (part2) / 29508 (part3).
"""
from __future__ import annotations

import argparse
from dataclasses import asdict, dataclass, field
from typing import Optional


@dataclass
class TrainConfig:
    part: str = "part3"                 # part1 | part2a | part2a_extra | part2b | part3
    sync: Optional[str] = None          # none | gather_scatter | p2p | allreduce | flat | ddp
    model: str = "VGG11"
    batch_size: Optional[int] = None    # per rank; None -> reference default for the part
    epochs: int = 1
    lr: float = 0.1
    momentum: float = 0.9
    weight_decay: float = 1e-4
    seed: int = 5000
    data_seed: int = 0
    master_ip: Optional[str] = None
    num_nodes: Optional[int] = None     # world size
    rank: Optional[int] = None
    port: Optional[int] = None
    backend: Optional[str] = None       # gloo | nccl (RCCL) | None=auto
    device: str = "auto"                # auto | cpu | cuda
    # auto: the native HIP engine whenever the run is on a GPU, autograd + gloo on CPU
    engine: str = "auto"                # auto | torch (nn.Module + autograd) | native (fused HIP engine)
    # auto: native engine -> rccl (one GPU per rank), or staged when ranks outnumber the GPUs
    # (RCCL refuses two ranks on one device); torch engine -> torch.distributed
    comm: str = "auto"                  # auto | torch | rccl | staged
    # xGMI-sized buckets closed at layer boundaries; the reference's DDP
    # bucketing is --bucket-policy size --bucket-mb 25
    bucket_mb: float = 4.0
    first_bucket_mb: float = 1.0
    bucket_policy: str = "layer"        # layer (xGMI-sized) | size (torch DDP semantics) | single
    coalesce: bool = False              # coalesced variants of the faithful sync modes
    max_steps: Optional[int] = None     # cap iterations per epoch (None = full epoch)
    train_size: Optional[int] = None    # synthetic dataset size override
    test_size: Optional[int] = None
    eval: bool = True
    log_every: int = 20
    all_ranks_print: bool = False
    threads: Optional[int] = None       # CPU intra-op threads (reference: 4)
    checkpoint: Optional[str] = None    # path to write at the end of training
    resume: Optional[str] = None        # path to load before training
    check_sync_every: int = 0           # cross-rank parameter checksum every K steps (0 = off)
    metrics_jsonl: Optional[str] = None
    timeout_s: float = 1800.0           # collective timeout / native step watchdog (reference: gloo's 30 min)
    check_comm_every: int = 20          # native engine: poll the communicator's async error every K steps
    extra: dict = field(default_factory=dict)

    def resolved_batch_size(self) -> int:
        if self.batch_size is not None:
            return self.batch_size
        return 256 if self.part == "part1" else 64

    def resolved_sync(self) -> str:
        if self.sync is not None:
            return self.sync
        return {"part1": "none", "part2a": "gather_scatter", "part2a_extra": "p2p",
                "part2b": "allreduce", "part3": "ddp"}.get(self.part, "ddp")

    def on_gpu(self) -> bool:
        import torch
        return self.device == "cuda" or (self.device == "auto" and torch.cuda.is_available())

    def resolved_engine(self) -> str:
        if self.engine != "auto":
            return self.engine
        return "native" if self.on_gpu() and self.model.upper().startswith("VGG") else "torch"

    def resolved_comm(self, world: int = 1) -> str:
        if self.comm != "auto":
            return self.comm
        if self.resolved_engine() != "native":
            return "torch"
        import torch
        return "staged" if world > max(torch.cuda.device_count(), 1) else "rccl"

    def resolved_port(self) -> int:
        if self.port is not None:
            return self.port
        return 29508 if self.part == "part3" else 29501

    def to_dict(self) -> dict:
        return asdict(self)


def add_reference_flags(p: argparse.ArgumentParser) -> None:
    """The reference's three flags, verbatim (`master/part2b/part2b.py:129-136`)."""
    p.add_argument("--master-ip", dest="master_ip", type=str, default=None, help="master ip, 10.10.1.1")
    p.add_argument("--num-nodes", dest="num_nodes", type=int, default=None, help="number of nodes, 4")
    p.add_argument("--rank", dest="rank", type=int, default=None, help="rank, 0")


def add_engine_flags(p: argparse.ArgumentParser) -> None:
    p.add_argument("--local-rank", "--local_rank", dest="local_rank", type=int, default=None)
    p.add_argument("--sync", type=str, default=None,
                   choices=["none", "gather_scatter", "p2p", "allreduce", "flat", "ddp"])
    p.add_argument("--model", type=str, default="VGG11")
    p.add_argument("--batch-size", type=int, default=None)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--weight-decay", type=float, default=1e-4)
    p.add_argument("--seed", type=int, default=5000)
    p.add_argument("--port", type=int, default=None)
    p.add_argument("--backend", type=str, default=None, choices=["gloo", "nccl"])
    p.add_argument("--device", type=str, default="auto", choices=["auto", "cpu", "cuda"])
    p.add_argument("--engine", type=str, default="auto", choices=["auto", "torch", "native"])
    p.add_argument("--comm", type=str, default="auto", choices=["auto", "torch", "rccl", "staged"])
    p.add_argument("--bucket-mb", type=float, default=4.0)
    p.add_argument("--first-bucket-mb", type=float, default=1.0)
    p.add_argument("--bucket-policy", type=str, default="layer", choices=["layer", "size", "single"])
    p.add_argument("--coalesce", action="store_true")
    p.add_argument("--steps", dest="max_steps", type=int, default=None)
    p.add_argument("--train-size", type=int, default=None)
    p.add_argument("--test-size", type=int, default=None)
    p.add_argument("--no-eval", dest="eval", action="store_false")
    p.add_argument("--log-every", type=int, default=20)
    p.add_argument("--all-ranks-print", action="store_true")
    p.add_argument("--threads", type=int, default=None)
    p.add_argument("--checkpoint", type=str, default=None)
    p.add_argument("--resume", type=str, default=None)
    p.add_argument("--check-sync-every", type=int, default=0)
    p.add_argument("--metrics-jsonl", type=str, default=None)
    p.add_argument("--timeout-s", type=float, default=1800.0)
    p.add_argument("--check-comm-every", type=int, default=20)


def config_from_args(part: str, argv=None) -> TrainConfig:
    p = argparse.ArgumentParser(description=f"{part} (MI355X-native CS744 tutorial engine)")
    add_reference_flags(p)
    add_engine_flags(p)
    a = p.parse_args(argv)
    d = vars(a)
    local_rank = d.pop("local_rank")
    cfg = TrainConfig(part=part, **d)
    if local_rank is not None:
        cfg.extra["local_rank"] = local_rank
    return cfg
