"""Training / evaluation loops (reference L4) and the shared
runner behind every part entrypoint.

``train_model`` / ``test_model`` mirror the reference signatures and print
formats (`master/part1/part1.py:20-62`, `master/part2b/part2b.py:23-70`):
zero_grad -> forward -> CE loss -> backward -> [gradient sync] -> SGD step,
loss printed every 20 iterations, the reference's ``average time`` line (with
its /9 formula) plus the true mean.

Fixed reference defects (documented divergences): the accuracy of every rank is
reduced to rank 0 with an all-reduce of (correct, count) instead of the
unmatched ``isend`` that hangs in the reference (C-4,
`slave/part2b/part2b.py:68-69`); ``sampler.set_epoch`` is called each epoch; the
world size is not hard-coded.
"""
from __future__ import annotations

import math
import time
from typing import Optional

import torch
import torch.nn as nn

from . import distributed as D
from .config import TrainConfig
from .models.vgg import VGG
from .parallel.ddp import DistributedDataParallel
from .parallel.comm import make_comm
from .parallel.sync import GradSync, NoSync, make_sync
from .utils import data as data_mod
from .utils import faults
from .utils.checkpoint import load_training_state, save_training_state
from .utils.metrics import IterTimer, RankLogger
from .utils.seed import seed_everything


def train_model(model: nn.Module, train_loader, optimizer: torch.optim.Optimizer, criterion: nn.Module, epoch: int,
                rank: int = 0, sync: Optional[GradSync] = None, logger: Optional[RankLogger] = None,
                max_steps: Optional[int] = None, device: Optional[torch.device] = None, log_every: int = 20,
                check_sync_every: int = 0) -> dict:
    logger = logger or RankLogger(rank)
    sync = sync or NoSync([])
    device = device or next(model.parameters()).device
    timer = IterTimer(sync_cuda=device.type == "cuda")
    model.train()
    losses = []
    n_seen = 0
    t0 = time.perf_counter()
    for batch_idx, (data, target) in enumerate(train_loader):
        if max_steps is not None and batch_idx >= max_steps:
            break
        data, target = data.to(device, non_blocking=True), target.to(device, non_blocking=True)
        optimizer.zero_grad()
        output = model(data)
        train_loss = criterion(output, target)
        train_loss.backward()
        sync()
        optimizer.step()
        n_seen += data.shape[0]
        if batch_idx <= 10:
            timer.stamp()
        if batch_idx % log_every == 0:
            lv = train_loss.item()
            losses.append((batch_idx, lv))
            logger.loss_line(batch_idx, lv)
        if batch_idx == 10:
            ref = timer.reference_formula()
            logger.average_time_line(ref)
            true = timer.true_mean(first=0)
            logger.print(f"(true mean over iters 1..10: {true:.6f} s; the line above uses the reference /9 formula)")
        if check_sync_every and batch_idx % check_sync_every == 0:
            faults.assert_replicas_in_sync([p.data for p in model.parameters()], rtol=1e-12)
    if device.type == "cuda":
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    return {"losses": losses, "images": n_seen, "seconds": elapsed,
            "last_loss": float(train_loss.item()) if n_seen else math.nan}


def test_model(model: nn.Module, test_loader, criterion: nn.Module, logger: Optional[RankLogger] = None,
               device: Optional[torch.device] = None, reduce_across_ranks: bool = True) -> dict:
    logger = logger or RankLogger(D.get_rank())
    device = device or next(model.parameters()).device
    model.eval()
    test_loss = torch.zeros((), dtype=torch.float64, device=device)
    correct = torch.zeros((), dtype=torch.int64, device=device)
    total = 0
    nb = 0
    with torch.no_grad():
        for data, target in test_loader:
            data, target = data.to(device), target.to(device)
            output = model(data)
            test_loss += criterion(output, target).double()
            pred = output.max(1, keepdim=True)[1]
            correct += pred.eq(target.view_as(pred)).sum()
            total += target.numel()
            nb += 1
    avg = float(test_loss.item()) / max(nb, 1)
    c = int(correct.item())
    local = {"avg_loss": avg, "correct": c, "total": total}
    logger.test_line(avg, c, total)
    if reduce_across_ranks and D.get_world_size() > 1:
        # intended semantics of the reference's unmatched isend (C-4): global accuracy on rank 0
        gc = int(D.all_reduce_scalar(float(c)))
        gt = int(D.all_reduce_scalar(float(total)))
        local.update(global_correct=gc, global_total=gt)
        if D.get_rank() == 0:
            logger.print(f"All ranks: Accuracy: {gc}/{gt} ({100.0 * gc / max(gt, 1):.0f}%)")
    return local


def resolve_device(cfg: TrainConfig) -> torch.device:
    if cfg.device == "cpu":
        return torch.device("cpu")
    if cfg.device == "cuda" or (cfg.device == "auto" and torch.cuda.is_available()):
        if D.is_initialized() and D.get_backend() == "nccl":
            return D.device()
        return torch.device("cuda", cfg.extra.get("local_rank", 0) if torch.cuda.device_count() > 1 else 0)
    return torch.device("cpu")


def init_from_config(cfg: TrainConfig) -> None:
    distributed = cfg.part != "part1" and ((cfg.num_nodes or 0) > 1 or "WORLD_SIZE" in __import__("os").environ)
    if distributed:
        backend = cfg.backend
        if backend is None:
            backend = "gloo" if cfg.device == "cpu" else D.default_backend()
        import os
        # torchrun owns MASTER_PORT (its agent hosts the store); only the reference-style
        # manual launch uses the part's default port (29501 / 29508)
        port = cfg.port if cfg.port is not None else (None if "MASTER_PORT" in os.environ else cfg.resolved_port())
        D.init_process_group(backend=backend, rank=cfg.rank, world_size=cfg.num_nodes,
                             master_addr=cfg.master_ip, master_port=port,
                             timeout_s=cfg.timeout_s, local_rank=cfg.extra.get("local_rank"))


def run(cfg: TrainConfig) -> dict:
    """Build data/model/optimizer/sync for ``cfg.part`` and train + evaluate."""
    from . import ensure_hw_queues
    ensure_hw_queues()  # before anything below initialises HIP (no-op with a warning if too late)
    if cfg.threads:
        torch.set_num_threads(cfg.threads)
    init_from_config(cfg)
    rank, world = D.get_rank(), D.get_world_size()
    device = resolve_device(cfg)
    logger = RankLogger(rank, all_ranks=cfg.all_ranks_print, jsonl_path=cfg.metrics_jsonl)
    if cfg.resolved_engine() == "native" and device.type == "cuda":
        from .runtime.engine import run_native
        return run_native(cfg, device, logger)

    seed_everything(cfg.seed)  # identical init on every rank (reference S1)
    bs = cfg.resolved_batch_size()
    train_set = data_mod.SyntheticCIFAR10(train=True, size=cfg.train_size, seed=cfg.data_seed)
    test_set = data_mod.SyntheticCIFAR10(train=False, size=cfg.test_size, seed=cfg.data_seed)
    sampler = data_mod.DistributedSampler(len(train_set), num_replicas=world, rank=rank, shuffle=True, seed=0) \
        if world > 1 else None
    if device.type == "cuda":
        train_loader = data_mod.DeviceDataLoader(train_set, bs, sampler=sampler, train=True, device=device,
                                                 seed=cfg.data_seed)
        test_loader = data_mod.DeviceDataLoader(test_set, bs, sampler=None, train=False, device=device,
                                                seed=cfg.data_seed)
    else:
        train_set.transform = data_mod.train_transform()
        test_set.transform = data_mod.test_transform()
        if sampler is None:
            train_loader = data_mod.make_cpu_loader(train_set, bs, shuffle=True)
        else:
            train_loader = data_mod.make_cpu_loader(train_set, bs, sampler=sampler)
        test_loader = data_mod.make_cpu_loader(test_set, bs, shuffle=False)

    model = VGG(cfg.model).to(device)
    mode = cfg.resolved_sync() if world > 1 else "none"
    if mode == "ddp":
        comm = make_comm(cfg.resolved_comm(world))
        net: nn.Module = DistributedDataParallel(model, comm=comm, bucket_cap_mb=cfg.bucket_mb,
                                                 first_bucket_cap_mb=cfg.first_bucket_mb,
                                                 bucket_policy=cfg.bucket_policy)
        sync = NoSync([])
    else:
        net = model
        kw = {"coalesce": True} if cfg.coalesce and mode in ("gather_scatter", "p2p") else {}
        sync = make_sync(mode, model.parameters(), group=D.new_group(list(range(world))) if world > 1 else None,
                         **kw)
    criterion = nn.CrossEntropyLoss().to(device)
    optimizer = torch.optim.SGD(net.parameters(), lr=cfg.lr, momentum=cfg.momentum, weight_decay=cfg.weight_decay)
    start_epoch = 0
    if cfg.resume:
        st = load_training_state(cfg.resume, net, optimizer)
        start_epoch = int(st.get("epoch", 0))
    results = {"rank": rank, "world": world, "sync": mode, "engine": "torch", "epochs": []}
    for epoch in range(start_epoch, start_epoch + cfg.epochs):
        if hasattr(train_loader, "set_epoch"):
            train_loader.set_epoch(epoch)
        elif sampler is not None:
            sampler.set_epoch(epoch)
        tr = train_model(net, train_loader, optimizer, criterion, epoch, rank, sync=sync, logger=logger,
                         max_steps=cfg.max_steps, device=device, log_every=cfg.log_every,
                         check_sync_every=cfg.check_sync_every)
        ips = tr["images"] * world / max(tr["seconds"], 1e-9)
        logger.metric(kind="train_epoch", epoch=epoch, sync=mode, world=world, images_per_s=ips, **{
            k: v for k, v in tr.items() if k != "losses"})
        te = test_model(net, test_loader, criterion, logger=logger, device=device) if cfg.eval else None
        results["epochs"].append({"train": tr, "test": te, "images_per_s": ips})
    if cfg.checkpoint:
        save_training_state(cfg.checkpoint, net, optimizer, start_epoch + cfg.epochs, 0, 0, world, rank)
    results["final_params"] = [p.detach().cpu() for p in model.parameters()]
    return results
