#!/usr/bin/env python3
"""Headline benchmark: VGG-11 training throughput on synthetic CIFAR-10-shaped data.

Metric (BASELINE.json): images/sec for the WHOLE node, VGG-11, 3x32x32 -> 10
classes, per-GPU batch 64 (the reference's part2/part3 per-rank batch,
`master/part2b/part2b.py:20`), SGD(0.1, 0.9, 1e-4), fp32 (the reference's
precision), one process per GPU, data-parallel gradient averaging with part3
(DDP) semantics: bucketed all-reduce(AVG) over RCCL/xGMI overlapped with the
backward pass. Weak scaling: per-GPU batch fixed, global batch = 64 * N.

Default engine = ``native``: the C++ VggEngine (hand-written gfx950 kernels for
every op, eager C++ step (hipGraph optional), native RcclComm). ``--engine torch`` runs the
same model through stock PyTorch-ROCm modules + the framework's DDP (the
comparison baseline). ``--model resnet50`` / ``--model llama-tiny`` etc. run the
BASELINE.json extension configs through the autograd-path trainer.

Contract: ``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched by
``torch.distributed.run`` (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from env). W untimed
warmup steps, then EXACTLY K timed steps bracketed by barrier + device sync on
both sides; the max over ranks is reported; rank 0 prints ONE JSON line.

Every timed step does the full work: batch gather + augmentation on device,
forward, loss, backward, gradient all-reduce (N > 1), SGD update.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# raise GPU_MAX_HW_QUEUES before anything initialises HIP (package ensure_hw_queues)
import cs744_pytorch_distributed_tutorial_amd as _pkg  # noqa: E402

_pkg.ensure_hw_queues()
import torch  # noqa: E402

from cs744_pytorch_distributed_tutorial_amd import distributed as D  # noqa: E402

# best reference configuration (part3 DDP, N=4, local CPU repro) = 554 img/s.
BASELINE_IMG_S = 554.0
# The same-chip comparator: stock PyTorch-ROCm (MIOpen convolutions, ATen BN/ReLU/pool, torch.optim
# SGD) on one MI355X, VGG-11 fp32, 64 images per GPU — `bench.py --engine torch`, measured in round 5
# (profiles/r5_extras.jsonl: 29,893 img/s, 2.141 ms/step). Reported as vs_stock_torch_per_gpu.
STOCK_TORCH_IMG_S_PER_GPU = 29893.0


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch-size", type=int, default=None, help="per-GPU batch (default: 64 VGG, 256 ResNet, 8 Llama)")
    p.add_argument("--model", type=str, default="VGG11")
    p.add_argument("--engine", type=str, default=os.environ.get("CS744_BENCH_ENGINE", "native"),
                   choices=["torch", "native"])
    p.add_argument("--sync", type=str, default="ddp",
                   choices=["ddp", "allreduce", "gather_scatter", "p2p", "flat"])
    p.add_argument("--comm", type=str, default="rccl", choices=["torch", "rccl", "staged"],
                   help="gradient transport at N > 1: rccl = the native RCCL communicator over xGMI (one GPU per "
                        "rank); torch = torch.distributed; staged = the native C++ step over a gloo process group "
                        "with host staging (several ranks may share one GPU: the N > 1 code path on a 1-GPU box)")
    p.add_argument("--busbw-iters", type=int, default=10,
                   help="N > 1: all-reduce timings per bucket size after the timed steps (0 = skip)")
    p.add_argument("--bucket-mb", type=float, default=4.0,
                   help="DDP bucket cap; buckets close at layer boundaries (VGG-11: 9|9|9|4.5|3.7 MiB)")
    p.add_argument("--bucket-policy", type=str, default="layer", choices=["size", "layer", "single"])
    p.add_argument("--dtype", type=str, default=None, choices=["fp32", "bf16"],
                   help="compute dtype (default: fp32 for the CNNs, the reference's; bf16 for the Llama LMs, "
                        "the BASELINE config's)")
    p.add_argument("--seq-len", type=int, default=0, help="decoder LM sequence length")
    p.add_argument("--no-graph", action="store_true", help="native engine: same as --graph none")
    p.add_argument("--graph", type=str, default="auto", choices=["auto", "full", "segments", "none"])
    p.add_argument("--json-out", type=str, default=None)
    p.add_argument("--watchdog-s", type=float, default=600.0,
                   help="abort the communicator and exit(18) if one step stalls this long (0 = off)")
    p.add_argument("--comm-probe", type=str, default=None,
                   help="native engine, world 1, measurement only: run the data-parallel step (bucket "
                        "all-reduces, buffer broadcast, fork/join) against a one-rank communicator: "
                        "'1' = RCCL, 'order' = scrambling probe, 'xgmi:G:W:us[:ctas]' = modelled ring")
    p.add_argument("--phases", type=int, default=0,
                   help="native engine: after the timed steps, N more steps with per-phase device timing "
                        "(forward / bucket backward / all-reduce wait / SGD), printed to stderr as JSON")
    return p.parse_args(argv)


def is_vgg(name: str) -> bool:
    return name.upper().startswith("VGG")


def make_trainer(args, device, rank, world):
    if args.engine == "native" and is_vgg(args.model):
        from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
        return NativeTrainer.from_bench_args(args, device, rank, world, probe=args.comm_probe)
    from cs744_pytorch_distributed_tutorial_amd.runtime.torch_trainer import TorchTrainer
    return TorchTrainer(args.model, args.batch_size, device, rank, world, sync=args.sync, comm=args.comm,
                        bucket_mb=args.bucket_mb, bucket_policy=args.bucket_policy, dtype=args.dtype,
                        seq_len=args.seq_len)


def describe(args, trainer, world):
    name = args.model
    if is_vgg(name):
        return (f"images/sec (whole node) {name[:3]}-{name[3:]} CIFAR-shape", "images/s",
                args.batch_size * world, None, BASELINE_IMG_S,
                "synthetic (CIFAR-10 shape 3x32x32 uint8, on-device augmentation), random-init weights")
    if getattr(trainer, "is_lm", False):
        seq = trainer.data.tokens.shape[1] - 1
        return (f"tokens/sec (whole node) {name} decoder LM", "tokens/s", args.batch_size * world, seq, None,
                "synthetic random token ids, random-init weights")
    return (f"images/sec (whole node) {name} ImageNet-shape", "images/s", args.batch_size * world, None, None,
            "synthetic (ImageNet shape 3x224x224 uint8 pool on device), random-init weights")


def comm_kind(trainer, world: int) -> str:
    """The gradient transport the timed steps actually used."""
    kind = getattr(trainer, "comm_kind", None)  # native engine
    if world == 1:  # a one-rank measurement communicator (--comm-probe) or none
        return kind if kind and kind.startswith("probe") else "none"
    if kind:
        return kind
    net = getattr(trainer, "net", None)
    comm = getattr(net, "comm", None)  # framework DDP (TorchTrainer)
    return getattr(comm, "kind", "torch") if comm is not None else "torch"


def comm_ctas_used(trainer):
    native = getattr(trainer, "native_comm", None)
    if native is None:
        native = getattr(getattr(getattr(trainer, "net", None), "comm", None), "native", None)
    return getattr(native, "max_ctas", None)


def _sysfs_card(device) -> str | None:
    """/sys/class/drm/cardN/device of the GPU torch calls `device` (matched by PCI address)."""
    import glob
    try:
        p = torch.cuda.get_device_properties(device)
        want = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}."
    except Exception:  # noqa: BLE001
        return None
    for d in sorted(glob.glob("/sys/class/drm/card*/device")):
        if os.path.basename(os.path.realpath(d)).startswith(want):
            return d
    return None


def _dpm_current(path: str):
    """The active level of a pp_dpm_* table ('1: 2400Mhz *' -> 2400)."""
    try:
        for line in open(path):
            if line.rstrip().endswith("*"):
                return int("".join(ch for ch in line.split(":", 1)[1] if ch.isdigit()))
    except (OSError, ValueError, IndexError):
        pass
    return None


def calibration(device) -> dict:
    """Box fingerprint taken AFTER the timed steps (it never touches `value`): the GPU's current
    shader / memory clock levels and power cap from sysfs, and the throughput of a fixed bf16 MFMA
    GEMM (hipBLASLt, 4096^3, ~1 ms per call) — so a slow box and a slow code change can be told
    apart when two runs of the same tree disagree."""
    out = {}
    card = _sysfs_card(device)
    if card:
        out["sclk_mhz"] = _dpm_current(os.path.join(card, "pp_dpm_sclk"))
        out["mclk_mhz"] = _dpm_current(os.path.join(card, "pp_dpm_mclk"))
        import glob
        for h in glob.glob(os.path.join(card, "hwmon", "hwmon*")):
            for key, name in (("power_cap_w", "power1_cap"), ("power_w", "power1_average")):
                try:
                    out[key] = round(int(open(os.path.join(h, name)).read()) / 1e6, 1)
                except (OSError, ValueError):
                    pass
    try:
        n = 4096
        a = torch.randn(n, n, device=device, dtype=torch.bfloat16)
        b = torch.randn(n, n, device=device, dtype=torch.bfloat16)
        for _ in range(3):
            torch.mm(a, b)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            torch.mm(a, b)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out["mfma_bf16_gemm_tflops"] = round(2 * n ** 3 / (ms * 1e-3) / 1e12, 1)
    except Exception as e:  # noqa: BLE001
        out["mfma_error"] = str(e)[:80]
    return out


def rccl_versions():
    """{runtime, header} RCCL version codes: the library actually loaded (torch's) and the header the
    native communicator was compiled against (they differ on this image: 2.26 vs 2.27)."""
    try:
        from cs744_pytorch_distributed_tutorial_amd.ops import native
        rt, hdr = native.C().rccl_version()
        return {"runtime": int(rt), "header": int(hdr)}
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)[:120]}


def _bench_comm(trainer):
    """The native DeviceComm the steps used (VGG engine, or the framework DDP's), or None."""
    native = getattr(trainer, "native_comm", None)
    if native is None:
        native = getattr(getattr(getattr(trainer, "net", None), "comm", None), "native", None)
    return native


def measure_busbw(trainer, world: int, device, iters: int = 10, warm: int = 3) -> dict:
    """All-reduce(AVG) bus bandwidth (GB/s, nccl-tests factor 2(N-1)/N) per distinct gradient-bucket
    size of the trainer's plan (VGG-11 at the 4 MiB cap: 9.0 / 4.5 / 3.4 / 0.3 MiB ...; 1/4/16/64 MiB
    for the autograd trainers), on the communicator the timed steps used; time = max over ranks.
    Reference: the gloo all_reduce of `master/part2b/part2b.py:43-45`, BASELINE.md busBW rows."""
    native = _bench_comm(trainer)
    ranges = getattr(trainer, "bucket_ranges", None)
    sizes = sorted({int(n) for _, n in ranges}, reverse=True) if ranges else [(k << 20) // 4 for k in (1, 4, 16, 64)]
    out = {}
    for n in sizes:
        buf = torch.ones(n, dtype=torch.float32, device=device)

        def run():
            if native is not None:
                native.all_reduce(buf, "avg")
            else:
                D.all_reduce(buf, op=D.ReduceOp.AVG)
        for _ in range(warm):
            run()
        if native is not None:
            native.join()
        torch.cuda.synchronize()
        D.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            run()
        if native is not None:
            native.join()
        torch.cuda.synchronize()
        t = D.all_reduce_scalar((time.perf_counter() - t0) / iters, op=D.ReduceOp.MAX)
        out[f"{4 * n / 2 ** 20:.2f}MiB"] = round(4 * n / t / 1e9 * 2 * (world - 1) / world, 3)
    return out


def main(argv=None) -> int:
    args = parse(argv)
    if args.batch_size is None:
        # Llama-3-8B: 8 x 2048 tokens per GPU (measured on MI355X with the round-2 kernels: 19.8-20.1k /
        # 20.0k / 20.7k tokens/s at B = 4 / 6 / 8 — the fp32 master-weight SGD step and, at N > 1, the
        # gradient all-reduce amortise over more tokens)
        m = args.model.lower()
        # ResNet: 256 images per GPU (channels-last native path on MI355X, bf16: 7255 img/s vs 6387 at B=128)
        args.batch_size = 64 if is_vgg(args.model) else (8 if "llama" in m or "8b" in m else 256)
    if args.dtype is None:
        args.dtype = "bf16" if "llama" in args.model.lower() else "fp32"
    if args.seq_len == 0 and "8b" in args.model.lower():
        args.seq_len = 2048  # the round-1 measurements' context (the model's max_seq is 8192)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    # one GPU per rank (local rank modulo the count — the identity on a full node; on a smaller box the
    # staged transport, and the rccl fallback test, let ranks share GPUs; device_count() does not
    # initialise HIP on this stack)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev_index = local % max(torch.cuda.device_count(), 1)
    if args.engine == "native" and is_vgg(args.model):
        # before the process group or anything else creates streams: the native engine's side
        # stream must own a hardware queue (measured 4x slower steps when it shares one)
        from cs744_pytorch_distributed_tutorial_amd.ops import native
        torch.cuda.set_device(dev_index)
        native.C().reserve_streams()
    native_vgg = args.engine == "native" and is_vgg(args.model)
    if world_env > 1:
        # control plane only (barriers, the unique-id exchange, the max-over-ranks time): gloo whenever
        # the gradients travel on a native communicator, so the native RcclComm is the ONLY RCCL
        # communicator per rank — a ProcessGroupNCCL next to it would bring its own channels, CTAs and
        # proxy threads for no traffic. The autograd trainers' DDP all-reduces through the process
        # group itself, so they keep the nccl backend.
        control_gloo = args.comm == "staged" or (native_vgg and args.comm == "rccl")
        D.init_process_group(backend="gloo" if control_gloo else "nccl")
    rank, world = D.get_rank(), D.get_world_size()
    if world != args.gpus and rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    device = D.device() if world > 1 and D.get_backend() == "nccl" else torch.device("cuda", dev_index)
    torch.cuda.set_device(device)
    trainer = make_trainer(args, device, rank, world)
    # a dead peer leaves RCCL kernels spinning forever: the watchdog turns that into ncclCommAbort
    # + a prompt non-zero exit; kicked once per step, nothing on the device
    from cs744_pytorch_distributed_tutorial_amd.utils.faults import Watchdog
    wd = Watchdog(args.watchdog_s, "bench step", on_timeout=getattr(trainer, "abort", None)).start() \
        if args.watchdog_s > 0 else None

    # no Python garbage-collector pass inside the timed steps: a full collection of the
    # interpreter's heap takes milliseconds, as long as a short window's whole budget (one
    # 20-step run measured a one-off 0.98 ms/step against 0.72-0.74 in five repeats). Collect
    # before the warmup steps, not between them and the timed ones, so the timed window does not
    # start behind a millisecond of idle GPU (profiles/r4_bench_windows.jsonl)
    import gc
    gc.collect()
    gc.disable()
    for _ in range(args.warmup):
        trainer.step()
        if wd is not None:
            wd.kick()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.step()
        if wd is not None:
            wd.kick()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    gc.enable()
    if wd is not None:
        wd.stop()
    if hasattr(trainer, "check_comm"):
        trainer.check_comm()  # async RCCL errors surface here instead of as a silent bad number
    elapsed = D.all_reduce_scalar(elapsed, op=D.ReduceOp.MAX) if world > 1 else elapsed
    # after the timed window (it never changes `value`): all-reduce bus bandwidth per gradient-bucket
    # size on the communicator the steps used — BASELINE.json's metric also names it
    busbw = measure_busbw(trainer, world, device, args.busbw_iters) if world > 1 and args.busbw_iters > 0 else None
    comm_used = comm_kind(trainer, world)
    loss = trainer.last_loss()
    metric, unit, gbatch, seq, baseline, data = describe(args, trainer, world)
    per_step = gbatch * (seq or 1)
    value = per_step * args.steps / elapsed
    engine = args.engine if is_vgg(args.model) else "torch"
    out = {
        "metric": metric,
        "value": round(value, 2),
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / baseline, 2) if baseline else None,
        "dtype": args.dtype,
        "data": data,
        "config": {"model": args.model, "global_batch": gbatch, "per_gpu_batch": args.batch_size, "seq_len": seq,
                   "parallelism": f"dp{world}", "sync": args.sync if world > 1 else "none", "engine": engine,
                   "comm": comm_used, "comm_requested": args.comm if world > 1 else None,
                   "comm_ctas": comm_ctas_used(trainer), "hw_queues": _pkg.hw_queues(), "bucket_mb": args.bucket_mb,
                   "optimizer": "SGD(lr=0.1, momentum=0.9, wd=1e-4)", "final_loss": round(loss, 4),
                   "baseline_img_s": baseline},
    }
    if busbw is not None:
        out["busbw_GBps"] = busbw
    if is_vgg(args.model) and args.model.upper() == "VGG11" and args.batch_size == 64 and args.dtype == "fp32":
        out["vs_stock_torch_per_gpu"] = round(value / world / STOCK_TORCH_IMG_S_PER_GPU, 3)
    if getattr(trainer, "queue_shared", None) is not None:
        out["config"]["hw_queue_shared"] = trainer.queue_shared
    if world > 1 or args.comm_probe:
        out["config"]["control_plane"] = D.get_backend() if world > 1 else "none"
        out["config"]["rccl_version"] = rccl_versions()
    # a scaling run must never read a number from another transport as the native one: the
    # fallback keeps its (valid, full-step) number, says so at the top level, and exits 0
    out["comm_fallback"] = bool(world > 1 and args.comm in ("rccl", "staged") and comm_used != args.comm)
    if hasattr(trainer, "tile_table"):
        # which MFMA math the autotuner picked per conv GEMM: f32-input MFMA, or the fp32-accurate
        # split-bf16 x6 kernels (3 bf16 pieces per operand, 6 MFMAs; f64-checked like the f32 path)
        maths = [t["math"] for t in trainer.tile_table()]
        out["config"]["conv_gemm_math"] = {m: maths.count(m) for m in sorted(set(maths))}
        out["config"]["conv_tiles"] = getattr(trainer, "tile_source", None)
        out["config"]["comm_defer"] = getattr(trainer, "comm_defer", None)
        out["config"]["wgrad_side_stream"] = getattr(trainer, "overlap_wgrad", None)
    out["config"]["grad_comm_dtype"] = getattr(trainer, "grad_comm_dtype", "fp32")
    if os.environ.get("CS744_BENCH_CALIBRATE", "1") != "0":
        out["calibration"] = calibration(device)
    if args.phases > 0 and hasattr(trainer, "phase_breakdown"):
        ph = trainer.phase_breakdown(args.phases)
        if rank == 0:
            print(json.dumps({"phases_ms": {k: round(v, 4) for k, v in ph.items()}, "rank": rank}),
                  file=sys.stderr, flush=True)
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "a") as f:
                f.write(line + "\n")
    if hasattr(trainer, "close"):
        trainer.close()
    if world > 1:
        D.barrier()
        D.destroy_process_group()
    if out["comm_fallback"]:
        # the number above ran on the fallback transport (torch.distributed, collectives issued from
        # Python), not the native communicator: top-level "comm_fallback": true and config.comm say
        # which; the measurement itself is a valid full step, so the exit status stays 0
        print(f"[bench] warning: --comm {args.comm} requested but the job ran on {comm_used!r} (native "
              "communicator construction failed on some rank); see comm_fallback / config.comm",
              file=sys.stderr, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
