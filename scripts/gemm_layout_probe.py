"""Probe: time the Llama-3-8B weight-gradient GEMM dW = gy^T @ x ([out, T] x [T, in], T = 8192 tokens)
in the operand layouts / output dtypes torch can hand hipBLASLt, to pick the fastest formulation
for ops.lm._LinearShadow. Prints one JSON line per shape."""
import json
import torch

T = 8192
SHAPES = [(4096, 4096), (1024, 4096), (14336, 4096), (4096, 14336), (128256, 4096)]


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3  # us


for out_f, in_f in SHAPES:
    gy = torch.randn(T, out_f, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, in_f, device="cuda", dtype=torch.bfloat16)
    r = {"out": out_f, "in": in_f}
    r["gyT_x_f32"] = timeit(lambda: torch.mm(gy.t(), x, out_dtype=torch.float32))
    r["gyT_x_bf16"] = timeit(lambda: torch.mm(gy.t(), x))
    r["xT_gy_f32_T"] = timeit(lambda: torch.mm(x.t(), gy, out_dtype=torch.float32))
    r["xT_gy_bf16_T"] = timeit(lambda: torch.mm(x.t(), gy))
    w = torch.randn(out_f, in_f, device="cuda", dtype=torch.bfloat16)
    r["fwd_x_wT"] = timeit(lambda: torch.mm(x, w.t()))
    r["dgrad_gy_w"] = timeit(lambda: torch.mm(gy, w))
    fl = 2.0 * T * out_f * in_f
    r["tflops_best_wgrad"] = round(fl / min(r["gyT_x_f32"], r["xT_gy_f32_T"]) / 1e6, 1)
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
