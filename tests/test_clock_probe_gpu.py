"""The diagnostic shader-clock sampler (csrc/kernels/clock_probe.hip, scripts/ramp_clock.py): it
stops when told, its samples are ordered, and the clock it reads is a plausible gfx950 shader clock."""
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_clock_sampler_stops_and_reads_a_plausible_clock():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    C = native.C()
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    n = 1 << 18  # ~7 us per sample: ~1.8 s of room
    a = torch.randn(4096, 4096, device=dev)
    (a @ a).sum().item()  # library kernels loaded before the sampler starts
    out = torch.zeros(2 * (n + 1), dtype=torch.int64, device=dev)
    stop = torch.zeros(1, dtype=torch.int32, device=dev)
    slots = torch.zeros(2, dtype=torch.int64, device=dev)
    C.clock_sampler(out, stop, s.cuda_stream)
    time.sleep(0.005)
    C.clock_stamp(slots, 0)
    for _ in range(20):
        c = a @ a  # keep the chip busy for a few ms
    C.clock_stamp(slots, 1)
    del c
    C.clock_stop(stop)
    torch.cuda.synchronize()
    o = out.view(-1, 2).cpu()
    k = int((o[:, 0] == 0).nonzero()[0]) if bool((o[:, 0] == 0).any()) else n
    assert 2 <= k < n, k  # stopped by the stop word, not by running out of samples
    real, clk = o[:k, 0], o[:k, 1]
    assert bool((real[1:] >= real[:-1]).all()) and bool((clk[1:] >= clk[:-1]).all())
    st = slots.cpu()
    assert real[0] <= st[0] < st[1] <= real[-1]
    mhz = 100.0 * float(clk[-1] - clk[0]) / float(real[-1] - real[0])
    assert 300.0 < mhz < 3000.0, mhz
