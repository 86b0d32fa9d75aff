"""The K-loop schedules of the bf16 GEMM (csrc/kernels/gemm_bf16.hip) agree bit for bit (MI355X
only): 0 = 8 waves, 4-phase counted-vmcnt pipeline; 1 = 8 waves, one barrier per K-tile; 2 = 4
waves of 128 x 128, BK = 32 in 4 buffers. All accumulate every output in the same k order (one
32-deep MFMA per k-step, increasing k)."""
import pytest
import torch

from test_gemm_bf16_gpu import C, LAYOUTS, LID, SHAPES, _operands  # noqa: F401  (C: the module fixture)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("layout", LAYOUTS, ids=LID)
@pytest.mark.parametrize("sched", [1, 2])
def test_gemm_sched_matches_sched0(C, layout, sched):
    """every schedule gives the bits of the 4-phase pipeline on every shape, every output mode"""
    prev = C.gemm_bf16_sched(-1)
    try:
        for M, N, K in SHAPES + [(512, 512, 96), (256, 512, 160)]:  # + 3 and 5 K-tiles of 32
            g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
            a, b = _operands(M, N, K, layout, g)
            acc = torch.randn(M, N, device="cuda", generator=g)
            outs = []
            for s in (0, sched):
                C.gemm_bf16_sched(s)
                outs.append((C.mm_bf16(a, b, True, splits=1), C.mm_bf16(a, b), C.mm_bf16(a, b, acc=acc.clone(), splits=1),
                             C.mm_bf16(a, b, True)))
            for x, y in zip(*outs):
                assert torch.equal(x, y), (M, N, K)
    finally:
        C.gemm_bf16_sched(prev)
