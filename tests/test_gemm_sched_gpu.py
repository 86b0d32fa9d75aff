"""The two K-loop schedules of the bf16 GEMM (csrc/kernels/gemm_bf16.hip) agree bit for bit
(MI355X only)."""
import pytest
import torch

from test_gemm_bf16_gpu import C, LAYOUTS, LID, SHAPES, _operands  # noqa: F401  (C: the module fixture)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("layout", LAYOUTS, ids=LID)
def test_gemm_sched1_matches_sched0(C, layout):
    """the one-barrier-per-K-tile K loop gives the same bits as the 4-phase pipeline (same
    MFMA order per accumulator) on every shape"""
    prev = C.gemm_bf16_sched(-1)
    try:
        for M, N, K in SHAPES:
            g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
            a, b = _operands(M, N, K, layout, g)
            C.gemm_bf16_sched(0)
            c0 = C.mm_bf16(a, b, True, splits=1)
            C.gemm_bf16_sched(1)
            c1 = C.mm_bf16(a, b, True, splits=1)
            assert torch.equal(c0, c1), (M, N, K)
    finally:
        C.gemm_bf16_sched(prev)
