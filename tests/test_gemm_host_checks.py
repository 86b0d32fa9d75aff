"""Host-side argument checks of the bf16 GEMM launcher (csrc/kernels/gemm_bf16.hip) and its
split-K heuristic, on CPU: with no GPU, a call that passes every check fails only at the launch
(hipErrorNoDevice), one that fails a check returns hipErrorInvalidValue. Never run where a GPU
exists (the fake operand addresses would be launched)."""
import ctypes
import os

import pytest
import torch

SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                  "cs744_pytorch_distributed_tutorial_amd", "_C.so")
HIP_INVALID_VALUE, HIP_NO_DEVICE = 1, 100

pytestmark = pytest.mark.skipif(torch.cuda.is_available() or not os.path.exists(SO),
                                reason="CPU-only check of the built extension")


@pytest.fixture(scope="module")
def lib():
    L = ctypes.CDLL(SO)
    g = L._Z12cs_gemm_bf16iPKvliS0_lPvliiiiilP12ihipStream_t
    g.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                  ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_int64, ctypes.c_void_p]
    s = L._Z19cs_gemm_bf16_splitsiii
    s.argtypes = [ctypes.c_int] * 3
    return g, s


# (M, N, K) of weight-gradient GEMMs: ResNet-50 at B = 256 (Co, Kp, pixels) and Llama-3-8B
WGRAD = [(64, 256, 802816), (256, 64, 802816), (128, 512, 200704), (512, 256, 200704), (256, 2304, 50176),
         (2048, 512, 12544), (1024, 4096, 16384), (14336, 4096, 16384), (4096, 14336, 16384)]


@pytest.mark.parametrize("M,N,K", WGRAD)
def test_default_splits_pass_the_launcher_checks(lib, M, N, K):
    gemm, splits = lib
    S = splits(M, N, K)
    assert 1 <= S <= 256
    kper = ((K + S - 1) // S + 63) // 64 * 64
    assert kper * (S - 1) < K  # no empty split
    assert gemm(0, 0x10000, M, 0, 0x20000, N, 0x30000, N, M, N, K, 1, S, M * N, None) == HIP_NO_DEVICE


def test_launcher_rejects_bad_arguments(lib):
    gemm, _ = lib
    ok = dict(ak=1, A=0x10000, lda=4096, bk=1, B=0x20000, ldb=4096, C=0x30000, ldc=1024, M=512, N=1024, K=4096, mode=0,
              S=1, slab=0)

    def call(**kw):
        a = dict(ok, **kw)
        return gemm(a["ak"], a["A"], a["lda"], a["bk"], a["B"], a["ldb"], a["C"], a["ldc"], a["M"], a["N"], a["K"],
                    a["mode"], a["S"], a["slab"], None)

    assert call() == HIP_NO_DEVICE
    assert call(K=4092, lda=4096, ldb=4096) == HIP_INVALID_VALUE  # K-major K % 8
    assert call(A=0x10008) == HIP_INVALID_VALUE                   # 16-byte operand alignment
    assert call(N=1022, ldc=1022) == HIP_INVALID_VALUE            # N % 4
    assert call(mode=0, S=2, slab=512 * 1024) == HIP_INVALID_VALUE  # split-K needs fp32 slabs
    assert call(mode=1, S=100, slab=512 * 1024) == HIP_INVALID_VALUE  # empty splits
    assert call(mode=4) == HIP_INVALID_VALUE
