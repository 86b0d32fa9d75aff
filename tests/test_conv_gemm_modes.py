"""CPU checks of which convolution GEMMs each CS_CONV_GEMM mode sends to the native bf16 GEMM
(ops/cnn_nhwc.py _native_gemm); the numerics of every mode are GPU-tested in
tests/test_gemm_bf16_gpu.py (test_resnet_bottleneck_native_gemm_close_to_blas)."""
import os
import subprocess
import sys

import pytest
import torch

from cs744_pytorch_distributed_tutorial_amd.ops import cnn_nhwc


@pytest.mark.parametrize("mode,fwd_wide,fwd_narrow,wg_wide,wg_narrow", [
    ("blas", False, False, False, False),
    ("native", True, True, True, True),
    ("auto", True, False, True, False),
    ("wgrad", False, False, True, False),
])
def test_mode_selection(monkeypatch, mode, fwd_wide, fwd_narrow, wg_wide, wg_narrow):
    monkeypatch.setattr(cnn_nhwc, "_CONV_GEMM", mode)
    a = torch.empty(4, 4, dtype=torch.bfloat16)
    assert cnn_nhwc._native_gemm(a, 512) == fwd_wide
    assert cnn_nhwc._native_gemm(a, 64) == fwd_narrow
    assert cnn_nhwc._native_gemm(a, 512, wgrad=True, m=512) == wg_wide
    assert cnn_nhwc._native_gemm(a, 64, wgrad=True, m=512) == wg_narrow
    if mode == "wgrad":  # few output rows: hipBLASLt
        assert not cnn_nhwc._native_gemm(a, 512, wgrad=True, m=128)
    # fp32 operands never take the bf16 GEMM
    assert not cnn_nhwc._native_gemm(a.float(), 512, wgrad=True)


def test_unknown_mode_rejected():
    env = dict(os.environ, CS_CONV_GEMM="fast")
    r = subprocess.run([sys.executable, "-c", "import cs744_pytorch_distributed_tutorial_amd.ops.cnn_nhwc"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "CS_CONV_GEMM" in r.stderr
