// torch-side helpers shared by the binding TUs. On ROCm builds torch devices are
// typed "cuda" (masquerading), so guards/streams must use the *MasqueradingAsCUDA forms.
#pragma once
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

namespace csb {
using DevGuard = c10::hip::HIPGuardMasqueradingAsCUDA;
inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
}  // namespace csb

#define CS_CHECK_CUDA(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CS_CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CS_CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CS_LAUNCH(expr)                                                                  \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    TORCH_CHECK(_e == hipSuccess, "kernel launch failed: ", hipGetErrorString(_e));      \
  } while (0)
