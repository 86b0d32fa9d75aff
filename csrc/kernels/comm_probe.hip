// Kernels of the world-1 ordering probe communicator (runtime/staged_comm.h ProbeComm):
// a bounded spin on the comm stream (stretches every collective so a missing stream
// fork/join in the engine becomes a visible race) and an exact, invertible scramble of
// the buffer (x2 / x0.5 for floats — exact barring overflow; +1 / -1 for integers).
#include "common.h"
#include "launchers.h"

namespace {

__global__ __launch_bounds__(64) void spin_kernel(uint64_t ticks) {
  // s_memrealtime: 100 MHz constant clock; the loop always ends (ticks is bounded by the host)
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

// stand-in for an RCCL collective's CTAs: `gridDim.x` workgroups of 256 threads that keep their
// CUs' vector pipes busy (dependent FMA chains, no sleep) for the collective's modelled duration,
// so compute overlapping it loses those CUs' issue slots the way a copy-reduce CTA takes them
__global__ __launch_bounds__(256) void busy_kernel(uint64_t ticks, float* __restrict__ sink) {
  const uint64_t t0 = wall_clock64();
  float a = (float)threadIdx.x, b = 1.0f;
  while (wall_clock64() - t0 < ticks) {
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      a = fmaf(a, 0.999f, b);
      b = fmaf(b, 1.001f, a);
    }
  }
  if (a == 1234.5f && b == 0.f) sink[threadIdx.x] = a;  // keeps the chains live; never true
}

__global__ __launch_bounds__(256) void scramble_f32_kernel(float* __restrict__ x, int64_t n, float s) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = x[i] * s;
}

template <typename T>
__global__ __launch_bounds__(256) void scramble_int_kernel(T* __restrict__ x, int64_t n, T d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = x[i] + d;
}

int grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

}  // namespace

hipError_t cs_comm_spin(double us, hipStream_t stream, int ctas, float* sink) {
  if (us <= 0.0) return hipSuccess;
  const double capped = us > 1e5 ? 1e5 : us;  // never more than 0.1 s per call
  if (ctas > 0) {
    if (ctas > 256 || sink == nullptr) return hipErrorInvalidValue;
    hipLaunchKernelGGL(busy_kernel, dim3(ctas), dim3(256), 0, stream, (uint64_t)(capped * 100.0), sink);
  } else {
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, stream, (uint64_t)(capped * 100.0));
  }
  return hipGetLastError();
}

hipError_t cs_comm_scramble(void* buf, int64_t n, int kind, int inverse, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (kind == CS_SCRAMBLE_F32) {
    hipLaunchKernelGGL(scramble_f32_kernel, dim3(grid_for(n)), dim3(256), 0, stream, (float*)buf, n,
                       inverse ? 0.5f : 2.0f);
  } else if (kind == CS_SCRAMBLE_I64) {
    hipLaunchKernelGGL(scramble_int_kernel<int64_t>, dim3(grid_for(n)), dim3(256), 0, stream, (int64_t*)buf, n,
                       (int64_t)(inverse ? -1 : 1));
  } else if (kind == CS_SCRAMBLE_I32) {
    hipLaunchKernelGGL(scramble_int_kernel<int32_t>, dim3(grid_for(n)), dim3(256), 0, stream, (int32_t*)buf, n,
                       inverse ? -1 : 1);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
