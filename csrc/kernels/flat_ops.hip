// Elementwise combines for the tutorial's faithful gradient-sync modes on the native
// engine's flat gradient buffer (parallel/flat_sync.py), replacing ATen's mean / add_ / div_
// on that path:
//  * rows_mean — part2a's gather -> mean on the root (`master/part2a/part2a.py:42-52`):
//    dst[i] = (sum_r src[r][i]) / rows, rows summed in rank order 0..rows-1 (fixed order: the
//    root's result does not depend on the launch shape); optionally the mean is also written
//    over every gathered row, which then is the scatter list the root sends back;
//  * accumulate — part2a_extra's star on the root (`master/part2a/part2a_extra.py:41-58`):
//    g += t for each received peer buffer, and on the last one g = (g + t) / div (the same two
//    roundings as the reference's add then divide).
//  * cast_grad — bf16 gradient transport of the framework DDP (parallel/ddp.py grad_comm_dtype):
//    a bucket's fp32 gradients -> bf16 (round to nearest even, the wire format of the bf16
//    all-reduce: half the xGMI bytes, SURVEY.md §2.3 / §7.1's 16 GB per Llama-3-8B step), and the
//    averaged bf16 bucket back into the fp32 gradient view the optimizer reads.
// All are HBM-streaming: float4 grid-stride loops, a few waves per CU, scalar tail.
#include "common.h"
#include "launchers.h"

namespace {

// bcast: also write the mean back over every row of src (the root's scatter list: every rank
// receives the mean); each thread reads all rows of its elements before writing any of them
__global__ __launch_bounds__(256) void rows_mean_kernel(float* __restrict__ src, int rows, int64_t n,
                                                        float* __restrict__ dst, int bcast) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const float fr = (float)rows;
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 s = reinterpret_cast<const float4*>(src)[i];
    for (int r = 1; r < rows; ++r) {
      const float4 v = reinterpret_cast<const float4*>(src + (int64_t)r * n)[i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const float4 m = make_float4(s.x / fr, s.y / fr, s.z / fr, s.w / fr);
    reinterpret_cast<float4*>(dst)[i] = m;
    if (bcast)
      for (int r = 0; r < rows; ++r) reinterpret_cast<float4*>(src + (int64_t)r * n)[i] = m;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float s = src[i];
    for (int r = 1; r < rows; ++r) s += src[(int64_t)r * n + i];
    dst[i] = s / fr;
    if (bcast)
      for (int r = 0; r < rows; ++r) src[(int64_t)r * n + i] = s / fr;
  }
}

__global__ __launch_bounds__(256) void accumulate_kernel(float* __restrict__ g, const float* __restrict__ t,
                                                         int64_t n, float div) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 a = reinterpret_cast<float4*>(g)[i];
    const float4 b = reinterpret_cast<const float4*>(t)[i];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    if (div > 0.f) { a.x /= div; a.y /= div; a.z /= div; a.w /= div; }
    reinterpret_cast<float4*>(g)[i] = a;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float a = g[i] + t[i];
    if (div > 0.f) a /= div;
    g[i] = a;
  }
}

__device__ __forceinline__ unsigned short bf16_rne(float x) {
  const __bf16 h = (__bf16)x;  // v_cvt_pk_bf16_f32: round to nearest even, NaN stays NaN
  return __builtin_bit_cast(unsigned short, h);
}

__global__ __launch_bounds__(256) void f32_to_bf16_kernel(const float* __restrict__ x, unsigned short* __restrict__ y,
                                                          int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    ushort4 o;
    o.x = bf16_rne(v.x); o.y = bf16_rne(v.y); o.z = bf16_rne(v.z); o.w = bf16_rne(v.w);
    reinterpret_cast<ushort4*>(y)[i] = o;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = bf16_rne(x[i]);
}

__global__ __launch_bounds__(256) void bf16_to_f32_kernel(const unsigned short* __restrict__ x, float* __restrict__ y,
                                                          int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const ushort4 v = reinterpret_cast<const ushort4*>(x)[i];
    reinterpret_cast<float4*>(y)[i] = make_float4(__uint_as_float((unsigned)v.x << 16), __uint_as_float((unsigned)v.y << 16),
                                                  __uint_as_float((unsigned)v.z << 16), __uint_as_float((unsigned)v.w << 16));
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = __uint_as_float((unsigned)x[i] << 16);
}

int grid_for(int64_t n) {
  const int64_t b = ((n + 3) / 4 + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

}  // namespace

hipError_t cs_rows_mean(float* src, int rows, int64_t n, float* dst, int bcast, hipStream_t stream) {
  if (n <= 0 || rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(rows_mean_kernel, dim3(grid_for(n)), dim3(256), 0, stream, src, rows, n, dst, bcast);
  return hipGetLastError();
}

hipError_t cs_accumulate(float* g, const float* t, int64_t n, float div, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(accumulate_kernel, dim3(grid_for(n)), dim3(256), 0, stream, g, t, n, div);
  return hipGetLastError();
}

hipError_t cs_cast_grad(const void* src, void* dst, int64_t n, int to_bf16, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (to_bf16)
    hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, stream, static_cast<const float*>(src),
                       static_cast<unsigned short*>(dst), n);
  else
    hipLaunchKernelGGL(bf16_to_f32_kernel, dim3(grid_for(n)), dim3(256), 0, stream,
                       static_cast<const unsigned short*>(src), static_cast<float*>(dst), n);
  return hipGetLastError();
}
