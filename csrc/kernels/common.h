// Shared helpers for the gfx950 (MI355X / CDNA4) kernels.
// Wave size is 64 on CDNA: every lane/wave constant below is written for 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CS_WAVE 64

#define CS_HIP_CHECK(expr)                                                             \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess) {                                                            \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__,      \
              __LINE__);                                                               \
      return _e;                                                                       \
    }                                                                                  \
  } while (0)

namespace cs {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024). `red` needs 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = (threadIdx.x < (unsigned)nw) ? red[threadIdx.x] : 0.f;
  if (wid == 0) r = wave_sum(r);
  if (threadIdx.x == 0) red[0] = r;
  __syncthreads();
  return red[0];
}

// The F3 conv math's operand bounds (launchers.h CS_AMAX_*): a producer workgroup folds |its values|
// into ONE atomic max on shard blockIdx % 64 (the float bits of a non-negative value order like
// unsigned ints; a NaN, above +inf, wins). Every thread of the block calls it (a barrier inside).
__device__ __forceinline__ void block_amax_publish(float v, float* amax) {
  __shared__ float red[16];
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < nw; ++w) v = fmaxf(v, red[w]);
    atomicMax(reinterpret_cast<unsigned*>(amax) + (blockIdx.x & 63) * 32, __float_as_uint(v));
  }
}

// Several bounds at once (the SGD's per-block weight bounds): v[k] folded into amax[k] (k < n,
// n <= 16; null amax[k] skipped). Every thread of the block calls it (a barrier inside).
__device__ __forceinline__ void block_amax_publish_n(const float (&v)[16], float* const (&amax)[16], int n) {
  __shared__ float red[16][16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k >= n) break;
    const float w = wave_max(v[k]);
    if (lane == 0) red[wid][k] = w;
  }
  __syncthreads();
  if ((int)threadIdx.x < n && amax[threadIdx.x] != nullptr) {
    float m = 0.f;
    for (int i = 0; i < nw; ++i) m = fmaxf(m, red[i][threadIdx.x]);
    atomicMax(reinterpret_cast<unsigned*>(amax[threadIdx.x]) + (blockIdx.x & 63) * 32, __float_as_uint(m));
  }
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5, "XCD swizzle must be
// bijective"): blocks b and b+8 share an XCD, so hand each XCD a contiguous range.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

}  // namespace cs
