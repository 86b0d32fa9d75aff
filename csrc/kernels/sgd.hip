// Fused SGD (momentum, weight decay, dampening, optional grad scale) — one launch
// for the whole model (reference optimizer: torch.optim.SGD(lr .1, mom .9, wd 1e-4),
// master/part1/part1.py:98-99).
//
// Same arithmetic order as torch's foreach SGD so results match to rounding:
//   d = g*scale + wd*p ; buf = first ? d : buf*mom + (1-damp)*d ; p = p - lr*buf
// Memory-bound (16 B read/write per element per tensor): float4 vectorised,
// grid-stride, sized to a few waves per CU. (Measured round 2: 4 or 8 float4 groups per
// thread with every load issued first ran no faster — 30.1 / 31.4 / 32.2 us for the
// 9.2M-parameter pass, 83.3-84.1k img/s in the bench either way — so the pass is bandwidth-
// bound, not latency-bound, and stays this simple loop.)
#include "common.h"
#include "launchers.h"
#include "sgd_device.h"

namespace {

struct SgdArgs {
  float lr, mom, wd, damp, scale;
  int first;
};

__device__ __forceinline__ void sgd1(float& p, float g, float& m, const SgdArgs& a) {
  cs_sgd::step1(p, g, m, a.lr, a.mom, a.wd, a.damp, a.scale, a.first);
}

__global__ __launch_bounds__(256) void sgd_flat_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ m, int64_t n, SgdArgs a,
                                                       int64_t* __restrict__ counter, CsWeightBounds wb) {
  if (counter != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *counter += 1;
  float vm[CS_WB_MAX] = {};  // the weight bounds (F3 conv math), wb.n > 0
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* m4 = reinterpret_cast<float4*>(m);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = p4[i], gv = g4[i];
    float4 mv = a.first ? make_float4(0.f, 0.f, 0.f, 0.f) : m4[i];
    sgd1(pv.x, gv.x, mv.x, a);
    sgd1(pv.y, gv.y, mv.y, a);
    sgd1(pv.z, gv.z, mv.z, a);
    sgd1(pv.w, gv.w, mv.w, a);
    p4[i] = pv;
    if (a.mom != 0.f) m4[i] = mv;
    if (wb.n > 0) cs_sgd::wb_fold(wb, i << 2, fmaxf(fmaxf(fabsf(pv.x), fabsf(pv.y)), fmaxf(fabsf(pv.z), fabsf(pv.w))), vm);
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pv = p[i], mv = a.first ? 0.f : m[i];
    sgd1(pv, g[i], mv, a);
    p[i] = pv;
    if (a.mom != 0.f) m[i] = mv;
    if (wb.n > 0) cs_sgd::wb_fold(wb, i, fabsf(pv), vm);
  }
  if (wb.n > 0) cs::block_amax_publish_n(vm, wb.amax, wb.n);
}

__global__ __launch_bounds__(256) void amax_rotate_kernel(float* __restrict__ cur, float* __restrict__ next,
                                                          unsigned mask, int L) {
  const int i = blockIdx.x * 256 + threadIdx.x, l = i / CS_AMAX_SHARDS;
  if (l < L && ((mask >> l) & 1u)) {
    const size_t o = (size_t)l * CS_AMAX_SLOT + (i % CS_AMAX_SHARDS) * CS_AMAX_STRIDE;
    cur[o] = next[o];
    next[o] = 0.f;
  }
}

__global__ __launch_bounds__(256) void amax_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ amax) {
  float vm = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) vm = fmaxf(vm, fabsf(x[i]));
  cs::block_amax_publish(vm, amax);
}

// Multi-tensor form: table of {p, g, m, n}; each block walks chunks of 4096 elements.
__global__ __launch_bounds__(256) void sgd_multi_kernel(const CsTensorEntry* __restrict__ tab, int ntens,
                                                        const int64_t* __restrict__ chunk_start, int nchunks,
                                                        SgdArgs a) {
  for (int c = blockIdx.x; c < nchunks; c += gridDim.x) {
    // binary search tensor id for chunk c
    int lo = 0, hi = ntens - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (chunk_start[mid] <= c) lo = mid; else hi = mid - 1;
    }
    const CsTensorEntry e = tab[lo];
    const int64_t base = (int64_t)(c - chunk_start[lo]) * 4096;
    const int64_t end = base + 4096 < e.n ? base + 4096 : e.n;
    for (int64_t i = base + threadIdx.x; i < end; i += blockDim.x) {
      float pv = e.p[i], mv = a.first ? 0.f : e.m[i];
      sgd1(pv, e.g[i], mv, a);
      e.p[i] = pv;
      if (a.mom != 0.f) e.m[i] = mv;
      if (e.shadow != nullptr) {  // round-to-nearest-even bf16 of the new value (NaN kept quiet)
        const uint32_t u = __float_as_uint(pv);
        e.shadow[i] = (pv != pv) ? (uint16_t)((u >> 16) | 0x40u) : (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
      }
    }
  }
}

}  // namespace

hipError_t cs_sgd_flat(float* p, const float* g, float* m, int64_t n, float lr, float mom, float wd, float damp,
                       float scale, int first, hipStream_t stream, int64_t* counter, const CsWeightBounds* wb) {
  if (n <= 0) return hipSuccess;
  SgdArgs a{lr, mom, wd, damp, scale, first};
  const int64_t work = (n + 3) / 4;
  int blocks = (int)((work + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(sgd_flat_kernel, dim3(blocks), dim3(256), 0, stream, p, g, m, n, a, counter,
                     wb != nullptr ? *wb : CsWeightBounds{});
  return hipGetLastError();
}

hipError_t cs_amax_rotate(float* cur, float* next, unsigned mask, int L, hipStream_t stream) {
  if (mask == 0 || L <= 0) return hipSuccess;
  hipLaunchKernelGGL(amax_rotate_kernel, dim3((L * CS_AMAX_SHARDS + 255) / 256), dim3(256), 0, stream, cur, next, mask,
                     L);
  return hipGetLastError();
}

hipError_t cs_amax(const float* x, int64_t n, float* amax, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  int blocks = (int)((n + 1023) / 1024);
  if (blocks > 256) blocks = 256;
  hipLaunchKernelGGL(amax_kernel, dim3(blocks), dim3(256), 0, stream, x, n, amax);
  return hipGetLastError();
}

hipError_t cs_sgd_multi(const CsTensorEntry* tab_dev, int ntens, const int64_t* chunk_start_dev, int nchunks,
                        float lr, float mom, float wd, float damp, float scale, int first, hipStream_t stream) {
  if (nchunks <= 0) return hipSuccess;
  SgdArgs a{lr, mom, wd, damp, scale, first};
  int blocks = nchunks < 2048 ? nchunks : 2048;
  hipLaunchKernelGGL(sgd_multi_kernel, dim3(blocks), dim3(256), 0, stream, tab_dev, ntens, chunk_start_dev, nchunks,
                     a);
  return hipGetLastError();
}
