// The SGD element update shared by the flat optimizer pass (sgd.hip) and the optimizer blocks
// appended to a GEMM launch (conv_gemm.hip, CsConvArgs::sgd): one definition, so both are bit-equal.
// torch.optim.SGD's order (master/part1/part1.py:98-99):
//   d = g*scale + wd*p ; buf = first ? d : buf*mom + (1-damp)*d ; p = p - lr*buf
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "launchers.h"

namespace cs_sgd {

// Every rounding is spelled out (explicit fma, contraction off): the launches that inline this
// update (the flat pass, the GEMM-tail blocks, conv0's fold) must produce the same bits whatever
// code surrounds them — left to the compiler, `m * mom + (1 - damp) * d` contracted differently in
// two kernels and the data-parallel step drifted from the world-1 step by an ulp.
__device__ __forceinline__ void step1(float& p, float g, float& m, float lr, float mom, float wd, float damp,
                                      float scale, int first) {
#pragma clang fp contract(off)
  float d = g * scale;
  if (wd != 0.f) d = __builtin_fmaf(wd, p, d);  // grad.add(param, alpha=wd)
  if (mom != 0.f) {
    m = first ? d : __builtin_fmaf(1.f - damp, d, m * mom);  // buf.mul_(mom).add_(d, alpha=1-damp)
    d = m;
  }
  p = __builtin_fmaf(-lr, d, p);  // param.add_(buf, alpha=-lr)
}

// the update of [0, t.n) of t's range by block `blk` of `nblk` (grid-stride, float4 + scalar tail);
// every lane of the calling block runs it (t.amax: a wave reduction at the end)
// |value| into the bound of the weight interval holding element i (CsWeightBounds)
__device__ __forceinline__ void wb_fold(const CsWeightBounds& wb, int64_t i, float a, float (&vm)[CS_WB_MAX]) {
#pragma unroll
  for (int k = 0; k < CS_WB_MAX; ++k)
    if (k < wb.n && i >= wb.lo[k] && i < wb.hi[k]) vm[k] = fmaxf(vm[k], a);
}

__device__ __forceinline__ void tail_body(const CsSgdTail& t, int blk, int nblk) {
  const int64_t n4 = t.n >> 2, stride = (int64_t)nblk * blockDim.x;
  float vm[CS_WB_MAX] = {};
  float4* p4 = reinterpret_cast<float4*>(t.p);
  const float4* g4 = reinterpret_cast<const float4*>(t.g);
  float4* m4 = reinterpret_cast<float4*>(t.m);
  for (int64_t i = (int64_t)blk * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = p4[i];
    const float4 gv = g4[i];
    float4 mv = t.first ? make_float4(0.f, 0.f, 0.f, 0.f) : m4[i];
    step1(pv.x, gv.x, mv.x, t.lr, t.mom, t.wd, t.damp, 1.0f, t.first);
    step1(pv.y, gv.y, mv.y, t.lr, t.mom, t.wd, t.damp, 1.0f, t.first);
    step1(pv.z, gv.z, mv.z, t.lr, t.mom, t.wd, t.damp, 1.0f, t.first);
    step1(pv.w, gv.w, mv.w, t.lr, t.mom, t.wd, t.damp, 1.0f, t.first);
    p4[i] = pv;
    if (t.mom != 0.f) m4[i] = mv;
    // (conv weight intervals are float4-aligned: the 4 elements share one interval)
    if (t.wb.n > 0) wb_fold(t.wb, i << 2, fmaxf(fmaxf(fabsf(pv.x), fabsf(pv.y)), fmaxf(fabsf(pv.z), fabsf(pv.w))), vm);
  }
  for (int64_t i = (n4 << 2) + (int64_t)blk * blockDim.x + threadIdx.x; i < t.n; i += stride) {
    float pv = t.p[i], mv = t.first ? 0.f : t.m[i];
    step1(pv, t.g[i], mv, t.lr, t.mom, t.wd, t.damp, 1.0f, t.first);
    t.p[i] = pv;
    if (t.mom != 0.f) t.m[i] = mv;
    if (t.wb.n > 0) wb_fold(t.wb, i, fabsf(pv), vm);
  }
  if (t.wb.n > 0) cs::block_amax_publish_n(vm, t.wb.amax, t.wb.n);
}

}  // namespace cs_sgd
