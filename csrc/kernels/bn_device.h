// Device-side BN backward pieces shared by bn.hip and conv_gemm.hip: the per-element visit
// (recompute relu(bn(y)) and the 2x2 pool argmax, route the incoming gradient) and the
// per-channel partial-sum body of the backward reduce. conv_gemm.hip runs that body in extra
// blocks appended to a weight-gradient GEMM launch (CsConvArgs::red) — the same code, block
// partition and summation order as the standalone reduce launch, so the partials are
// bit-identical.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "launchers.h"

namespace cs_bn {

// ------------------------------------------------------------------ backward
// Visit every full-resolution element once: unit = a 2x2 window (pool) or a pixel.
// APPLY = false: accumulate per-channel partials; APPLY = true: write dZ.
template <bool APPLY, bool POOL>
__device__ __forceinline__ void bwd_visit(const float* __restrict__ y, const float* __restrict__ G, int B, int H,
                                          int W, int C, int cq, int unit, const float* scale, const float* shift,
                                          const float* mean, const float* invstd, const float* coef, float* dz,
                                          float (&acc)[3][4], int coef_c0 = 0, float* vmax = nullptr) {
  const int C4 = C >> 2;
  float sc[4], sh[4], mu[4], is[4], k1[4], k2[4], k3[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 4 * cq + q;
    sc[q] = scale[c]; sh[q] = shift[c]; mu[q] = mean[c]; is[q] = invstd[c];
    if (APPLY) {  // coef holds channels from coef_c0 on (an LDS copy in the single-launch kernel)
      k1[q] = coef[3 * (c - coef_c0)]; k2[q] = coef[3 * (c - coef_c0) + 1]; k3[q] = coef[3 * (c - coef_c0) + 2];
    }
  }
  const float4 g4 = reinterpret_cast<const float4*>(G)[(size_t)unit * C4 + cq];
  const float gin[4] = {g4.x, g4.y, g4.z, g4.w};
  constexpr int NP = POOL ? 4 : 1;
  size_t off[NP];
  if (POOL) {
    const int Wo = W >> 1, Ho = H >> 1;
    const int wo = unit % Wo, ho = (unit / Wo) % Ho, b = unit / (Wo * Ho);
    const size_t base = (((size_t)b * H + 2 * ho) * W + 2 * wo) * C4 + cq;
    off[0] = base;
    if (POOL) {
      off[1 % NP] = base + C4;
      off[2 % NP] = base + (size_t)W * C4;
      off[3 % NP] = base + (size_t)W * C4 + C4;
    }
  } else {
    off[0] = (size_t)unit * C4 + cq;
  }
  float yv[NP][4];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const float4 v = reinterpret_cast<const float4*>(y)[off[p]];
    yv[p][0] = v.x; yv[p][1] = v.y; yv[p][2] = v.z; yv[p][3] = v.w;
  }
  float out[NP][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float z[NP];
    int am = 0;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      z[p] = fmaxf(yv[p][q] * sc[q] + sh[q], 0.f);
      if (p > 0 && z[p] > z[am]) am = p;
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const float g = (p == am && z[p] > 0.f) ? gin[q] : 0.f;
      const float xh = (yv[p][q] - mu[q]) * is[q];
      if (APPLY) {
        out[p][q] = k1[q] * (g - k2[q] - xh * k3[q]);
      } else {
        acc[0][q] += g;
        acc[1][q] += g * xh;
        acc[2][q] += xh;
      }
    }
  }
  if (APPLY) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
      reinterpret_cast<float4*>(dz)[off[p]] = make_float4(out[p][0], out[p][1], out[p][2], out[p][3]);
    if (vmax != nullptr)  // the dZ bound the F3 conv math scales by
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) *vmax = fmaxf(*vmax, fabsf(out[p][q]));
  }
}


// The same per-element visit for ONE channel of one incoming-gradient value g, when the
// gradient is still in the registers of the GEMM (or split-K combine) that produced it: i0 is
// the element's index in y (the window's first element with pooling), C the channel count and
// W2 y's width. Decisions and sums are bwd_visit's, so the partials only differ from the
// standalone reduce pass in their (fixed) summation order.
template <bool POOL>
__device__ __forceinline__ void bwd_point(const float* __restrict__ y, size_t i0, int C, int W2, float g, float sc,
                                          float sh, float mu, float is, float& s0, float& s1, float& s2) {
  constexpr int NP = POOL ? 4 : 1;
  float yv[NP];
  yv[0] = y[i0];
  if (POOL) {
    yv[1 % NP] = y[i0 + C];
    yv[2 % NP] = y[i0 + (size_t)W2 * C];
    yv[3 % NP] = y[i0 + (size_t)W2 * C + C];
  }
  float z[NP];
  int am = 0;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    z[p] = fmaxf(yv[p] * sc + sh, 0.f);
    if (p > 0 && z[p] > z[am]) am = p;
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const float gp = (p == am && z[p] > 0.f) ? g : 0.f;
    const float xh = (yv[p] - mu) * is;
    s0 += gp;
    s1 += gp * xh;
    s2 += xh;
  }
}

__device__ __forceinline__ float f4get(const float4& v, int q) {
  return q == 0 ? v.x : (q == 1 ? v.y : (q == 2 ? v.z : v.w));
}

// bwd_point for 4 consecutive channels (i0 16-B aligned): one float4 load of y per window
// position, the per-channel BN vectors as float4; s[k][q] += the k-th term of channel q
template <bool POOL>
__device__ __forceinline__ void bwd_point4(const float* __restrict__ y, size_t i0, int C, int W2, float4 g,
                                           float4 sc, float4 sh, float4 mu, float4 is, float (&s)[3][4]) {
  constexpr int NP = POOL ? 4 : 1;
  float4 yv[NP];
  yv[0] = *reinterpret_cast<const float4*>(y + i0);
  if (POOL) {
    yv[1 % NP] = *reinterpret_cast<const float4*>(y + i0 + C);
    yv[2 % NP] = *reinterpret_cast<const float4*>(y + i0 + (size_t)W2 * C);
    yv[3 % NP] = *reinterpret_cast<const float4*>(y + i0 + (size_t)W2 * C + C);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float scq = f4get(sc, q), shq = f4get(sh, q), muq = f4get(mu, q), isq = f4get(is, q), gq = f4get(g, q);
    float yq[NP], z[NP];
    int am = 0;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      yq[p] = f4get(yv[p], q);
      z[p] = fmaxf(yq[p] * scq + shq, 0.f);
      if (p > 0 && z[p] > z[am]) am = p;
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const float gp = (p == am && z[p] > 0.f) ? gq : 0.f;
      const float xh = (yq[p] - muq) * isq;
      s[0][q] += gp;
      s[1][q] += gp * xh;
      s[2][q] += xh;
    }
  }
}

// index in y (full resolution, NHWC, C channels) of output-gradient row m's first element;
// the gradient rows are pixels of an H x W (= y's size halved with pooling) image
template <bool POOL>
__device__ __forceinline__ size_t bwd_point_index(int m, int n, int lgH, int lgW, int C) {
  if (!POOL) return (size_t)m * C + n;
  const int W = 1 << lgW, H = 1 << lgH;
  const int wo = m & (W - 1), ho = (m >> lgW) & (H - 1), b = m >> (lgW + lgH);
  return (((size_t)b * 2 * H + 2 * ho) * 2 * W + 2 * wo) * C + n;
}

// Partials of block `blk` of `nblk` (part [nblk][C][3]); 256 working threads (more are idle),
// red = rows * C * 3 floats of LDS (cs_bn_red_lds)
template <bool POOL>
__device__ __forceinline__ void bn_red_body(const CsBnRed& r, int blk, int nblk, float* red) {
  const int C = r.C, C4 = C >> 2;
  const int rows = 256 / C4;  // C <= 1024
  const int cq = threadIdx.x % C4, rl = threadIdx.x / C4;
  const int units = POOL ? r.B * (r.H >> 1) * (r.W >> 1) : r.B * r.H * r.W;
  float acc[3][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  if (rl < rows && threadIdx.x < 256) {
    for (int u = blk * rows + rl; u < units; u += nblk * rows)
      bwd_visit<false, POOL>(r.y, r.G, r.B, r.H, r.W, C, cq, u, r.scale, r.shift, r.mean, r.invstd, nullptr, nullptr,
                             acc);
    for (int k = 0; k < 3; ++k)
      for (int q = 0; q < 4; ++q) red[((size_t)rl * C + 4 * cq + q) * 3 + k] = acc[k][q];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < C * 3; e += blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < rows; ++q) s += red[(size_t)q * C * 3 + e];
    r.part[(size_t)blk * C * 3 + e] = s;
  }
}

}  // namespace cs_bn
