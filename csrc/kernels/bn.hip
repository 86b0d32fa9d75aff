// BatchNorm2d (training statistics, eps 1e-5, momentum 0.1) + ReLU + optional
// MaxPool2d(2,2), forward and backward, NHWC fp32 — the reference block
// Conv -> BatchNorm2d -> ReLU(inplace) [-> MaxPool2d] (master/part1/model.py:16-25;
// SURVEY.md §2.2 N4-N7).
//
// Forward:  the conv GEMM epilogue already produced per-row-tile (mean, M2) partials;
//   bn_finalize combines them with Chan's parallel update (numerically robust,
//   deterministic), updates running_mean / running_var (unbiased) /
//   num_batches_tracked, and emits per-channel scale/shift; bn_apply then computes
//   relu(y*scale+shift) and the 2x2 max in ONE pass (the un-pooled activation is
//   never written).
// Backward: bn_bwd_reduce recomputes z = relu(bn(y)) and the pool argmax (first
//   maximum in window scan order, as ATen) from y, routes the incoming gradient,
//   and accumulates per-channel (sum g, sum g*xhat, sum xhat); bn_bwd_finalize
//   emits dgamma, dbeta, the conv-bias gradient (exact chain rule:
//   sum_m dZ = -gamma*invstd*mean(g*xhat)*sum(xhat)) and the dZ coefficients;
//   bn_bwd_apply writes dZ = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat)).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "launchers.h"
#include "bn_device.h"

namespace {

using cs_bn::bwd_visit;

__device__ __forceinline__ void chan_combine(float& n, float& m, float& M2, float nb, float mb, float M2b) {
  if (nb == 0.f) return;
  if (n == 0.f) {
    n = nb; m = mb; M2 = M2b;
    return;
  }
  const float nn = n + nb, d = mb - m;
  m = m + d * (nb / nn);
  M2 = M2 + M2b + d * d * (n * nb / nn);
  n = nn;
}

// gamma / beta / running stats of channel c, loaded at kernel entry so their memory latency
// overlaps the partial-sum gather instead of following it
struct FinChan {
  float g = 0.f, b = 0.f, rm = 0.f, rv = 0.f;
};
__device__ __forceinline__ FinChan finalize_load(int c, int C, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, const float* running_mean,
                                                 const float* running_var) {
  FinChan f;
  if (c < C) {
    f.g = gamma[c];
    f.b = beta[c];
    if (running_mean != nullptr) {
      f.rm = running_mean[c];
      f.rv = running_var[c];
    }
  }
  return f;
}

// scale/shift, saved batch statistics and the running-stat update of channel c from its
// combined (count, mean, M2)
__device__ __forceinline__ void finalize_store(int c, float n, float m, float M2, const FinChan& f,
                                               float* running_mean, float* running_var, float momentum, float eps,
                                               float* __restrict__ scale, float* __restrict__ shift,
                                               float* __restrict__ save_mean, float* __restrict__ save_invstd) {
  const float var = M2 / n;
  const float inv = 1.0f / sqrtf(var + eps);
  scale[c] = f.g * inv;
  shift[c] = f.b - m * f.g * inv;
  save_mean[c] = m;
  save_invstd[c] = inv;
  if (running_mean != nullptr) {
    const float unb = n > 1.f ? M2 / (n - 1.f) : var;
    running_mean[c] = (1.f - momentum) * f.rm + momentum * m;
    running_var[c] = (1.f - momentum) * f.rv + momentum * unb;
  }
}

// Chan-combine channel c's partials t = first, first + stride, ... (tile t covers rows
// [t*R, min(t*R+R, M))). The loads of 8 tiles are issued before any combine: a plain loop
// waits one full memory latency per tile (measured ~0.6 us each on conv0's 16 tiles per lane).
__device__ __forceinline__ void finalize_gather(const float* __restrict__ part, int T, int R, int M, int C, int c,
                                                int first, int stride, float& n, float& m, float& M2) {
  for (int t0 = first; t0 < T; t0 += 8 * stride) {
    float2 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = t0 + j * stride;
      v[j] = t < T ? *reinterpret_cast<const float2*>(part + ((size_t)t * C + c) * 2) : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = t0 + j * stride;
      if (t < T) chan_combine(n, m, M2, (float)((M - t * R) < R ? (M - t * R) : R), v[j].x, v[j].y);
    }
  }
}

// 256 threads = 4 waves = 4 channels; the 64 lanes of a channel's wave each combine every
// 64th tile partial, then a 6-step butterfly (fixed order: deterministic). One wave per
// channel keeps even conv0's 1024-4096 partials per channel to <= 64 serial combines.
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ part, int T, int R, int M, int C,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* running_mean,
                                                          float* running_var, int64_t* nbt, float momentum, float eps,
                                                          float* __restrict__ scale, float* __restrict__ shift,
                                                          float* __restrict__ save_mean,
                                                          float* __restrict__ save_invstd) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  float n = 0.f, m = 0.f, M2 = 0.f;
  const FinChan fc = finalize_load(c, C, gamma, beta, running_mean, running_var);
  if (c < C) finalize_gather(part, T, R, M, C, c, lane, 64, n, m, M2);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float nb = __shfl_xor(n, off, 64), mb = __shfl_xor(m, off, 64), M2b = __shfl_xor(M2, off, 64);
    chan_combine(n, m, M2, nb, mb, M2b);
  }
  if (lane == 0 && c < C)
    finalize_store(c, n, m, M2, fc, running_mean, running_var, momentum, eps, scale, shift, save_mean, save_invstd);
  if (nbt != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
}

// Many-partials variant (conv0: 4096 row tiles x 64 channels at B=64). The one-wave-per-channel
// kernel reads each channel's partials at a C*8-byte stride (one cache line per lane per load)
// from only C waves; here a 1024-thread block owns 8 consecutive channels and 128 tile slices,
// so every wave load covers 8 tiles x 64 contiguous bytes, and the 128 slice states are combined
// through LDS in a fixed tree (deterministic).
constexpr int kFinWideC = 8, kFinWideS = 128;
__global__ __launch_bounds__(1024) void bn_finalize_wide_kernel(
    const float* __restrict__ part, int T, int R, int M, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps,
    float* __restrict__ scale, float* __restrict__ shift, float* __restrict__ save_mean,
    float* __restrict__ save_invstd) {
  __shared__ float sn[kFinWideS][kFinWideC], sm[kFinWideS][kFinWideC], sM2[kFinWideS][kFinWideC];
  const int cl = threadIdx.x % kFinWideC, sl = threadIdx.x / kFinWideC;
  const int c = blockIdx.x * kFinWideC + cl;
  float n = 0.f, m = 0.f, M2 = 0.f;
  const FinChan fc = finalize_load(c, C, gamma, beta, running_mean, running_var);
  if (c < C) finalize_gather(part, T, R, M, C, c, sl, kFinWideS, n, m, M2);
  sn[sl][cl] = n;
  sm[sl][cl] = m;
  sM2[sl][cl] = M2;
  __syncthreads();
#pragma unroll
  for (int h = kFinWideS / 2; h > 0; h >>= 1) {
    if (sl < h) {
      chan_combine(n, m, M2, sn[sl + h][cl], sm[sl + h][cl], sM2[sl + h][cl]);
      sn[sl][cl] = n;
      sm[sl][cl] = m;
      sM2[sl][cl] = M2;
    }
    __syncthreads();
  }
  if (sl == 0 && c < C)
    finalize_store(c, n, m, M2, fc, running_mean, running_var, momentum, eps, scale, shift, save_mean, save_invstd);
  if (nbt != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
}

__global__ void bn_eval_coeffs_kernel(const float* gamma, const float* beta, const float* rm, const float* rv, int C,
                                      float eps, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) {
    const float inv = 1.0f / sqrtf(rv[c] + eps);
    scale[c] = gamma[c] * inv;
    shift[c] = beta[c] - rm[c] * gamma[c] * inv;
  }
}

__device__ __forceinline__ float4 bnrelu4(float4 y, float4 s, float4 t) {
  return make_float4(fmaxf(y.x * s.x + t.x, 0.f), fmaxf(y.y * s.y + t.y, 0.f), fmaxf(y.z * s.z + t.z, 0.f),
                     fmaxf(y.w * s.w + t.w, 0.f));
}

// one thread per (output position, 4 channels)
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ y, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, float* __restrict__ out,
                                                       int B, int H, int W, int C, int pool, float* __restrict__ amax) {
  const int C4 = C >> 2;
  const int Ho = pool ? H >> 1 : H, Wo = pool ? W >> 1 : W;
  const int total = B * Ho * Wo * C4;
  const int t0 = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = t0 < total;
  const int t = live ? t0 : 0;  // (every lane stays for the wave's bound)
  const int cq = t % C4, pos = t / C4;
  const float4 s = reinterpret_cast<const float4*>(scale)[cq];
  const float4 sh = reinterpret_cast<const float4*>(shift)[cq];
  float4 r;
  if (!pool) {
    r = bnrelu4(reinterpret_cast<const float4*>(y)[t], s, sh);
  } else {
    const int wo = pos % Wo, ho = (pos / Wo) % Ho, b = pos / (Wo * Ho);
    const size_t base = (((size_t)b * H + 2 * ho) * W + 2 * wo) * C4 + cq;
    const float4* y4 = reinterpret_cast<const float4*>(y);
    const float4 a0 = bnrelu4(y4[base], s, sh), a1 = bnrelu4(y4[base + C4], s, sh);
    const float4 a2 = bnrelu4(y4[base + (size_t)W * C4], s, sh), a3 = bnrelu4(y4[base + (size_t)W * C4 + C4], s, sh);
    r = make_float4(fmaxf(fmaxf(a0.x, a1.x), fmaxf(a2.x, a3.x)), fmaxf(fmaxf(a0.y, a1.y), fmaxf(a2.y, a3.y)),
                    fmaxf(fmaxf(a0.z, a1.z), fmaxf(a2.z, a3.z)), fmaxf(fmaxf(a0.w, a1.w), fmaxf(a2.w, a3.w)));
  }
  if (live) reinterpret_cast<float4*>(out)[t] = r;
  // the output bound the next conv's F3 math scales by (ReLU output: non-negative)
  if (amax != nullptr) cs::block_amax_publish(live ? fmaxf(fmaxf(r.x, r.y), fmaxf(r.z, r.w)) : 0.f, amax);
}

template <bool APPLY, bool POOL>
__global__ __launch_bounds__(256) void bn_bwd_kernel(const float* __restrict__ y, const float* __restrict__ G, int B,
                                                     int H, int W, int C, const float* __restrict__ scale,
                                                     const float* __restrict__ shift, const float* __restrict__ mean,
                                                     const float* __restrict__ invstd, const float* __restrict__ coef,
                                                     float* __restrict__ dz, float* __restrict__ part,
                                                     unsigned long long* __restrict__ signal, float* __restrict__ amax) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [rows][C][3] (reduce only)
  // a deferred stream-link signal (device_comm.h StreamLink::defer): this launch started, so the
  // kernels before it on the stream completed
  if (signal != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_fetch_add(signal, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if constexpr (!APPLY) {  // the shared body (also run inside weight-gradient GEMM launches)
    const CsBnRed r{y, G, scale, shift, mean, invstd, part, B, H, W, C, POOL ? 1 : 0, (int)gridDim.x};
    cs_bn::bn_red_body<POOL>(r, blockIdx.x, gridDim.x, red);
    return;
  }
  const int C4 = C >> 2;
  const int rows = 256 / C4;  // C <= 1024
  const int cq = threadIdx.x % C4, rl = threadIdx.x / C4;
  const int units = POOL ? B * (H >> 1) * (W >> 1) : B * H * W;
  float acc[3][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  float vm = 0.f;
  if (rl < rows) {
    for (int u = blockIdx.x * rows + rl; u < units; u += gridDim.x * rows)
      bwd_visit<APPLY, POOL>(y, G, B, H, W, C, cq, u, scale, shift, mean, invstd, coef, dz, acc, 0,
                             APPLY && amax != nullptr ? &vm : nullptr);
  }
  if (APPLY) {
    if (amax != nullptr) cs::block_amax_publish(vm, amax);  // the dZ bound (F3 conv math)
    return;
  }
  if (rl < rows) {
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[((size_t)rl * C + 4 * cq + q) * 3 + k] = acc[k][q];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < C * 3; e += blockDim.x) {
    float s = 0.f;
    for (int r = 0; r < rows; ++r) s += red[(size_t)r * C * 3 + e];
    part[(size_t)blockIdx.x * C * 3 + e] = s;
  }
}

// 256 threads = 4 waves = 4 channels: each lane sums every 64th block's partials, then
// a wave butterfly (fixed order: deterministic).
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ part, int P, int C, int M,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ invstd,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              float* __restrict__ dbias, float* __restrict__ coef,
                                                              unsigned long long* __restrict__ signal) {
  // a deferred stream-link signal (the kernels before this launch on its stream completed)
  if (signal != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_fetch_add(signal, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  float sg = 0.f, sgx = 0.f, sx = 0.f;
  // per-channel operands first, then 8 partial loads in flight per lane (same summation order)
  const float gam = c < C ? gamma[c] : 0.f, ist = c < C ? invstd[c] : 0.f;
  if (c < C) {
    for (int p0 = lane; p0 < P; p0 += 8 * 64) {
      float v[8][3];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int p = p0 + j * 64;
        const float* q = part + ((size_t)p * C + c) * 3;
        v[j][0] = p < P ? q[0] : 0.f;
        v[j][1] = p < P ? q[1] : 0.f;
        v[j][2] = p < P ? q[2] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sg += v[j][0];
        sgx += v[j][1];
        sx += v[j][2];
      }
    }
  }
  sg = cs::wave_sum(sg);
  sgx = cs::wave_sum(sgx);
  sx = cs::wave_sum(sx);
  if (lane != 0 || c >= C) return;
  const float k1 = gam * ist, k2 = sg / (float)M, k3 = sgx / (float)M;
  if (dgamma) dgamma[c] = sgx;
  if (dbeta) dbeta[c] = sg;
  if (dbias) dbias[c] = -k1 * k3 * sx;
  coef[3 * c] = k1;
  coef[3 * c + 1] = k2;
  coef[3 * c + 2] = k3;
}

// ------------------------------------------------------------------ single-kernel BN for small layers
// One block owns 16 channels (4 float4 lanes x 64 row lanes) and ALL rows of them, so the
// statistics -> coefficients -> apply dependency stays inside the block: forward = finalize
// + normalize/ReLU/pool, backward = reduce + finalize + apply, each ONE launch instead of
// two / three (each launch boundary plus its dependent global round trip costs ~3-5 us on
// MI355X, more than these layers' data movement). Reductions run in a fixed order
// (row-lane butterfly, then the 4 waves in order): deterministic. Used where the rows per
// block are few (the engine's small-spatial layers).
constexpr int kFusedCh = 16;

// fixed-order Chan combine of 64 row lanes (tid = rl*4 + cq) -> lanes with rl == 0
__device__ __forceinline__ void chan_reduce_block(float (&n)[4], float (&m)[4], float (&M2)[4], float* lds) {
#pragma unroll
  for (int off = 4; off < 64; off <<= 1)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float nb = __shfl_xor(n[q], off, 64), mb = __shfl_xor(m[q], off, 64), M2b = __shfl_xor(M2[q], off, 64);
      chan_combine(n[q], m[q], M2[q], nb, mb, M2b);
    }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, cq = threadIdx.x & 3;
  if (lane < 4)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      lds[((wv * 4 + cq) * 4 + q) * 3 + 0] = n[q];
      lds[((wv * 4 + cq) * 4 + q) * 3 + 1] = m[q];
      lds[((wv * 4 + cq) * 4 + q) * 3 + 2] = M2[q];
    }
  __syncthreads();
  if (threadIdx.x < 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      n[q] = m[q] = M2[q] = 0.f;
      for (int w = 0; w < 4; ++w)
        chan_combine(n[q], m[q], M2[q], lds[((w * 4 + cq) * 4 + q) * 3], lds[((w * 4 + cq) * 4 + q) * 3 + 1],
                     lds[((w * 4 + cq) * 4 + q) * 3 + 2]);
    }
  }
}

// fixed-order sum of 3x4 per-thread accumulators over the 64 row lanes -> threads < 4
__device__ __forceinline__ void sum_reduce_block(float (&acc)[3][4], float* lds) {
#pragma unroll
  for (int off = 4; off < 64; off <<= 1)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[k][q] += __shfl_xor(acc[k][q], off, 64);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, cq = threadIdx.x & 3;
  if (lane < 4)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int q = 0; q < 4; ++q) lds[((wv * 4 + cq) * 3 + k) * 4 + q] = acc[k][q];
  __syncthreads();
  if (threadIdx.x < 4)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float s = 0.f;
        for (int w = 0; w < 4; ++w) s += lds[((w * 4 + cq) * 3 + k) * 4 + q];
        acc[k][q] = s;
      }
}

// grid (C/16, row chunks): every block finalizes its 16 channels from the T tile partials
// (identical fixed-order combine in every block), block row 0 publishes bnv / running stats,
// and each block normalizes its chunk of `upb` output units.
__global__ __launch_bounds__(256) void bn_fused_fwd_kernel(const float* __restrict__ part, int T, int R, int M,
                                                           int C, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float* running_mean,
                                                           float* running_var, int64_t* nbt, float momentum,
                                                           float eps, float* __restrict__ bnv, const float* __restrict__ y,
                                                           float* __restrict__ out, int B, int H, int W, int pool,
                                                           int upb) {
  __shared__ float lds[4 * 4 * 4 * 3];
  __shared__ float4 sc_sh[2][4];
  const int cq = threadIdx.x & 3, rl = threadIdx.x >> 2;
  const int cqg = blockIdx.x * 4 + cq;  // global channel quad
  const bool lead = blockIdx.y == 0;
  const int C4 = C >> 2;
  const int Ho = pool ? H >> 1 : H, Wo = pool ? W >> 1 : W;
  const int u0 = blockIdx.y * upb + rl;
  const int u_end = min(B * Ho * Wo, (int)(blockIdx.y + 1) * upb);
  const float4* y4 = reinterpret_cast<const float4*>(y);
  // Everything that does not depend on the statistics is loaded first, so its memory latency
  // overlaps the partial gather: this block's first y rows (4 units without pooling, the first
  // unit's 2x2 window with it) and the lead threads' per-channel operands
  float4 pre[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) pre[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!pool) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (u0 + 64 * j < u_end) pre[j] = y4[(size_t)(u0 + 64 * j) * C4 + cqg];
  } else if (u0 < u_end) {
    const int wo = u0 % Wo, ho = (u0 / Wo) % Ho, b = u0 / (Wo * Ho);
    const size_t base = (((size_t)b * H + 2 * ho) * W + 2 * wo) * C4 + cqg;
    pre[0] = y4[base];
    pre[1] = y4[base + C4];
    pre[2] = y4[base + (size_t)W * C4];
    pre[3] = y4[base + (size_t)W * C4 + C4];
  }
  float gq[4] = {0.f, 0.f, 0.f, 0.f}, bq[4] = {0.f, 0.f, 0.f, 0.f}, rmq[4] = {0.f, 0.f, 0.f, 0.f},
        rvq[4] = {0.f, 0.f, 0.f, 0.f};
  if (threadIdx.x < 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 4 * cqg + q;
      gq[q] = gamma[c];
      bq[q] = beta[c];
      if (lead && running_mean != nullptr) {
        rmq[q] = running_mean[c];
        rvq[q] = running_var[c];
      }
    }
  }
  float n[4] = {0.f, 0.f, 0.f, 0.f}, m[4] = {0.f, 0.f, 0.f, 0.f}, M2[4] = {0.f, 0.f, 0.f, 0.f};
  for (int t = rl; t < T; t += 64) {
    const int cnt = (M - t * R) < R ? (M - t * R) : R;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float2 pm = *reinterpret_cast<const float2*>(part + ((size_t)t * C + 4 * cqg + q) * 2);
      chan_combine(n[q], m[q], M2[q], (float)cnt, pm.x, pm.y);
    }
  }
  chan_reduce_block(n, m, M2, lds);
  if (threadIdx.x < 4) {
    float sc[4], sh[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 4 * cqg + q;
      const float var = M2[q] / n[q], inv = 1.0f / sqrtf(var + eps);
      sc[q] = gq[q] * inv;
      sh[q] = bq[q] - m[q] * gq[q] * inv;
      if (!lead) continue;
      bnv[c] = sc[q];
      bnv[C + c] = sh[q];
      bnv[2 * C + c] = m[q];
      bnv[3 * C + c] = inv;
      if (running_mean != nullptr) {
        const float unb = n[q] > 1.f ? M2[q] / (n[q] - 1.f) : var;
        running_mean[c] = (1.f - momentum) * rmq[q] + momentum * m[q];
        running_var[c] = (1.f - momentum) * rvq[q] + momentum * unb;
      }
    }
    sc_sh[0][cq] = make_float4(sc[0], sc[1], sc[2], sc[3]);
    sc_sh[1][cq] = make_float4(sh[0], sh[1], sh[2], sh[3]);
  }
  if (nbt != nullptr && lead && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
  __syncthreads();
  const float4 s = sc_sh[0][cq], t = sc_sh[1][cq];
  float4* out4 = reinterpret_cast<float4*>(out);
  if (!pool) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (u0 + 64 * j < u_end) out4[(size_t)(u0 + 64 * j) * C4 + cqg] = bnrelu4(pre[j], s, t);
  } else if (u0 < u_end) {
    const float4 a0 = bnrelu4(pre[0], s, t), a1 = bnrelu4(pre[1], s, t);
    const float4 a2 = bnrelu4(pre[2], s, t), a3 = bnrelu4(pre[3], s, t);
    out4[(size_t)u0 * C4 + cqg] =
        make_float4(fmaxf(fmaxf(a0.x, a1.x), fmaxf(a2.x, a3.x)), fmaxf(fmaxf(a0.y, a1.y), fmaxf(a2.y, a3.y)),
                    fmaxf(fmaxf(a0.z, a1.z), fmaxf(a2.z, a3.z)), fmaxf(fmaxf(a0.w, a1.w), fmaxf(a2.w, a3.w)));
  }
  for (int u = u0 + (pool ? 64 : 256); u < u_end; u += 64) {
    float4 r;
    if (!pool) {
      r = bnrelu4(y4[(size_t)u * C4 + cqg], s, t);
    } else {
      const int wo = u % Wo, ho = (u / Wo) % Ho, b = u / (Wo * Ho);
      const size_t base = (((size_t)b * H + 2 * ho) * W + 2 * wo) * C4 + cqg;
      const float4 a0 = bnrelu4(y4[base], s, t), a1 = bnrelu4(y4[base + C4], s, t);
      const float4 a2 = bnrelu4(y4[base + (size_t)W * C4], s, t), a3 = bnrelu4(y4[base + (size_t)W * C4 + C4], s, t);
      r = make_float4(fmaxf(fmaxf(a0.x, a1.x), fmaxf(a2.x, a3.x)), fmaxf(fmaxf(a0.y, a1.y), fmaxf(a2.y, a3.y)),
                      fmaxf(fmaxf(a0.z, a1.z), fmaxf(a2.z, a3.z)), fmaxf(fmaxf(a0.w, a1.w), fmaxf(a2.w, a3.w)));
    }
    reinterpret_cast<float4*>(out)[(size_t)u * C4 + cqg] = r;
  }
}

template <bool POOL>
__global__ __launch_bounds__(256) void bn_fused_bwd_kernel(const float* __restrict__ y, const float* __restrict__ G,
                                                           int B, int H, int W, int C, const float* __restrict__ bnv,
                                                           const float* __restrict__ gamma, float* __restrict__ coef,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                           float* __restrict__ dbias, float* __restrict__ dz,
                                                           unsigned long long* __restrict__ signal,
                                                           float* __restrict__ amax) {
  __shared__ float lds[4 * 4 * 3 * 4];
  __shared__ float coef_sh[3 * kFusedCh];  // this block's 16 channels' dZ coefficients
  // a deferred stream-link signal (device_comm.h StreamLink::defer): this launch started, so the
  // kernels before it on the stream completed
  if (signal != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_fetch_add(signal, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int cq = threadIdx.x & 3, rl = threadIdx.x >> 2;
  const int cqg = blockIdx.x * 4 + cq;
  const float* scale = bnv;
  const float* shift = bnv + C;
  const float* mean = bnv + 2 * C;
  const float* invstd = bnv + 3 * C;
  const int units = POOL ? B * (H >> 1) * (W >> 1) : B * H * W;
  // gamma * invstd loaded up front (its latency overlaps the reduce pass)
  float k1q[4] = {0.f, 0.f, 0.f, 0.f};
  if (threadIdx.x < 4)
#pragma unroll
    for (int q = 0; q < 4; ++q) k1q[q] = gamma[4 * cqg + q] * invstd[4 * cqg + q];
  float acc[3][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  for (int u = rl; u < units; u += 64)
    bwd_visit<false, POOL>(y, G, B, H, W, C, cqg, u, scale, shift, mean, invstd, coef, dz, acc);
  sum_reduce_block(acc, lds);
  const int c0 = blockIdx.x * kFusedCh;
  if (threadIdx.x < 4) {
    const float Mf = (float)(B * H * W);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 4 * cqg + q;
      const float k1 = k1q[q], k2 = acc[0][q] / Mf, k3 = acc[1][q] / Mf;
      if (dgamma) dgamma[c] = acc[1][q];
      if (dbeta) dbeta[c] = acc[0][q];
      if (dbias) dbias[c] = -k1 * k3 * acc[2][q];
      coef[3 * c] = k1;
      coef[3 * c + 1] = k2;
      coef[3 * c + 2] = k3;
      coef_sh[3 * (c - c0)] = k1;
      coef_sh[3 * (c - c0) + 1] = k2;
      coef_sh[3 * (c - c0) + 2] = k3;
    }
  }
  __syncthreads();  // the apply pass reads the coefficients from LDS (no global round trip)
  float dummy[3][4];
  float vm = 0.f;
  for (int u = rl; u < units; u += 64)
    bwd_visit<true, POOL>(y, G, B, H, W, C, cqg, u, scale, shift, mean, invstd, coef_sh, dz, dummy, c0,
                          amax != nullptr ? &vm : nullptr);
  if (amax != nullptr) cs::block_amax_publish(vm, amax);  // the dZ bound (F3 conv math)
}

// grid (C/16, row chunks): finalize the BN backward of this block's 16 channels from the P
// partials [P][C][3] (sum g, sum g*xhat, sum xhat) — thread (rl, cq) sums partials rl, rl + 64, ...
// of its channel quad, then the fixed-order block reduce: identical in every block — block row 0
// publishes the coefficients and the parameter gradients, and every block writes dZ for its chunk
// of `upb` units. The first statistics-independent loads (the chunk's first unit of G and y) are
// issued before the partial gather so their latency overlaps it.
template <bool POOL>
__global__ __launch_bounds__(256) void bn_bwd_tail_fused_kernel(const float* __restrict__ y, const float* __restrict__ G,
                                                                int B, int H, int W, int C,
                                                                const float* __restrict__ bnv,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ part, int P,
                                                                float* __restrict__ coef, float* __restrict__ dgamma,
                                                                float* __restrict__ dbeta, float* __restrict__ dbias,
                                                                float* __restrict__ dz, int upb,
                                                                unsigned long long* __restrict__ signal) {
  __shared__ float lds[4 * 4 * 3 * 4];
  __shared__ float coef_sh[3 * kFusedCh];
  if (signal != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    __hip_atomic_fetch_add(signal, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int cq = threadIdx.x & 3, rl = threadIdx.x >> 2;
  const int cqg = blockIdx.x * 4 + cq;
  const bool lead = blockIdx.y == 0;
  const float* invstd = bnv + 3 * C;
  float k1q[4] = {0.f, 0.f, 0.f, 0.f};
  if (threadIdx.x < 4)
#pragma unroll
    for (int q = 0; q < 4; ++q) k1q[q] = gamma[4 * cqg + q] * invstd[4 * cqg + q];
  float acc[3][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  // 4 partials in flight per lane before their adds (same ascending order per lane)
  for (int p0 = rl; p0 < P; p0 += 4 * 64) {
    float4 v[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = p0 + 64 * j;
      const float* q = part + ((size_t)p * C + 4 * cqg) * 3;
      v[j][0] = p < P ? *reinterpret_cast<const float4*>(q) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[j][1] = p < P ? *reinterpret_cast<const float4*>(q + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[j][2] = p < P ? *reinterpret_cast<const float4*>(q + 8) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // 12 floats = channels 4cqg..4cqg+3 x (g, g*xhat, xhat), channel-major
      const float f[12] = {v[j][0].x, v[j][0].y, v[j][0].z, v[j][0].w, v[j][1].x, v[j][1].y,
                           v[j][1].z, v[j][1].w, v[j][2].x, v[j][2].y, v[j][2].z, v[j][2].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < 3; ++k) acc[k][q] += f[3 * q + k];
    }
  }
  sum_reduce_block(acc, lds);
  const int c0 = blockIdx.x * kFusedCh;
  if (threadIdx.x < 4) {
    const float Mf = (float)(B * H * W);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 4 * cqg + q;
      const float k1 = k1q[q], k2 = acc[0][q] / Mf, k3 = acc[1][q] / Mf;
      if (lead) {
        if (dgamma) dgamma[c] = acc[1][q];
        if (dbeta) dbeta[c] = acc[0][q];
        if (dbias) dbias[c] = -k1 * k3 * acc[2][q];
        coef[3 * c] = k1;
        coef[3 * c + 1] = k2;
        coef[3 * c + 2] = k3;
      }
      coef_sh[3 * (c - c0)] = k1;
      coef_sh[3 * (c - c0) + 1] = k2;
      coef_sh[3 * (c - c0) + 2] = k3;
    }
  }
  __syncthreads();
  const int units = POOL ? B * (H >> 1) * (W >> 1) : B * H * W;
  const int u_end = min(units, (int)(blockIdx.y + 1) * upb);
  float dummy[3][4];
  for (int u = blockIdx.y * upb + rl; u < u_end; u += 64)
    bwd_visit<true, POOL>(y, G, B, H, W, C, cqg, u, bnv, bnv + C, bnv + 2 * C, invstd, coef_sh, dz, dummy, c0);
}

}  // namespace

int cs_bn_bwd_blocks(int B, int H, int W, int C, int pool) {
  const int units = pool ? B * (H / 2) * (W / 2) : B * H * W;
  const int rows = 256 / (C / 4);
  int blocks = (units + rows - 1) / rows;
  return blocks < 256 ? blocks : 256;
}

// partial count from which the 8-channel / 1024-thread finalize runs
constexpr int kFinWideMin = 512;

hipError_t cs_bn_finalize(const float* part, int T, int R, int M, int C, const float* gamma, const float* beta,
                          float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps,
                          float* scale, float* shift, float* save_mean, float* save_invstd, hipStream_t stream) {
  if (T >= kFinWideMin && C % kFinWideC == 0)
    hipLaunchKernelGGL(bn_finalize_wide_kernel, dim3(C / kFinWideC), dim3(1024), 0, stream, part, T, R, M, C, gamma,
                       beta, running_mean, running_var, nbt, momentum, eps, scale, shift, save_mean, save_invstd);
  else
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 3) / 4), dim3(256), 0, stream, part, T, R, M, C, gamma, beta,
                       running_mean, running_var, nbt, momentum, eps, scale, shift, save_mean, save_invstd);
  return hipGetLastError();
}

hipError_t cs_bn_eval_coeffs(const float* gamma, const float* beta, const float* rm, const float* rv, int C, float eps,
                             float* scale, float* shift, hipStream_t stream) {
  hipLaunchKernelGGL(bn_eval_coeffs_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, gamma, beta, rm, rv, C, eps,
                     scale, shift);
  return hipGetLastError();
}

hipError_t cs_bn_apply(const float* y, const float* scale, const float* shift, float* out, int B, int H, int W, int C,
                       int pool, hipStream_t stream, float* amax) {
  if (C % 4 != 0 || (pool && ((H | W) & 1))) return hipErrorInvalidValue;
  const int total = B * (pool ? H / 2 : H) * (pool ? W / 2 : W) * (C / 4);
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(bn_apply_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, y, scale, shift, out, B, H, W,
                     C, pool, amax);
  return hipGetLastError();
}

hipError_t cs_bn_bwd(const float* y, const float* G, int B, int H, int W, int C, int pool, const float* scale,
                     const float* shift, const float* mean, const float* invstd, const float* gamma, float* part,
                     float* coef, float* dgamma, float* dbeta, float* dbias, float* dz, hipStream_t stream,
                     float* amax) {
  if (C % 4 != 0 || C > 1024 || (pool && ((H | W) & 1))) return hipErrorInvalidValue;
  const int P = cs_bn_bwd_blocks(B, H, W, C, pool);
  const int rows = 256 / (C / 4);
  const size_t lds = (size_t)rows * C * 3 * sizeof(float);
  if (pool) {
    hipLaunchKernelGGL((bn_bwd_kernel<false, true>), dim3(P), dim3(256), lds, stream, y, G, B, H, W, C, scale, shift,
                       mean, invstd, nullptr, nullptr, part, nullptr, nullptr);
  } else {
    hipLaunchKernelGGL((bn_bwd_kernel<false, false>), dim3(P), dim3(256), lds, stream, y, G, B, H, W, C, scale, shift,
                       mean, invstd, nullptr, nullptr, part, nullptr, nullptr);
  }
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  return cs_bn_bwd_tail(y, G, B, H, W, C, pool, scale, shift, mean, invstd, gamma, part, P, coef, dgamma, dbeta,
                        dbias, dz, stream, nullptr, amax);
}

hipError_t cs_bn_bwd_finalize(const float* part, int P, int C, int M, const float* gamma, const float* invstd,
                              float* coef, float* dgamma, float* dbeta, float* dbias, hipStream_t stream,
                              unsigned long long* signal) {
  if (C % 4 != 0 || P < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 3) / 4), dim3(256), 0, stream, part, P, C, M, gamma, invstd,
                     dgamma, dbeta, dbias, coef, signal);
  return hipGetLastError();
}

hipError_t cs_bn_bwd_tail(const float* y, const float* G, int B, int H, int W, int C, int pool, const float* scale,
                          const float* shift, const float* mean, const float* invstd, const float* gamma,
                          const float* part, int P, float* coef, float* dgamma, float* dbeta, float* dbias, float* dz,
                          hipStream_t stream, unsigned long long* signal, float* amax) {
  if (C % 4 != 0 || C > 1024 || (pool && ((H | W) & 1)) || P < 1) return hipErrorInvalidValue;
  const int M = B * H * W;
  const int rows = 256 / (C / 4);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 3) / 4), dim3(256), 0, stream, part, P, C, M, gamma, invstd,
                     dgamma, dbeta, dbias, coef, signal);
  // the apply pass is sized for bandwidth, independent of the reduce's P
  const int units = pool ? B * (H / 2) * (W / 2) : B * H * W;
  int blocks = (units + rows - 1) / rows;
  if (blocks > 2048) blocks = 2048;
  if (pool) {
    hipLaunchKernelGGL((bn_bwd_kernel<true, true>), dim3(blocks), dim3(256), 0, stream, y, G, B, H, W, C, scale, shift,
                       mean, invstd, coef, dz, nullptr, nullptr, amax);
  } else {
    hipLaunchKernelGGL((bn_bwd_kernel<true, false>), dim3(blocks), dim3(256), 0, stream, y, G, B, H, W, C, scale,
                       shift, mean, invstd, coef, dz, nullptr, nullptr, amax);
  }
  return hipGetLastError();
}

hipError_t cs_bn_bwd_apply(const float* y, const float* G, int B, int H, int W, int C, int pool, const float* scale,
                           const float* shift, const float* mean, const float* invstd, const float* coef, float* dz,
                           hipStream_t stream, unsigned long long* signal) {
  if (C % 4 != 0 || C > 1024 || (pool && ((H | W) & 1))) return hipErrorInvalidValue;
  const int rows = 256 / (C / 4);
  const int units = pool ? B * (H / 2) * (W / 2) : B * H * W;
  int blocks = (units + rows - 1) / rows;
  if (blocks > 2048) blocks = 2048;
  if (pool)
    hipLaunchKernelGGL((bn_bwd_kernel<true, true>), dim3(blocks), dim3(256), 0, stream, y, G, B, H, W, C, scale, shift,
                       mean, invstd, coef, dz, nullptr, signal, nullptr);
  else
    hipLaunchKernelGGL((bn_bwd_kernel<true, false>), dim3(blocks), dim3(256), 0, stream, y, G, B, H, W, C, scale,
                       shift, mean, invstd, coef, dz, nullptr, signal, nullptr);
  return hipGetLastError();
}

hipError_t cs_bn_fused_fwd(const float* part, int T, int R, int M, int C, const float* gamma, const float* beta,
                           float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps,
                           float* bnv, const float* y, float* out, int B, int H, int W, int pool, hipStream_t stream) {
  if (C % kFusedCh != 0 || (pool && ((H | W) & 1))) return hipErrorInvalidValue;
  // row chunks of >= 256 output units (4 per row lane), ~512 blocks at most
  const int units = B * (pool ? H / 2 : H) * (pool ? W / 2 : W);
  const int cg = C / kFusedCh;
  int chunks = std::max(1, std::min((units + 255) / 256, std::max(1, 512 / cg)));
  const int upb = (units + chunks - 1) / chunks;
  chunks = (units + upb - 1) / upb;
  hipLaunchKernelGGL(bn_fused_fwd_kernel, dim3(cg, chunks), dim3(256), 0, stream, part, T, R, M, C, gamma, beta,
                     running_mean, running_var, nbt, momentum, eps, bnv, y, out, B, H, W, pool, upb);
  return hipGetLastError();
}

hipError_t cs_bn_bwd_tail_fused(const float* y, const float* G, int B, int H, int W, int C, int pool, const float* bnv,
                                const float* gamma, const float* part, int P, float* coef, float* dgamma, float* dbeta,
                                float* dbias, float* dz, hipStream_t stream, unsigned long long* signal) {
  if (C % kFusedCh != 0 || C > 1024 || (pool && ((H | W) & 1)) || P < 1) return hipErrorInvalidValue;
  // row chunks of >= 64 units (one per row lane), ~512 blocks at most (as cs_bn_fused_fwd)
  const int units = B * (pool ? H / 2 : H) * (pool ? W / 2 : W);
  const int cg = C / kFusedCh;
  int chunks = std::max(1, std::min((units + 63) / 64, std::max(1, 512 / cg)));
  const int upb = (units + chunks - 1) / chunks;
  chunks = (units + upb - 1) / upb;
  if (pool)
    hipLaunchKernelGGL((bn_bwd_tail_fused_kernel<true>), dim3(cg, chunks), dim3(256), 0, stream, y, G, B, H, W, C, bnv,
                       gamma, part, P, coef, dgamma, dbeta, dbias, dz, upb, signal);
  else
    hipLaunchKernelGGL((bn_bwd_tail_fused_kernel<false>), dim3(cg, chunks), dim3(256), 0, stream, y, G, B, H, W, C,
                       bnv, gamma, part, P, coef, dgamma, dbeta, dbias, dz, upb, signal);
  return hipGetLastError();
}

hipError_t cs_bn_fused_bwd(const float* y, const float* G, int B, int H, int W, int C, int pool, const float* bnv,
                           const float* gamma, float* coef, float* dgamma, float* dbeta, float* dbias, float* dz,
                           hipStream_t stream, unsigned long long* signal, float* amax) {
  if (C % kFusedCh != 0 || (pool && ((H | W) & 1))) return hipErrorInvalidValue;
  if (pool)
    hipLaunchKernelGGL((bn_fused_bwd_kernel<true>), dim3(C / kFusedCh), dim3(256), 0, stream, y, G, B, H, W, C, bnv,
                       gamma, coef, dgamma, dbeta, dbias, dz, signal, amax);
  else
    hipLaunchKernelGGL((bn_fused_bwd_kernel<false>), dim3(C / kFusedCh), dim3(256), 0, stream, y, G, B, H, W, C, bnv,
                       gamma, coef, dgamma, dbeta, dbias, dz, signal, amax);
  return hipGetLastError();
}
