// Shared pieces of the conv implicit-GEMM kernels (conv_gemm.hip: register / LDS-DMA staged
// fp32 operands; conv_xp.hip: pre-split bf16 operand planes): buffer-resource addressing,
// the 3x3 tap mask, the in-launch split-K combine and the common epilogue (K-group partial
// sums, bias, output / split-K slab stores, BN tile statistics, conv0's OIHW scatter).
// Every block computes one BMxBN output tile with 4 spatial waves (2x2, (BM/2)x(BN/2) each,
// 32x32 MFMA tiles) per K-group.
#pragma once
#include "bn_device.h"
#include "bn_fin.h"
#include "common.h"
#include "launchers.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

// byte offset past every descriptor's range: loads return 0, stores are dropped
constexpr int kOOB = 0x7ffffff0;

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// the whole offset goes in voffset: the range check is only guaranteed to cover it
__device__ __forceinline__ float4 bload4(rsrc_t r, int voff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}
__device__ __forceinline__ void bstore1(rsrc_t r, float v, int voff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, voff, 0, 0);
}

// 9-bit mask of the 3x3 taps whose source pixel (h + s*dh, w + s*dw) is inside the image
// (s = +1 for FWD / WGRAD, -1 for DGRAD's flipped kernel); bit t = tap t = 3*(dh+1)+(dw+1)
__device__ __forceinline__ unsigned tap_mask(int h, int w, int H, int W, int s) {
  unsigned m = 0;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int hh = h + s * (t / 3 - 1), ww = w + s * (t % 3 - 1);
    if ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W) m |= 1u << t;
  }
  return m;
}

// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt left at their maxima), gfx9 encoding
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// DGRAD epilogue with CsConvArgs::ered: this tile's BN-backward partial sums of the block below
// (bn.hip's reduce pass, per channel: sum g, sum g*xhat, sum xhat over its full-resolution
// elements) from the output gradient values of K-group 0. The tile goes through LDS first
// (dgrad_bn_stage, inline), then a NON-inlined pass gathers y and sums: it runs after the
// accumulators are dead and gets its own register allocation, so the main loop's does not
// grow (inlined, it cost the 1024-thread tiles VGPR spills). Every wave of the block shares
// the gathers: thread t owns column t % BN and every (NT/BN)-th row; the row groups' sums are
// added in a fixed order -> ered.part [mt][N][3]. LDS: BM x (BN + 4) floats (launch_k sizes
// the launch for it). Every thread of the block takes part (barriers inside).
template <int BM, int BN>
__device__ __forceinline__ void dgrad_bn_stage(const f32x16 (&acc)[BM / 64][BN / 64], bool owner, float* smem) {
  constexpr int RM = BM / 64, RN = BN / 64, WM = BM / 2, WN = BN / 2, TP = BN + 4;
  const int lane = threadIdx.x & 63, wsp = (threadIdx.x >> 6) & 3;
  const int wm = wsp >> 1, wn = wsp & 1, r = lane & 31, hh = lane >> 5;
  if (owner) {
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int el = 0; el < 16; ++el)
          smem[(wm * WM + i * 32 + (el & 3) + 8 * (el >> 2) + 4 * hh) * TP + wn * WN + j * 32 + r] = acc[i][j][el];
  }
  __syncthreads();
}

template <int BM, int BN, int NT, bool POOL>
__device__ __noinline__ void dgrad_bn_partials(const float* __restrict__ y, const float* __restrict__ bnv_scale,
                                               const float* __restrict__ bnv_shift, const float* __restrict__ bnv_mean,
                                               const float* __restrict__ bnv_invstd, float* __restrict__ part, int M,
                                               int N, int lgH, int lgW, int mt, int m0, int n0, float* img, bool fin) {
  // thread: channel quad cq (float4 loads of the image, y and the BN vectors), every RG-th row
  constexpr int TP = BN + 4, CQ = BN / 4, RG = NT / CQ, NW = NT / 64;
  static_assert(NT % CQ == 0 && 64 % CQ == 0 && NW * BN * 3 <= BM * TP, "wave partials must fit the tile image");
  const int tid = threadIdx.x, lane = tid & 63, cq = tid % CQ, rg = tid / CQ, n = n0 + 4 * cq;
  const bool nok = n < N;
  const int nc = nok ? n : 0;
  const float4 sc = *reinterpret_cast<const float4*>(bnv_scale + nc), sh = *reinterpret_cast<const float4*>(bnv_shift + nc);
  const float4 mu = *reinterpret_cast<const float4*>(bnv_mean + nc), is = *reinterpret_cast<const float4*>(bnv_invstd + nc);
  float s[3][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll 2
  for (int row = rg; row < BM; row += RG) {
    const int m = m0 + row;
    const bool ok = nok && m < M;
    float t[3][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    cs_bn::bwd_point4<POOL>(y, cs_bn::bwd_point_index<POOL>(ok ? m : 0, nc, lgH, lgW, N), N, 2 << lgW,
                            *reinterpret_cast<const float4*>(img + row * TP + 4 * cq), sc, sh, mu, is, t);
    if (ok)
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int q = 0; q < 4; ++q) s[k][q] += t[k][q];
  }
  // the wave's row groups (lane / CQ), then the waves in order
#pragma unroll
  for (int off = CQ; off < 64; off <<= 1)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int q = 0; q < 4; ++q) s[k][q] += __shfl_xor(s[k][q], off, 64);
  __syncthreads();  // every image read done: the wave sums reuse the space
  if (lane < CQ)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int q = 0; q < 4; ++q) img[((tid >> 6) * BN + 4 * cq + q) * 3 + k] = s[k][q];
  __syncthreads();
  if (tid < BN && n0 + tid < N) {
    float t[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      t[k] = 0.f;
      for (int w = 0; w < NW; ++w) t[k] += img[(w * BN + tid) * 3 + k];
    }
    if (fin) {  // [T][N][4], write-through for the launch's last arriver (bn_fin.h)
      cs_fin::put_sums(part, N, mt, n0 + tid, t[0], t[1], t[2]);
    } else {
#pragma unroll
      for (int k = 0; k < 3; ++k) part[((size_t)mt * N + n0 + tid) * 3 + k] = t[k];
    }
  }
}

// Epilogue of one output tile: `acc` holds each spatial wave's (BM/2)x(BN/2) partial sums of
// this block's K range (K-group kg's share when KG > 1). The caller's main loop has ended
// on a barrier (every wave's LDS reads done): smem is free.
template <int BM, int BN, int MODE, int KG>
__device__ __forceinline__ void conv_epilogue(const CsConvArgs& a, f32x16 (&acc)[BM / 64][BN / 64], const int tile,
                                              const int split, const int nsplit, float* smem) {
  constexpr int RM = BM / 64, RN = BN / 64, WM = BM / 2, WN = BN / 2;
  const int ntn = (a.N + BN - 1) / BN;
  const int mt = tile / ntn, nt = tile - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kg = wid >> 2, wsp = wid & 3;
  const int wm = wsp >> 1, wn = wsp & 1, r = lane & 31, hh = lane >> 5;
  if constexpr (KG > 1) {
    // K-group partials -> group 0, summed in group order through LDS (the main loop ended on
    // a barrier; every group's last LDS reads are done)
    float* red = smem;  // [KG-1][4 spatial waves][RM*RN*16][64 lanes]
    constexpr int PER = RM * RN * 16 * 64;
    if (kg > 0) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) red[((kg - 1) * 4 + wsp) * PER + ((i * RN + j) * 16 + e) * 64 + lane] = acc[i][j][e];
    }
    __syncthreads();
    if (kg == 0) {
#pragma unroll
      for (int q = 0; q < KG - 1; ++q)
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] += red[(q * 4 + wsp) * PER + ((i * RN + j) * 16 + e) * 64 + lane];
    }
    __syncthreads();
  }
  const bool owner = kg == 0;  // only K-group 0 holds the full sums; the others' stores are dropped

  // ------------------------------------------------------------------ epilogue
  // C/D map (32x32 f32 MFMA): col = lane & 31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5).
  // Stores go through a buffer descriptor: rows/cols outside the GEMM get kOOB (dropped).
  const bool slab = nsplit > 1;
  if (slab || MODE == CS_CONV_DGRAD || (MODE == CS_CONV_WGRAD && !a.w_oihw)) {
    float* dst = slab ? a.ws + (size_t)split * a.M * a.N : a.out;
    const rsrc_t ro = make_rsrc(dst, (int64_t)a.M * a.N * 4);
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int n = n0 + wn * WN + j * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
          bstore1(ro, acc[i][j][e], (owner && m < a.M && n < a.N) ? (m * a.N + n) * 4 : kOOB);
        }
      }
    if constexpr (MODE == CS_CONV_DGRAD) {
      if (!slab && a.ered.part != nullptr) {  // (split-K: the combine launch takes them)
        dgrad_bn_stage<BM, BN>(acc, owner, smem);
        const CsBnRed& e = a.ered;
        const bool fin = a.fin.cnt != nullptr;
        if (e.pool)
          dgrad_bn_partials<BM, BN, 256 * KG, true>(e.y, e.scale, e.shift, e.mean, e.invstd, e.part, a.M, a.N, a.lgH,
                                                    a.lgW, mt, m0, n0, smem, fin);
        else
          dgrad_bn_partials<BM, BN, 256 * KG, false>(e.y, e.scale, e.shift, e.mean, e.invstd, e.part, a.M, a.N, a.lgH,
                                                     a.lgW, mt, m0, n0, smem, fin);
        // the last block of the column finalizes the block below's BN backward (coef, dgamma, ...)
        if (fin) cs_fin::arrive<true, BN>(a.fin, e.part, a.N, mt, nt, n0, smem);
      }
    }
    if (slab || MODE != CS_CONV_FWD) return;
  }
  if constexpr (MODE == CS_CONV_WGRAD) {  // conv0: scatter the padded (tap, ci) columns to OIHW
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int n = n0 + wn * WN + j * 32 + r;
        const int tap = n >> 2, ci = n & 3;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
          if (owner && m < a.M && n < a.N && ci < 3) a.out[(size_t)m * 27 + ci * 9 + tap] = acc[i][j][e];
        }
      }
    return;
  }
  if constexpr (MODE == CS_CONV_FWD) {
    // bias, store, and this tile's per-channel (mean, M2) for the BN statistics
    float* red = smem;  // [2][BN] after the main loop's final barrier
    const int cnt = (a.M - m0) < BM ? (a.M - m0) : BM;
    const rsrc_t ro = make_rsrc(a.out, (int64_t)a.M * a.N * 4);
    float colsum[RN];
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int n = n0 + wn * WN + j * 32 + r;
      const float bv = (a.bias != nullptr && n < a.N) ? a.bias[n] : 0.f;
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
          const float v = acc[i][j][e] + bv;
          acc[i][j][e] = v;
          s += m < a.M ? v : 0.f;
          bstore1(ro, v, (owner && m < a.M && n < a.N) ? (m * a.N + n) * 4 : kOOB);
        }
      colsum[j] = s + __shfl_xor(s, 32, 64);
    }
    if (a.stats == nullptr) return;
#pragma unroll
    for (int j = 0; j < RN; ++j)
      if (owner && hh == 0) red[wm * BN + wn * WN + j * 32 + r] = colsum[j];
    __syncthreads();
    float mean[RN];
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int c = wn * WN + j * 32 + r;
      mean[j] = (red[c] + red[BN + c]) / (float)cnt;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
          const float d = acc[i][j][e] - mean[j];
          s += m < a.M ? d * d : 0.f;
        }
      s += __shfl_xor(s, 32, 64);
      if (owner && hh == 0) red[wm * BN + wn * WN + j * 32 + r] = s;
    }
    __syncthreads();
    const bool fin = a.fin.cnt != nullptr;
    if (owner && wm == 0 && hh == 0) {
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int c = wn * WN + j * 32 + r, n = n0 + c;
        if (n < a.N) {
          if (fin) {  // write-through for the launch's last arriver (bn_fin.h)
            cs_fin::put_stats(a.stats, a.N, mt, n, mean[j], red[c] + red[BN + c]);
          } else {
            a.stats[((size_t)mt * a.N + n) * 2 + 0] = mean[j];
            a.stats[((size_t)mt * a.N + n) * 2 + 1] = red[c] + red[BN + c];
          }
        }
      }
    }
    // the last block of the column finalizes the BN forward: scale / shift / mean / invstd,
    // running stats (the separate bn_finalize launch is gone)
    if (fin) cs_fin::arrive<false, BN>(a.fin, a.stats, a.N, mt, nt, n0, smem);
  }
}

}  // namespace
