// 3x3 / stride 1 / pad 1 convolution as implicit GEMM on CDNA4 fp32 MFMA
// (v_mfma_f32_32x32x2_f32: exact f32, 64 FLOP/clk/SIMD), NHWC activations.
// Replaces ATen conv2d forward / backward-data / backward-weight of the reference
// (nn.Conv2d at master/part1/model.py:18-23; SURVEY.md §2.2 N1-N3, §2.4 shapes).
//
//   FWD  : Y [M=B*H*W][N=Cout]  = im2col(X)[M][K=9*Cin] . W^T      (+bias, +BN tile stats)
//   DGRAD: dX[M=B*H*W][N=Cin]   = shift(dZ)[M][K=9*Cout] . W        (flipped taps)
//   WGRAD: dW[M=Cout][N=9*Cin]  = dZ^T[Cout][K=B*H*W] . im2col(X)
//
// Tiling: 256 threads = 4 waves (2x2), block tile BMxBN, K-step BK (16 or 32),
// wave tile (BM/2)x(BN/2) built from 32x32 MFMA tiles. Global -> registers -> LDS
// double buffer with one barrier per K-step; the next K-step's global loads are
// issued before the current step's MFMAs so HBM/L2 latency hides under matrix work.
// K is permuted inside a K-step so each lane's BK/2 A (and B) values are contiguous
// in LDS: lane-half h feeds k = (BK/2)h + s at MFMA sub-step s, turning the operand
// fetch into BK/8 ds_read_b128 per tile ([row][BK+4] padded rows), or BK/2
// conflict-free ds_read_b32 for operands that are staged K-major ([k][rows+4]).
// Split-K over blockIdx.z writes fp32 slabs that `splitk_reduce` sums in a fixed
// order (deterministic, no float atomics). Tiles are dealt to XCDs in contiguous
// ranges (common.h xcd_remap) so neighbouring tiles share an L2.
#include <stdlib.h>

#include "common.h"
#include "launchers.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void pix_decode(int p, const CsConvArgs& a, int& b, int& h, int& w) {
  w = p & (a.W - 1);
  h = (p >> a.lgW) & (a.H - 1);
  b = p >> (a.lgW + a.lgH);
}

template <int MODE>
struct Traits;
template <>
struct Traits<CS_CONV_FWD> {
  static constexpr bool A_KC = true, B_KC = true;
};
template <>
struct Traits<CS_CONV_DGRAD> {
  static constexpr bool A_KC = true, B_KC = false;
};
template <>
struct Traits<CS_CONV_WGRAD> {
  static constexpr bool A_KC = false, B_KC = false;
};

template <int BM, int BN, int MODE, int BK>
struct Tile {
  static constexpr bool A_KC = Traits<MODE>::A_KC, B_KC = Traits<MODE>::B_KC;
  static constexpr int A_ELEMS = A_KC ? BM * (BK + 4) : BK * (BM + 4);
  static constexpr int B_ELEMS = B_KC ? BN * (BK + 4) : BK * (BN + 4);
  static constexpr int STAGE = A_ELEMS + B_ELEMS;
  static constexpr int AC = BM * BK / 1024;  // float4 chunks per thread per stage
  static constexpr int BC = BN * BK / 1024;
  static constexpr int KQ = BK / 4;          // float4 chunks per K-contiguous row
  static constexpr int HK = BK / 2;          // MFMA sub-steps per K-step
  static constexpr int WM = BM / 2, WN = BN / 2, RM = WM / 32, RN = WN / 32;
};

template <int BM, int BN, int MODE, int BK>
struct Loader {
  using T = Tile<BM, BN, MODE, BK>;
  // per-thread precomputed row info for K-contiguous A rows (FWD/DGRAD: pixel rows)
  int a_b[T::AC], a_h[T::AC], a_w[T::AC];
  bool a_ok[T::AC];
  float4 ra[2][T::AC], rb[2][T::BC];  // two register stages (tile k+1 and k+2 in flight)

  __device__ void init(const CsConvArgs& a, int m0) {
    if constexpr (T::A_KC) {
#pragma unroll
      for (int i = 0; i < T::AC; ++i) {
        const int q = threadIdx.x + 256 * i, row = q / T::KQ, m = m0 + row;
        a_ok[i] = m < a.M;
        pix_decode(a_ok[i] ? m : 0, a, a_b[i], a_h[i], a_w[i]);
      }
    }
  }

  // Branch-free loads: an out-of-range / padding element loads from the (valid) base
  // pointer and is zeroed at store time through its flag, so every load is issued
  // unconditionally and the compiler can count outstanding loads exactly (partial
  // vmcnt) instead of draining the queue around exec-masked branches.
  bool oka[2][T::AC], okb[2][T::BC];

  template <int S>
  __device__ void load(const CsConvArgs& a, int m0, int n0, int k0) {
    // ---------------- A operand
#pragma unroll
    for (int i = 0; i < T::AC; ++i) {
      const int q = threadIdx.x + 256 * i;
      size_t off = 0;
      bool ok;
      const float* src;
      if constexpr (MODE == CS_CONV_FWD || MODE == CS_CONV_DGRAD) {
        const int c = q % T::KQ, kk = k0 + 4 * c;
        const int lgC = (MODE == CS_CONV_FWD) ? a.lgCin : a.lgCout;
        const int tap = kk >> lgC, ch = kk & ((1 << lgC) - 1);
        const int t3 = tap / 3, dh = t3 - 1, dw = tap - 3 * t3 - 1;
        const int hh = (MODE == CS_CONV_FWD) ? a_h[i] + dh : a_h[i] - dh;
        const int ww = (MODE == CS_CONV_FWD) ? a_w[i] + dw : a_w[i] - dw;
        ok = a_ok[i] && tap < 9 && (unsigned)hh < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
        src = (MODE == CS_CONV_FWD) ? a.x : a.dz;
        if (ok) off = ((((size_t)a_b[i] * a.H + hh) * a.W + ww) << lgC) + ch;
      } else {  // WGRAD: A[k = pixel][m' = cout]  (K-major staging)
        constexpr int CPR = BM / 4;
        const int kr = q / CPR, c = q - kr * CPR, p = k0 + kr;
        ok = p < a.K && m0 + 4 * c < a.M;
        src = a.dz;
        if (ok) off = ((size_t)p << a.lgCout) + m0 + 4 * c;
      }
      ra[S][i] = *reinterpret_cast<const float4*>(src + off);
      oka[S][i] = ok;
    }
    // ---------------- B operand
#pragma unroll
    for (int i = 0; i < T::BC; ++i) {
      const int q = threadIdx.x + 256 * i;
      size_t off = 0;
      bool ok;
      if constexpr (MODE == CS_CONV_FWD) {
        const int row = q / T::KQ, c = q % T::KQ, n = n0 + row, kk = k0 + 4 * c;
        ok = n < a.N && kk < a.K;
        if (!a.w_oihw) {
          if (ok) off = (size_t)n * a.K + kk;
          rb[S][i] = *reinterpret_cast<const float4*>(a.w + off);
        } else {  // conv0: OIHW [Cout][3][3x3], K = 9 taps x 4 (padded) channels
          if (ok) off = (size_t)n * 27 + (kk >> 2);
          const float* wr = a.w + off;
          rb[S][i] = make_float4(wr[0], wr[9], wr[18], 0.f);
        }
      } else if constexpr (MODE == CS_CONV_DGRAD) {  // B[k = (tap, cout)][n = cin]
        constexpr int CPR = BN / 4;
        const int kr = q / CPR, c = q - kr * CPR, kk = k0 + kr;
        const int tap = kk >> a.lgCout, co = kk & (a.Cout - 1);
        ok = kk < a.K && n0 + 4 * c < a.N;
        if (ok) off = ((size_t)co * 9 + tap) * a.Cin + n0 + 4 * c;
        rb[S][i] = *reinterpret_cast<const float4*>(a.w + off);
      } else {  // WGRAD: B[k = pixel][n' = (tap, cin)]
        constexpr int CPR = BN / 4;
        const int kr = q / CPR, c = q - kr * CPR, p = k0 + kr, nn = n0 + 4 * c;
        const int tap = nn >> a.lgCin, ci = nn & (a.Cin - 1);
        int b, h, w;
        pix_decode(p, a, b, h, w);
        const int t3 = tap / 3, hh = h + t3 - 1, ww = w + (tap - 3 * t3) - 1;
        ok = p < a.K && nn < a.N && tap < 9 && (unsigned)hh < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
        if (ok) off = ((((size_t)b * a.H + hh) * a.W + ww) << a.lgCin) + ci;
        rb[S][i] = *reinterpret_cast<const float4*>(a.x + off);
      }
      okb[S][i] = ok;
    }
  }

  __device__ static float4 keep(float4 v, bool ok) {
    return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  }

  template <int S>
  __device__ void store(float* As, float* Bs) const {
#pragma unroll
    for (int i = 0; i < T::AC; ++i) {
      const int q = threadIdx.x + 256 * i;
      if constexpr (T::A_KC) {
        *reinterpret_cast<float4*>(As + (q / T::KQ) * (BK + 4) + 4 * (q % T::KQ)) = keep(ra[S][i], oka[S][i]);
      } else {
        constexpr int CPR = BM / 4;
        const int kr = q / CPR, c = q - kr * CPR;
        *reinterpret_cast<float4*>(As + kr * (BM + 4) + 4 * c) = keep(ra[S][i], oka[S][i]);
      }
    }
#pragma unroll
    for (int i = 0; i < T::BC; ++i) {
      const int q = threadIdx.x + 256 * i;
      if constexpr (T::B_KC) {
        *reinterpret_cast<float4*>(Bs + (q / T::KQ) * (BK + 4) + 4 * (q % T::KQ)) = keep(rb[S][i], okb[S][i]);
      } else {
        constexpr int CPR = BN / 4;
        const int kr = q / CPR, c = q - kr * CPR;
        *reinterpret_cast<float4*>(Bs + kr * (BN + 4) + 4 * c) = keep(rb[S][i], okb[S][i]);
      }
    }
  }
};

// One K-step on a staged LDS tile: every fragment read is issued first (one
// lgkmcnt wait), then the BK/2 x RM x RN MFMA chain runs back to back.
template <int BM, int BN, int MODE, int BK, int SCHED>
__device__ __forceinline__ void mma_stage(const float* __restrict__ As, const float* __restrict__ Bs,
                                          f32x16 (&acc)[Tile<BM, BN, MODE, BK>::RM][Tile<BM, BN, MODE, BK>::RN],
                                          int wm, int wn, int r, int hh) {
  using T = Tile<BM, BN, MODE, BK>;
  float af[T::RM][T::HK], bf[T::RN][T::HK];
#pragma unroll
  for (int i = 0; i < T::RM; ++i) {
    const int row = wm * T::WM + i * 32 + r;
    if constexpr (T::A_KC) {
#pragma unroll
      for (int c4 = 0; c4 < T::HK / 4; ++c4) {
        const float4 v = *reinterpret_cast<const float4*>(As + row * (BK + 4) + T::HK * hh + 4 * c4);
        af[i][4 * c4 + 0] = v.x; af[i][4 * c4 + 1] = v.y; af[i][4 * c4 + 2] = v.z; af[i][4 * c4 + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int s = 0; s < T::HK; ++s) af[i][s] = As[(T::HK * hh + s) * (BM + 4) + row];
    }
  }
#pragma unroll
  for (int j = 0; j < T::RN; ++j) {
    const int col = wn * T::WN + j * 32 + r;
    if constexpr (T::B_KC) {
#pragma unroll
      for (int c4 = 0; c4 < T::HK / 4; ++c4) {
        const float4 v = *reinterpret_cast<const float4*>(Bs + col * (BK + 4) + T::HK * hh + 4 * c4);
        bf[j][4 * c4 + 0] = v.x; bf[j][4 * c4 + 1] = v.y; bf[j][4 * c4 + 2] = v.z; bf[j][4 * c4 + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int s = 0; s < T::HK; ++s) bf[j][s] = Bs[(T::HK * hh + s) * (BN + 4) + col];
    }
  }
  if constexpr (SCHED != 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < T::HK; ++s)
#pragma unroll
    for (int i = 0; i < T::RM; ++i)
#pragma unroll
      for (int j = 0; j < T::RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
}

// SCHED: instruction-schedule variant of the main loop (A/B-tested on MI355X):
//   0 = next tile's loads, then fragment reads, sched barrier, MFMA chain
//   1 = same without the sched barrier (compiler interleaves freely)
//   2 = fragment reads, MFMA chain, then the next tile's loads (their address VALU
//       overlaps the tail of the matrix pipe)
template <int BM, int BN, int MODE, int BK, int SCHED>
__global__ __launch_bounds__(256) void conv_gemm_kernel(CsConvArgs a) {
  using T = Tile<BM, BN, MODE, BK>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int ntn = (a.N + BN - 1) / BN;
  const int ntiles = ((a.M + BM - 1) / BM) * ntn;
  const int tile = cs::xcd_remap(blockIdx.x, ntiles);
  const int mt = tile / ntn, nt = tile - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int split = blockIdx.z;
  const int ks_begin = split * a.ksteps_per_split;
  int ks_end = ks_begin + a.ksteps_per_split;
  if (ks_end > a.total_ksteps) ks_end = a.total_ksteps;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1, r = lane & 31, hh = lane >> 5;

  f32x16 acc[T::RM][T::RN];
#pragma unroll
  for (int i = 0; i < T::RM; ++i)
#pragma unroll
    for (int j = 0; j < T::RN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  Loader<BM, BN, MODE, BK> ld;
  ld.init(a, m0);
  float* lds0 = smem;
  float* lds1 = smem + T::STAGE;
  // Pipeline: LDS double buffer + two register stages, so a tile's global loads are
  // issued two K-steps before its LDS store (they survive the plain s_barrier; the
  // store waits with a partial vmcnt that leaves the newer stage in flight).
  // Unrolled by two so every register-stage index is a compile-time constant.
  const int nks = ks_end - ks_begin;
  if (nks > 0) {
    ld.template load<0>(a, m0, n0, ks_begin * BK);
    ld.template store<0>(lds0, lds0 + T::A_ELEMS);
    if (nks > 1) ld.template load<1>(a, m0, n0, (ks_begin + 1) * BK);
  }
  __syncthreads();
  for (int t = 0; t < nks; t += 2) {
    // even step: tile t in lds0, tile t+1 in registers[1]
    if (SCHED != 2 && t + 2 < nks) ld.template load<0>(a, m0, n0, (ks_begin + t + 2) * BK);
    mma_stage<BM, BN, MODE, BK, SCHED>(lds0, lds0 + T::A_ELEMS, acc, wm, wn, r, hh);
    if (SCHED == 2 && t + 2 < nks) ld.template load<0>(a, m0, n0, (ks_begin + t + 2) * BK);
    if (t + 1 < nks) ld.template store<1>(lds1, lds1 + T::A_ELEMS);
    __syncthreads();
    if (t + 1 >= nks) break;
    // odd step: tile t+1 in lds1, tile t+2 in registers[0]
    if (SCHED != 2 && t + 3 < nks) ld.template load<1>(a, m0, n0, (ks_begin + t + 3) * BK);
    mma_stage<BM, BN, MODE, BK, SCHED>(lds1, lds1 + T::A_ELEMS, acc, wm, wn, r, hh);
    if (SCHED == 2 && t + 3 < nks) ld.template load<1>(a, m0, n0, (ks_begin + t + 3) * BK);
    if (t + 2 < nks) ld.template store<0>(lds0, lds0 + T::A_ELEMS);
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  // C/D map (32x32 f32 MFMA): col = lane & 31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
  const bool slab = gridDim.z > 1;
  if (slab) {
    float* dst = a.ws + (size_t)split * a.M * a.N;
#pragma unroll
    for (int i = 0; i < T::RM; ++i)
#pragma unroll
      for (int j = 0; j < T::RN; ++j) {
        const int n = n0 + wn * T::WN + j * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * T::WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
          if (m < a.M && n < a.N) dst[(size_t)m * a.N + n] = acc[i][j][e];
        }
      }
    return;
  }
  if constexpr (MODE == CS_CONV_WGRAD) {
#pragma unroll
    for (int i = 0; i < T::RM; ++i)
#pragma unroll
      for (int j = 0; j < T::RN; ++j) {
        const int n = n0 + wn * T::WN + j * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * T::WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
          if (m < a.M && n < a.N) {
            if (!a.w_oihw) {
              a.out[(size_t)m * a.N + n] = acc[i][j][e];
            } else {
              const int tap = n >> 2, ci = n & 3;
              if (ci < 3) a.out[(size_t)m * 27 + ci * 9 + tap] = acc[i][j][e];
            }
          }
        }
      }
    return;
  }
  if constexpr (MODE == CS_CONV_DGRAD) {
#pragma unroll
    for (int i = 0; i < T::RM; ++i)
#pragma unroll
      for (int j = 0; j < T::RN; ++j) {
        const int n = n0 + wn * T::WN + j * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * T::WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
          if (m < a.M && n < a.N) a.out[(size_t)m * a.N + n] = acc[i][j][e];
        }
      }
    return;
  }
  if constexpr (MODE == CS_CONV_FWD) {
    // bias, store, and this tile's per-channel (mean, M2) for the BN statistics
    float* red = smem;  // [2][BN] after the main loop's final barrier
    const int cnt = (a.M - m0) < BM ? (a.M - m0) : BM;
    float colsum[T::RN];
#pragma unroll
    for (int j = 0; j < T::RN; ++j) {
      const int n = n0 + wn * T::WN + j * 32 + r;
      const float bv = (a.bias != nullptr && n < a.N) ? a.bias[n] : 0.f;
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < T::RM; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * T::WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
          const float v = acc[i][j][e] + bv;
          acc[i][j][e] = v;
          if (m < a.M) {
            s += v;
            if (n < a.N) a.out[(size_t)m * a.N + n] = v;
          }
        }
      colsum[j] = s + __shfl_xor(s, 32, 64);
    }
    if (a.stats == nullptr) return;
#pragma unroll
    for (int j = 0; j < T::RN; ++j)
      if (hh == 0) red[wm * BN + wn * T::WN + j * 32 + r] = colsum[j];
    __syncthreads();
    float mean[T::RN];
#pragma unroll
    for (int j = 0; j < T::RN; ++j) {
      const int c = wn * T::WN + j * 32 + r;
      mean[j] = (red[c] + red[BN + c]) / (float)cnt;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < T::RN; ++j) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < T::RM; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * T::WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
          const float d = acc[i][j][e] - mean[j];
          if (m < a.M) s += d * d;
        }
      s += __shfl_xor(s, 32, 64);
      if (hh == 0) red[wm * BN + wn * T::WN + j * 32 + r] = s;
    }
    __syncthreads();
    if (wm == 0 && hh == 0) {
#pragma unroll
      for (int j = 0; j < T::RN; ++j) {
        const int c = wn * T::WN + j * 32 + r, n = n0 + c;
        if (n < a.N) {
          a.stats[((size_t)mt * a.N + n) * 2 + 0] = mean[j];
          a.stats[((size_t)mt * a.N + n) * 2 + 1] = red[c] + red[BN + c];
        }
      }
    }
  }
}

// Deterministic split-K combine: out = sum_z ws[z] (+bias, +BN tile stats for FWD;
// OIHW scatter for the conv0 weight gradient). Tile = 16 rows x 64 columns (one row
// and one float4 per thread) so even an M = 256 GEMM gets enough blocks to stream
// the slabs at HBM rate. Large split counts are first folded in groups of
// kFold slabs (pre-pass, in place into the group's first slab), so no thread
// walks more than ~kFold dependent loads. Summation order is fixed.
constexpr int kRedRows = 16;
constexpr int kFold = 16;

__global__ __launch_bounds__(256) void splitk_fold_kernel(float* __restrict__ ws, size_t slab, int splits) {
  // grid.y = group g: ws[g*kFold] = sum_{z in group} ws[z]
  const size_t n4 = slab >> 2;
  const int z0 = blockIdx.y * kFold;
  const int z1 = min(splits, z0 + kFold);
  float4* w4 = reinterpret_cast<float4*>(ws);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    float4 acc = w4[(size_t)z0 * n4 + i];
    for (int z = z0 + 1; z < z1; ++z) {
      const float4 t = w4[(size_t)z * n4 + i];
      acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
    }
    w4[(size_t)z0 * n4 + i] = acc;
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(CsConvArgs a, int mode, int nslab, int zstep) {
  __shared__ float red[kRedRows][64];
  __shared__ float meanv[64];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int ntn = (a.N + 63) / 64;
  const int mt = blockIdx.x / ntn, nt = blockIdx.x - mt * ntn;
  const int m0 = mt * kRedRows, n0 = nt * 64, n = n0 + 4 * tx, m = m0 + ty;
  const size_t slab = (size_t)a.M * a.N;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool in = m < a.M && n < a.N;
  if (in) {
    const float* p = a.ws + (size_t)m * a.N + n;
    for (int z = 0; z < nslab; ++z) {
      const float4 t = *reinterpret_cast<const float4*>(p + (size_t)z * zstep * slab);
      acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
    }
    if (mode == CS_CONV_FWD && a.bias != nullptr) {
      const float4 bv = *reinterpret_cast<const float4*>(a.bias + n);
      acc.x += bv.x; acc.y += bv.y; acc.z += bv.z; acc.w += bv.w;
    }
    if (mode == CS_CONV_WGRAD && a.w_oihw) {
      const float vals[4] = {acc.x, acc.y, acc.z, acc.w};
      for (int q = 0; q < 4; ++q) {
        const int nn = n + q, tap = nn >> 2, ci = nn & 3;
        if (ci < 3) a.out[(size_t)m * 27 + ci * 9 + tap] = vals[q];
      }
    } else {
      *reinterpret_cast<float4*>(a.out + (size_t)m * a.N + n) = acc;
    }
  }
  if (mode != CS_CONV_FWD || a.stats == nullptr) return;
  // per-column (mean, M2) of this 16-row tile (two-pass inside the tile: robust)
  const int cnt = (a.M - m0) < kRedRows ? (a.M - m0) : kRedRows;
  red[ty][4 * tx + 0] = in ? acc.x : 0.f;
  red[ty][4 * tx + 1] = in ? acc.y : 0.f;
  red[ty][4 * tx + 2] = in ? acc.z : 0.f;
  red[ty][4 * tx + 3] = in ? acc.w : 0.f;
  __syncthreads();
  if (threadIdx.x < 64) {
    float sum = 0.f;
    for (int k = 0; k < kRedRows; ++k) sum += red[k][threadIdx.x];
    meanv[threadIdx.x] = sum / (float)cnt;
  }
  __syncthreads();
  const float dx = in ? acc.x - meanv[4 * tx] : 0.f, dy = in ? acc.y - meanv[4 * tx + 1] : 0.f;
  const float dz = in ? acc.z - meanv[4 * tx + 2] : 0.f, dw = in ? acc.w - meanv[4 * tx + 3] : 0.f;
  __syncthreads();
  red[ty][4 * tx + 0] = dx * dx;
  red[ty][4 * tx + 1] = dy * dy;
  red[ty][4 * tx + 2] = dz * dz;
  red[ty][4 * tx + 3] = dw * dw;
  __syncthreads();
  if (threadIdx.x < 64 && n0 + (int)threadIdx.x < a.N) {
    float sq = 0.f;
    for (int k = 0; k < kRedRows; ++k) sq += red[k][threadIdx.x];
    a.stats[((size_t)mt * a.N + n0 + threadIdx.x) * 2 + 0] = meanv[threadIdx.x];
    a.stats[((size_t)mt * a.N + n0 + threadIdx.x) * 2 + 1] = sq;
  }
}

hipError_t launch_reduce(const CsConvArgs& a, int mode, int splits, hipStream_t stream) {
  int nslab = splits, zstep = 1;
  if (splits > 2 * kFold) {
    const size_t slab = (size_t)a.M * a.N;
    const int groups = (splits + kFold - 1) / kFold;
    int bx = (int)((slab / 4 + 255) / 256);
    if (bx > 1024) bx = 1024;
    hipLaunchKernelGGL(splitk_fold_kernel, dim3(bx, groups), dim3(256), 0, stream, a.ws, slab, splits);
    nslab = groups;
    zstep = kFold;
  }
  const int nt = ((a.M + kRedRows - 1) / kRedRows) * ((a.N + 63) / 64);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(nt), dim3(256), 0, stream, a, mode, nslab, zstep);
  return hipGetLastError();
}

int conv_sched() {
  static int v = [] {
    const char* e = getenv("CS_CONV_SCHED");
    return e ? atoi(e) : 1;  // default: measured 3-5% faster than 0 and 2 on MI355X
  }();
  return v;
}

template <int BM, int BN, int MODE, int BK>
hipError_t launch_gemm(const CsConvArgs& a, int splits, hipStream_t stream) {
  using T = Tile<BM, BN, MODE, BK>;
  const int ntiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const size_t lds = 2 * T::STAGE * sizeof(float);
  const dim3 grid(ntiles, 1, splits);
  switch (conv_sched()) {
    case 1: hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, MODE, BK, 1>), grid, dim3(256), lds, stream, a); break;
    case 2: hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, MODE, BK, 2>), grid, dim3(256), lds, stream, a); break;
    case 0: hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, MODE, BK, 0>), grid, dim3(256), lds, stream, a); break;
    default: hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, MODE, BK, 1>), grid, dim3(256), lds, stream, a); break;
  }
  return hipGetLastError();
}

int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

}  // namespace

int cs_conv_lg(int v) { return ilog2(v); }

void cs_conv_fill_dims(CsConvArgs* a, int mode) {
  a->lgH = ilog2(a->H);
  a->lgW = ilog2(a->W);
  a->lgCin = ilog2(a->Cin);
  a->lgCout = ilog2(a->Cout);
  const int pix = a->B * a->H * a->W;
  if (mode == CS_CONV_FWD) {
    a->M = pix;
    a->N = a->Cout;
    a->K = 9 * a->Cin;
  } else if (mode == CS_CONV_DGRAD) {
    a->M = pix;
    a->N = a->Cin;
    a->K = 9 * a->Cout;
  } else {
    a->M = a->Cout;
    a->N = 9 * a->Cin;
    a->K = pix;
  }
}

int cs_conv_effective_splits(int K, int bk, int splits) {
  const int ks = (K + bk - 1) / bk;
  int s = splits < 1 ? 1 : (splits > ks ? ks : splits);
  const int per = (ks + s - 1) / s;
  return (ks + per - 1) / per;
}

hipError_t cs_conv_gemm(CsConvArgs a, int mode, int bm, int bn, int bk, int splits, hipStream_t stream) {
  if (bk != 16 && bk != 32) return hipErrorInvalidValue;
  cs_conv_fill_dims(&a, mode);
  a.total_ksteps = (a.K + bk - 1) / bk;
  splits = cs_conv_effective_splits(a.K, bk, splits);
  a.ksteps_per_split = (a.total_ksteps + splits - 1) / splits;
  if (splits > 1 && a.ws == nullptr) return hipErrorInvalidValue;
#define CS_DISPATCH(BM_, BN_, BK_)                                                                       \
  if (bm == BM_ && bn == BN_ && bk == BK_) {                                                             \
    hipError_t e;                                                                                        \
    if (mode == CS_CONV_FWD) e = launch_gemm<BM_, BN_, CS_CONV_FWD, BK_>(a, splits, stream);            \
    else if (mode == CS_CONV_DGRAD) e = launch_gemm<BM_, BN_, CS_CONV_DGRAD, BK_>(a, splits, stream);   \
    else e = launch_gemm<BM_, BN_, CS_CONV_WGRAD, BK_>(a, splits, stream);                              \
    if (e != hipSuccess || splits == 1) return e;                                                        \
    return launch_reduce(a, mode, splits, stream);                                                       \
  }
  CS_DISPATCH(64, 64, 16)
  CS_DISPATCH(128, 64, 16)
  CS_DISPATCH(64, 128, 16)
  CS_DISPATCH(128, 128, 16)
  CS_DISPATCH(64, 64, 32)
  CS_DISPATCH(128, 64, 32)
  CS_DISPATCH(64, 128, 32)
  CS_DISPATCH(128, 128, 32)
#undef CS_DISPATCH
  return hipErrorInvalidValue;
}
