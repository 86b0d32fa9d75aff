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
// double buffer with one barrier per K-step and two register stages (a tile's
// global loads are issued two K-steps before its LDS store).
//
// Addressing is built for the CDNA4 buffer unit, not for flat pointers:
//  * every operand is read through a buffer resource (32-bit byte offsets, one
//    SGPR descriptor per tensor); a padding / out-of-range element gets an offset
//    past the descriptor's size, and the range check returns 0 — no selects, no
//    branches, no 64-bit address math in the K loop;
//  * the per-K-step part of every offset is wave-uniform (the 3x3 tap and the
//    channel base of a K-step: BK divides the channel count), so it lives in an
//    SGPR (added to the fixed per-thread part with one VALU add, so the range check
//    sees the whole offset); per-thread parts (pixel row, channel lane) are fixed for the whole
//    loop, and the padding test is one bit of a 9-bit per-row tap mask built once.
// K is permuted inside a K-step so each lane's BK/2 A (and B) values are contiguous
// in LDS: lane-half h feeds k = (BK/2)h + s at MFMA sub-step s, so K-contiguous
// operands ([row][BK+4] padded rows) are fetched with ds_read_b128 and K-major
// operands ([k][rows+4]) with conflict-free ds_read_b32. The MFMA chain is
// software-pipelined one 4-deep chunk ahead of its fragment reads.
// Split-K over blockIdx.z writes fp32 slabs that `splitk_reduce` sums in a fixed
// order (deterministic, no float atomics). Tiles are dealt to XCDs in contiguous
// ranges (common.h xcd_remap) so neighbouring tiles share an L2.
#include <stdlib.h>

#include <algorithm>

#include "conv_common.h"
#include "sgd_device.h"
#include "xent_device.h"

namespace {


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

// GL = LDS-DMA staging (buffer_load ... lds): images are lane-linear, so unpadded; a
// K-contiguous row (BK = 32 -> 8 float4 chunks) stores logical chunk c at physical chunk
// c ^ ((row >> 1) & 7), which makes the ds_read_b128 fragment reads conflict-free.
// KG = K-groups: the block has 4*KG waves; wave group g multiplies sub-step chunks
// [g*NG/KG, (g+1)*NG/KG) of every K-step on the shared LDS tile, and the KG partial
// accumulators are summed through LDS (fixed order) before the epilogue — more waves per
// SIMD for latency hiding without more split-K slabs.
template <int BM, int BN, int MODE, int BK, bool GL = false, int KG = 1>
struct Tile {
  static constexpr int NT = 256 * KG;  // threads per block
  static constexpr bool A_KC = Traits<MODE>::A_KC, B_KC = Traits<MODE>::B_KC;
  static constexpr int A_ELEMS = GL ? BM * BK : (A_KC ? BM * (BK + 4) : BK * (BM + 4));
  static constexpr int B_ELEMS = GL ? BN * BK : (B_KC ? BN * (BK + 4) : BK * (BN + 4));
  static constexpr int STAGE = A_ELEMS + B_ELEMS;
  static constexpr int AC = BM * BK / (4 * NT);  // float4 chunks per thread per stage
  static constexpr int BC = BN * BK / (4 * NT);
  static_assert(AC >= 1 && BC >= 1, "tile too small for this many threads");
  static constexpr int KQ = BK / 4;          // float4 chunks per K-contiguous row
  static constexpr int HK = BK / 2;          // MFMA sub-steps per K-step
  static constexpr int NG = HK / 4;          // 4-deep sub-step chunks per K-step
  static constexpr int WM = BM / 2, WN = BN / 2, RM = WM / 32, RN = WN / 32;
};

// C4: FWD of the padded conv0 (Cin = 4 < BK, OIHW weights) — a compile-time variant so
// the common kernels carry no branch for it.
//
// GL: the same per-chunk offsets feed LDS-DMA instead of registers. Chunk i of a thread is
// then slot s = (wave * AC + i) * 64 + lane of the operand's lane-linear LDS image (one
// 1 KiB wave-instruction per chunk index), instead of q = tid + 256 * i.
template <int BM, int BN, int MODE, int BK, bool C4 = false, bool GL = false, int KG = 1>
struct Loader {
  using T = Tile<BM, BN, MODE, BK, GL, KG>;
  rsrc_t ra_, rb_;
  int av[T::AC], bv[T::BC];        // per-thread fixed byte offsets
  unsigned am[T::AC], bm_[T::BC];  // per-thread tap masks / flags
  int lds_a[T::AC], lds_b[T::BC];  // LDS float offsets of this thread's chunks (register staging)
  int kb[T::BC];                   // WGRAD B: the chunk's pixel row within the K-step
  float4 ra[GL ? 1 : 2][T::AC], rb[GL ? 1 : 2][T::BC];

  // chunk -> (row or k-row, logical float4 chunk) of the operand image
  template <int CHUNKS>
  __device__ static void slot_kc(int i, int& row, int& c) {
    if constexpr (GL) {
      const int s = (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * CHUNKS + i) * 64 + (threadIdx.x & 63);
      row = s / T::KQ;
      c = (s % T::KQ) ^ ((row >> 1) & 7);
    } else {
      const int q = threadIdx.x + T::NT * i;
      row = q / T::KQ;
      c = q % T::KQ;
    }
  }
  template <int ROWS, int CHUNKS>
  __device__ static void slot_km(int i, int& kr, int& c) {
    constexpr int CPR = ROWS / 4;
    const int s = GL ? (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * CHUNKS + i) * 64 + (threadIdx.x & 63)
                     : threadIdx.x + T::NT * i;
    kr = s / CPR;
    c = s - kr * CPR;
  }

  __device__ void init(const CsConvArgs& a, int m0, int n0) {
    const int pix = a.B * a.H * a.W;
    const int64_t xbytes = (int64_t)pix * a.Cin * 4, zbytes = (int64_t)pix * a.Cout * 4;
    const int64_t wbytes = (a.w_oihw ? (int64_t)a.Cout * 27 : (int64_t)a.Cout * 9 * a.Cin) * 4;
#pragma unroll
    for (int i = 0; i < T::AC; ++i) {
      if constexpr (T::A_KC) {  // FWD / DGRAD: A[m = pixel][k = (tap, ch)], one pixel row per chunk
        int row, c;
        slot_kc<T::AC>(i, row, c);
        const int m = m0 + row;
        const int w = m & (a.W - 1), h = (m >> a.lgW) & (a.H - 1);
        const int lgC = (MODE == CS_CONV_FWD) ? a.lgCin : a.lgCout;
        am[i] = m < a.M ? tap_mask(h, w, a.H, a.W, MODE == CS_CONV_FWD ? 1 : -1) : 0u;
        av[i] = ((m << lgC) + 4 * c) * 4;
        lds_a[i] = row * (BK + 4) + 4 * c;
      } else {  // WGRAD: A[m = cout][k = pixel] from dZ [pixel][cout], K-major staging
        int kr, c;
        slot_km<BM, T::AC>(i, kr, c);
        am[i] = (m0 + 4 * c < a.M) ? 1u : 0u;
        av[i] = ((kr << a.lgCout) + m0 + 4 * c) * 4;
        lds_a[i] = kr * (BM + 4) + 4 * c;
      }
    }
#pragma unroll
    for (int i = 0; i < T::BC; ++i) {
      if constexpr (MODE == CS_CONV_FWD) {  // B[n = cout][k]: weights [Cout][K] (K-contiguous)
        int row, c;
        slot_kc<T::BC>(i, row, c);
        const int n = n0 + row;
        bm_[i] = n < a.N ? 1u : 0u;
        bv[i] = C4 ? (n * 27 + c) : (n * a.K + 4 * c) * 4;  // conv0: element index (gather path)
        lds_b[i] = row * (BK + 4) + 4 * c;
      } else if constexpr (MODE == CS_CONV_DGRAD) {  // B[k = (tap, cout)][n = cin]: OHWI weights, K-major
        int kr, c;
        slot_km<BN, T::BC>(i, kr, c);
        bm_[i] = (n0 + 4 * c < a.N) ? 1u : 0u;
        bv[i] = (kr * 9 * a.Cin + n0 + 4 * c) * 4;
        lds_b[i] = kr * (BN + 4) + 4 * c;
      } else {  // WGRAD: B[k = pixel][n = (tap, cin)] = X[pixel + tap shift][cin], K-major
        int kr, c;
        slot_km<BN, T::BC>(i, kr, c);
        const int nn = n0 + 4 * c;
        kb[i] = kr;
        const int tap = nn >> a.lgCin, ci = nn & (a.Cin - 1);
        const int t3 = tap / 3, dh = t3 - 1, dw = tap - 3 * t3 - 1;
        // flag bits: [0] column valid, [4..] signed tap delta (dh, dw) packed as (dh+1)*3+(dw+1)
        bm_[i] = (nn < a.N && tap < 9) ? (1u | ((unsigned)tap << 4)) : 0u;
        bv[i] = (((dh * a.W + dw) << a.lgCin) + ci) * 4;  // + (pixel << lgCin)*4 per K-step
        lds_b[i] = kr * (BN + 4) + 4 * c;
      }
    }
    if constexpr (MODE == CS_CONV_FWD) {
      ra_ = make_rsrc(a.x, xbytes);
      rb_ = make_rsrc(a.w, wbytes);
    } else if constexpr (MODE == CS_CONV_DGRAD) {
      ra_ = make_rsrc(a.dz, zbytes);
      rb_ = make_rsrc(a.w, wbytes);
    } else {
      ra_ = make_rsrc(a.dz, (int64_t)a.K * a.Cout * 4);  // pixels >= K fall off the end: zero
      rb_ = make_rsrc(a.x, xbytes);
    }
  }

  // byte offset (or kOOB) of A chunk i / B chunk i for the K-step starting at k0 (non-C4)
  __device__ __forceinline__ int a_off(const CsConvArgs& a, int k0, int i) const {
    if constexpr (T::A_KC) {
      const int lgC = (MODE == CS_CONV_FWD) ? a.lgCin : a.lgCout;
      const int tap = k0 >> lgC, ch0 = k0 & ((1 << lgC) - 1);
      const int t3 = tap / 3, dh = t3 - 1, dw = tap - 3 * t3 - 1;
      const int sh = (MODE == CS_CONV_FWD) ? (dh * a.W + dw) : -(dh * a.W + dw);
      return ((am[i] >> tap) & 1u) ? av[i] + ((sh << lgC) + ch0) * 4 : kOOB;
    } else {
      return am[i] ? av[i] + ((k0 << a.lgCout) * 4) : kOOB;
    }
  }
  __device__ __forceinline__ int b_off(const CsConvArgs& a, int k0, int i) const {
    if constexpr (MODE == CS_CONV_FWD) {
      return bm_[i] ? bv[i] + k0 * 4 : kOOB;
    } else if constexpr (MODE == CS_CONV_DGRAD) {
      const int tap = k0 >> a.lgCout, co0 = k0 & (a.Cout - 1);
      return bm_[i] ? bv[i] + (((co0 * 9 + tap) << a.lgCin) * 4) : kOOB;
    } else {
      const int p = k0 + kb[i];
      const int w = p & (a.W - 1), h = (p >> a.lgW) & (a.H - 1);
      const int tap = (int)(bm_[i] >> 4), t3 = tap / 3;
      const int hh = h + t3 - 1, ww = w + (tap - 3 * t3) - 1;
      const bool ok = (bm_[i] & 1u) && p < a.K && (unsigned)hh < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      return ok ? bv[i] + ((p << a.lgCin) * 4) : kOOB;
    }
  }

  // LDS-DMA staging of the K-step at k0 into an operand image pair (GL only): one
  // buffer_load_dwordx4 ... lds per chunk; out-of-range offsets land as zeros.
  __device__ __forceinline__ void gload(const CsConvArgs& a, int k0, float* As, float* Bs) const {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int i = 0; i < T::AC; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra_, (__attribute__((address_space(3))) void*)(As + (wv * T::AC + i) * 256),
                                               16, a_off(a, k0, i), 0, 0, 0);
#pragma unroll
    for (int i = 0; i < T::BC; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb_, (__attribute__((address_space(3))) void*)(Bs + (wv * T::BC + i) * 256),
                                               16, b_off(a, k0, i), 0, 0, 0);
  }

  template <int S>
  __device__ __forceinline__ void load(const CsConvArgs& a, int k0) {
    // ---------------- A operand
    if constexpr (!C4) {
#pragma unroll
      for (int i = 0; i < T::AC; ++i) ra[S][i] = bload4(ra_, a_off(a, k0, i));
    } else {  // conv0 (C = 4 < BK): each float4 is its own tap
      const int lgC = a.lgCin;
#pragma unroll
      for (int i = 0; i < T::AC; ++i) {
        const int c = (threadIdx.x + T::NT * i) % T::KQ;
        const int tap = (k0 >> lgC) + c;
        const int t3 = tap / 3, dh = t3 - 1, dw = tap - 3 * t3 - 1;
        const int sh = dh * a.W + dw;
        const int off = (tap < 9 && ((am[i] >> tap) & 1u)) ? av[i] - 16 * c + (sh << lgC) * 4 : kOOB;
        ra[S][i] = bload4(ra_, off);
      }
    }
    // ---------------- B operand
#pragma unroll
    for (int i = 0; i < T::BC; ++i) {
      if constexpr (MODE == CS_CONV_FWD && C4) {  // conv0: OIHW [Cout][3][3x3], K = 9 taps x 4 (padded) channels
        const int tap = (k0 >> 2) + (threadIdx.x + T::NT * i) % T::KQ;
        const bool ok = bm_[i] && tap < 9;
        const int e = bv[i] - ((threadIdx.x + T::NT * i) % T::KQ) + tap;  // n*27 + tap
        const float* wr = a.w + (ok ? e : 0);
        rb[S][i] = ok ? make_float4(wr[0], wr[9], wr[18], 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        rb[S][i] = bload4(rb_, b_off(a, k0, i));
      }
    }
  }

  template <int S>
  __device__ __forceinline__ void store(float* As, float* Bs) const {
#pragma unroll
    for (int i = 0; i < T::AC; ++i) *reinterpret_cast<float4*>(As + lds_a[i]) = ra[S][i];
#pragma unroll
    for (int i = 0; i < T::BC; ++i) *reinterpret_cast<float4*>(Bs + lds_b[i]) = rb[S][i];
  }
};

// Fragment reads of 4-deep sub-step chunk g (sub-steps 4g..4g+3) of one staged tile.
// Register-staged images are padded ([row][BK+4] / [k][rows+4]); LDS-DMA images (GL) are
// unpadded, K-contiguous rows chunk-swizzled (Tile).
template <int BM, int BN, int MODE, int BK, bool GL = false>
__device__ __forceinline__ void read_chunk(const float* __restrict__ As, const float* __restrict__ Bs, int g,
                                           float (&af)[Tile<BM, BN, MODE, BK, GL>::RM][4],
                                           float (&bf)[Tile<BM, BN, MODE, BK, GL>::RN][4], int wm, int wn, int r,
                                           int hh) {
  using T = Tile<BM, BN, MODE, BK, GL>;
  constexpr int KP = GL ? BK : BK + 4;  // K-contiguous row pitch
#pragma unroll
  for (int i = 0; i < T::RM; ++i) {
    const int row = wm * T::WM + i * 32 + r;
    if constexpr (T::A_KC) {
      const int ch = GL ? ((T::HK / 4 * hh + g) ^ ((row >> 1) & 7)) : (T::HK / 4 * hh + g);
      const float4 v = *reinterpret_cast<const float4*>(As + row * KP + 4 * ch);
      af[i][0] = v.x; af[i][1] = v.y; af[i][2] = v.z; af[i][3] = v.w;
    } else {
      constexpr int RP = GL ? BM : BM + 4;
#pragma unroll
      for (int s = 0; s < 4; ++s) af[i][s] = As[(T::HK * hh + 4 * g + s) * RP + row];
    }
  }
#pragma unroll
  for (int j = 0; j < T::RN; ++j) {
    const int col = wn * T::WN + j * 32 + r;
    if constexpr (T::B_KC) {
      const int ch = GL ? ((T::HK / 4 * hh + g) ^ ((col >> 1) & 7)) : (T::HK / 4 * hh + g);
      const float4 v = *reinterpret_cast<const float4*>(Bs + col * KP + 4 * ch);
      bf[j][0] = v.x; bf[j][1] = v.y; bf[j][2] = v.z; bf[j][3] = v.w;
    } else {
      constexpr int RP = GL ? BN : BN + 4;
#pragma unroll
      for (int s = 0; s < 4; ++s) bf[j][s] = Bs[(T::HK * hh + 4 * g + s) * RP + col];
    }
  }
}

template <int RM, int RN>
__device__ __forceinline__ void mma_chunk(const float (&af)[RM][4], const float (&bf)[RN][4],
                                          f32x16 (&acc)[RM][RN]) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
}

// ---------------------------------------------------------------- fp32-accurate split-bf16 math (X6)
// gfx950 has no xf32, and its bf16 MFMA (v_mfma_f32_32x32x16_bf16: 32 cyc / 32K FLOP) runs 16x
// the rate of the f32-input one (32x32x2f32: 64 cyc / 4K FLOP). Each f32 operand is split
// exactly into three bf16 pieces by round-to-nearest: x = h + m + l, |m| <= 2^-9 |x|,
// |l| <= 2^-18 |x| (the residuals x - h and r - m are exact in f32). The product is the six
// terms down to 2^-18 relative — hh + hm + mh + mm + hl + lh — accumulated in f32 by the MFMA;
// the dropped ml + lm + ll are <= 2^-26 |a||b|, below f32's own product rounding (2^-24). So
// a K=16 step costs 6 x 32 = 192 MFMA cycles instead of 8 x 64 = 512, with f32-level error
// (tests/test_conv_bn_gpu.py checks it against the f64 reference next to the f32 path).
// Fragment mapping: two 4-deep f32 sub-step chunks (k = base + 0..3 and base + 4..7 of the
// lane half) are the 8 bf16 elements j of one 32x32x16 fragment; A and B use the same k
// order, so the K permutation cancels in the dot product.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3(const float (&x0)[4], const float (&x1)[4], bf16x8& h, bf16x8& m,
                                       bf16x8& l) {
#ifdef CS_X6_PROBE  // measurement only: no split arithmetic (wrong numbers), prices the split VALU
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 hj = (__bf16)(j < 4 ? x0[j] : x1[j - 4]);
    h[j] = hj; m[j] = hj; l[j] = hj;
  }
  return;
#endif
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = j < 4 ? x0[j] : x1[j - 4];
    const __bf16 hj = (__bf16)x;
    const float r = x - (float)hj;
    const __bf16 mj = (__bf16)r;
    h[j] = hj;
    m[j] = mj;
    l[j] = (__bf16)(r - (float)mj);
  }
}

template <int RM, int RN>
__device__ __forceinline__ void mma_x6f(const bf16x8 (&ah)[RM], const bf16x8 (&am)[RM], const bf16x8 (&al)[RM],
                                        const bf16x8 (&bh)[RN], const bf16x8 (&bm)[RN], const bf16x8 (&bl)[RN],
                                        f32x16 (&acc)[RM][RN]) {
  // small terms first (they are exact products; the f32 chain rounds once per MFMA)
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
    }
}

template <int RM, int RN>
__device__ __forceinline__ void mma_x6(const float (&a0)[RM][4], const float (&a1)[RM][4], const float (&b0)[RN][4],
                                       const float (&b1)[RN][4], f32x16 (&acc)[RM][RN]) {
  bf16x8 ah[RM], am[RM], al[RM], bh[RN], bm[RN], bl[RN];
#pragma unroll
  for (int i = 0; i < RM; ++i) split3(a0[i], a1[i], ah[i], am[i], al[i]);
#pragma unroll
  for (int j = 0; j < RN; ++j) split3(b0[j], b1[j], bh[j], bm[j], bl[j]);
  mma_x6f<RM, RN>(ah, am, al, bh, bm, bl, acc);
}

// SCHED 2 (X6 math): one K-step as pairs of sub-step chunks, each pair one split-bf16 MFMA
// group; the next tiles' global loads go out after the first pair, the LDS store after the
// second (or the first when the K-group owns a single pair).
template <int BM, int BN, int MODE, int BK, int LS, int SS, bool C4, int KG>
__device__ __forceinline__ void kstep_x6(Loader<BM, BN, MODE, BK, C4, false, KG>& ld, const CsConvArgs& a,
                                         const float* cur, float* nxt,
                                         f32x16 (&acc)[Tile<BM, BN, MODE, BK>::RM][Tile<BM, BN, MODE, BK>::RN],
                                         int wm, int wn, int r, int hh, int kg, int k_load) {
  using T = Tile<BM, BN, MODE, BK>;
  constexpr int NGK = T::NG / KG;
  static_assert(NGK >= 2 && NGK % 2 == 0, "X6 math needs pairs of sub-step chunks per K-group");
  const int g0 = kg * NGK;
#pragma unroll
  for (int gp = 0; gp < NGK; gp += 2) {
    float af[2][T::RM][4], bf[2][T::RN][4];
    read_chunk<BM, BN, MODE, BK>(cur, cur + T::A_ELEMS, g0 + gp, af[0], bf[0], wm, wn, r, hh);
    read_chunk<BM, BN, MODE, BK>(cur, cur + T::A_ELEMS, g0 + gp + 1, af[1], bf[1], wm, wn, r, hh);
    mma_x6<T::RM, T::RN>(af[0], af[1], bf[0], bf[1], acc);
    if (gp == 0) ld.template load<LS>(a, k_load);
    if (gp == (NGK > 2 ? 2 : 0)) ld.template store<SS>(nxt, nxt + T::A_ELEMS);
  }
}

// ---------------------------------------------------------------- X6S: split once, at the LDS store
// SCHED 3: the register-staged tile is split into three bf16 planes as it is written to LDS
// (once per element per block, instead of once per element per consuming wave), and the
// fragment reads take bf16 directly: ds_read_b128 from K-contiguous planes [row][BK+8], and
// for K-major operands two ds_read_b64_tr_b16 per plane from [k][rows+32] images (the
// hardware transpose delivers 4 k-values of one row per lane; +32 pads make the 4 rows of a
// 16-lane block and the two blocks of a 32-lane half hit 8 distinct 8-bank ranges).
// (s_setprio(1) around the MFMA chain measured -1%: 81.2-81.6k vs 82.3-82.6k img/s.)
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));

// NP = bf16 planes per operand: 3 (h, m, l: the fp32-accurate X6S math) or 1 (h only: plain
// bf16 operands with f32 accumulation, the native engine's opt-in bf16 mode)
template <int BM, int BN, int MODE, int BK, int NP = 3>
struct TileXS {
  using T = Tile<BM, BN, MODE, BK>;
  static constexpr int PA = T::A_KC ? BK + 8 : BM + 32;  // plane pitch (bf16 elements)
  static constexpr int PB = T::B_KC ? BK + 8 : BN + 32;
  static constexpr int PLA = (T::A_KC ? BM : BK) * PA;  // one plane
  static constexpr int PLB = (T::B_KC ? BN : BK) * PB;
  static constexpr int A16 = NP * PLA, STAGE16 = NP * PLA + NP * PLB;
  static constexpr size_t BYTES = 2 * (size_t)STAGE16 * 2;  // double buffer
};

__device__ __forceinline__ void split4(const float4 v, bf16x4& h, bf16x4& m, bf16x4& l) {
  const float x[4] = {v.x, v.y, v.z, v.w};
#ifdef CS_X6_PROBE  // measurement only (wrong numbers): prices the split arithmetic of the X6S store
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const __bf16 hj = (__bf16)x[j];
    h[j] = hj; m[j] = hj; l[j] = hj;
  }
  return;
#endif
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const __bf16 hj = (__bf16)x[j];
    const float r = x[j] - (float)hj;
    const __bf16 mj = (__bf16)r;
    h[j] = hj;
    m[j] = mj;
    l[j] = (__bf16)(r - (float)mj);
  }
}

// bf16 plane offset of this thread's register-staged chunk i (Loader's slot map q = tid + NT*i)
template <int ROWS, bool KC, int P, int BK, int NT>
__device__ __forceinline__ int xs_off(int i) {
  const int q = threadIdx.x + NT * i;
  if constexpr (KC) {
    constexpr int KQ = BK / 4;
    return (q / KQ) * P + 4 * (q % KQ);
  } else {
    constexpr int CPR = ROWS / 4;
    const int kr = q / CPR;
    return kr * P + 4 * (q - kr * CPR);
  }
}

__device__ __forceinline__ bf16x4 round4(const float4 v) {
  bf16x4 h;
  h[0] = (__bf16)v.x; h[1] = (__bf16)v.y; h[2] = (__bf16)v.z; h[3] = (__bf16)v.w;
  return h;
}

// ---------------------------------------------------------------- F3: scaled fp16 hi/lo, 3 MFMAs
// gfx950's f16 MFMA (v_mfma_f32_32x32x16_f16) runs at the bf16 rate with 11-bit significands, so
// two fp16 pieces carry 22 bits where bf16 needs three: x*2^s = h + l, h = fp16(x*2^s) and
// l = fp16(x*2^s - h) (the residual is exact in f32; |l| <= 2^-11 |x*2^s|, its rounding <= 2^-23).
// fp16's range is the catch: each operand tensor gets one power-of-two scale 2^s from its absolute
// maximum (CsConvArgs::amax_a / amax_b, written by the operand's producer) so that its largest
// element lands in [2^14, 2^15) — nothing overflows, and the subnormal floor (2^-25 absolute) is
// 2^-40 of the tensor's maximum. The product is hl + lh + hh (the dropped ll <= 2^-22 |a||b|),
// accumulated in f32 by the MFMA, then scaled back by 2^-(sa+sb) in the epilogue (exact): a
// 32x32x16 product costs 3 x 32 MFMA cycles (X6S: 6 x 32) and the LDS holds two planes, not three.
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// 2^s for an operand whose absolute maximum is the largest of its CS_AMAX_SHARDS shards (the
// producers' atomic-max shards, launchers.h): its largest element scales into [2^14, 2^15). Lane i
// of every wave reads shard i; the wave's max is every lane's (all 64 lanes active).
__device__ __forceinline__ int f3_exp(const float* amax) {
  if (amax == nullptr) return 0;
  static_assert(CS_AMAX_SHARDS == 64, "one shard per lane");
  unsigned bits = __builtin_bit_cast(unsigned, amax[(threadIdx.x & 63) * CS_AMAX_STRIDE]) & 0x7fffffffu;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {  // as bit patterns: a NaN (above +inf) wins and gives s = 0
    const unsigned o = (unsigned)__shfl_xor((int)bits, off, 64);
    bits = o > bits ? o : bits;
  }
  const int e = (int)(bits >> 23);
  if (e == 0 || e == 255) return 0;  // zero / subnormal max, or inf / nan (propagates as is)
  const int s = 14 - (e - 127);
  return s < -100 ? -100 : (s > 100 ? 100 : s);
}
__device__ __forceinline__ float exp2i(int s) { return __builtin_bit_cast(float, (unsigned)(s + 127) << 23); }

// One packed pair of the split: h = (fp16(x0*sc), fp16(x1*sc)) and l = (fp16(x0*sc - h0),
// fp16(x1*sc - h1)), four v_fma_mix (f32 x and sc, f16 h picked by op_sel; mixlo / mixhi write
// the low / high half). Each rounds the exact value once (x*sc is exact: sc is a power of two),
// so the pieces are the ones the plain casts give. Left to itself hipcc mixes v_pk_mul /
// v_cvt_pk / unpack / re-pack sequences and element shuffles (6-7 VALU per pair, not 4).
// Pure VALU on register operands: no memory, no hazard inside the statement.
__device__ __forceinline__ void split_pair(float x0, float x1, float sc, unsigned& h, unsigned& l) {
  asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(h), "=&v"(l)
      : "v"(x0), "v"(x1), "v"(sc));
}

__device__ __forceinline__ void split2h(const float4 v, float sc, bf16x4& h, bf16x4& l) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  unsigned h0, h1, l0, l1;
  split_pair(v.x, v.y, sc, h0, l0);
  split_pair(v.z, v.w, sc, h1, l1);
  h = __builtin_bit_cast(bf16x4, u32x2{h0, h1});
  l = __builtin_bit_cast(bf16x4, u32x2{l0, l1});
}

template <int RM, int RN>
__device__ __forceinline__ void mma_f3(const bf16x8 (&ah)[RM], const bf16x8 (&al)[RM], const bf16x8 (&bh)[RN],
                                       const bf16x8 (&bl)[RN], f32x16 (&acc)[RM][RN]) {
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) {  // small terms first
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, ah[i]),
                                                         __builtin_bit_cast(f16x8, bl[j]), acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, al[i]),
                                                         __builtin_bit_cast(f16x8, bh[j]), acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, ah[i]),
                                                         __builtin_bit_cast(f16x8, bh[j]), acc[i][j], 0, 0, 0);
    }
}

// NP = 3: X6S split (h, m, l bf16); 2: F3 split (h, l fp16 of the scaled value, as 16-bit words);
// 1: bf16 rounding
template <int BM, int BN, int MODE, int BK, bool C4, int KG, int S, int NP = 3>
__device__ __forceinline__ void store_xs(const Loader<BM, BN, MODE, BK, C4, false, KG>& ld, __bf16* As, __bf16* Bs,
                                         const int (&oa)[Tile<BM, BN, MODE, BK, false, KG>::AC],
                                         const int (&ob)[Tile<BM, BN, MODE, BK, false, KG>::BC], float sa = 1.f,
                                         float sb = 1.f) {
  using T = Tile<BM, BN, MODE, BK, false, KG>;  // chunk counts depend on the block's thread count
  using X = TileXS<BM, BN, MODE, BK, NP>;
#pragma unroll
  for (int i = 0; i < T::AC; ++i) {
    if constexpr (NP == 1) {
      *reinterpret_cast<bf16x4*>(As + oa[i]) = round4(ld.ra[S][i]);
    } else if constexpr (NP == 2) {
      bf16x4 h, l;
      split2h(ld.ra[S][i], sa, h, l);
      *reinterpret_cast<bf16x4*>(As + oa[i]) = h;
      *reinterpret_cast<bf16x4*>(As + X::PLA + oa[i]) = l;
    } else {
      bf16x4 h, m, l;
      split4(ld.ra[S][i], h, m, l);
      *reinterpret_cast<bf16x4*>(As + oa[i]) = h;
      *reinterpret_cast<bf16x4*>(As + X::PLA + oa[i]) = m;
      *reinterpret_cast<bf16x4*>(As + 2 * X::PLA + oa[i]) = l;
    }
  }
#pragma unroll
  for (int i = 0; i < T::BC; ++i) {
    if constexpr (NP == 1) {
      *reinterpret_cast<bf16x4*>(Bs + ob[i]) = round4(ld.rb[S][i]);
    } else if constexpr (NP == 2) {
      bf16x4 h, l;
      split2h(ld.rb[S][i], sb, h, l);
      *reinterpret_cast<bf16x4*>(Bs + ob[i]) = h;
      *reinterpret_cast<bf16x4*>(Bs + X::PLB + ob[i]) = l;
    } else {
      bf16x4 h, m, l;
      split4(ld.rb[S][i], h, m, l);
      *reinterpret_cast<bf16x4*>(Bs + ob[i]) = h;
      *reinterpret_cast<bf16x4*>(Bs + X::PLB + ob[i]) = m;
      *reinterpret_cast<bf16x4*>(Bs + 2 * X::PLB + ob[i]) = l;
    }
  }
}

// 32x32x16 fragments (element j <-> k = (BK/2)*hh + 4*g0 + j) of R 32-row groups from one plane
template <int R, bool KC, int P, int BK>
__device__ __forceinline__ void read_xs(const __bf16* pl, int base, int g0, int lane, bf16x8 (&f)[R]) {
#pragma unroll
  for (int i = 0; i < R; ++i) {
    if constexpr (KC) {
      const int row = base + i * 32 + (lane & 31);
      f[i] = *reinterpret_cast<const bf16x8*>(pl + row * P + (BK / 2) * (lane >> 5) + 4 * g0);
    } else {
      const int grp = lane >> 4, l16 = lane & 15;
      const int col = base + i * 32 + 16 * (grp & 1) + 4 * (l16 & 3);
      const int kr = (BK / 2) * (grp >> 1) + 4 * g0 + (l16 >> 2);
      const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) i16x4*)(pl + kr * P + col));
      const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) i16x4*)(pl + (kr + 4) * P + col));
      const bf16x4 blo = __builtin_bit_cast(bf16x4, lo), bhi = __builtin_bit_cast(bf16x4, hi);
      f[i] = __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
}

template <int BM, int BN, int MODE, int BK, int LS, int SS, bool C4, int KG, int NP = 3>
__device__ __forceinline__ void kstep_xs(Loader<BM, BN, MODE, BK, C4, false, KG>& ld, const CsConvArgs& a,
                                         const __bf16* cur, __bf16* nxt,
                                         f32x16 (&acc)[Tile<BM, BN, MODE, BK>::RM][Tile<BM, BN, MODE, BK>::RN],
                                         int wm, int wn, int kg, int k_load,
                                         const int (&oa)[Tile<BM, BN, MODE, BK, false, KG>::AC],
                                         const int (&ob)[Tile<BM, BN, MODE, BK, false, KG>::BC], float sa,
                                         float sb) {
  using T = Tile<BM, BN, MODE, BK>;
  using X = TileXS<BM, BN, MODE, BK, NP>;
  constexpr int NGK = T::NG / KG;
  static_assert(NGK >= 2 && NGK % 2 == 0, "X6 math needs pairs of sub-step chunks per K-group");
  const int g0 = kg * NGK, lane = threadIdx.x & 63;
  const __bf16* Bc = cur + X::A16;
#pragma unroll
  for (int gp = 0; gp < NGK; gp += 2) {
    bf16x8 ah[T::RM], bh[T::RN];
    read_xs<T::RM, T::A_KC, X::PA, BK>(cur, wm * T::WM, g0 + gp, lane, ah);
    read_xs<T::RN, T::B_KC, X::PB, BK>(Bc, wn * T::WN, g0 + gp, lane, bh);
    if constexpr (NP == 1) {
#pragma unroll
      for (int i = 0; i < T::RM; ++i)
#pragma unroll
        for (int j = 0; j < T::RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
    } else if constexpr (NP == 2) {
      bf16x8 al[T::RM], bl[T::RN];
      read_xs<T::RM, T::A_KC, X::PA, BK>(cur + X::PLA, wm * T::WM, g0 + gp, lane, al);
      read_xs<T::RN, T::B_KC, X::PB, BK>(Bc + X::PLB, wn * T::WN, g0 + gp, lane, bl);
      mma_f3<T::RM, T::RN>(ah, al, bh, bl, acc);
    } else {
      bf16x8 am[T::RM], al[T::RM], bm[T::RN], bl[T::RN];
      read_xs<T::RM, T::A_KC, X::PA, BK>(cur + X::PLA, wm * T::WM, g0 + gp, lane, am);
      read_xs<T::RM, T::A_KC, X::PA, BK>(cur + 2 * X::PLA, wm * T::WM, g0 + gp, lane, al);
      read_xs<T::RN, T::B_KC, X::PB, BK>(Bc + X::PLB, wn * T::WN, g0 + gp, lane, bm);
      read_xs<T::RN, T::B_KC, X::PB, BK>(Bc + 2 * X::PLB, wn * T::WN, g0 + gp, lane, bl);
      mma_x6f<T::RM, T::RN>(ah, am, al, bh, bm, bl, acc);
    }
    if (gp == 0) ld.template load<LS>(a, k_load);
    if (gp == (NGK > 2 ? 2 : 0)) store_xs<BM, BN, MODE, BK, C4, KG, SS, NP>(ld, nxt, nxt + X::A16, oa, ob, sa, sb);
  }
}

// One K-step on a staged LDS tile, with the next tiles' global loads (tile t+2 -> register
// stage LS) and LDS store (tile t+1, register stage SS -> the other LDS buffer) folded in.
// Both are unconditional (no branch around a load: hipcc would drain vmcnt there): past the
// split's last K-step they fetch a neighbouring range or zeros (range check) into a
// register stage / LDS buffer that is never read again.
// SCHED 0: the MFMA chain runs one chunk behind its fragment reads; the global loads
//          go out after the first chunk, the LDS store after the second (sched barriers
//          pin the phases so hipcc cannot hoist every read ahead of the chain).
template <int BM, int BN, int MODE, int BK, int SCHED, int LS, int SS, bool C4, int KG>
__device__ __forceinline__ void kstep(Loader<BM, BN, MODE, BK, C4, false, KG>& ld, const CsConvArgs& a,
                                      const float* cur, float* nxt,
                                      f32x16 (&acc)[Tile<BM, BN, MODE, BK>::RM][Tile<BM, BN, MODE, BK>::RN],
                                      int wm, int wn, int r, int hh, int kg, int k_load) {
  using T = Tile<BM, BN, MODE, BK>;
  constexpr int NGK = T::NG / KG;  // chunks of this K-group
  static_assert(NGK >= 1, "K-step too short for the K-groups");
  const int g0 = kg * NGK;
  float af[2][T::RM][4], bf[2][T::RN][4];
  read_chunk<BM, BN, MODE, BK>(cur, cur + T::A_ELEMS, g0, af[0], bf[0], wm, wn, r, hh);
#pragma unroll
  for (int g = 0; g < NGK; ++g) {
    if (g + 1 < NGK) read_chunk<BM, BN, MODE, BK>(cur, cur + T::A_ELEMS, g0 + g + 1, af[(g + 1) & 1],
                                                  bf[(g + 1) & 1], wm, wn, r, hh);
    if constexpr (SCHED == 0) __builtin_amdgcn_sched_barrier(0);
    mma_chunk<T::RM, T::RN>(af[g & 1], bf[g & 1], acc);
    if (g == 0) ld.template load<LS>(a, k_load);
    if (g == (NGK > 1 ? 1 : 0)) ld.template store<SS>(nxt, nxt + T::A_ELEMS);
    if constexpr (SCHED == 0) __builtin_amdgcn_sched_barrier(0);
  }
}


// One K-step's MFMA chain on a staged LDS-DMA tile (GL): fragment reads one chunk ahead.
template <int BM, int BN, int MODE, int BK, bool X6 = false>
__device__ __forceinline__ void kcompute_gl(const float* cur,
                                            f32x16 (&acc)[Tile<BM, BN, MODE, BK, true>::RM][Tile<BM, BN, MODE, BK, true>::RN],
                                            int wm, int wn, int r, int hh) {
  using T = Tile<BM, BN, MODE, BK, true>;
  if constexpr (X6) {
    static_assert(T::NG % 2 == 0, "X6 math needs pairs of sub-step chunks");
#pragma unroll
    for (int gp = 0; gp < T::NG; gp += 2) {
      float a2[2][T::RM][4], b2[2][T::RN][4];
      read_chunk<BM, BN, MODE, BK, true>(cur, cur + T::A_ELEMS, gp, a2[0], b2[0], wm, wn, r, hh);
      read_chunk<BM, BN, MODE, BK, true>(cur, cur + T::A_ELEMS, gp + 1, a2[1], b2[1], wm, wn, r, hh);
      mma_x6<T::RM, T::RN>(a2[0], a2[1], b2[0], b2[1], acc);
    }
    return;
  }
  float af[2][T::RM][4], bf[2][T::RN][4];
  read_chunk<BM, BN, MODE, BK, true>(cur, cur + T::A_ELEMS, 0, af[0], bf[0], wm, wn, r, hh);
#pragma unroll
  for (int g = 0; g < T::NG; ++g) {
    if (g + 1 < T::NG)
      read_chunk<BM, BN, MODE, BK, true>(cur, cur + T::A_ELEMS, g + 1, af[(g + 1) & 1], bf[(g + 1) & 1], wm, wn, r, hh);
    __builtin_amdgcn_sched_barrier(0);
    mma_chunk<T::RM, T::RN>(af[g & 1], bf[g & 1], acc);
    __builtin_amdgcn_sched_barrier(0);
  }
}


// GL > 0: LDS-DMA staging through a GL-deep ring of LDS images — tile t+GL-1 is fetched
// while tile t is multiplied, one raw s_barrier per K-step after a counted vmcnt (tile t
// landed, newer tiles may still be in flight); no register stage, no ds_write.
// One output tile (`tile`, already XCD-remapped) x one K split of a conv GEMM; the body of
// the GEMM kernel.
template <int BM, int BN, int MODE, int BK, int SCHED, bool C4, int GL, int KG = 1>
__device__ __forceinline__ void gemm_body(const CsConvArgs& a, const int tile, const int split, const int nsplit,
                                          float* smem) {
  static_assert(KG == 1 || GL == 0, "K-groups use register staging");
  using T = Tile<BM, BN, MODE, BK>;
  const int ntn = (a.N + BN - 1) / BN;
  const int mt = tile / ntn, nt = tile - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int ks_begin = split * a.ksteps_per_split;
  int ks_end = ks_begin + a.ksteps_per_split;
  if (ks_end > a.total_ksteps) ks_end = a.total_ksteps;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kg = wid >> 2, wsp = wid & 3;  // K-group, spatial wave (2x2)
  const int wm = wsp >> 1, wn = wsp & 1, r = lane & 31, hh = lane >> 5;

  f32x16 acc[T::RM][T::RN];
#pragma unroll
  for (int i = 0; i < T::RM; ++i)
#pragma unroll
    for (int j = 0; j < T::RN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nks = ks_end - ks_begin;
  if constexpr (GL > 0) {
    using TG = Tile<BM, BN, MODE, BK, true>;
    constexpr int NI = TG::AC + TG::BC;  // LDS-DMA instructions per wave per tile
    constexpr int NB = GL;               // ring depth: tiles t+1 .. t+NB-1 in flight during tile t
    Loader<BM, BN, MODE, BK, false, true> ld;
    ld.init(a, m0, n0);
#pragma unroll
    for (int p = 0; p < NB - 1; ++p)
      if (p < nks) ld.gload(a, (ks_begin + p) * BK, smem + p * TG::STAGE, smem + p * TG::STAGE + TG::A_ELEMS);
    int cur = 0;
    for (int t = 0; t < nks; ++t) {
      // tile t has landed once at most `ahead` newer tiles are outstanding (loads retire in order)
      const int ahead = min(NB - 2, nks - 1 - t);
      if (ahead >= 4) wait_vmcnt<4 * NI>();
      else if (ahead == 3) wait_vmcnt<3 * NI>();
      else if (ahead == 2) wait_vmcnt<2 * NI>();
      else if (ahead == 1) wait_vmcnt<NI>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + NB - 1 < nks) {
        const int nx = cur == 0 ? NB - 1 : cur - 1;  // (t + NB - 1) % NB: the buffer read at step t-1
        ld.gload(a, (ks_begin + t + NB - 1) * BK, smem + nx * TG::STAGE, smem + nx * TG::STAGE + TG::A_ELEMS);
      }
      kcompute_gl<BM, BN, MODE, BK, SCHED == 2>(smem + cur * TG::STAGE, acc, wm, wn, r, hh);
      cur = cur == NB - 1 ? 0 : cur + 1;
    }
    __syncthreads();  // every wave's fragment reads are done before the epilogue reuses LDS
  } else if constexpr (SCHED == 3 || SCHED == 5 || SCHED == 6) {
    // SCHED 5: bf16 operands (h plane only); SCHED 6: F3 (scaled fp16 h / l planes)
    constexpr int NP = SCHED == 5 ? 1 : (SCHED == 6 ? 2 : 3);
    using X = TileXS<BM, BN, MODE, BK, NP>;
    const int ea = SCHED == 6 ? f3_exp(a.amax_a) : 0, eb = SCHED == 6 ? f3_exp(a.amax_b) : 0;
    const float sa = exp2i(ea), sb = exp2i(eb);
    Loader<BM, BN, MODE, BK, C4, false, KG> ld;
    ld.init(a, m0, n0);
    using TK = Tile<BM, BN, MODE, BK, false, KG>;
    int oa[TK::AC], ob[TK::BC];
#pragma unroll
    for (int i = 0; i < TK::AC; ++i) oa[i] = xs_off<BM, T::A_KC, X::PA, BK, TK::NT>(i);
#pragma unroll
    for (int i = 0; i < TK::BC; ++i) ob[i] = xs_off<BN, T::B_KC, X::PB, BK, TK::NT>(i);
    __bf16* l0 = reinterpret_cast<__bf16*>(smem);
    __bf16* l1 = l0 + X::STAGE16;
    if (nks > 0) {
      ld.template load<0>(a, ks_begin * BK);
      if (nks > 1) ld.template load<1>(a, (ks_begin + 1) * BK);
      store_xs<BM, BN, MODE, BK, C4, KG, 0, NP>(ld, l0, l0 + X::A16, oa, ob, sa, sb);
    }
    __syncthreads();
    // one exit: an odd last K-step is peeled after the loop instead of a break between the
    // halves (with two exits hipcc kept the accumulator in different registers at each and
    // copied it inside the loop, behind an MFMA-result stall)
    int t = 0;
    for (; t + 1 < nks; t += 2) {
      kstep_xs<BM, BN, MODE, BK, 0, 1, C4, KG, NP>(ld, a, l0, l1, acc, wm, wn, kg, (ks_begin + t + 2) * BK, oa, ob,
                                                   sa, sb);
      __syncthreads();
      kstep_xs<BM, BN, MODE, BK, 1, 0, C4, KG, NP>(ld, a, l1, l0, acc, wm, wn, kg, (ks_begin + t + 3) * BK, oa, ob,
                                                   sa, sb);
      __syncthreads();
    }
    if (t < nks) {
      kstep_xs<BM, BN, MODE, BK, 0, 1, C4, KG, NP>(ld, a, l0, l1, acc, wm, wn, kg, (ks_begin + t + 2) * BK, oa, ob,
                                                   sa, sb);
      __syncthreads();
    }
    if constexpr (SCHED == 6) {  // back to the operands' scale (a power of two: exact)
      const float un = exp2i(-(ea + eb));
#pragma unroll
      for (int i = 0; i < T::RM; ++i)
#pragma unroll
        for (int j = 0; j < T::RN; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][j][e] *= un;
    }
  } else {
  Loader<BM, BN, MODE, BK, C4, false, KG> ld;
  ld.init(a, m0, n0);
  float* lds0 = smem;
  float* lds1 = smem + T::STAGE;
  if (nks > 0) {
    ld.template load<0>(a, ks_begin * BK);
    if (nks > 1) ld.template load<1>(a, (ks_begin + 1) * BK);
    ld.template store<0>(lds0, lds0 + T::A_ELEMS);
  }
  __syncthreads();
  // even step t: tile t in lds0, tile t+1 in registers[1] -> lds1, tile t+2 -> registers[0];
  // one loop exit, an odd last step peeled (as in the split-operand loop above)
  int t = 0;
  for (; t + 1 < nks; t += 2) {
    if constexpr (SCHED == 2)
      kstep_x6<BM, BN, MODE, BK, 0, 1, C4, KG>(ld, a, lds0, lds1, acc, wm, wn, r, hh, kg, (ks_begin + t + 2) * BK);
    else
      kstep<BM, BN, MODE, BK, SCHED, 0, 1, C4, KG>(ld, a, lds0, lds1, acc, wm, wn, r, hh, kg, (ks_begin + t + 2) * BK);
    __syncthreads();
    if constexpr (SCHED == 2)
      kstep_x6<BM, BN, MODE, BK, 1, 0, C4, KG>(ld, a, lds1, lds0, acc, wm, wn, r, hh, kg, (ks_begin + t + 3) * BK);
    else
      kstep<BM, BN, MODE, BK, SCHED, 1, 0, C4, KG>(ld, a, lds1, lds0, acc, wm, wn, r, hh, kg, (ks_begin + t + 3) * BK);
    __syncthreads();
  }
  if (t < nks) {
    if constexpr (SCHED == 2)
      kstep_x6<BM, BN, MODE, BK, 0, 1, C4, KG>(ld, a, lds0, lds1, acc, wm, wn, r, hh, kg, (ks_begin + t + 2) * BK);
    else
      kstep<BM, BN, MODE, BK, SCHED, 0, 1, C4, KG>(ld, a, lds0, lds1, acc, wm, wn, r, hh, kg, (ks_begin + t + 2) * BK);
    __syncthreads();
  }
  }

  conv_epilogue<BM, BN, MODE, KG>(a, acc, tile, split, nsplit, smem);
}

template <int BM, int BN, int MODE, int BK, int SCHED, bool C4, int GL, int KG = 1>
__global__ __launch_bounds__(256 * KG) void conv_gemm_kernel(CsConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int ntiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  // linear grid: ntiles x nsplit GEMM blocks (x fastest, as the old (ntiles, 1, nsplit) grid
  // dispatched them), then sgd.P blocks of an independent SGD update that run in the GEMM's tail
  const int nsplit = (a.total_ksteps + a.ksteps_per_split - 1) / a.ksteps_per_split;
  const int ng = ntiles * nsplit, lin = blockIdx.x;
  if (lin >= ng) {
    cs_sgd::tail_body(a.sgd, lin - ng, a.sgd.P);
    return;
  }
  gemm_body<BM, BN, MODE, BK, SCHED, C4, GL, KG>(a, cs::xcd_remap(lin % ntiles, ntiles), lin / ntiles, nsplit, smem);
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
    // every load of the group in flight before the adds (same ascending-z order)
    float4 t[kFold];
#pragma unroll
    for (int j = 0; j < kFold; ++j)
      t[j] = z0 + j < z1 ? w4[(size_t)(z0 + j) * n4 + i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 acc = t[0];
#pragma unroll
    for (int j = 1; j < kFold; ++j)
      if (z0 + j < z1) {
        acc.x += t[j].x; acc.y += t[j].y; acc.z += t[j].z; acc.w += t[j].w;
      }
    w4[(size_t)z0 * n4 + i] = acc;
  }
}

// smem: >= kRedLds floats (the row image, the column means, and bn_fin.h's combine space)
constexpr int kRedLds = 1024 + 80;
__device__ __forceinline__ void splitk_reduce_body(const CsConvArgs& a, int mode, int nslab, int zstep, int blk,
                                                   float* smem) {
  float(&red)[kRedRows][64] = *reinterpret_cast<float(*)[kRedRows][64]>(smem);
  float* meanv = smem + kRedRows * 64;
  const bool fin = a.fin.cnt != nullptr;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int ntn = (a.N + 63) / 64;
  const int mt = blk / ntn, nt = blk - mt * ntn;
  const int m0 = mt * kRedRows, n0 = nt * 64, n = n0 + 4 * tx, m = m0 + ty;
  const size_t slab = (size_t)a.M * a.N;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool in = m < a.M && n < a.N;
  if (in) {
    const bool add_bias = mode == CS_CONV_FWD && a.bias != nullptr;
    const float4 bv = add_bias ? *reinterpret_cast<const float4*>(a.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float* p = a.ws + (size_t)m * a.N + n;
    // 8 slab loads in flight before the adds (a plain loop waits one memory latency per
    // slab); the summation order is unchanged: z ascending, then the bias
    for (int z0 = 0; z0 < nslab; z0 += 8) {
      float4 t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        t[j] = z0 + j < nslab ? *reinterpret_cast<const float4*>(p + (size_t)(z0 + j) * zstep * slab)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (z0 + j < nslab) {
          acc.x += t[j].x; acc.y += t[j].y; acc.z += t[j].z; acc.w += t[j].w;
        }
    }
    if (add_bias) {
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
  if (mode == CS_CONV_DGRAD && a.ered.part != nullptr) {
    // BN-backward partials of the block below over this 16-row tile (conv_common.h
    // dgrad_bn_partials): each thread's 4 channels at its row, then the 16 rows in order
    const CsBnRed& e = a.ered;
    float tot[3] = {0.f, 0.f, 0.f};
    float s[3][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    if (in) {
      const float4 sc = *reinterpret_cast<const float4*>(e.scale + n), sh = *reinterpret_cast<const float4*>(e.shift + n);
      const float4 mu = *reinterpret_cast<const float4*>(e.mean + n), is = *reinterpret_cast<const float4*>(e.invstd + n);
      if (e.pool)
        cs_bn::bwd_point4<true>(e.y, cs_bn::bwd_point_index<true>(m, n, a.lgH, a.lgW, a.N), a.N, 2 * a.W, acc, sc, sh,
                                mu, is, s);
      else
        cs_bn::bwd_point4<false>(e.y, cs_bn::bwd_point_index<false>(m, n, a.lgH, a.lgW, a.N), a.N, 2 * a.W, acc, sc,
                                 sh, mu, is, s);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
      for (int q = 0; q < 4; ++q) red[ty][4 * tx + q] = s[k][q];
      __syncthreads();
      if (threadIdx.x < 64 && n0 + (int)threadIdx.x < a.N) {
        float t = 0.f;
        for (int r = 0; r < kRedRows; ++r) t += red[r][threadIdx.x];
        if (fin) tot[k] = t;
        else e.part[((size_t)mt * a.N + n0 + threadIdx.x) * 3 + k] = t;
      }
      __syncthreads();
    }
    if (fin) {  // [T][N][4] write-through, then the launch's last arriver finalizes (bn_fin.h)
      if (threadIdx.x < 64 && n0 + (int)threadIdx.x < a.N)
        cs_fin::put_sums(e.part, a.N, mt, n0 + threadIdx.x, tot[0], tot[1], tot[2]);
      cs_fin::arrive<true, 64>(a.fin, e.part, a.N, mt, nt, n0, smem);
    }
    return;
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
    if (fin) {
      cs_fin::put_stats(a.stats, a.N, mt, n0 + threadIdx.x, meanv[threadIdx.x], sq);
    } else {
      a.stats[((size_t)mt * a.N + n0 + threadIdx.x) * 2 + 0] = meanv[threadIdx.x];
      a.stats[((size_t)mt * a.N + n0 + threadIdx.x) * 2 + 1] = sq;
    }
  }
  if (fin) cs_fin::arrive<false, 64>(a.fin, a.stats, a.N, mt, nt, n0, smem);
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(CsConvArgs a, int mode, int nslab, int zstep) {
  __shared__ float smem[kRedLds];
  splitk_reduce_body(a, mode, nslab, zstep, blockIdx.x, smem);
}

int reduce_blocks(const CsConvArgs& a) { return ((a.M + kRedRows - 1) / kRedRows) * ((a.N + 63) / 64); }

// fold pre-pass for large split counts; returns (nslab, zstep) for the combine
void fold_if_needed(const CsConvArgs& a, int splits, hipStream_t stream, int& nslab, int& zstep) {
  nslab = splits;
  zstep = 1;
  if (splits > 2 * kFold) {
    const size_t slab = (size_t)a.M * a.N;
    const int groups = (splits + kFold - 1) / kFold;
    int bx = (int)((slab / 4 + 255) / 256);
    if (bx > 1024) bx = 1024;
    hipLaunchKernelGGL(splitk_fold_kernel, dim3(bx, groups), dim3(256), 0, stream, a.ws, slab, splits);
    nslab = groups;
    zstep = kFold;
  }
}

hipError_t launch_reduce(const CsConvArgs& a, int mode, int splits, hipStream_t stream) {
  int nslab, zstep;
  fold_if_needed(a, splits, stream, nslab, zstep);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(reduce_blocks(a)), dim3(256), 0, stream, a, mode, nslab, zstep);
  return hipGetLastError();
}

template <int BM, int BN, int MODE, int BK, int SCHED, bool C4, int GL, int KG = 1>
hipError_t launch_k(dim3 grid, size_t lds, hipStream_t stream, const CsConvArgs& a) {
  size_t l = std::max(lds, (size_t)(1024 + 16) * sizeof(float));  // bn_fin.h's combine space
  if (MODE == CS_CONV_DGRAD && a.ered.part != nullptr) l = std::max(l, (size_t)BM * (BN + 4) * sizeof(float));
  hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, MODE, BK, SCHED, C4, GL, KG>), grid, dim3(256 * KG), l, stream, a);
  return hipGetLastError();
}

// MATH 0: f32 MFMA; MATH 2: X6 split-bf16 kernels;
// MATH 3: X6 split at the LDS store (register staging only)
template <int BM, int BN, int MODE, int BK, int MATH>
hipError_t launch_gemm_m(const CsConvArgs& a, int splits, int stage, hipStream_t stream) {
  using T = Tile<BM, BN, MODE, BK>;
  using TG = Tile<BM, BN, MODE, BK, true>;
  const int ntiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const size_t lds = MATH == 3   ? TileXS<BM, BN, MODE, BK>::BYTES
                     : MATH == 5 ? TileXS<BM, BN, MODE, BK, 1>::BYTES
                     : MATH == 6 ? TileXS<BM, BN, MODE, BK, 2>::BYTES
                                 : 2 * T::STAGE * sizeof(float);
  const dim3 grid(ntiles * splits + a.sgd.P);
  constexpr bool deep_fits = (BM + BN) * BK * 4 * 5 < 160 * 1024;
  if constexpr (BK != 64 && MATH == 0) {
    if (MODE == CS_CONV_FWD && a.w_oihw)  // padded conv0: Cin = 4 < BK
      return launch_k<BM, BN, MODE, BK, 0, true, 0>(grid, lds, stream, a);
  }
  if constexpr (BK == 32 && MATH != 3 && MATH != 5 && MATH != 6) {
    if (stage == CS_STAGE_LDS_DMA)
      return launch_k<BM, BN, MODE, BK, MATH, false, 3>(grid, 3 * TG::STAGE * sizeof(float), stream, a);
    if constexpr (deep_fits) {
      if (stage == CS_STAGE_LDS_DMA_DEEP)
        return launch_k<BM, BN, MODE, BK, MATH, false, 5>(grid, 5 * TG::STAGE * sizeof(float), stream, a);
    }
  }
  // K-groups: the LDS tile ring must also hold the (KG-1) partial-accumulator images
  if constexpr (BK >= 32 && BM * BK >= 2048 && BN * BK >= 2048 && (MATH != 3 || BK == 32 || (BM == 64 && BN == 64)) &&
                (MATH != 6 || BK == 32 || !(BM == 128 && BN == 128))) {
    if (stage == CS_STAGE_KG2) {
      const size_t red = (size_t)1 * 4 * (BM / 64) * (BN / 64) * 16 * 64 * sizeof(float);
      return launch_k<BM, BN, MODE, BK, MATH, false, 0, 2>(grid, std::max(lds, red), stream, a);
    }
  }
  if constexpr (BK == 64 && BM * BK >= 4096 && BN * BK >= 4096 && (MATH != 3 || (BM == 64 && BN == 64)) &&
                (MATH != 6 || !(BM == 128 && BN == 128))) {
    if (stage == CS_STAGE_KG4) {
      const size_t red = (size_t)3 * 4 * (BM / 64) * (BN / 64) * 16 * 64 * sizeof(float);
      return launch_k<BM, BN, MODE, BK, MATH, false, 0, 4>(grid, std::max(lds, red), stream, a);
    }
  }
  if (stage != CS_STAGE_REGS) return hipErrorInvalidValue;
  if constexpr ((MATH == 3 && BK == 64 && !(BM == 64 && BN == 64)) ||
                ((MATH == 5 || MATH == 6) && BK == 64 && BM == 128 && BN == 128)) {
    return hipErrorInvalidValue;  // bf16 planes of a wider bk-64 tile exceed the 160 KiB LDS
  } else if constexpr (MATH >= 2) {
    return launch_k<BM, BN, MODE, BK, MATH, false, 0>(grid, lds, stream, a);
  } else {
    return launch_k<BM, BN, MODE, BK, 0, false, 0>(grid, lds, stream, a);
  }
}

template <int BM, int BN, int MODE, int BK>
hipError_t launch_gemm(const CsConvArgs& a, int splits, int stage, hipStream_t stream) {
  if (stage & CS_STAGE_BF16) return launch_gemm_m<BM, BN, MODE, BK, 5>(a, splits, stage & ~CS_STAGE_BF16, stream);
  if (stage & CS_STAGE_F3) return launch_gemm_m<BM, BN, MODE, BK, 6>(a, splits, stage & ~CS_STAGE_F3, stream);
  if (stage & CS_STAGE_X6S) return launch_gemm_m<BM, BN, MODE, BK, 3>(a, splits, stage & ~CS_STAGE_X6S, stream);
  if (stage & CS_STAGE_X6) return launch_gemm_m<BM, BN, MODE, BK, 2>(a, splits, stage & ~CS_STAGE_X6, stream);
  return launch_gemm_m<BM, BN, MODE, BK, 0>(a, splits, stage, stream);
}

// hipcc (ROCm 7.2) leaves some host-side kernel stubs undefined when they are only
// implicitly instantiated through launch_k (an undefined-symbol error at import, seen for
// the LDS-DMA variants); explicit instantiation of every launched variant emits them all.
#define CS_K(BM_, BN_, MODE_, BK_, SCHED_, C4_, GL_) \
  template __global__ void conv_gemm_kernel<BM_, BN_, MODE_, BK_, SCHED_, C4_, GL_>(CsConvArgs);
#define CS_MODE(BM_, BN_, MODE_)                                            \
  CS_K(BM_, BN_, MODE_, 16, 0, false, 0)                                      \
  CS_K(BM_, BN_, MODE_, 32, 0, false, 0)                                      \
  CS_K(BM_, BN_, MODE_, 32, 0, false, 3)                                      \
  CS_K(BM_, BN_, MODE_, 16, 2, false, 0) CS_K(BM_, BN_, MODE_, 32, 2, false, 0) \
  CS_K(BM_, BN_, MODE_, 32, 2, false, 3)                                      \
  CS_K(BM_, BN_, MODE_, 16, 3, false, 0) CS_K(BM_, BN_, MODE_, 32, 3, false, 0)     \
  CS_K(BM_, BN_, MODE_, 16, 5, false, 0) CS_K(BM_, BN_, MODE_, 32, 5, false, 0)     \
  CS_K(BM_, BN_, MODE_, 16, 6, false, 0) CS_K(BM_, BN_, MODE_, 32, 6, false, 0)
#define CS_TILE(BM_, BN_)                                                                       \
  CS_MODE(BM_, BN_, CS_CONV_FWD) CS_MODE(BM_, BN_, CS_CONV_DGRAD) CS_MODE(BM_, BN_, CS_CONV_WGRAD) \
  CS_K(BM_, BN_, CS_CONV_FWD, 16, 0, true, 0) CS_K(BM_, BN_, CS_CONV_FWD, 32, 0, true, 0)
CS_TILE(64, 64)
CS_TILE(64, 128)
CS_TILE(128, 64)
CS_TILE(128, 128)
#define CS_BK64(BM_, BN_, MODE_) \
  CS_K(BM_, BN_, MODE_, 64, 0, false, 0) CS_K(BM_, BN_, MODE_, 64, 2, false, 0)
#define CS_TILE64(BM_, BN_) CS_BK64(BM_, BN_, CS_CONV_FWD) CS_BK64(BM_, BN_, CS_CONV_DGRAD) CS_BK64(BM_, BN_, CS_CONV_WGRAD)
CS_TILE64(64, 64)
CS_TILE64(128, 64)
CS_TILE64(64, 128)
CS_K(64, 64, CS_CONV_FWD, 64, 5, false, 0)
CS_K(64, 64, CS_CONV_DGRAD, 64, 5, false, 0)
CS_K(64, 64, CS_CONV_WGRAD, 64, 5, false, 0)
CS_K(128, 64, CS_CONV_FWD, 64, 5, false, 0)
CS_K(128, 64, CS_CONV_DGRAD, 64, 5, false, 0)
CS_K(128, 64, CS_CONV_WGRAD, 64, 5, false, 0)
CS_K(64, 128, CS_CONV_FWD, 64, 5, false, 0)
CS_K(64, 128, CS_CONV_DGRAD, 64, 5, false, 0)
CS_K(64, 128, CS_CONV_WGRAD, 64, 5, false, 0)
CS_K(64, 64, CS_CONV_FWD, 64, 3, false, 0)
CS_K(64, 64, CS_CONV_DGRAD, 64, 3, false, 0)
CS_K(64, 64, CS_CONV_WGRAD, 64, 3, false, 0)
#define CS_F3_64(BM_, BN_) \
  CS_K(BM_, BN_, CS_CONV_FWD, 64, 6, false, 0) CS_K(BM_, BN_, CS_CONV_DGRAD, 64, 6, false, 0) \
  CS_K(BM_, BN_, CS_CONV_WGRAD, 64, 6, false, 0)
CS_F3_64(64, 64)
CS_F3_64(128, 64)
CS_F3_64(64, 128)
#undef CS_F3_64
#undef CS_TILE64
#undef CS_BK64
#define CS_KG1(BM_, BN_, BK_, KG_, M_)                                                            \
  template __global__ void conv_gemm_kernel<BM_, BN_, CS_CONV_FWD, BK_, M_, false, 0, KG_>(CsConvArgs);   \
  template __global__ void conv_gemm_kernel<BM_, BN_, CS_CONV_DGRAD, BK_, M_, false, 0, KG_>(CsConvArgs); \
  template __global__ void conv_gemm_kernel<BM_, BN_, CS_CONV_WGRAD, BK_, M_, false, 0, KG_>(CsConvArgs);
#define CS_KG(BM_, BN_, BK_, KG_) CS_KG1(BM_, BN_, BK_, KG_, 0) CS_KG1(BM_, BN_, BK_, KG_, 2)
CS_KG(64, 64, 32, 2)
CS_KG(128, 64, 32, 2)
CS_KG(64, 128, 32, 2)
CS_KG(128, 128, 32, 2)
CS_KG1(64, 64, 32, 2, 3)
CS_KG1(128, 64, 32, 2, 3)
CS_KG1(64, 128, 32, 2, 3)
CS_KG1(128, 128, 32, 2, 3)
CS_KG1(64, 64, 64, 2, 3)
CS_KG1(64, 64, 64, 4, 3)
CS_KG1(64, 64, 32, 2, 6)
CS_KG1(128, 64, 32, 2, 6)
CS_KG1(64, 128, 32, 2, 6)
CS_KG1(128, 128, 32, 2, 6)
CS_KG1(64, 64, 64, 2, 6)
CS_KG1(128, 64, 64, 2, 6)
CS_KG1(64, 128, 64, 2, 6)
CS_KG1(64, 64, 64, 4, 6)
CS_KG1(128, 64, 64, 4, 6)
CS_KG1(64, 128, 64, 4, 6)
CS_KG1(64, 64, 32, 2, 5)
CS_KG1(128, 64, 32, 2, 5)
CS_KG1(64, 128, 32, 2, 5)
CS_KG1(128, 128, 32, 2, 5)
CS_KG1(64, 64, 64, 2, 5)
CS_KG1(128, 64, 64, 2, 5)
CS_KG1(64, 128, 64, 2, 5)
CS_KG1(64, 64, 64, 4, 5)
CS_KG1(128, 64, 64, 4, 5)
CS_KG1(64, 128, 64, 4, 5)
CS_KG(64, 64, 64, 2)
CS_KG(128, 64, 64, 2)
CS_KG(64, 128, 64, 2)
CS_KG(64, 64, 64, 4)
CS_KG(128, 64, 64, 4)
CS_KG(64, 128, 64, 4)
#undef CS_KG
#undef CS_KG1
#define CS_DEEP1(BM_, BN_, M_)                                                                \
  CS_K(BM_, BN_, CS_CONV_FWD, 32, M_, false, 5) CS_K(BM_, BN_, CS_CONV_DGRAD, 32, M_, false, 5) \
  CS_K(BM_, BN_, CS_CONV_WGRAD, 32, M_, false, 5)
#define CS_DEEP(BM_, BN_) CS_DEEP1(BM_, BN_, 0) CS_DEEP1(BM_, BN_, 2)
CS_DEEP(64, 64)
CS_DEEP(64, 128)
CS_DEEP(128, 64)
#undef CS_DEEP
#undef CS_DEEP1
#undef CS_TILE
#undef CS_MODE
#undef CS_K

int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

}  // namespace

int cs_conv_lg(int v) { return ilog2(v); }

hipError_t cs_conv_splitk_reduce(const CsConvArgs& a, int mode, int splits, hipStream_t stream) {
  return launch_reduce(a, mode, splits, stream);
}

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

bool cs_conv_stage_ok(int stage, int bm, int bn, int bk, bool conv0_fwd) {
  const int maths = ((stage & CS_STAGE_X6) != 0) + ((stage & CS_STAGE_X6S) != 0) + ((stage & CS_STAGE_BF16) != 0) +
                    ((stage & CS_STAGE_F3) != 0);
  if (maths > 1) return false;
  if (stage & CS_STAGE_F3) {  // two fp16 planes: register staging / K-groups; bk 64 up to 128x64 tiles
    stage &= ~CS_STAGE_F3;
    if (conv0_fwd || (stage != CS_STAGE_REGS && stage != CS_STAGE_KG2 && stage != CS_STAGE_KG4)) return false;
    if (bk == 64 && bm == 128 && bn == 128) return false;
  }
  if (stage & CS_STAGE_BF16) {  // bf16 operands (one plane): register staging / K-groups
    stage &= ~CS_STAGE_BF16;
    if (conv0_fwd || (stage != CS_STAGE_REGS && stage != CS_STAGE_KG2 && stage != CS_STAGE_KG4)) return false;
  }
  if (stage & CS_STAGE_X6) {  // split-bf16 math: every staging, except the padded conv0 forward
    if (conv0_fwd) return false;
    stage &= ~CS_STAGE_X6;
  }
  if (stage & CS_STAGE_X6S) {  // split at the LDS store: register staging, bf16 planes within 160 KiB
    stage &= ~CS_STAGE_X6S;
    if (conv0_fwd || (stage != CS_STAGE_REGS && stage != CS_STAGE_KG2 && stage != CS_STAGE_KG4)) return false;
    if (bk == 64 && !(bm == 64 && bn == 64)) return false;
  }
  if (conv0_fwd && stage != CS_STAGE_REGS) return false;
  switch (stage) {
    case CS_STAGE_REGS: return bk != 64 || !(bm == 128 && bn == 128);
    case CS_STAGE_LDS_DMA: return bk == 32;
    case CS_STAGE_LDS_DMA_DEEP: return bk == 32 && (bm + bn) * bk * 4 * 5 < 160 * 1024;
    case CS_STAGE_KG2: return bk >= 32 && !(bk == 64 && bm == 128 && bn == 128);
    case CS_STAGE_KG4: return bk == 64 && !(bm == 128 && bn == 128);
    default: return false;
  }
}

int cs_conv_stat_rows(int K, int bm, int bk, int splits) {
  return cs_conv_effective_splits(K, bk, splits) == 1 ? bm : CS_SPLITK_STAT_ROWS;
}

int cs_conv_ered_rows(int K, int bm, int bk, int splits) {
  return cs_conv_effective_splits(K, bk, splits) == 1 ? bm : CS_SPLITK_STAT_ROWS;
}

int cs_conv_effective_splits(int K, int bk, int splits) {
  const int ks = (K + bk - 1) / bk;
  int s = splits < 1 ? 1 : (splits > ks ? ks : splits);
  const int per = (ks + s - 1) / s;
  return (ks + per - 1) / per;
}

namespace {
// dims, K-step split and size checks; -> effective splits or -1
int prep_gemm(CsConvArgs& a, int mode, int bk, int splits) {
  if (bk != 16 && bk != 32 && bk != 64) return -1;
  if (bk == 64 && mode == CS_CONV_FWD && a.w_oihw) return -1;  // conv0's K = 36
  cs_conv_fill_dims(&a, mode);
  // 32-bit buffer offsets: every operand / output / workspace must stay below 2 GiB
  const int64_t pix = (int64_t)a.B * a.H * a.W;
  const int64_t big = std::max<int64_t>(pix * std::max(a.Cin, a.Cout), (int64_t)a.M * a.N) * 4;
  if (big >= 0x7ffffff0ll) return -1;
  a.total_ksteps = (a.K + bk - 1) / bk;
  splits = cs_conv_effective_splits(a.K, bk, splits);
  a.ksteps_per_split = (a.total_ksteps + splits - 1) / splits;
  if (splits > 1 && a.ws == nullptr) return -1;
  if (splits > 1 && (int64_t)splits * a.M * a.N * 4 >= 0x7ffffff0ll) return -1;
  return splits;
}
}  // namespace

hipError_t cs_conv_gemm(CsConvArgs a, int mode, int bm, int bn, int bk, int splits, hipStream_t stream, int stage) {
  if (!cs_conv_stage_ok(stage, bm, bn, bk, a.w_oihw && mode == CS_CONV_FWD)) return hipErrorInvalidValue;
  splits = prep_gemm(a, mode, bk, splits);
  if (splits < 0) return hipErrorInvalidValue;
  if ((stage & CS_STAGE_F3) && (a.amax_a == nullptr || a.amax_b == nullptr)) return hipErrorInvalidValue;
  a.sgd.P = a.sgd.n > 0 ? (int)std::min<int64_t>(256, (a.sgd.n / 4 + 255) / 256) : 0;
  if (a.fin.cnt != nullptr) {  // last-arriver BN finalize: its statistics must exist in this launch pair
    if (mode == CS_CONV_WGRAD || (mode == CS_CONV_FWD && a.stats == nullptr) ||
        (mode == CS_CONV_DGRAD && a.ered.part == nullptr))
      return hipErrorInvalidValue;
    const int R = cs_conv_stat_rows(a.K, bm, bk, splits), nc = splits > 1 ? 64 : bn;
    if (a.fin.R != R || a.fin.M != a.M || a.fin.T != (a.M + R - 1) / R || a.fin.grp == nullptr) return hipErrorInvalidValue;
    (void)nc;
  }
#define CS_DISPATCH(BM_, BN_, BK_)                                                                       \
  if (bm == BM_ && bn == BN_ && bk == BK_) {                                                             \
    hipError_t e;                                                                                        \
    if (mode == CS_CONV_FWD) e = launch_gemm<BM_, BN_, CS_CONV_FWD, BK_>(a, splits, stage, stream);     \
    else if (mode == CS_CONV_DGRAD) e = launch_gemm<BM_, BN_, CS_CONV_DGRAD, BK_>(a, splits, stage, stream); \
    else e = launch_gemm<BM_, BN_, CS_CONV_WGRAD, BK_>(a, splits, stage, stream);                       \
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
  CS_DISPATCH(64, 64, 64)
  CS_DISPATCH(128, 64, 64)
  CS_DISPATCH(64, 128, 64)
#undef CS_DISPATCH
  return hipErrorInvalidValue;
}
