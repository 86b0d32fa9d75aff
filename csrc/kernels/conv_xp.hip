// 3x3 / stride 1 / pad 1 convolution as implicit GEMM on PRE-SPLIT operands ("XP"):
// fp32-accurate split-bf16 maths (X6: x = h + m + l, six v_mfma_f32_32x32x16_bf16 per
// 32x32x16 product, conv_gemm.hip "X6") where every operand arrives already split into
// three bf16 planes, written by the kernel that produced it (BN apply -> x3, BN backward ->
// dz3, SGD -> w3; cs_split3 for anything else). Replaces ATen conv2d forward / backward-data
// / backward-weight of the reference (nn.Conv2d at master/part1/model.py:18-23; SURVEY.md
// §2.2 N1-N3, §2.4 shapes).
//
// Why pre-split: with the split inside the GEMM (X6 / X6S) every K-step pays the split VALU
// and a register-staged ds_write of 1.5x the fp32 bytes, and the K-loop measured 21-28 %
// MFMA busy (profiles/r2_pmc_conv_ta_lds_mfma.txt) — staging-bound, not MFMA-bound. Here the
// operand images reach LDS by LDS-DMA alone (buffer_load_dwordx4 ... lds: no VGPR staging,
// no ds_write, no split arithmetic in the loop), so the loop is fragment reads + MFMAs:
//
//   stage ring: NB LDS images of one K-step (BK) each; tile t+NB-1 is fetched while tile t is
//   multiplied; one counted vmcnt + one raw s_barrier per K-step (cdna_hip_programming.md §5
//   "Pipelining across barriers").
//
// Plane layout in memory ("P3"): a tensor of n fp32 elements becomes bf16 T3[n/8][3][8] — every
// 8-element chunk is followed by its three planes (h, m, l) as three 16-B slots, so one K-step
// of one operand row (BK elements, all planes) is ONE contiguous 6*BK-byte run (measured: with
// separate planes a BK = 32 row was three 64-B half-line reads and the K-loop stalled on the
// TA/TCP path). Element (flat index f, plane p) sits at 3*(f & ~7) + 8p + (f & 7).
// LDS images hold 16-B slots (8 bf16 of one plane) row by row: a row is its S chunks of each
// plane, slot u = plane * S + chunk XOR-swizzled by the row, so (i) the fragment reads are
// bank-conflict-free and (ii) one 64-slot LDS-DMA instruction fetches whole contiguous P3 rows
// (the swizzle lives on the DMA's per-lane SOURCE address; the LDS side is lane-linear):
//   K-contiguous operand (A of FWD/DGRAD, B of FWD): [row][3 * BK/8], read by ds_read_b128
//   (lane (r, h) of sub-step s takes k = 16s + 8h .. +7 of row r);
//   K-major operand (B of DGRAD, A/B of WGRAD): [k][3 * cols/8], read by two
//   ds_read_b64_tr_b16 (the hardware transpose hands each lane 4 k-values of one column).
// Both give lane-half h the k = 16s + 8h + j order, so A and B fragments agree.
// Blocks: 256*KG threads = KG K-groups of 4 spatial waves (2x2, (BM/2)x(BN/2) each); group g
// multiplies sub-steps [g*NG/KG, (g+1)*NG/KG) of every staged K-step and the groups' partial
// sums meet in the shared epilogue (conv_common.h). Split-K slabs are combined by the same
// deterministic reduce as conv_gemm.hip.
#include <stdlib.h>

#include "conv_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));

template <int MODE>
struct XpTraits;
template <>
struct XpTraits<CS_CONV_FWD> {
  static constexpr bool A_KC = true, B_KC = true;
};
template <>
struct XpTraits<CS_CONV_DGRAD> {
  static constexpr bool A_KC = true, B_KC = false;
};
template <>
struct XpTraits<CS_CONV_WGRAD> {
  static constexpr bool A_KC = false, B_KC = false;
};

// slot swizzles (involutions on the slot index within one row)
template <int S>  // K-contiguous rows of S = BK/8 slots
__device__ __forceinline__ int swz_kc(int row) {
  static_assert(S == 4 || S == 8, "BK 32 or 64");
  return S == 4 ? ((row >> 2) & 3) : ((row >> 1) & 7);
}
template <int S>  // K-major rows of S = cols/8 slots
__device__ __forceinline__ int swz_km(int kr) {
  static_assert(S == 4 || S == 8 || S == 16, "32, 64 or 128 columns");
  return S == 4 ? 0 : (S == 8 ? (((kr >> 1) & 1) << 2) : ((kr & 3) << 2));
}

template <int BM, int BN, int MODE, int BK, int KG, int NBX = 0>
struct XpTile {
  static constexpr int NT = 256 * KG;
  static constexpr bool A_KC = XpTraits<MODE>::A_KC, B_KC = XpTraits<MODE>::B_KC;
  static constexpr int SA = 3 * BM * BK / 8, SB = 3 * BN * BK / 8;  // 16-B slots per operand image
  static constexpr int IA = SA / NT, IB = SB / NT;                  // LDS-DMA instructions per wave per stage
  static_assert(SA % NT == 0 && SB % NT == 0, "operand image must split evenly over the block's waves");
  static constexpr int NI = IA + IB;
  static constexpr int STAGE = (SA + SB) * 16;  // bytes per ring stage
  static constexpr int NB_FIT = (147456 / STAGE) > 6 ? 6 : (147456 / STAGE);
  static constexpr int NB = NBX > 0 ? NBX : NB_FIT;  // NBX: a shallower ring so 2+ blocks share a CU
  static_assert(NB >= 2, "one stage must fit twice in LDS");
  static_assert((NB - 2) * NI <= 63, "vmcnt range");
  static constexpr int RM = BM / 64, RN = BN / 64, WM = BM / 2, WN = BN / 2;
  static constexpr int NG = BK / 16, NGK = NG / KG;  // MFMA sub-steps per K-step / per K-group
  static_assert(NGK >= 1 && NG % KG == 0, "K-groups must split the sub-steps");
};

// Per-lane LDS-DMA offsets of one operand image: instruction i of this wave fills slot
// (wave * I + i) * 64 + lane. `fix` = fixed element offset, `msk` = tap mask / flags.
template <int BM, int BN, int MODE, int BK, int KG>
struct XpLoader {
  using T = XpTile<BM, BN, MODE, BK, KG>;
  rsrc_t ra, rb;
  int afix[T::IA], bfix[T::IB];
  unsigned amsk[T::IA], bmsk[T::IB];
  int akr[T::A_KC ? 1 : T::IA], bkr[T::B_KC ? 1 : T::IB];  // K-major: the slot's k-row in the K-step

  // (plane, row-or-k-row, 8-element chunk) of slot s of an operand image over R rows/cols
  template <bool KC, int R>
  __device__ static void slot(int s, int& p, int& row, int& c) {
    constexpr int S = KC ? BK / 8 : R / 8;
    row = s / (3 * S);
    int sw;
    if constexpr (KC) sw = swz_kc<S>(row);
    else sw = swz_km<S>(row);
    const int u = (s - row * (3 * S)) ^ sw;
    p = u / S;
    c = u - p * S;
  }

  __device__ void init(const CsConvArgs& a, int m0, int n0) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < T::IA; ++i) {
      int p, row, c;
      slot<T::A_KC, BM>((wv * T::IA + i) * 64 + lane, p, row, c);
      if constexpr (MODE == CS_CONV_FWD || MODE == CS_CONV_DGRAD) {  // A[m = pixel][k = (tap, ch)]
        const int m = m0 + row;
        const int w = m & (a.W - 1), h = (m >> a.lgW) & (a.H - 1);
        const int C = MODE == CS_CONV_FWD ? a.Cin : a.Cout;
        amsk[i] = m < a.M ? tap_mask(h, w, a.H, a.W, MODE == CS_CONV_FWD ? 1 : -1) : 0u;
        afix[i] = 3 * (m * C + 8 * c) + 8 * p;
      } else {  // WGRAD A[m = cout][k = pixel] from dz3 [pixel][cout]: k-row `row`, cols m0 + 8c
        const int m = m0 + 8 * c;
        amsk[i] = m < a.M ? 1u : 0u;
        akr[i] = row;
        afix[i] = 3 * (row * a.Cout + m) + 8 * p;
      }
    }
#pragma unroll
    for (int i = 0; i < T::IB; ++i) {
      int p, row, c;
      slot<T::B_KC, BN>((wv * T::IB + i) * 64 + lane, p, row, c);
      if constexpr (MODE == CS_CONV_FWD) {  // B[n = cout][k]: w3 [Cout][K]
        const int n = n0 + row;
        bmsk[i] = n < a.N ? 1u : 0u;
        bfix[i] = 3 * (n * a.K + 8 * c) + 8 * p;
      } else if constexpr (MODE == CS_CONV_DGRAD) {  // B[k = (tap, cout)][n = cin]: w3 [Cout][9][Cin]
        const int n = n0 + 8 * c;
        bmsk[i] = n < a.N ? 1u : 0u;
        bkr[i] = row;
        bfix[i] = 3 * (row * 9 * a.Cin + n) + 8 * p;
      } else {  // WGRAD B[k = pixel][n = (tap, cin)] = x3[pixel + tap shift][cin]
        const int nn = n0 + 8 * c;
        const int tap = nn >> a.lgCin, ci = nn & (a.Cin - 1);
        const int t3 = tap / 3, dh = t3 - 1, dw = tap - 3 * t3 - 1;
        bmsk[i] = (nn < a.N && tap < 9) ? (1u | ((unsigned)tap << 4)) : 0u;
        bkr[i] = row;
        bfix[i] = 3 * ((dh * a.W + dw) * a.Cin + ci) + 8 * p;
      }
    }
    const int64_t pix = (int64_t)a.B * a.H * a.W;
    if constexpr (MODE == CS_CONV_FWD) {
      ra = make_rsrc(a.x3, 6 * pix * a.Cin);
      rb = make_rsrc(a.w3, 6 * (int64_t)a.Cout * 9 * a.Cin);
    } else if constexpr (MODE == CS_CONV_DGRAD) {
      ra = make_rsrc(a.dz3, 6 * pix * a.Cout);
      rb = make_rsrc(a.w3, 6 * (int64_t)a.Cout * 9 * a.Cin);
    } else {
      ra = make_rsrc(a.dz3, 6 * pix * a.Cout);
      rb = make_rsrc(a.x3, 6 * pix * a.Cin);
    }
  }

  // byte offset (or kOOB) of this lane's slot of A instruction i / B instruction i, K-step at k0
  __device__ __forceinline__ int a_off(const CsConvArgs& a, int k0, int i) const {
    if constexpr (MODE == CS_CONV_FWD || MODE == CS_CONV_DGRAD) {
      const int lgC = MODE == CS_CONV_FWD ? a.lgCin : a.lgCout;
      const int tap = k0 >> lgC, ch0 = k0 & ((1 << lgC) - 1);
      const int t3 = tap / 3, dh = t3 - 1, dw = tap - 3 * t3 - 1;
      const int sh = MODE == CS_CONV_FWD ? (dh * a.W + dw) : -(dh * a.W + dw);
      return ((amsk[i] >> tap) & 1u) ? (afix[i] + 3 * ((sh << lgC) + ch0)) * 2 : kOOB;
    } else {
      return (amsk[i] && k0 + akr[i] < a.K) ? (afix[i] + 3 * (k0 << a.lgCout)) * 2 : kOOB;
    }
  }
  __device__ __forceinline__ int b_off(const CsConvArgs& a, int k0, int i) const {
    if constexpr (MODE == CS_CONV_FWD) {
      return bmsk[i] ? (bfix[i] + 3 * k0) * 2 : kOOB;
    } else if constexpr (MODE == CS_CONV_DGRAD) {
      const int tap = k0 >> a.lgCout, co0 = k0 & (a.Cout - 1);
      return bmsk[i] ? (bfix[i] + 3 * ((co0 * 9 + tap) << a.lgCin)) * 2 : kOOB;
    } else {
      const int p = k0 + bkr[i];
      const int w = p & (a.W - 1), h = (p >> a.lgW) & (a.H - 1);
      const int tap = (int)(bmsk[i] >> 4), t3 = tap / 3;
      const int hh = h + t3 - 1, ww = w + (tap - 3 * t3) - 1;
      const bool ok = (bmsk[i] & 1u) && p < a.K && (unsigned)hh < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      return ok ? (bfix[i] + 3 * (p << a.lgCin)) * 2 : kOOB;
    }
  }

  // one ring stage: every wave's share of the A and B images, K-step at k0
  __device__ __forceinline__ void issue(const CsConvArgs& a, int k0, char* stage) const {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    char* As = stage;
    char* Bs = stage + T::SA * 16;
#pragma unroll
    for (int i = 0; i < T::IA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ra, (__attribute__((address_space(3))) void*)(As + (wv * T::IA + i) * 1024), 16, a_off(a, k0, i), 0, 0, 0);
#pragma unroll
    for (int i = 0; i < T::IB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (__attribute__((address_space(3))) void*)(Bs + (wv * T::IB + i) * 1024), 16, b_off(a, k0, i), 0, 0, 0);
  }
};

// Fragments (3 planes) of sub-step s for R/32 32-wide groups starting at `base` of one image.
template <bool KC, int R, int BK, int NR>
__device__ __forceinline__ void xp_frags(const char* img, int base, int s, int lane, bf16x8 (&f)[3][NR]) {
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      if constexpr (KC) {
        constexpr int S = BK / 8;
        const int row = base + i * 32 + (lane & 31);
        const int kc = 2 * s + (lane >> 5);
        const int sl = row * (3 * S) + ((p * S + kc) ^ swz_kc<S>(row));
        f[p][i] = *reinterpret_cast<const bf16x8*>(img + sl * 16);
      } else {
        constexpr int S = R / 8;
        const int grp = lane >> 4, l16 = lane & 15;
        const int col = base + i * 32 + 16 * (grp & 1) + 4 * (l16 & 3);
        const int kr = 16 * s + 8 * (grp >> 1) + (l16 >> 2);
        const int c8 = col >> 3, in = (col & 7) * 2;
        const int lo = (kr * (3 * S) + ((p * S + c8) ^ swz_km<S>(kr))) * 16 + in;
        const int hi = ((kr + 4) * (3 * S) + ((p * S + c8) ^ swz_km<S>(kr + 4))) * 16 + in;
        const i16x4 vlo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(img + lo));
        const i16x4 vhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(img + hi));
        f[p][i] = __builtin_shufflevector(__builtin_bit_cast(bf16x4, vlo), __builtin_bit_cast(bf16x4, vhi), 0, 1, 2, 3,
                                          4, 5, 6, 7);
      }
    }
}

// six split-bf16 products of one sub-step, small terms first (conv_gemm.hip mma_x6f order)
template <int RM, int RN>
__device__ __forceinline__ void xp_mma(const bf16x8 (&fa)[3][RM], const bf16x8 (&fb)[3][RN], f32x16 (&acc)[RM][RN]) {
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[1][j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[2][j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2][i], fb[0][j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[1][j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[0][j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
    }
}

// counted wait: tile t landed once at most `ahead` newer stages are outstanding (in-order retire)
template <int NI, int MAXA>
__device__ __forceinline__ void wait_ahead(int ahead) {
  if constexpr (MAXA >= 4) {
    if (ahead >= 4) { wait_vmcnt<4 * NI>(); return; }
  }
  if constexpr (MAXA >= 3) {
    if (ahead == 3) { wait_vmcnt<3 * NI>(); return; }
  }
  if constexpr (MAXA >= 2) {
    if (ahead == 2) { wait_vmcnt<2 * NI>(); return; }
  }
  if constexpr (MAXA >= 1) {
    if (ahead == 1) { wait_vmcnt<NI>(); return; }
  }
  wait_vmcnt<0>();
}

// PROBE (measurement only, wrong numbers; CS_XP_PROBE): 1 = no LDS-DMA in the K-loop (fragment
// reads + MFMAs + barriers on stale stages), 2 = no MFMAs (operands kept live), 3 = no fragment
// reads and no MFMAs (DMA + barriers only)
template <int BM, int BN, int MODE, int BK, int KG, int NBX, int PROBE = 0>
__device__ __forceinline__ void xp_body(const CsConvArgs& a, const int tile, const int split, const int nsplit,
                                        char* smem) {
  using T = XpTile<BM, BN, MODE, BK, KG, NBX>;
  constexpr int NB = T::NB;
  const int ntn = (a.N + BN - 1) / BN;
  const int mt = tile / ntn, nt = tile - mt * ntn;
  const int ks_begin = split * a.ksteps_per_split;
  const int ks_end = min(ks_begin + a.ksteps_per_split, a.total_ksteps);
  const int nks = ks_end - ks_begin;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int kg = wid >> 2, wsp = wid & 3, wm = wsp >> 1, wn = wsp & 1;

  f32x16 acc[T::RM][T::RN];
#pragma unroll
  for (int i = 0; i < T::RM; ++i)
#pragma unroll
    for (int j = 0; j < T::RN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  XpLoader<BM, BN, MODE, BK, KG> ld;
  ld.init(a, mt * BM, nt * BN);
#pragma unroll
  for (int p = 0; p < NB - 1; ++p)
    if (p < nks) ld.issue(a, (ks_begin + p) * BK, smem + p * T::STAGE);
  int cur = 0;
  for (int t = 0; t < nks; ++t) {
    wait_ahead<T::NI, NB - 2>(min(NB - 2, nks - 1 - t));
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (PROBE != 1 && t + NB - 1 < nks) {
      const int nx = cur == 0 ? NB - 1 : cur - 1;  // (t + NB - 1) % NB: the stage read at step t-1
      ld.issue(a, (ks_begin + t + NB - 1) * BK, smem + nx * T::STAGE);
    }
    const char* As = smem + cur * T::STAGE;
    const char* Bs = As + T::SA * 16;
    if constexpr (PROBE != 3) {
      bf16x8 fa[2][3][T::RM], fb[2][3][T::RN];
      const int s0 = kg * T::NGK;
      xp_frags<T::A_KC, BM, BK, T::RM>(As, wm * T::WM, s0, lane, fa[0]);
      xp_frags<T::B_KC, BN, BK, T::RN>(Bs, wn * T::WN, s0, lane, fb[0]);
#pragma unroll
      for (int s = 0; s < T::NGK; ++s) {
        if (s + 1 < T::NGK) {
          xp_frags<T::A_KC, BM, BK, T::RM>(As, wm * T::WM, s0 + s + 1, lane, fa[(s + 1) & 1]);
          xp_frags<T::B_KC, BN, BK, T::RN>(Bs, wn * T::WN, s0 + s + 1, lane, fb[(s + 1) & 1]);
        }
        if constexpr (PROBE == 2) {
#pragma unroll
          for (int q = 0; q < 3; ++q) {
#pragma unroll
            for (int i = 0; i < T::RM; ++i) asm volatile("" ::"v"(fa[s & 1][q][i]));
#pragma unroll
            for (int j = 0; j < T::RN; ++j) asm volatile("" ::"v"(fb[s & 1][q][j]));
          }
        } else {
          xp_mma<T::RM, T::RN>(fa[s & 1], fb[s & 1], acc);
        }
      }
    }
    cur = cur == NB - 1 ? 0 : cur + 1;
  }
  __syncthreads();  // every wave's fragment reads are done before the epilogue reuses LDS
  conv_epilogue<BM, BN, MODE, KG>(a, acc, tile, split, nsplit, reinterpret_cast<float*>(smem));
}

template <int BM, int BN, int MODE, int BK, int KG, int NBX, int PROBE = 0>
__global__ __launch_bounds__(256 * KG) void conv_xp_kernel(CsConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char xsm[];
  const int ntiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const int nsplit = (a.total_ksteps + a.ksteps_per_split - 1) / a.ksteps_per_split;
  const int ng = ntiles * nsplit, lin = blockIdx.x;
  if (lin >= ng) {  // appended BN-backward reduce blocks (conv_gemm.hip conv_gemm_kernel)
    if (a.red.pool) cs_bn::bn_red_body<true>(a.red, lin - ng, a.red.P, reinterpret_cast<float*>(xsm));
    else cs_bn::bn_red_body<false>(a.red, lin - ng, a.red.P, reinterpret_cast<float*>(xsm));
    return;
  }
  xp_body<BM, BN, MODE, BK, KG, NBX, PROBE>(a, cs::xcd_remap(lin % ntiles, ntiles), lin / ntiles, nsplit, xsm);
}

// ---------------------------------------------------------------- producers
// x (fp32, n elements, n % 8 == 0) -> P3 chunks [n/8][3][8] bf16: x = h + m + l up to 2^-26 |x|
// (round-to-nearest at each level; conv_gemm.hip "X6")
__device__ __forceinline__ void split8(const float4 v0, const float4 v1, bf16x8& h, bf16x8& m, bf16x8& l) {
  const float x[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 hj = (__bf16)x[j];
    const float r = x[j] - (float)hj;
    const __bf16 mj = (__bf16)r;
    h[j] = hj;
    m[j] = mj;
    l[j] = (__bf16)(r - (float)mj);
  }
}

__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ x, __bf16* __restrict__ out,
                                                     int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const float4 v0 = reinterpret_cast<const float4*>(x)[2 * i];
    const float4 v1 = reinterpret_cast<const float4*>(x)[2 * i + 1];
    bf16x8 h, m, l;
    split8(v0, v1, h, m, l);
    *reinterpret_cast<bf16x8*>(out + 24 * i) = h;
    *reinterpret_cast<bf16x8*>(out + 24 * i + 8) = m;
    *reinterpret_cast<bf16x8*>(out + 24 * i + 16) = l;
  }
}

template <int BM, int BN, int MODE, int BK, int KG, int NBX, int PROBE = 0>
hipError_t launch_xp(const CsConvArgs& a, int splits, hipStream_t stream) {
  using T = XpTile<BM, BN, MODE, BK, KG, NBX>;
  const int ntiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  size_t lds = (size_t)T::NB * T::STAGE;
  const size_t red = (size_t)(KG - 1) * 4 * T::RM * T::RN * 16 * 64 * sizeof(float);
  if (red > lds) lds = red;
  if (a.red.P > 0) lds = std::max(lds, cs_bn_red_lds(a.red.C));
  hipLaunchKernelGGL((conv_xp_kernel<BM, BN, MODE, BK, KG, NBX, PROBE>), dim3(ntiles * splits + a.red.P), dim3(256 * KG), lds,
                     stream, a);
  return hipGetLastError();
}

template <int BM, int BN, int BK, int KG, int NBX>
hipError_t launch_xp_mode(const CsConvArgs& a, int mode, int splits, hipStream_t stream) {
  if (mode == CS_CONV_FWD) return launch_xp<BM, BN, CS_CONV_FWD, BK, KG, NBX>(a, splits, stream);
  if (mode == CS_CONV_DGRAD) return launch_xp<BM, BN, CS_CONV_DGRAD, BK, KG, NBX>(a, splits, stream);
  return launch_xp<BM, BN, CS_CONV_WGRAD, BK, KG, NBX>(a, splits, stream);
}

}  // namespace

hipError_t cs_split3(const float* x, uint16_t* out, int64_t n, hipStream_t stream) {
  if (n % 8 != 0) return hipErrorInvalidValue;
  const int64_t n8 = n / 8;
  int64_t blocks = (n8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(split3_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x, reinterpret_cast<__bf16*>(out),
                     n8);
  return hipGetLastError();
}

bool cs_conv_xp_ok(int bm, int bn, int bk, int kg, int nb) {
  if ((bm != 64 && bm != 128) || (bn != 64 && bn != 128) || (bk != 32 && bk != 64) || (kg != 1 && kg != 2))
    return false;
  if (bk == 64 && bm == 128 && bn == 128) return false;  // one stage would not fit twice
  const int nt = 256 * kg;
  if (!((3 * bm * bk / 8) % nt == 0 && (3 * bn * bk / 8) % nt == 0 && (bk / 16) % kg == 0)) return false;
  // shallow rings (two blocks per CU): 64x64 bk32 with 2 or 3 stages, 128x64 / 64x128 bk32 with 2
  if (nb == 0) return true;
  if (kg != 1 || bk != 32) return false;
  return (bm == 64 && bn == 64 && (nb == 2 || nb == 3)) || (bm + bn == 192 && nb == 2);
}

hipError_t cs_conv_xp(CsConvArgs a, int mode, int bm, int bn, int bk, int splits, int kg, int nb, hipStream_t stream) {
  if (!cs_conv_xp_ok(bm, bn, bk, kg, nb)) return hipErrorInvalidValue;
  cs_conv_fill_dims(&a, mode);
  const int64_t pix = (int64_t)a.B * a.H * a.W;
  // operand planes: 3 planes per tensor, 32-bit byte offsets in one buffer descriptor each
  if (a.w_oihw || a.Cin < 64 || a.Cout < 64) return hipErrorInvalidValue;
  const bool needx = mode != CS_CONV_DGRAD, needz = mode != CS_CONV_FWD, needw = mode != CS_CONV_WGRAD;
  if ((needx && (a.x3 == nullptr || 6 * pix * a.Cin >= 0x7ffffff0ll)) ||
      (needz && (a.dz3 == nullptr || 6 * pix * a.Cout >= 0x7ffffff0ll)) ||
      (needw && (a.w3 == nullptr || 6 * (int64_t)a.Cout * 9 * a.Cin >= 0x7ffffff0ll)))
    return hipErrorInvalidValue;
  if ((int64_t)a.M * a.N * 4 >= 0x7ffffff0ll) return hipErrorInvalidValue;
  a.total_ksteps = (a.K + bk - 1) / bk;
  splits = cs_conv_effective_splits(a.K, bk, splits);
  a.ksteps_per_split = (a.total_ksteps + splits - 1) / splits;
  if (splits > 1 && (a.ws == nullptr || (int64_t)splits * a.M * a.N * 4 >= 0x7ffffff0ll)) return hipErrorInvalidValue;
  a.counters = nullptr;
  hipError_t e = hipErrorInvalidValue;
  static const int probe = [] {
    const char* v = getenv("CS_XP_PROBE");
    return v ? atoi(v) : 0;
  }();
  if (probe > 0 && mode == CS_CONV_FWD && kg == 2 && nb == 0 && bm == bn && bm + bk == 128) {
#define CS_XPP(BM_, BK_, P_)                                                                                 \
  if (bm == BM_ && probe == P_) e = launch_xp<BM_, BM_, CS_CONV_FWD, BK_, 2, 0, P_>(a, splits, stream);
    CS_XPP(64, 64, 1) CS_XPP(64, 64, 2) CS_XPP(64, 64, 3) CS_XPP(128, 32, 1) CS_XPP(128, 32, 2) CS_XPP(128, 32, 3)
#undef CS_XPP
    if (e != hipSuccess || splits == 1) return e;
    return cs_conv_splitk_reduce(a, mode, splits, stream);
  }
#define CS_XP(BM_, BN_, BK_, KG_, NB_)                                  \
  if (bm == BM_ && bn == BN_ && bk == BK_ && kg == KG_ && nb == NB_) \
    e = launch_xp_mode<BM_, BN_, BK_, KG_, NB_>(a, mode, splits, stream);
  CS_XP(64, 64, 32, 1, 0)
  CS_XP(128, 64, 32, 1, 0)
  CS_XP(64, 128, 32, 1, 0)
  CS_XP(128, 128, 32, 1, 0)
  CS_XP(64, 64, 64, 1, 0)
  CS_XP(128, 64, 64, 1, 0)
  CS_XP(64, 128, 64, 1, 0)
  CS_XP(128, 128, 32, 2, 0)
  CS_XP(64, 64, 64, 2, 0)
  CS_XP(128, 64, 64, 2, 0)
  CS_XP(64, 128, 64, 2, 0)
  CS_XP(64, 64, 32, 1, 2)
  CS_XP(64, 64, 32, 1, 3)
  CS_XP(128, 64, 32, 1, 2)
  CS_XP(64, 128, 32, 1, 2)
#undef CS_XP
  if (e != hipSuccess || splits == 1) return e;
  return cs_conv_splitk_reduce(a, mode, splits, stream);
}
