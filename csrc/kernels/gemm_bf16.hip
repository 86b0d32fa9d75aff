// bf16 GEMM on the gfx950 matrix cores for the decoder-LM projections and the ResNet 1x1 convs:
//   C[M, N] (=, +=) sum_k A(m, k) B(n, k)      (bf16 operands, fp32 accumulate)
// Each operand is stored either K-major ([rows][K], the reduction contiguous) or M-major
// ([K][rows], the output dimension contiguous), which covers all three GEMMs of a linear layer
// with no transpose pass: y = x W^T (A = x [T][in] K-major, B = W [out][in] K-major),
// dx = dy W (A = dy K-major, B = W [out][in] read M-major), dW = dy^T x (both M-major: tokens are
// the reduction). A channels-last 1x1 conv is the same three products. Output bf16 or fp32
// (optionally accumulated into).
//
// MI355X design (cdna_hip_programming.md §5, 'The 256² 8-phase template' and §5.5 T1-T5, T10):
//  - 256 x 256 output tile per workgroup, BK = 64, 8 waves as 2 (M) x 4 (N): 128 x 64 per wave as
//    8 x 4 tiles of v_mfma_f32_16x16x32_bf16 (128 accumulator registers). The MFMA's A operand is
//    the B-matrix tile and its B operand the A-matrix tile, so the accumulator's 4 registers are 4
//    consecutive output COLUMNS of one row: one 8-byte (bf16) / 16-byte (fp32) store per register
//    quad instead of four scattered 2-byte stores.
//  - Operands reach LDS by LDS-DMA (buffer_load ... lds, 16 bytes per lane): no staging registers,
//    no ds_write pass. The DMA writes 1 KiB lane-linearly per wave-instruction, so every LDS
//    swizzle is applied to the per-lane SOURCE address (guide §5.4 rule 21). Out-of-range rows,
//    columns and k get an out-of-range buffer offset and land as zeros: no padding anywhere.
//    K-major image: [256 rows][64 k], 128-byte rows, 16-byte chunk c of row r at c ^ ((r >> 1) & 7)
//    -> the 16 lanes of a ds_read_b128 group (16 consecutive rows, one chunk) hit 16 distinct
//    16-byte bank slots. M-major image: 2 halves x [64 k][128 columns], 256-byte k rows, chunk c of
//    k row kr at c ^ 2((kr & 3) | ((kr >> 3) & 1) << 2), read with ds_read_b64_tr_b16 (T10): the
//    8 k rows one 32-lane half reads land on 8 distinct 32-byte bank slots.
//  - Two LDS buffers (2 x 64 KiB, one workgroup per CU). Each K-tile is computed in 4 phases, one
//    per quadrant of the wave tile (64 rows x 32 cols, 16 MFMAs). Phase p of tile t first waits
//    (counted vmcnt) for the half-tiles it reads, passes a raw s_barrier, then stages one
//    half-tile of tile t + 1 (2 DMA instructions per wave) and runs its quadrant. Quadrant order
//    (A0 B0) (A0 B1) (A1 B1) (A1 B0) against staging order A0 B0 B1 A1 (A_h = the 128 A rows
//    with (r >> 6) & 1 == h, the rows every wave's quadrant h reads; B_h likewise by (r >> 5) & 1)
//    keeps one operand half in registers from phase to phase (28 fragment reads per K-tile, not
//    48), and every phase needs at most the half-tile staged 2 phases before it: vmcnt(4) = 2
//    half-tiles stay in flight across each barrier and every DMA has >= 3 phases (~1500 clocks)
//    to land. Nothing drains the load queue inside the K loop (guide T3+T4).
//    WAR: phase p stages into the buffer tile t - 1 read; its last read of that half-tile was in
//    tile t - 1, and every wave has passed phase p's barrier after consuming those reads.
//    RAW: the waiting wave's own vmcnt retires its DMAs; the barrier after it orders every other
//    wave's (guide: 'Read a staged buffer one phase AFTER the wait that retires it').
//  - s_setprio(1) around each MFMA cluster keeps hipcc from moving MFMAs across the barriers
//    (guide T5). One __shared__ array for all LDS (guide §5 'Projection GEMM' item 4(a)).
//  - XCD-aware tile order (T1, the bijective remap) then GROUP_M = 8 tile grouping: the 32 blocks
//    an XCD runs at once cover 8 row tiles x 4 column tiles and share their operand panels in
//    that XCD's L2.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "launchers.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

constexpr int kTile = 256, kBK = 64, kThreads = 512;
constexpr int kImg = kTile * kBK * 2;  // bytes of one [256][64] bf16 operand image
constexpr int kBuf = 2 * kImg;         // A image + B image
constexpr int kOOB = 0x7ffffff0;

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

// K-major operand, memory [rows][K] (row stride ld elements), tile rows [row0, row0 + 256).
// Half-tile h = the rows r with (r >> HS) & 1 == h (HS = 6 for A, 5 for B) = 16 groups of 8
// consecutive rows; wave w issues groups 2w and 2w + 1. The per-lane byte offsets of the 4 DMA
// instructions a wave issues per K-tile are fixed but for + 2 k0: computed once (kOOB for rows
// past the end).
template <int HS>
struct OpK {
  static constexpr bool kRowRead = true;
  __amdgpu_buffer_rsrc_t rs;
  int off[2][2];  // [half][instruction] at k0 = 0
  int kch[2][2];  // the lane's k offset (elements) within the K-tile
  int lds[2][2];  // image byte offset of the instruction's first row (wave-uniform)
  int K;
  // base: element (row0, 0); nrows: valid rows from row0
  __device__ OpK(const __bf16* base, int64_t ld, int nrows, int K_) : K(K_) {
    const int64_t bytes = nrows > 0 ? (int64_t)(nrows - 1) * ld * 2 + (int64_t)K_ * 2 : 0;
    rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(base), (short)0,
                                           (int)(bytes < 0x7fffffff ? bytes : 0x7fffffff), 0x00020000);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    constexpr int RUN = 1 << HS;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int pr0 = 8 * (2 * wv + i);  // first row of the group within the half
        const int r0 = (pr0 / RUN) * 2 * RUN + h * RUN + (pr0 % RUN);
        const int r = r0 + (lane >> 3), kc = ((lane & 7) ^ swz(r)) << 3;
        kch[h][i] = kc;
        off[h][i] = r < nrows ? r * (int)(ld * 2) + kc * 2 : kOOB;
        lds[h][i] = r0 * 128;
      }
  }
  template <bool KTAIL>
  __device__ __forceinline__ void stage(char* img, int h, int k0) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int o = off[h][i] == kOOB ? kOOB : off[h][i] + 2 * k0;
      if constexpr (KTAIL) o = k0 + kch[h][i] < K ? o : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(img + lds[h][i]), 16, o,
                                               0, 0, 0);
    }
  }
  // MFMA operand fragment of the 16-row subtile starting at tile row r0, k-step s (32 k): lane l
  // gets row r0 + (l & 15), k = 32 s + 8 (l >> 4) + j
  __device__ __forceinline__ bf16x8 frag(const char* img, int r0, int s, int lane) const {
    const int r = r0 + (lane & 15), ch = s * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + r * 128 + ((ch ^ swz(r)) << 4));
  }
};

__device__ __forceinline__ int xs(int kr) { return 2 * ((kr & 3) | (((kr >> 3) & 1) << 2)); }

// M-major operand, memory [K][cols] (row stride ld elements), tile columns [col0, col0 + 256)
// contiguous in memory. Image: 2 halves x [64 k][128 local columns]; half h = the tile columns c
// with (c >> HS) & 1 == h, local column lc = (c >> (HS + 1)) << HS | (c & (RUN - 1)). A DMA
// instruction fills 4 k rows of one half (wave w: k rows 8w .. 8w + 7 of each half). The buffer
// resource is re-based at every K-tile (scalar work), so offsets stay 32-bit for any K and k
// rows past K fall outside its range (zeros).
template <int HS>
struct OpM {
  static constexpr bool kRowRead = false;
  const __bf16* base;  // element (0, col0)
  int64_t ld;
  int ncols, K;
  int off[2][2];
  int lds[2][2];
  __device__ OpM(const __bf16* base_, int64_t ld_, int ncols_, int K_) : base(base_), ld(ld_), ncols(ncols_), K(K_) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    constexpr int RUN = 1 << HS;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int kr0 = 4 * (2 * wv + i), kr = kr0 + (lane >> 4);
        const int lc = ((lane & 15) ^ xs(kr)) << 3;
        const int c = ((lc >> HS) << (HS + 1)) | (h << HS) | (lc & (RUN - 1));
        off[h][i] = c < ncols ? kr * (int)(ld * 2) + c * 2 : kOOB;
        lds[h][i] = h * (kImg / 2) + kr0 * 256;
      }
  }
  template <bool KTAIL>
  __device__ __forceinline__ void stage(char* img, int h, int k0) const {
    const int rows = K - k0 < kBK ? K - k0 : kBK;
    const int bytes = (int)((int64_t)(rows - 1) * ld * 2 + (int64_t)ncols * 2);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(base + (int64_t)k0 * ld), (short)0, bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(img + lds[h][i]), 16,
                                               off[h][i], 0, 0, 0);
  }
  // the same fragment as OpK::frag, by two transposed reads (T10): lane 4q + p of group g supplies
  // k row 32 s + 8 g + q (then + 4), columns c0 + 4p .. + 3; lane i of the group receives column
  // c0 + i of those 4 k rows
  __device__ __forceinline__ bf16x8 frag(const char* img, int c0, int s, int lane) const {
    constexpr int RUN = 1 << HS;
    const int h = (c0 >> HS) & 1, lc0 = ((c0 >> (HS + 1)) << HS) | (c0 & (RUN - 1));
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int kr = s * 32 + 8 * g + q, ch = (lc0 >> 3) + (p >> 1);
    const char* a0 = img + h * (kImg / 2) + kr * 256 + ((ch ^ xs(kr)) << 4) + 8 * (p & 1);
    // inline asm: the builtin form makes hipcc wait vmcnt(0) (all LDS-DMA) before every
    // transposed read; the quadrant waits lgkmcnt(0) for these itself (see quadrant())
    const unsigned ad = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)a0;
    i32x2 lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(ad) : "memory");
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:1024" : "=v"(hi) : "v"(ad) : "memory");
    const bf16x4 blo = __builtin_bit_cast(bf16x4, lo), bhi = __builtin_bit_cast(bf16x4, hi);
    return __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
}

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

struct Tile {
  f32x4 acc[8][4];
};

// fragments of the wave tile's A rows of half MH (4 subtiles) / B rows of half NH (2 subtiles)
// for both 32-deep k-steps of the K-tile in `buf`
template <int MH, class SA>
__device__ __forceinline__ void load_a(bf16x8 (&fa)[4][2], const char* buf, const SA& sa, int wr, int lane) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i][s] = sa.frag(buf, wr * 128 + MH * 64 + i * 16, s, lane);
}
template <int NH, class SB>
__device__ __forceinline__ void load_b(bf16x8 (&fb)[2][2], const char* buf, const SB& sb, int wc, int lane) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int q = 0; q < 2; ++q) fb[q][s] = sb.frag(buf + kImg, wc * 64 + NH * 32 + q * 16, s, lane);
}

// quadrant (MH, NH) of the wave tile: 16 MFMAs on fragments already in registers
template <int MH, int NH, bool ASM_READS>
__device__ __forceinline__ void mma(Tile& t, const bf16x8 (&fa)[4][2], const bf16x8 (&fb)[2][2]) {
  if constexpr (ASM_READS) {
    // inline-asm transposed reads are invisible to hipcc's waitcnt insertion (and an asm wait
    // does not order the register-only MFMAs after it without the sched_barrier: guide §5.4 rule 18)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        t.acc[MH * 4 + i][NH * 2 + q] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[q][s], fa[i][s], t.acc[MH * 4 + i][NH * 2 + q], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

// one K-tile: 4 phases, quadrant order (A0 B0) (A0 B1) (A1 B1) (A1 B0), so consecutive phases share
// one operand half in registers: 28 fragment reads per K-tile instead of 48 (LDS read bandwidth,
// not the MFMA, bounds the 16x16x32 wave tile otherwise). STAGE: tile k0n is staged into `nxt`
// meanwhile, in the order its phases need it (A0 B0 B1 A1); W: vmcnt before phases 1-3.
template <bool STAGE, bool KTAIL, int W, class SA, class SB>
__device__ __forceinline__ void ktile(Tile& t, const char* cur, char* nxt, const SA& sa, const SB& sb, int k0n, int wr,
                                      int wc, int lane) {
  constexpr bool ASM = !SA::kRowRead || !SB::kRowRead;
  bf16x8 fa[4][2], fb[2][2];
  wait_vm<W>();
  barrier();
  if constexpr (STAGE) sa.template stage<KTAIL>(nxt, 0, k0n);
  load_a<0>(fa, cur, sa, wr, lane);
  load_b<0>(fb, cur, sb, wc, lane);
  mma<0, 0, ASM>(t, fa, fb);
  wait_vm<W>();
  barrier();
  if constexpr (STAGE) sb.template stage<KTAIL>(nxt + kImg, 0, k0n);
  load_b<1>(fb, cur, sb, wc, lane);
  mma<0, 1, ASM>(t, fa, fb);
  wait_vm<W>();
  barrier();
  if constexpr (STAGE) sb.template stage<KTAIL>(nxt + kImg, 1, k0n);
  load_a<1>(fa, cur, sa, wr, lane);
  mma<1, 1, ASM>(t, fa, fb);
  barrier();
  if constexpr (STAGE) sa.template stage<KTAIL>(nxt, 1, k0n);
  load_b<0>(fb, cur, sb, wc, lane);
  mma<1, 0, ASM>(t, fa, fb);
}

template <bool KM, int HS>
struct Op;
template <int HS>
struct Op<true, HS> {
  using T = OpK<HS>;
  // base: the matrix; stored [rows][K]
  __device__ static T make(const __bf16* p, int64_t ld, int r0, int rows, int K) {
    return T(p + (int64_t)r0 * ld, ld, rows - r0 < kTile ? rows - r0 : kTile, K);
  }
};
template <int HS>
struct Op<false, HS> {
  using T = OpM<HS>;
  // stored [K][rows]
  __device__ static T make(const __bf16* p, int64_t ld, int r0, int rows, int K) {
    return T(p + r0, ld, rows - r0 < kTile ? rows - r0 : kTile, K);
  }
};

// OUT: 0 = bf16 C, 1 = fp32 C, 2 = fp32 C += product, 3 = bf16 C += product (summed in fp32, one
// rounding); AK / BK: operand K-major
// BatchNorm statistics of the bf16-rounded outputs of one 256-row tile (the values the BN pass
// reads back), per column: the mean over the tile's valid rows, then M2 = sum (y - mean)^2 around
// that mean (two passes over the accumulators, no cancellation), combined across the 16 lanes of
// a column group by xor-shuffles and across the two wave rows through LDS (`red`: 512 floats).
// The finalize Chan-combines the tiles in a fixed order (cs_bn_nhwc_fwd_tiles).
__device__ __forceinline__ void tile_stats(const Tile& t, int M, int N, int m0, int n0, int tm, int wr, int wc,
                                           int lane, float* red, float* __restrict__ stats) {
  const int rows = M - m0 < kTile ? M - m0 : kTile;
  float v[4][4];  // [j][e]: column n0 + wc*64 + j*16 + (lane >> 4)*4 + e
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    float mean[4][4];
    if (pass == 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = wc * 64 + j * 16 + (lane >> 4) * 4 + e;
          mean[j][e] = (red[c] + red[256 + c]) / (float)rows;
        }
      __syncthreads();  // every wave has its means before red is overwritten
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool ok = m0 + wr * 128 + i * 16 + (lane & 15) < M;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float y = (float)(__bf16)t.acc[i][j][e];
          const float d = pass == 0 ? y : y - mean[j][e];
          v[j][e] += ok ? (pass == 0 ? d : d * d) : 0.f;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = v[j][e];
        x += __shfl_xor(x, 1);
        x += __shfl_xor(x, 2);
        x += __shfl_xor(x, 4);
        x += __shfl_xor(x, 8);
        if ((lane & 15) == 0) red[wr * 256 + wc * 64 + j * 16 + (lane >> 4) * 4 + e] = x;
      }
    __syncthreads();
    if (pass == 1 && wr == 0 && (lane & 15) == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = wc * 64 + j * 16 + (lane >> 4) * 4 + e;
          if (n0 + c < N)
            *reinterpret_cast<float2*>(stats + ((int64_t)tm * N + n0 + c) * 2) =
                make_float2(mean[j][e], red[c] + red[256 + c]);
        }
    }
  }
}

// split-K: workgroup row blockIdx.y = split s takes k in [s * kper, (s + 1) * kper) and writes its
// own C slab C + s * slab (fp32 partials, summed by cs_slab_sum)
// STATS (bf16 C, no split): per-channel BatchNorm statistics of this tile's bf16 outputs, tile
// mean and M2 = sum (y - mean)^2 per column, into stats[tile row][N][2] (see tile_stats below)
template <int OUT, bool AK, bool BK, bool STATS = false>
__global__ __launch_bounds__(kThreads, 1) void gemm_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                        void* __restrict__ C, int M, int N, int K, int64_t lda,
                                                        int64_t ldb, int64_t ldc, int kper, int64_t slab,
                                                        float* __restrict__ stats) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * kBuf];
  const int nM = (M + kTile - 1) / kTile, nN = (N + kTile - 1) / kTile, nwg = nM * nN;
  // XCD remap (bijective for any nwg), then GROUP_M tile order
  const int orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  constexpr int G = 8;
  const int per = G * nN, grp = wg / per, first = grp * G, gm = nM - first < G ? nM - first : G;
  const int tm = first + (wg % per) % gm, tn = (wg % per) / gm;
  const int m0 = tm * kTile, n0 = tn * kTile;

  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wr = wv >> 2, wc = wv & 3;
  const int kb = blockIdx.y * kper;
  K = K - kb < kper ? K - kb : kper;
  A += AK ? (int64_t)kb : (int64_t)kb * lda;
  B += BK ? (int64_t)kb : (int64_t)kb * ldb;
  if constexpr (OUT == 0 || OUT == 3) C = static_cast<__bf16*>(C) + blockIdx.y * slab;
  else C = static_cast<float*>(C) + blockIdx.y * slab;
  const auto sa = Op<AK, 6>::make(A, lda, m0, M, K);
  const auto sb = Op<BK, 5>::make(B, ldb, n0, N, K);

  Tile t;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) t.acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + kBK - 1) / kBK;
  // prologue: all of K-tile 0 (A0 B0 B1 A1, the order the loop's phases stage in)
  sa.template stage<true>(smem, 0, 0);
  sb.template stage<true>(smem + kImg, 0, 0);
  sb.template stage<true>(smem + kImg, 1, 0);
  sa.template stage<true>(smem, 1, 0);
  int kt = 0;
  // the last K-tile may be partial (K % 64 != 0): only its staging checks k against K
  for (; kt + 2 < nk; ++kt) {
    char* cur = smem + (kt & 1) * kBuf;
    char* nxt = smem + ((kt + 1) & 1) * kBuf;
    ktile<true, false, 4>(t, cur, nxt, sa, sb, (kt + 1) * kBK, wr, wc, lane);
  }
  if (kt + 1 < nk) {
    ktile<true, true, 4>(t, smem + (kt & 1) * kBuf, smem + ((kt + 1) & 1) * kBuf, sa, sb, (kt + 1) * kBK, wr, wc,
                         lane);
    ++kt;
  }
  ktile<false, false, 0>(t, smem + (kt & 1) * kBuf, nullptr, sa, sb, 0, wr, wc, lane);

  // epilogue: acc[i][j] register e = C[row m0 + wr*128 + i*16 + (lane & 15)][col n0 + wc*64 + j*16 + (lane >> 4)*4 + e]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wc * 64 + j * 16 + (lane >> 4) * 4;
      if (n >= N) continue;
      const f32x4 v = t.acc[i][j];
      if constexpr (OUT == 0 || OUT == 3) {
        bf16x4* p = reinterpret_cast<bf16x4*>(static_cast<__bf16*>(C) + (int64_t)m * ldc + n);
        f32x4 w = v;
        if constexpr (OUT == 3) {
          const bf16x4 old = *p;
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] += (float)old[e];
        }
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (__bf16)w[e];
        *p = o;
      } else {
        f32x4* p = reinterpret_cast<f32x4*>(static_cast<float*>(C) + (int64_t)m * ldc + n);
        if constexpr (OUT == 2) *p = *p + v;
        else *p = v;
      }
    }
  }
  if constexpr (STATS) {
    __syncthreads();  // every wave is past its last reads of the operand images: reuse the LDS
    tile_stats(t, M, N, m0, n0, tm, wr, wc, lane, reinterpret_cast<float*>(smem), stats);
  }
}

struct Geo {
  int M, N, K;
  int64_t lda, ldb, ldc;
  int kper;
  int64_t slab;
};

template <int OUT, bool AK, bool BK>
void launch(const __bf16* a, const __bf16* b, void* c, const Geo& g, dim3 grid, hipStream_t stream) {
  hipLaunchKernelGGL((gemm_kernel<OUT, AK, BK>), grid, dim3(kThreads), 0, stream, a, b, c, g.M, g.N, g.K, g.lda, g.ldb,
                     g.ldc, g.kper, g.slab, nullptr);
}

template <int OUT>
void launch_layout(int ak, int bk, const __bf16* a, const __bf16* b, void* c, const Geo& g, dim3 grid,
                   hipStream_t stream) {
  if (ak && bk) launch<OUT, true, true>(a, b, c, g, grid, stream);
  else if (ak) launch<OUT, true, false>(a, b, c, g, grid, stream);
  else if (bk) launch<OUT, false, true>(a, b, c, g, grid, stream);
  else launch<OUT, false, false>(a, b, c, g, grid, stream);
}

}  // namespace

int cs_gemm_bf16_splits(int M, int N, int K) {
  // split the reduction only when the output alone leaves CUs idle: up to about two waves of
  // workgroups over the 256 CUs, >= 1024 k per split, fp32 slabs within 1 GiB
  const int64_t tiles = (int64_t)((M + kTile - 1) / kTile) * ((N + kTile - 1) / kTile);
  int s = 1;
  while (s < 256 && tiles * s * 2 <= 512 && K / (2 * s) >= 1024 && (int64_t)2 * s * M * N * 4 <= (1LL << 30)) s *= 2;
  // K per split is rounded up to whole K-tiles: keep every split non-empty
  while (s > 1 && (int64_t)(((K + s - 1) / s + kBK - 1) / kBK * kBK) * (s - 1) >= K) --s;
  return s;
}

hipError_t cs_gemm_bf16(int a_kmajor, const void* A, int64_t lda, int b_kmajor, const void* B, int64_t ldb, void* C,
                        int64_t ldc, int M, int N, int K, int out_mode, int splits, int64_t slab, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return hipSuccess;
  if (out_mode < 0 || out_mode > 3 || splits < 1 || (splits > 1 && out_mode != 1)) return hipErrorInvalidValue;
  // 16-byte source chunks (rows 16-byte aligned), 8/16-byte output quads
  if (lda % 8 || ldb % 8 || N % 4 || ldc % 4 || ldc < N) return hipErrorInvalidValue;
  if ((a_kmajor && K % 8) || (b_kmajor && K % 8)) return hipErrorInvalidValue;
  if (a_kmajor ? lda < K : lda < M) return hipErrorInvalidValue;
  if (b_kmajor ? ldb < K : ldb < N) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return hipErrorInvalidValue;
  if (reinterpret_cast<uintptr_t>(C) & (out_mode == 0 || out_mode == 3 ? 7 : 15)) return hipErrorInvalidValue;
  // 32-bit buffer offsets: a K-major operand addresses 256 rows, an M-major one 64 k rows
  if ((int64_t)(a_kmajor ? kTile : kBK) * lda * 2 >= 0x7fffffff) return hipErrorInvalidValue;
  if ((int64_t)(b_kmajor ? kTile : kBK) * ldb * 2 >= 0x7fffffff) return hipErrorInvalidValue;
  const int64_t tiles = (int64_t)((M + kTile - 1) / kTile) * ((N + kTile - 1) / kTile);
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  // K per split: a multiple of the K-tile (and of 8), every split non-empty
  const int kper = splits == 1 ? K : (int)(((K + splits - 1) / splits + kBK - 1) / kBK * kBK);
  if (splits > 1 && ((int64_t)kper * (splits - 1) >= K || slab < (int64_t)(M - 1) * ldc + N)) return hipErrorInvalidValue;
  const Geo g{M, N, K, lda, ldb, ldc, kper, slab};
  const dim3 grid((unsigned)tiles, (unsigned)splits);
  const auto* a = static_cast<const __bf16*>(A);
  const auto* b = static_cast<const __bf16*>(B);
  if (out_mode == 0) launch_layout<0>(a_kmajor, b_kmajor, a, b, C, g, grid, stream);
  else if (out_mode == 1) launch_layout<1>(a_kmajor, b_kmajor, a, b, C, g, grid, stream);
  else if (out_mode == 2) launch_layout<2>(a_kmajor, b_kmajor, a, b, C, g, grid, stream);
  else launch_layout<3>(a_kmajor, b_kmajor, a, b, C, g, grid, stream);
  return hipGetLastError();
}

hipError_t cs_gemm_bf16_bn_stats(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M,
                                 int N, int K, float* stats, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return hipSuccess;
  if (K % 8 || lda % 8 || ldb % 8 || N % 4 || ldc % 4 || ldc < N || lda < K || ldb < K) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15 || reinterpret_cast<uintptr_t>(C) & 7 ||
      reinterpret_cast<uintptr_t>(stats) & 7)
    return hipErrorInvalidValue;
  if ((int64_t)kTile * lda * 2 >= 0x7fffffff || (int64_t)kTile * ldb * 2 >= 0x7fffffff) return hipErrorInvalidValue;
  const int64_t tiles = (int64_t)((M + kTile - 1) / kTile) * ((N + kTile - 1) / kTile);
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm_kernel<0, true, true, true>), dim3((unsigned)tiles), dim3(kThreads), 0, stream,
                     static_cast<const __bf16*>(A), static_cast<const __bf16*>(B), C, M, N, K, lda, ldb, ldc, K,
                     (int64_t)0, stats);
  return hipGetLastError();
}
