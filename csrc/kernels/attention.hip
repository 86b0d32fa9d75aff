// Causal grouped-query attention (flash style) for gfx950, bf16 in / bf16 out, f32 softmax and
// accumulation: the attention of the Llama-3 extension config (models/llama.py; BASELINE.json
// "Llama-3 8B bf16 pure data-parallel"), replacing scaled_dot_product_attention's forward and
// backward. Tensors in the model's natural [B, S, H, D] layout (no transposes); D = 64 or 128.
//
// All products are v_mfma_f32_32x32x16_bf16. The score tile is computed transposed,
// S^T = K . Q^T (keys on the accumulator rows, the query on the lane), so a query's scores sit
// in one lane pair (lane, lane ^ 32): row max / row sum are in-register plus one xor-32 shuffle.
// The accumulator then feeds the next product as its B operand with no lane movement
// (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand"): registers
// 8s..8s+7 of a 32x32 tile, converted to bf16, are k-step s, with k (= key) order
// 16s + 8(j>>2) + 4h + (j&3) for element j of lane half h — the A operand (V^T, K^T, dO^T, Q^T)
// is read with ds_read_b64_tr_b16 in exactly that k order from a row-major [rows][D] LDS image.
// LDS images put 16-byte chunk ch of row r at ch ^ swz(r) (guide T10 layout (b)), which serves
// both the ds_read_b128 row reads and the transposed reads.
//
// Forward: one workgroup = 4 waves = 128 queries of one (batch, head); K/V tiles of 64 keys,
// LDS-DMA-staged into a double-buffered LDS image (one barrier per tile); online softmax in
// base 2 (c = log2(e)/sqrt(D)); writes O and the row log-sum-exp L2 = m + log2(l) (base 2).
// Backward (deterministic, no float atomics):
//   attn_delta: delta = rowsum(dO * O) per (b, head, query);
//   attn_dq:    per 128-query block, like the forward: S^T, P^T, dP^T = V . dO^T,
//               dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T;
//   attn_dkdv:  per 128-key block of one kv head, every query head of its group: S = Q K^T,
//               dP = dO V^T (key on the lane), dV^T += dO^T P, dK^T += Q^T dS; Q/dO tiles of 64
//               queries (+ their L2 and delta) double-buffered in LDS.
#include <math.h>

#include "common.h"
#include "launchers.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// [rows][D] bf16 image, 16-byte chunks XOR-swizzled per row
template <int D>
struct Img {
  static constexpr int NCH = D / 8;
  static constexpr int ROW = 2 * D;  // bytes
  __device__ static int off(int r, int ch) {
    const int sw = (((r & 3) << 2) | ((r >> 2) & 3)) & (NCH - 1);
    return ROW * r + 16 * (ch ^ sw);
  }
};

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int e = 0; e < 16; ++e) z[e] = 0.f;
  return z;
}

// row-read operand fragment: image row `row`, k = d = 16 kk + 8h + j (natural order)
template <int D>
__device__ __forceinline__ bf16x8 row_frag(const char* img, int row, int kk, int h) {
  return *reinterpret_cast<const bf16x8*>(img + Img<D>::off(row, 2 * kk + h));
}

// transposed-read operand fragment for "A . X" with X an accumulator tile: lane (r, h) gets
// column d = dbase + r of image rows k0 + 16s.. in the accumulator's k order
// (j -> row k0 + 8(j>>2) + 4h + (j&3)); k0 already includes 16s
template <int D>
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int k0, int dbase, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = k0 + 4 * (g >> 1) + q;
  const int ch = ((dbase + 16 * (g & 1)) >> 3) + (p >> 1);
  const char* a0 = img + Img<D>::off(row, ch) + 8 * (p & 1);
  const char* a1 = img + Img<D>::off(row + 8, ch) + 8 * (p & 1);
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(a0));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(a1));
  const bf16x4 blo = __builtin_bit_cast(bf16x4, lo), bhi = __builtin_bit_cast(bf16x4, hi);
  return __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// registers 8s..8s+7 of an accumulator tile as a bf16 operand fragment
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& x, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (__bf16)x[8 * s + j];
  return f;
}

__device__ __forceinline__ bf16x8 gload8(const __bf16* p, bool ok) {
  if (ok) return *reinterpret_cast<const bf16x8*>(p);
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
  return z;
}

// accumulator row of register e for lane half h
__device__ __forceinline__ int acc_row(int e, int h) { return (e & 3) + 8 * (e >> 2) + 4 * h; }

// store an O^T-shaped accumulator set (rows = d, lane = one row of the output) as bf16
template <int D>
__device__ __forceinline__ void store_rowT(const f32x16 (&acc)[D / 32], float mul, __bf16* dst, int h) {
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      bf16x4 v;
#pragma unroll
      for (int x = 0; x < 4; ++x) v[x] = (__bf16)(acc[dt][4 * g4 + x] * mul);
      *reinterpret_cast<bf16x4*>(dst + 32 * dt + 8 * g4 + 4 * h) = v;
    }
}

constexpr int kBM = 128;  // queries per workgroup (fwd, dq) / keys per workgroup (dkdv)
constexpr int kBN = 64;   // keys per K/V tile (fwd, dq) / queries per Q/dO tile (dkdv)

// LDS-DMA copy (buffer_load ... lds) of a 64-row [rows][D] global tile into an LDS image, no
// registers: each wave-instruction writes 64 16-byte pieces = 1 KiB of the image contiguously,
// so the swizzle is applied on the SOURCE side (image piece (row, pc) <- global chunk
// pc ^ swz(row)); rows >= nrows get an out-of-range offset and land as zeros.
constexpr int kOOB = 0x7ffffff0;

template <int D>
struct Dma {
  static constexpr int NCH = D / 8, PER_WAVE = kBN * NCH / (4 * 64);  // instructions per wave
  __amdgpu_buffer_rsrc_t rs;
  size_t stride;  // bytes between rows
  int nrows;
  __device__ Dma(const __bf16* base, size_t stride_elems, int nrows_) : stride(stride_elems * 2), nrows(nrows_) {
    const int64_t bytes = nrows_ > 0 ? (int64_t)(nrows_ - 1) * (int64_t)stride + 2 * D : 0;
    rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(base), (short)0, (int)bytes, 0x00020000);
  }
  __device__ __forceinline__ void issue(char* img, int row0) const {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int slot = (wv * PER_WAVE + i) * 64 + lane, row = slot / NCH, pc = slot % NCH;
      const int sw = (((row & 3) << 2) | ((row >> 2) & 3)) & (NCH - 1);
      const int grow = row0 + row;
      const int off = grow < nrows ? (int)((size_t)grow * stride) + 16 * (pc ^ sw) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(img + (wv * PER_WAVE + i) * 1024),
                                               16, off, 0, 0, 0);
    }
  }
};

// every wave's LDS-DMA has landed and every wave is past its reads of the other buffer
__device__ __forceinline__ void dma_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

template <int D>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                       const __bf16* __restrict__ v, __bf16* __restrict__ o,
                                                       float* __restrict__ lse, int S, int Hq, int Hkv, float c,
                                                       int causal) {
  constexpr int KK = D / 16, DT = D / 32, TILE = kBN * D * 2;  // bytes of one K or V image
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [2 buffers][K image, V image]
  const int nqb = (S + kBM - 1) / kBM;
  const int qb = nqb - 1 - (int)blockIdx.x;  // the longest (latest) query blocks first
  const int hq = blockIdx.y, b = blockIdx.z, hk = hq / (Hq / Hkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int q0 = qb * kBM, q0w = q0 + 32 * w, qi = q0w + r;
  const size_t qs = (size_t)Hq * D, ks = (size_t)Hkv * D;
  const __bf16* Q = q + (size_t)b * S * qs + (size_t)hq * D;
  const __bf16* K = k + (size_t)b * S * ks + (size_t)hk * D;
  const __bf16* V = v + (size_t)b * S * ks + (size_t)hk * D;

  bf16x8 qf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) qf[kk] = gload8(Q + (size_t)qi * qs + 16 * kk + 8 * h, qi < S);
  f32x16 acc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) acc[dt] = zero16();
  float m = -INFINITY, l = 0.f;

  const int kend = causal ? min(S, q0 + kBM) : S;
  const int nkt = (kend + kBN - 1) / kBN;
  const Dma<D> dk(K, ks, S), dv(V, ks, S);
  dk.issue(smem, 0);
  dv.issue(smem + TILE, 0);
  dma_barrier();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) {  // the other buffer: every wave finished reading it before the last barrier
      char* nx = smem + (cur ^ 1) * 2 * TILE;
      dk.issue(nx, (kt + 1) * kBN);
      dv.issue(nx + TILE, (kt + 1) * kBN);
    }
    const char* Kl = smem + cur * 2 * TILE;
    const char* Vl = Kl + TILE;
    const int k0 = kt * kBN;
    if (!causal || k0 <= q0w + 31) {  // wave-uniform: some key of the tile is visible to this wave
      f32x16 s[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s[t] = zero16();
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) s[t] = mfma(row_frag<D>(Kl, 32 * t + r, kk, h), qf[kk], s[t]);
      }
      const bool edge = (causal && k0 + kBN - 1 > q0w) || k0 + kBN > S;
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float x = s[t][e] * c;
          if (edge) {
            const int key = k0 + 32 * t + acc_row(e, h);
            if ((causal && key > qi) || key >= S) x = -INFINITY;
          }
          s[t][e] = x;
          mx = fmaxf(mx, x);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      const float mn = fmaxf(m, mx);
      const float mu = mn == -INFINITY ? 0.f : mn;
      const float alpha = __builtin_amdgcn_exp2f(m - mu);
      float rs = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float p = __builtin_amdgcn_exp2f(s[t][e] - mu);
          s[t][e] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 32);
      l = l * alpha + rs;
      m = mn;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[dt][e] *= alpha;
      bf16x8 pf[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) pf[t][ss] = acc_frag(s[t], ss);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) acc[dt] = mfma(tr_frag<D>(Vl, 32 * t + 16 * ss, 32 * dt, lane), pf[t][ss], acc[dt]);
    }
    dma_barrier();
  }
  if (qi < S) {
    store_rowT<D>(acc, l > 0.f ? 1.f / l : 0.f, o + ((size_t)b * S + qi) * qs + (size_t)hq * D, h);
    if (h == 0) lse[((size_t)b * Hq + hq) * S + qi] = m + __log2f(l);
  }
}

// delta[b, h, q] = sum_d dO * O (f32), one 16-lane group per (b, q, h) row
template <int D>
__global__ __launch_bounds__(256) void attn_delta_kernel(const __bf16* __restrict__ o, const __bf16* __restrict__ dout,
                                                         float* __restrict__ delta, int B, int S, int H) {
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4), l16 = threadIdx.x & 15;
  const int rows = B * S * H;
  float s = 0.f;
  if (row < rows) {
    const __bf16* op = o + (size_t)row * D;
    const __bf16* gp = dout + (size_t)row * D;
    for (int d = 8 * l16; d < D; d += 128) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(op + d);
      const bf16x8 g = *reinterpret_cast<const bf16x8*>(gp + d);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += (float)a[j] * (float)g[j];
    }
  }
#pragma unroll
  for (int x = 8; x >= 1; x >>= 1) s += __shfl_xor(s, x, 16);
  if (row < rows && l16 == 0) {
    const int hh = row % H, bq = row / H, qq = bq % S, bb = bq / S;
    delta[((size_t)bb * H + hh) * S + qq] = s;
  }
}

template <int D>
__device__ __forceinline__ void dq_body(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                      const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                      const float* __restrict__ lse, const float* __restrict__ delta,
                                                      __bf16* __restrict__ dq, int S, int Hq, int Hkv, float c,
                                                      float scale, int causal, int bx, int by, int bz) {
  constexpr int KK = D / 16, DT = D / 32, TILE = kBN * D * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = (S + kBM - 1) / kBM;
  const int qb = nqb - 1 - bx;
  const int hq = by, b = bz, hk = hq / (Hq / Hkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int q0 = qb * kBM, q0w = q0 + 32 * w, qi = q0w + r;
  const size_t qs = (size_t)Hq * D, ks = (size_t)Hkv * D;
  const size_t qrow = ((size_t)b * S + qi) * qs + (size_t)hq * D;
  const __bf16* K = k + (size_t)b * S * ks + (size_t)hk * D;
  const __bf16* V = v + (size_t)b * S * ks + (size_t)hk * D;
  bf16x8 qf[KK], gf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    qf[kk] = gload8(q + qrow + 16 * kk + 8 * h, qi < S);
    gf[kk] = gload8(dout + qrow + 16 * kk + 8 * h, qi < S);
  }
  const size_t st = ((size_t)b * Hq + hq) * S + qi;
  const float L2 = qi < S ? lse[st] : 0.f, dl = qi < S ? delta[st] : 0.f;
  f32x16 acc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) acc[dt] = zero16();

  const int kend = causal ? min(S, q0 + kBM) : S;
  const int nkt = (kend + kBN - 1) / kBN;
  const Dma<D> dmk(K, ks, S), dmv(V, ks, S);
  dmk.issue(smem, 0);
  dmv.issue(smem + TILE, 0);
  dma_barrier();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) {
      char* nx = smem + (cur ^ 1) * 2 * TILE;
      dmk.issue(nx, (kt + 1) * kBN);
      dmv.issue(nx + TILE, (kt + 1) * kBN);
    }
    const char* Kl = smem + cur * 2 * TILE;
    const char* Vl = Kl + TILE;
    const int k0 = kt * kBN;
    // one 32-key half of the tile at a time (no running max here: P = exp2(S c - L2) is final),
    // which keeps two score tiles live instead of four: two waves per SIMD fit
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (causal && k0 + 32 * t > q0w + 31) continue;  // wave-uniform: the half is above the diagonal
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        s = mfma(row_frag<D>(Kl, 32 * t + r, kk, h), qf[kk], s);
        dp = mfma(row_frag<D>(Vl, 32 * t + r, kk, h), gf[kk], dp);
      }
      const bool edge = (causal && k0 + 32 * t + 31 > q0w) || k0 + 32 * t + 32 > S;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        float p = __builtin_amdgcn_exp2f(s[e] * c - L2);
        if (edge) {
          const int key = k0 + 32 * t + acc_row(e, h);
          if ((causal && key > qi) || key >= S) p = 0.f;
        }
        s[e] = p * (dp[e] - dl);  // dS^T
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss)
          acc[dt] = mfma(tr_frag<D>(Kl, 32 * t + 16 * ss, 32 * dt, lane), acc_frag(s, ss), acc[dt]);
    }
    dma_barrier();
  }
  if (qi < S) store_rowT<D>(acc, scale, dq + qrow, h);
}

template <int D>
__global__ __launch_bounds__(256, 2) void attn_dq_kernel(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                      const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                      const float* __restrict__ lse, const float* __restrict__ delta,
                                                      __bf16* __restrict__ dq, int S, int Hq, int Hkv, float c,
                                                      float scale, int causal) {
  dq_body<D>(q, k, v, dout, lse, delta, dq, S, Hq, Hkv, c, scale, causal, blockIdx.x, blockIdx.y, blockIdx.z);
}

template <int D>
__device__ __forceinline__ void dkdv_body(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                        const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                        const float* __restrict__ lse, const float* __restrict__ delta,
                                                        __bf16* __restrict__ dk, __bf16* __restrict__ dv, int S, int Hq,
                                                        int Hkv, float c, float scale, int causal, int bx, int by, int bz) {
  constexpr int KK = D / 16, DT = D / 32, TILE = kBN * D * 2;
  // [2 buffers][Q image, dO image, L2[64], delta[64]]
  constexpr int BUF = 2 * TILE + 2 * kBN * 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nkb = (S + kBM - 1) / kBM;
  const int kb = causal ? bx : nkb - 1 - bx;  // causal: early keys see the most queries
  const int hk = by, b = bz, grp = Hq / Hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int kw0 = kb * kBM + 32 * w, kj = kw0 + r;  // this lane's key (the accumulator column)
  const size_t qs = (size_t)Hq * D, ks = (size_t)Hkv * D;
  const size_t krow = ((size_t)b * S + kj) * ks + (size_t)hk * D;
  bf16x8 kf[KK], vf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    kf[kk] = gload8(k + krow + 16 * kk + 8 * h, kj < S);
    vf[kk] = gload8(v + krow + 16 * kk + 8 * h, kj < S);
  }
  f32x16 adk[DT], adv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    adk[dt] = zero16();
    adv[dt] = zero16();
  }
  // query tiles of 64: from the block's first key (causal) to the end, for every head of the group
  const int qt0 = causal ? (kb * kBM) / kBN : 0;
  const int nqt = (S + kBN - 1) / kBN - qt0;
  const int total = nqt * grp;
  // Q / dO tiles by LDS-DMA; L2 / delta (64 floats each) through registers
  auto store = [&](int it, int buf) {
    char* base = smem + buf * BUF;
    {
      const int hq = hk * grp + it / nqt, q0 = (qt0 + it % nqt) * kBN;
      const Dma<D> dq_(q + (size_t)b * S * qs + (size_t)hq * D, qs, S), dg(dout + (size_t)b * S * qs + (size_t)hq * D, qs, S);
      dq_.issue(base, q0);
      dg.issue(base + TILE, q0);
    }
    if (threadIdx.x < 2 * kBN) {  // L2 and delta of the tile's 64 queries
      const int hq = hk * grp + it / nqt, q0 = (qt0 + it % nqt) * kBN;
      const int qq = q0 + (threadIdx.x & (kBN - 1));
      const float* src = threadIdx.x < kBN ? lse : delta;
      reinterpret_cast<float*>(base + 2 * TILE)[threadIdx.x] =
          qq < S ? src[((size_t)b * Hq + hq) * S + qq] : 0.f;
    }
  };
  if (total > 0) store(0, 0);
  dma_barrier();
  for (int it = 0; it < total; ++it) {
    const int cur = it & 1;
    if (it + 1 < total) store(it + 1, cur ^ 1);  // the other buffer: its readers passed the last barrier
    const char* Ql = smem + cur * BUF;
    const char* Gl = Ql + TILE;
    const float* L2s = reinterpret_cast<const float*>(Ql + 2 * TILE);
    const float* Dls = L2s + kBN;
    const int q0 = (qt0 + it % nqt) * kBN;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int qu = q0 + 32 * u;  // this 32-query slice
      if (causal && qu + 31 < kw0) continue;  // wave-uniform: every query precedes this wave's keys
      if (qu >= S) continue;
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        s = mfma(row_frag<D>(Ql, 32 * u + r, kk, h), kf[kk], s);
        dp = mfma(row_frag<D>(Gl, 32 * u + r, kk, h), vf[kk], dp);
      }
      // rows = queries (registers), column = this lane's key
      f32x16 ds;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int qr = 32 * u + acc_row(e, h), qq = q0 + qr;
        float p = __builtin_amdgcn_exp2f(s[e] * c - L2s[qr]);
        if ((causal && kj > qq) || qq >= S || kj >= S) p = 0.f;
        s[e] = p;
        ds[e] = p * (dp[e] - Dls[qr]);
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          adv[dt] = mfma(tr_frag<D>(Gl, 32 * u + 16 * ss, 32 * dt, lane), acc_frag(s, ss), adv[dt]);
          adk[dt] = mfma(tr_frag<D>(Ql, 32 * u + 16 * ss, 32 * dt, lane), acc_frag(ds, ss), adk[dt]);
        }
    }
    dma_barrier();
  }
  if (kj < S) {
    store_rowT<D>(adk, scale, dk + krow, h);
    store_rowT<D>(adv, 1.f, dv + krow, h);
  }
}

template <int D>
__global__ __launch_bounds__(256) void attn_dkdv_kernel(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                        const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                        const float* __restrict__ lse, const float* __restrict__ delta,
                                                        __bf16* __restrict__ dk, __bf16* __restrict__ dv, int S, int Hq,
                                                        int Hkv, int B, float c, float scale, int causal) {
  // 1-D grid, key block slowest-varying: every head's heaviest (earliest, causal) key blocks dispatch
  // first. At one wave per SIMD (356 VGPR+AGPR) the 512 blocks of the Llama-3-8B shape run in two
  // rounds on 256 CUs; heaviest-first keeps the second round from starting with a 16x-longer block.
  const int L = (int)blockIdx.x;
  dkdv_body<D>(q, k, v, dout, lse, delta, dk, dv, S, Hq, Hkv, c, scale, causal, L / (Hkv * B), L % Hkv,
               (L / Hkv) % B);
}

// Causal backward in ONE launch: the dK/dV blocks first (key block ascending = most query tiles
// first), then the dQ blocks (latest query block first). A dK/dV block of an early key block
// walks up to 16x the query tiles of a late one, so run alone that kernel leaves most CUs idle
// in its tail; here the dQ blocks (independent: they write only dQ) fill those CUs as the short
// dK/dV blocks retire. Same bodies, same arithmetic, same results as the two launches.
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_fused_kernel(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                             const __bf16* __restrict__ v,
                                                             const __bf16* __restrict__ dout,
                                                             const float* __restrict__ lse,
                                                             const float* __restrict__ delta, __bf16* __restrict__ dq,
                                                             __bf16* __restrict__ dk, __bf16* __restrict__ dv, int S,
                                                             int Hq, int Hkv, int B, float c, float scale, int causal) {
  const int nb = (S + kBM - 1) / kBM;
  const int n_kv = nb * Hkv * B;
  int L = (int)blockIdx.x;
  if (L < n_kv) {  // key block slowest-varying: all heads' heaviest key blocks dispatch first
    dkdv_body<D>(q, k, v, dout, lse, delta, dk, dv, S, Hq, Hkv, c, scale, causal, L / (Hkv * B), L % Hkv,
                 (L / Hkv) % B);
  } else {
    L -= n_kv;
    dq_body<D>(q, k, v, dout, lse, delta, dq, S, Hq, Hkv, c, scale, causal, L / (Hq * B), L % Hq, (L / Hq) % B);
  }
}

// The causal backward runs as one launch (attn_bwd_fused_kernel) by default; CS_ATTN_BWD_FUSED=0 gives
// dQ then dK/dV (heaviest-first grid). Llama-3-8B step on MI355X: two launches in grid order 18.79k
// tokens/s (dK/dV 1156 us), heaviest-first 19.76k (dK/dV 645 us), one launch 20.12k.
bool attn_bwd_fused() {
  static const bool on = [] {
    const char* e = getenv("CS_ATTN_BWD_FUSED");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}

template <int D>
size_t fwd_lds() { return 2 * 2 * (size_t)kBN * D * 2; }
template <int D>
size_t dkdv_lds() { return 2 * (2 * (size_t)kBN * D * 2 + 2 * kBN * 4); }

template <int D>
hipError_t launch_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int Hq, int Hkv,
                      float scale, int causal, hipStream_t st) {
  const dim3 grid((S + kBM - 1) / kBM, Hq, B);
  hipLaunchKernelGGL(attn_fwd_kernel<D>, grid, dim3(256), fwd_lds<D>(), st, (const __bf16*)q, (const __bf16*)k,
                     (const __bf16*)v, (__bf16*)o, lse, S, Hq, Hkv, scale * 1.4426950408889634f, causal);
  return hipGetLastError();
}

template <int D>
hipError_t launch_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                      float* delta, void* dq, void* dk, void* dv, int B, int S, int Hq, int Hkv, float scale, int causal,
                      hipStream_t st) {
  const int rows = B * S * Hq;
  hipLaunchKernelGGL(attn_delta_kernel<D>, dim3((rows + 15) / 16), dim3(256), 0, st, (const __bf16*)o,
                     (const __bf16*)dout, delta, B, S, Hq);
  const float c = scale * 1.4426950408889634f;
  const int nb = (S + kBM - 1) / kBM;
  if (causal && attn_bwd_fused()) {
    const size_t lds = dkdv_lds<D>() > fwd_lds<D>() ? dkdv_lds<D>() : fwd_lds<D>();
    hipLaunchKernelGGL(attn_bwd_fused_kernel<D>, dim3(nb * (Hkv + Hq) * B), dim3(256), lds, st, (const __bf16*)q,
                       (const __bf16*)k, (const __bf16*)v, (const __bf16*)dout, lse, delta, (__bf16*)dq, (__bf16*)dk,
                       (__bf16*)dv, S, Hq, Hkv, B, c, scale, causal);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(attn_dq_kernel<D>, dim3(nb, Hq, B), dim3(256), fwd_lds<D>(), st,
                     (const __bf16*)q, (const __bf16*)k, (const __bf16*)v, (const __bf16*)dout, lse, delta,
                     (__bf16*)dq, S, Hq, Hkv, c, scale, causal);
  hipLaunchKernelGGL(attn_dkdv_kernel<D>, dim3(nb * Hkv * B), dim3(256), dkdv_lds<D>(), st,
                     (const __bf16*)q, (const __bf16*)k, (const __bf16*)v, (const __bf16*)dout, lse, delta,
                     (__bf16*)dk, (__bf16*)dv, S, Hq, Hkv, B, c, scale, causal);
  return hipGetLastError();
}

}  // namespace

hipError_t cs_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int Hq, int Hkv,
                       int D, float scale, int causal, hipStream_t stream) {
  if (B == 0 || S == 0) return hipSuccess;
  if (D == 128) return launch_fwd<128>(q, k, v, o, lse, B, S, Hq, Hkv, scale, causal, stream);
  if (D == 64) return launch_fwd<64>(q, k, v, o, lse, B, S, Hq, Hkv, scale, causal, stream);
  return hipErrorInvalidValue;
}

hipError_t cs_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                       float* delta, void* dq, void* dk, void* dv, int B, int S, int Hq, int Hkv, int D, float scale,
                       int causal, hipStream_t stream) {
  if (B == 0 || S == 0) return hipSuccess;
  if (D == 128) return launch_bwd<128>(q, k, v, o, dout, lse, delta, dq, dk, dv, B, S, Hq, Hkv, scale, causal, stream);
  if (D == 64) return launch_bwd<64>(q, k, v, o, dout, lse, delta, dq, dk, dv, B, S, Hq, Hkv, scale, causal, stream);
  return hipErrorInvalidValue;
}
