// Channels-last (NHWC) CNN kernels for the ResNet family's native path (models/resnet.py,
// ops/cnn_nhwc.py; BASELINE.json "ResNet-50 on synthetic ImageNet-shape"). On MI355X the NCHW
// path spends ~20 % of a ResNet-50 bf16 step in MIOpen's NCHW<->NHWC batched transposes around
// its NHWC implicit-GEMM kernels (profiles/r2_resnet50_bf16_kernels.txt); keeping activations
// NHWC end to end makes every 1x1 convolution a plain [B*H*W, Cin] x [Cin, Cout] GEMM
// (hipBLASLt) and every k x k / strided one an im2col gather + the same GEMM, with:
//   * training BatchNorm2d (+ residual add) (+ ReLU): stats -> finalize -> apply forward,
//     reduce -> finalize -> apply backward, per-channel vectors of V = 16 bytes along C;
//   * 3x3/2 pad-1 max-pool (window position kept as uint8, gather-style backward);
//   * im2col (columns ordered (r, s, c), zero padding, K padded to Kp) and its gather-style
//     adjoint col2im (each input element sums the taps that read it: no atomics).
// Every reduction has a fixed shape and order: bitwise deterministic run to run.
#include <hip/hip_bf16.h>

#include "common.h"
#include "launchers.h"

namespace {

template <typename T>
struct E;
template <>
struct E<float> {
  __device__ static float ld(const float* p) { return *p; }
  __device__ static void st(float* p, float v) { *p = v; }
};
template <>
struct E<__hip_bfloat16> {
  __device__ static float ld(const __hip_bfloat16* p) { return __bfloat162float(*p); }
  __device__ static void st(__hip_bfloat16* p, float v) { *p = __float2bfloat16(v); }
};

// V consecutive channels through one 4/8/16-byte access (V == 1: scalar)
template <typename T, int V>
__device__ __forceinline__ void ldv(const T* p, float (&v)[V]) {
  if constexpr (V == 1) {
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = E<T>::ld(p + j);
  } else {
    typedef unsigned u32v __attribute__((ext_vector_type(V * sizeof(T) / 4)));
    const u32v raw = *reinterpret_cast<const u32v*>(p);
    const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = E<T>::ld(e + j);
  }
}
template <typename T, int V>
__device__ __forceinline__ void stv(T* p, const float (&v)[V]) {
  if constexpr (V == 1) {
#pragma unroll
    for (int j = 0; j < V; ++j) E<T>::st(p + j, v[j]);
  } else {
    typedef unsigned u32v __attribute__((ext_vector_type(V * sizeof(T) / 4)));
    u32v raw;
    T* e = reinterpret_cast<T*>(&raw);
#pragma unroll
    for (int j = 0; j < V; ++j) E<T>::st(e + j, v[j]);
    *reinterpret_cast<u32v*>(p) = raw;
  }
}

__device__ __forceinline__ float preact(float x, float scale, float shift, float res) {
  return fmaf(x, scale, shift) + res;
}

// ------------------------------------------------------------------------------ BatchNorm
// Block (p, g): rows [p*rpb, min(M, (p+1)*rpb)) x channel vectors [g*256, g*256 + nv). The
// nv vector lanes of a row are adjacent threads (coalesced row reads); 256/nv row lanes stride
// the rows. Per-channel accumulators are summed over the row lanes through LDS in lane order.
constexpr int kMaxV = 8;
struct RowSplit {
  int nv, lanes, cv, rl, c0;
};
__device__ __forceinline__ RowSplit row_split(int C, int V) {
  RowSplit s;
  const int CV = C / V, g0 = blockIdx.y * 256;
  s.nv = min(256, CV - g0);
  s.lanes = 256 / s.nv;
  s.cv = threadIdx.x % s.nv;
  s.rl = threadIdx.x / s.nv;
  s.c0 = (g0 + s.cv) * V;
  return s;
}

// two accumulators per channel -> part[p][c][2] (fixed lane order)
template <int V>
__device__ __forceinline__ void lanes_to_part(const RowSplit& s, const float (&a)[V], const float (&b)[V], float* sh,
                                              float* __restrict__ part, int C) {
  const int width = s.nv * V;  // channels of this block
  if (s.rl < s.lanes)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      sh[((size_t)s.rl * width + s.cv * V + j) * 2 + 0] = a[j];
      sh[((size_t)s.rl * width + s.cv * V + j) * 2 + 1] = b[j];
    }
  __syncthreads();
  const int cbase = blockIdx.y * 256 * V;
  for (int e = threadIdx.x; e < width; e += 256) {
    float x = 0.f, y = 0.f;
    for (int l = 0; l < s.lanes; ++l) {
      x += sh[((size_t)l * width + e) * 2 + 0];
      y += sh[((size_t)l * width + e) * 2 + 1];
    }
    part[((size_t)blockIdx.x * C + cbase + e) * 2 + 0] = x;
    part[((size_t)blockIdx.x * C + cbase + e) * 2 + 1] = y;
  }
}

// part[p][c] = {sum(x - K_c), sum((x - K_c)^2)} with K_c = x[row 0][c] (a shift that keeps the
// f32 partial sums well conditioned; the finalize combines them in f64)
template <typename T, int V>
__global__ __launch_bounds__(256) void stats_kernel(const T* __restrict__ x, int64_t M, int C, int rpb,
                                                    float* __restrict__ part) {
  __shared__ float sh[256 * kMaxV * 2];
  const RowSplit s = row_split(C, V);
  float s1[V], s2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) s1[j] = s2[j] = 0.f;
  if (s.rl < s.lanes) {
    float K[V];
    ldv<T, V>(x + s.c0, K);
    const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = min(M, r0 + rpb);
    for (int64_t r = r0 + s.rl; r < r1; r += s.lanes) {
      float v[V];
      ldv<T, V>(x + r * C + s.c0, v);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float d = v[j] - K[j];
        s1[j] += d;
        s2[j] = fmaf(d, d, s2[j]);
      }
    }
  }
  lanes_to_part<V>(s, s1, s2, sh, part, C);
}

// 256 threads = 8 channels x 32 partial lanes (f64 sums, lanes combined in a fixed tree):
// mean / biased var (normalisation) / unbiased var (running stats); stat = [scale, shift, mean,
// invstd][C]. 32 lanes keep even 1024 partials to 32 dependent adds per thread.
template <typename T>
__global__ __launch_bounds__(256) void finalize_fwd_kernel(const T* __restrict__ x, const float* __restrict__ part,
                                                           int P, int C, double M, const float* __restrict__ w,
                                                           const float* __restrict__ b, float* __restrict__ rm,
                                                           float* __restrict__ rv, float momentum, float eps,
                                                           float* __restrict__ stat, int64_t* __restrict__ nbt) {
  __shared__ double sh[32][8][2];
  const int cl = threadIdx.x & 7, pl = threadIdx.x >> 3, c = blockIdx.x * 8 + cl;
  double s1 = 0.0, s2 = 0.0;
  if (c < C)
#pragma unroll 4
    for (int p = pl; p < P; p += 32) {
      const float2 v = *reinterpret_cast<const float2*>(part + ((size_t)p * C + c) * 2);
      s1 += (double)v.x;
      s2 += (double)v.y;
    }
  sh[pl][cl][0] = s1;
  sh[pl][cl][1] = s2;
  __syncthreads();
#pragma unroll
  for (int h = 16; h > 0; h >>= 1) {
    if (pl < h) {
      sh[pl][cl][0] += sh[pl + h][cl][0];
      sh[pl][cl][1] += sh[pl + h][cl][1];
    }
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt != nullptr) *nbt += 1;  // num_batches_tracked
  if (pl != 0 || c >= C) return;
  s1 = sh[0][cl][0];
  s2 = sh[0][cl][1];
  const double K = (double)E<T>::ld(x + c);
  const double dm = s1 / M;
  double var = s2 / M - dm * dm;
  if (var < 0.0) var = 0.0;
  const double mean = K + dm;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float scale = (w != nullptr ? w[c] : 1.f) * invstd;
  stat[c] = scale;
  stat[C + c] = (b != nullptr ? b[c] : 0.f) - (float)mean * scale;
  stat[2 * C + c] = (float)mean;
  stat[3 * C + c] = invstd;
  if (rm != nullptr) {
    const double unbiased = M > 1.0 ? var * M / (M - 1.0) : var;
    rm[c] = (1.f - momentum) * rm[c] + momentum * (float)mean;
    rv[c] = (1.f - momentum) * rv[c] + momentum * (float)unbiased;
  }
}

// The same outputs from per-tile (mean, M2) partials of R-row tiles (the bf16 GEMM's statistics
// epilogue, gemm_bf16.hip tile_stats): tiles [T][C][2]. Lane pl Chan-combines tiles pl, pl + 32,
// ... in order (f64), then the 32 lane states combine in a fixed tree: deterministic.
__device__ __forceinline__ void chan64(double& n, double& m, double& M2, double nb, double mb, double M2b) {
  if (nb == 0.0) return;
  if (n == 0.0) {
    n = nb; m = mb; M2 = M2b;
    return;
  }
  const double nn = n + nb, d = mb - m;
  m += d * (nb / nn);
  M2 += M2b + d * d * (n * nb / nn);
  n = nn;
}

__global__ __launch_bounds__(256) void finalize_tiles_kernel(const float* __restrict__ tiles, int T, int R, int64_t M,
                                                             int C, const float* __restrict__ w,
                                                             const float* __restrict__ b, float* __restrict__ rm,
                                                             float* __restrict__ rv, float momentum, float eps,
                                                             float* __restrict__ stat, int64_t* __restrict__ nbt) {
  __shared__ double sh[32][8][3];
  const int cl = threadIdx.x & 7, pl = threadIdx.x >> 3, c = blockIdx.x * 8 + cl;
  double n = 0.0, m = 0.0, M2 = 0.0;
  if (c < C)
    for (int p = pl; p < T; p += 32) {
      const int64_t left = M - (int64_t)p * R;
      const float2 v = *reinterpret_cast<const float2*>(tiles + ((size_t)p * C + c) * 2);
      chan64(n, m, M2, (double)(left < R ? left : R), (double)v.x, (double)v.y);
    }
  sh[pl][cl][0] = n;
  sh[pl][cl][1] = m;
  sh[pl][cl][2] = M2;
  __syncthreads();
#pragma unroll
  for (int h = 16; h > 0; h >>= 1) {
    if (pl < h) {
      double a = sh[pl][cl][0], am = sh[pl][cl][1], a2 = sh[pl][cl][2];
      chan64(a, am, a2, sh[pl + h][cl][0], sh[pl + h][cl][1], sh[pl + h][cl][2]);
      sh[pl][cl][0] = a;
      sh[pl][cl][1] = am;
      sh[pl][cl][2] = a2;
    }
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt != nullptr) *nbt += 1;  // num_batches_tracked
  if (pl != 0 || c >= C) return;
  const double mean = sh[0][cl][1];
  double var = sh[0][cl][2] / (double)M;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float scale = (w != nullptr ? w[c] : 1.f) * invstd;
  stat[c] = scale;
  stat[C + c] = (b != nullptr ? b[c] : 0.f) - (float)mean * scale;
  stat[2 * C + c] = (float)mean;
  stat[3 * C + c] = invstd;
  if (rm != nullptr) {
    const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
    rm[c] = (1.f - momentum) * rm[c] + momentum * (float)mean;
    rv[c] = (1.f - momentum) * rv[c] + momentum * (float)unbiased;
  }
}

// Block (p, g): rows [p*rpb, ...) x this block's channel vectors (the stats kernel's split): each
// thread keeps its V channels' scale / shift in registers and walks rows.
template <typename T, int V>
__global__ __launch_bounds__(256) void apply_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                        const float* __restrict__ stat, T* __restrict__ y,
                                                        int64_t M, int C, int rpb, int relu,
                                                        unsigned char* __restrict__ mask) {
  const RowSplit s = row_split(C, V);
  if (s.rl >= s.lanes) return;
  float sc[V], sf[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    sc[j] = stat[s.c0 + j];
    sf[j] = stat[C + s.c0 + j];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = min(M, r0 + rpb);
#pragma unroll 2
  for (int64_t r = r0 + s.rl; r < r1; r += s.lanes) {
    const int64_t e = r * C + s.c0;
    float v[V], rr[V];
    ldv<T, V>(x + e, v);
    if (res != nullptr) ldv<T, V>(res + e, rr);
    unsigned live = 0;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float z = preact(v[j], sc[j], sf[j], res != nullptr ? rr[j] : 0.f);
      live |= (z > 0.f ? 1u : 0u) << j;
      v[j] = relu && !(z > 0.f) ? 0.f : z;
    }
    stv<T, V>(y + e, v);
    if (mask != nullptr) mask[e / V] = (unsigned char)live;
  }
}

// POOL: the BatchNorm's output went through the 3x3/2 max-pool (the ResNet stem) and dy is the
// pooled gradient: a row's incoming gradient is gathered from the <= 2x2 windows that hold it and
// picked it (maxpool_bwd_kernel's arithmetic, rounded to T as that kernel stores it) instead of
// being read from a full-resolution gradient tensor that would first have to be written.
struct PoolG {
  const unsigned char* pos;
  int H, W, Ho, Wo;
};
template <typename T, int V>
__device__ __forceinline__ void pool_grad(const T* __restrict__ dy, const PoolG& pg, int q, int C, int c0,
                                          float (&g)[V]) {
  const int iw = q % pg.W, ih = (q / pg.W) % pg.H, b = q / (pg.W * pg.H);
  const int oh0 = ih / 2, oh1 = min(pg.Ho - 1, (ih + 1) / 2);
  const int ow0 = iw / 2, ow1 = min(pg.Wo - 1, (iw + 1) / 2);
#pragma unroll
  for (int j = 0; j < V; ++j) g[j] = 0.f;
  for (int oh = oh0; oh <= oh1; ++oh)
    for (int ow = ow0; ow <= ow1; ++ow) {
      const int dh = ih - (2 * oh - 1), dw = iw - (2 * ow - 1);
      if (dh < 0 || dh > 2 || dw < 0 || dw > 2) continue;
      const int64_t o = (((int64_t)b * pg.Ho + oh) * pg.Wo + ow) * C + c0;
      float d[V];
      ldv<T, V>(dy + o, d);
#pragma unroll
      for (int j = 0; j < V; ++j)
        if (pg.pos[o + j] == dh * 3 + dw) g[j] += d[j];
    }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    T t;
    E<T>::st(&t, g[j]);
    g[j] = E<T>::ld(&t);
  }
}

// g = dy masked by the recomputed pre-activation; part[p][c] = {sum g, sum g*xhat}
template <typename T, int V, bool POOL>
__global__ __launch_bounds__(256) void bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                         const T* __restrict__ res, const float* __restrict__ stat,
                                                         int64_t M, int C, int rpb, int relu,
                                                         const unsigned char* __restrict__ mask,
                                                         float* __restrict__ part, PoolG pg) {
  __shared__ float sh[256 * kMaxV * 2];
  const RowSplit s = row_split(C, V);
  float sg[V], sgx[V];
#pragma unroll
  for (int j = 0; j < V; ++j) sg[j] = sgx[j] = 0.f;
  if (s.rl < s.lanes) {
    float sc[V], sf[V], mu[V], is[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      sc[j] = stat[s.c0 + j];
      sf[j] = stat[C + s.c0 + j];
      mu[j] = stat[2 * C + s.c0 + j];
      is[j] = stat[3 * C + s.c0 + j];
    }
    const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = min(M, r0 + rpb);
    for (int64_t r = r0 + s.rl; r < r1; r += s.lanes) {
      const int64_t off = r * C + s.c0;
      float g[V], v[V], rr[V];
      if constexpr (POOL)
        pool_grad<T, V>(dy, pg, (int)r, C, s.c0, g);
      else
        ldv<T, V>(dy + off, g);
      ldv<T, V>(x + off, v);
      unsigned live = 0;
      if (mask != nullptr) live = mask[off / V];
      else if (relu && res != nullptr) ldv<T, V>(res + off, rr);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        if (mask != nullptr ? !((live >> j) & 1u) : relu && !(preact(v[j], sc[j], sf[j], res != nullptr ? rr[j] : 0.f) > 0.f))
          g[j] = 0.f;
        sg[j] += g[j];
        sgx[j] = fmaf(g[j], (v[j] - mu[j]) * is[j], sgx[j]);
      }
    }
  }
  lanes_to_part<V>(s, sg, sgx, sh, part, C);
}

// dbeta = sum g, dgamma = sum g*xhat (8 channels x 32 partial lanes, as the forward finalize);
// coef = [gamma*invstd, sum g / M, sum g*xhat / M][C]
__global__ __launch_bounds__(256) void finalize_bwd_kernel(const float* __restrict__ part, int P, int C, double M,
                                                           const float* __restrict__ w, const float* __restrict__ stat,
                                                           float* __restrict__ dw, float* __restrict__ db,
                                                           float* __restrict__ coef) {
  __shared__ double sh[32][8][2];
  const int cl = threadIdx.x & 7, pl = threadIdx.x >> 3, c = blockIdx.x * 8 + cl;
  double sg = 0.0, sgx = 0.0;
  if (c < C)
#pragma unroll 4
    for (int p = pl; p < P; p += 32) {
      const float2 v = *reinterpret_cast<const float2*>(part + ((size_t)p * C + c) * 2);
      sg += (double)v.x;
      sgx += (double)v.y;
    }
  sh[pl][cl][0] = sg;
  sh[pl][cl][1] = sgx;
  __syncthreads();
#pragma unroll
  for (int h = 16; h > 0; h >>= 1) {
    if (pl < h) {
      sh[pl][cl][0] += sh[pl + h][cl][0];
      sh[pl][cl][1] += sh[pl + h][cl][1];
    }
    __syncthreads();
  }
  if (pl != 0 || c >= C) return;
  sg = sh[0][cl][0];
  sgx = sh[0][cl][1];
  if (dw != nullptr) dw[c] = (float)sgx;
  if (db != nullptr) db[c] = (float)sg;
  coef[c] = (w != nullptr ? w[c] : 1.f) * stat[3 * C + c];
  coef[C + c] = (float)(sg / M);
  coef[2 * C + c] = (float)(sgx / M);
}

// dx = k*(g - mean(g) - xhat*mean(g*xhat)), dres = g; per-channel operands in registers, rows walked
// as in apply_fwd_kernel
template <typename T, int V, bool POOL>
__global__ __launch_bounds__(256) void apply_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                        const T* __restrict__ res, const float* __restrict__ stat,
                                                        const float* __restrict__ coef, T* __restrict__ dx,
                                                        T* __restrict__ dres, int64_t M, int C, int rpb, int relu,
                                                        const unsigned char* __restrict__ mask, PoolG pg) {
  const RowSplit s = row_split(C, V);
  if (s.rl >= s.lanes) return;
  float sc[V], sf[V], mu[V], is[V], k[V], mg[V], mgx[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c = s.c0 + j;
    sc[j] = stat[c];
    sf[j] = stat[C + c];
    mu[j] = stat[2 * C + c];
    is[j] = stat[3 * C + c];
    k[j] = coef[c];
    mg[j] = coef[C + c];
    mgx[j] = coef[2 * C + c];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = min(M, r0 + rpb);
#pragma unroll 2
  for (int64_t r = r0 + s.rl; r < r1; r += s.lanes) {
    const int64_t e = r * C + s.c0;
    float g[V], v[V], rr[V];
    if constexpr (POOL)
      pool_grad<T, V>(dy, pg, (int)r, C, s.c0, g);
    else
      ldv<T, V>(dy + e, g);
    ldv<T, V>(x + e, v);
    unsigned live = 0;
    if (mask != nullptr) live = mask[e / V];
    else if (relu && res != nullptr) ldv<T, V>(res + e, rr);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      if (mask != nullptr ? !((live >> j) & 1u) : relu && !(preact(v[j], sc[j], sf[j], res != nullptr ? rr[j] : 0.f) > 0.f))
        g[j] = 0.f;
      const float xhat = (v[j] - mu[j]) * is[j];
      v[j] = k[j] * (g[j] - mg[j] - xhat * mgx[j]);
    }
    stv<T, V>(dx + e, v);
    if (dres != nullptr) stv<T, V>(dres + e, g);
  }
}

// ------------------------------------------------------------------------------ max-pool 3x3/2
// one thread per (output position, V channels); ties keep the first maximum in row-major window
// order and a NaN wins (ATen's rules). stat != nullptr: the input is a BatchNorm's pre-activation
// and each window element is first taken through that BatchNorm + ReLU and rounded to T — the
// same arithmetic as apply_fwd_kernel, so the result equals BN-apply then max-pool bit for bit,
// without the full-resolution activation ever being written (the ResNet stem).
template <typename T, int V>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          unsigned char* __restrict__ pos, int B, int H, int W, int C,
                                                          int Ho, int Wo, const float* __restrict__ stat) {
  const int CV = C / V;
  const int64_t total = (int64_t)B * Ho * Wo * CV;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ii = (int)i, cv = ii % CV, o32 = ii / CV;  // total < 2^31 (host check): 32-bit index math
    const int64_t o = o32;
    const int ow = o32 % Wo, oh = (o32 / Wo) % Ho, b = o32 / (Wo * Ho);
    float sc[V], sf[V];
    if (stat != nullptr)
#pragma unroll
      for (int j = 0; j < V; ++j) {
        sc[j] = stat[cv * V + j];
        sf[j] = stat[C + cv * V + j];
      }
    float best[V];
    int bp[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      best[j] = -INFINITY;
      bp[j] = -1;
    }
#pragma unroll
    for (int dh = 0; dh < 3; ++dh)
#pragma unroll
      for (int dw = 0; dw < 3; ++dw) {
        const int ih = 2 * oh - 1 + dh, iw = 2 * ow - 1 + dw;
        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
          float v[V];
          ldv<T, V>(x + (((int64_t)b * H + ih) * W + iw) * C + cv * V, v);
          if (stat != nullptr)
#pragma unroll
            for (int j = 0; j < V; ++j) {
              const float z = preact(v[j], sc[j], sf[j], 0.f);
              T t;
              E<T>::st(&t, !(z > 0.f) ? 0.f : z);
              v[j] = E<T>::ld(&t);
            }
#pragma unroll
          for (int j = 0; j < V; ++j)
            if (bp[j] < 0 || v[j] > best[j] || v[j] != v[j]) {
              best[j] = v[j];
              bp[j] = dh * 3 + dw;
            }
        }
      }
    stv<T, V>(y + o * C + cv * V, best);
#pragma unroll
    for (int j = 0; j < V; ++j) pos[o * C + cv * V + j] = (unsigned char)bp[j];
  }
}

template <typename T, int V>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const T* __restrict__ dy, const unsigned char* __restrict__ pos,
                                                          T* __restrict__ dx, int B, int H, int W, int C, int Ho,
                                                          int Wo) {
  const int CV = C / V;
  const int64_t total = (int64_t)B * H * W * CV;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ii = (int)i, cv = ii % CV, q32 = ii / CV;  // 32-bit index math (host check)
    const int64_t q = q32;
    const int iw = q32 % W, ih = (q32 / W) % H, b = q32 / (W * H);
    // outputs whose window [2o-1, 2o+1] holds this input, in row-major order
    const int oh0 = ih / 2, oh1 = min(Ho - 1, (ih + 1) / 2);
    const int ow0 = iw / 2, ow1 = min(Wo - 1, (iw + 1) / 2);
    float g[V];
#pragma unroll
    for (int j = 0; j < V; ++j) g[j] = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh)
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int dh = ih - (2 * oh - 1), dw = iw - (2 * ow - 1);
        if (dh < 0 || dh > 2 || dw < 0 || dw > 2) continue;
        const int64_t o = (((int64_t)b * Ho + oh) * Wo + ow) * C + cv * V;
        float d[V];
        ldv<T, V>(dy + o, d);
#pragma unroll
        for (int j = 0; j < V; ++j)
          if (pos[o + j] == dh * 3 + dw) g[j] += d[j];
      }
    stv<T, V>(dx + q * C + cv * V, g);
  }
}

// ------------------------------------------------------------------------------ im2col / col2im
// col[m][(r*S + s)*C + c] = x[b][oh*st - pad + r][ow*st - pad + s][c] (0 outside), columns
// K = R*S*C .. Kp-1 zero; m = (b*Ho + oh)*Wo + ow. One thread per V columns.
template <typename T, int V>
__global__ __launch_bounds__(256) void im2col_kernel(const T* __restrict__ x, T* __restrict__ col, int B, int H, int W,
                                                     int C, int R, int S, int st, int pad, int Ho, int Wo, int Kp) {
  const int KV = Kp / V, K = R * S * C;
  const int64_t total = (int64_t)B * Ho * Wo * KV;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ii = (int)i, k = (ii % KV) * V, m32 = ii / KV;  // 32-bit index math (host check)
    const int64_t m = m32;
    float v[V];
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = 0.f;
    if (k < K) {
      const int c = k % C, rs = k / C, s = rs % S, r = rs / S;
      const int ow = m32 % Wo, oh = (m32 / Wo) % Ho, b = m32 / (Wo * Ho);
      const int ih = oh * st - pad + r, iw = ow * st - pad + s;
      if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ldv<T, V>(x + (((int64_t)b * H + ih) * W + iw) * C + c, v);
    }
    stv<T, V>(col + m * Kp + k, v);
  }
}

// dx[b][ih][iw][c] = sum over the taps (r, s) that read it of dcol[m(oh, ow)][(r*S + s)*C + c],
// r and s ascending (fixed order, f32 accumulation)
template <typename T, int V>
__global__ __launch_bounds__(256) void col2im_kernel(const T* __restrict__ dcol, T* __restrict__ dx, int B, int H, int W,
                                                     int C, int R, int S, int st, int pad, int Ho, int Wo, int Kp) {
  const int CV = C / V;
  const int64_t total = (int64_t)B * H * W * CV;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ii = (int)i, c = (ii % CV) * V, q32 = ii / CV;  // 32-bit index math (host check)
    const int64_t q = q32;
    const int iw = q32 % W, ih = (q32 / W) % H, b = q32 / (W * H);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    for (int r = 0; r < R; ++r) {
      const int th = ih + pad - r;
      if (th < 0 || th % st != 0 || th / st >= Ho) continue;
      const int oh = th / st;
      for (int s = 0; s < S; ++s) {
        const int tw = iw + pad - s;
        if (tw < 0 || tw % st != 0 || tw / st >= Wo) continue;
        const int64_t m = ((int64_t)b * Ho + oh) * Wo + tw / st;
        float d[V];
        ldv<T, V>(dcol + m * Kp + (r * S + s) * C + c, d);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += d[j];
      }
    }
    stv<T, V>(dx + q * C + c, acc);
  }
}

// ------------------------------------------------------------------------------ host side
// the gather kernels index their work items in 32 bits (64-bit integer division is emulated):
// a launch covers at most kMaxItems items, larger tensors go in batch chunks (every image's
// gather is independent) — e.g. the 224-px stem im2col passes 2^31 items near B = 850
constexpr int64_t kMaxItems = (int64_t)1 << 31;

// images per launch so that one launch stays below kMaxItems items (>= 1: one image always fits
// for every shape these kernels serve; the callers check per_image < kMaxItems)
int batch_chunk(int B, int64_t per_image) {
  const int64_t c = (kMaxItems - 1) / per_image;
  return (int)(c < 1 ? 1 : (c > B ? B : c));
}

int grid_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

// V for a channel count: 16 bytes when C allows it, then 4 elements, then scalar
int vec_for(int C, int esize) {
  const int v16 = 16 / esize;
  if (C % v16 == 0) return v16;
  if (C % 4 == 0) return 4;
  return 1;
}

// rows per BN block: >= 16 rows per row lane, and ~1024 blocks for the big layers
struct BnGrid {
  int P, CG, rpb;
};
BnGrid bn_grid(int64_t M, int C, int V) {
  BnGrid g;
  const int CV = C / V;
  g.CG = (CV + 255) / 256;
  const int lanes = 256 / (CV < 256 ? CV : 256);
  const int64_t want = (1024 + g.CG - 1) / g.CG;
  int64_t rpb = (M + want - 1) / want;
  if (rpb < 16 * (int64_t)lanes) rpb = 16 * (int64_t)lanes;
  g.rpb = (int)rpb;
  g.P = (int)((M + rpb - 1) / rpb);
  return g;
}

// elementwise passes: ~2048 blocks of >= 4 rows per row lane
BnGrid apply_grid(int64_t M, int C, int V) {
  BnGrid g;
  const int CV = C / V;
  g.CG = (CV + 255) / 256;
  const int lanes = 256 / (CV < 256 ? CV : 256);
  const int64_t want = (2048 + g.CG - 1) / g.CG;
  int64_t rpb = (M + want - 1) / want;
  if (rpb < 4 * (int64_t)lanes) rpb = 4 * (int64_t)lanes;
  g.rpb = (int)rpb;
  g.P = (int)((M + rpb - 1) / rpb);
  return g;
}

template <typename T, int V>
void bn_fwd_t(const void* x, const void* res, const float* w, const float* b, float* rm, float* rv, int64_t* nbt,
              float momentum, float eps, int relu, void* y, float* stat, float* part, int64_t M, int C,
              unsigned char* mask, hipStream_t st) {
  const BnGrid g = bn_grid(M, C, V);
  hipLaunchKernelGGL((stats_kernel<T, V>), dim3(g.P, g.CG), dim3(256), 0, st, (const T*)x, M, C, g.rpb, part);
  hipLaunchKernelGGL(finalize_fwd_kernel<T>, dim3((C + 7) / 8), dim3(256), 0, st, (const T*)x, part, g.P, C,
                     (double)M, w, b, rm, rv, momentum, eps, stat, nbt);
  if (y == nullptr) return;  // statistics only (the apply is fused into the consumer)
  const BnGrid a = apply_grid(M, C, V);
  hipLaunchKernelGGL((apply_fwd_kernel<T, V>), dim3(a.P, a.CG), dim3(256), 0, st, (const T*)x, (const T*)res, stat,
                     (T*)y, M, C, a.rpb, relu, mask);
}

template <typename T, int V>
void bn_bwd_t(const void* dy, const void* x, const void* res, const float* w, const float* stat, int relu, void* dx,
              void* dres, float* dw, float* db, float* coef, float* part, int64_t M, int C, const unsigned char* mask,
              const PoolG* pool, hipStream_t st) {
  const BnGrid g = bn_grid(M, C, V);
  const PoolG pg = pool != nullptr ? *pool : PoolG{nullptr, 0, 0, 0, 0};
  if (pool != nullptr)
    hipLaunchKernelGGL((bwd_reduce_kernel<T, V, true>), dim3(g.P, g.CG), dim3(256), 0, st, (const T*)dy, (const T*)x,
                       (const T*)res, stat, M, C, g.rpb, relu, mask, part, pg);
  else
    hipLaunchKernelGGL((bwd_reduce_kernel<T, V, false>), dim3(g.P, g.CG), dim3(256), 0, st, (const T*)dy,
                       (const T*)x, (const T*)res, stat, M, C, g.rpb, relu, mask, part, pg);
  hipLaunchKernelGGL(finalize_bwd_kernel, dim3((C + 7) / 8), dim3(256), 0, st, part, g.P, C, (double)M, w, stat, dw,
                     db, coef);
  const BnGrid a = apply_grid(M, C, V);
  if (pool != nullptr)
    hipLaunchKernelGGL((apply_bwd_kernel<T, V, true>), dim3(a.P, a.CG), dim3(256), 0, st, (const T*)dy, (const T*)x,
                       (const T*)res, stat, coef, (T*)dx, (T*)dres, M, C, a.rpb, relu, mask, pg);
  else
    hipLaunchKernelGGL((apply_bwd_kernel<T, V, false>), dim3(a.P, a.CG), dim3(256), 0, st, (const T*)dy, (const T*)x,
                       (const T*)res, stat, coef, (T*)dx, (T*)dres, M, C, a.rpb, relu, mask, pg);
}

// dispatch on (dtype, V) for a functor F<T, V>::run(args...)
#define CS_NHWC_DISPATCH(dt, C, ...)                          \
  do {                                                         \
    if ((dt) == CS_BF16) {                                     \
      using T = __hip_bfloat16;                                \
      const int V_ = vec_for((C), 2);                          \
      if (V_ == 8) { constexpr int V = 8; __VA_ARGS__; }              \
      else if (V_ == 4) { constexpr int V = 4; __VA_ARGS__; }         \
      else { constexpr int V = 1; __VA_ARGS__; }                      \
    } else {                                                   \
      using T = float;                                         \
      const int V_ = vec_for((C), 4);                          \
      if (V_ == 4) { constexpr int V = 4; __VA_ARGS__; }              \
      else { constexpr int V = 1; __VA_ARGS__; }                      \
    }                                                          \
  } while (0)

}  // namespace

int cs_bn_nhwc_vec(int C, int dt) { return vec_for(C, dt == CS_BF16 ? 2 : 4); }

int cs_bn_nhwc_partials(int64_t M, int C, int dt) {
  const BnGrid g = bn_grid(M, C, vec_for(C, dt == CS_BF16 ? 2 : 4));
  return g.P * C * 2;
}

hipError_t cs_bn_nhwc_fwd(int dt, const void* x, const void* res, const float* w, const float* b, float* rm, float* rv,
                          int64_t* nbt, float momentum, float eps, int relu, void* y, float* stat, float* part,
                          int64_t M, int C, hipStream_t stream, unsigned char* mask) {
  if (M * C == 0) return hipSuccess;
  CS_NHWC_DISPATCH(dt, C, bn_fwd_t<T, V>(x, res, w, b, rm, rv, nbt, momentum, eps, relu, y, stat, part, M, C, mask, stream));
  return hipGetLastError();
}

hipError_t cs_bn_nhwc_fwd_tiles(int dt, const void* x, const void* res, const float* w, const float* b, float* rm,
                                float* rv, int64_t* nbt, float momentum, float eps, int relu, void* y, float* stat,
                                const float* tiles, int ntiles, int R, int64_t M, int C, hipStream_t stream,
                                unsigned char* mask) {
  if (M * C == 0) return hipSuccess;
  if (ntiles < 1 || R < 1 || (int64_t)(ntiles - 1) * R >= M || (int64_t)ntiles * R < M) return hipErrorInvalidValue;
  hipLaunchKernelGGL(finalize_tiles_kernel, dim3((C + 7) / 8), dim3(256), 0, stream, tiles, ntiles, R, M, C, w, b, rm, rv,
                     momentum, eps, stat, nbt);
  CS_NHWC_DISPATCH(dt, C, {
    const BnGrid a = apply_grid(M, C, V);
    hipLaunchKernelGGL((apply_fwd_kernel<T, V>), dim3(a.P, a.CG), dim3(256), 0, stream, (const T*)x, (const T*)res,
                       stat, (T*)y, M, C, a.rpb, relu, mask);
  });
  return hipGetLastError();
}

hipError_t cs_bn_nhwc_bwd(int dt, const void* dy, const void* x, const void* res, const float* w, const float* stat,
                          int relu, void* dx, void* dres, float* dw, float* db, float* coef, float* part, int64_t M,
                          int C, hipStream_t stream, const unsigned char* mask, const unsigned char* pool_pos,
                          int H, int W, int Ho, int Wo) {
  if (M * C == 0) return hipSuccess;
  if (pool_pos != nullptr && (M >= kMaxItems || (int64_t)H * W <= 0 || M % ((int64_t)H * W) != 0 ||
                              Ho != (H - 1) / 2 + 1 || Wo != (W - 1) / 2 + 1))
    return hipErrorInvalidValue;
  const PoolG pg{pool_pos, H, W, Ho, Wo};
  const PoolG* pp = pool_pos != nullptr ? &pg : nullptr;
  CS_NHWC_DISPATCH(dt, C, bn_bwd_t<T, V>(dy, x, res, w, stat, relu, dx, dres, dw, db, coef, part, M, C, mask, pp, stream));
  return hipGetLastError();
}

hipError_t cs_maxpool3s2_nhwc_fwd(int dt, const void* x, void* y, unsigned char* pos, int B, int H, int W, int C,
                                  int Ho, int Wo, hipStream_t stream, const float* stat) {
  const int64_t per = (int64_t)Ho * Wo * C;
  if (per * B == 0) return hipSuccess;
  if (per >= kMaxItems) return hipErrorInvalidValue;
  const int cb = batch_chunk(B, per);
  for (int b0 = 0; b0 < B; b0 += cb) {
    const int nb = B - b0 < cb ? B - b0 : cb;
    const int64_t xo = (int64_t)b0 * H * W * C, yo = (int64_t)b0 * per;
    CS_NHWC_DISPATCH(dt, C, hipLaunchKernelGGL((maxpool_fwd_kernel<T, V>), dim3(grid_for(nb * per / V)), dim3(256),
                                               0, stream, (const T*)x + xo, (T*)y + yo, pos + yo, nb, H, W, C, Ho,
                                               Wo, stat));
  }
  return hipGetLastError();
}

hipError_t cs_maxpool3s2_nhwc_bwd(int dt, const void* dy, const unsigned char* pos, void* dx, int B, int H, int W,
                                  int C, int Ho, int Wo, hipStream_t stream) {
  const int64_t per = (int64_t)H * W * C;
  if (per * B == 0) return hipSuccess;
  if (per >= kMaxItems) return hipErrorInvalidValue;
  const int cb = batch_chunk(B, per);
  for (int b0 = 0; b0 < B; b0 += cb) {
    const int nb = B - b0 < cb ? B - b0 : cb;
    const int64_t yo = (int64_t)b0 * Ho * Wo * C, xo = (int64_t)b0 * per;
    CS_NHWC_DISPATCH(dt, C, hipLaunchKernelGGL((maxpool_bwd_kernel<T, V>), dim3(grid_for(nb * per / V)), dim3(256),
                                               0, stream, (const T*)dy + yo, pos + yo, (T*)dx + xo, nb, H, W, C, Ho,
                                               Wo));
  }
  return hipGetLastError();
}

hipError_t cs_im2col_nhwc(int dt, const void* x, void* col, int B, int H, int W, int C, int R, int S, int stride,
                          int pad, int Ho, int Wo, int Kp, hipStream_t stream) {
  const int64_t per = (int64_t)Ho * Wo * Kp;
  if (per * B == 0) return hipSuccess;
  if (per >= kMaxItems) return hipErrorInvalidValue;
  // V must divide C (a vector stays inside one tap) and Kp
  const int vc = vec_for(C, dt == CS_BF16 ? 2 : 4);
  if (vc > 1 && Kp % vc != 0) return hipErrorInvalidValue;
  const int cb = batch_chunk(B, per);
  for (int b0 = 0; b0 < B; b0 += cb) {
    const int nb = B - b0 < cb ? B - b0 : cb;
    const int64_t xo = (int64_t)b0 * H * W * C, co = (int64_t)b0 * per;
    CS_NHWC_DISPATCH(dt, C, hipLaunchKernelGGL((im2col_kernel<T, V>), dim3(grid_for(nb * per / V)), dim3(256), 0,
                                               stream, (const T*)x + xo, (T*)col + co, nb, H, W, C, R, S, stride, pad,
                                               Ho, Wo, Kp));
  }
  return hipGetLastError();
}

hipError_t cs_col2im_nhwc(int dt, const void* dcol, void* dx, int B, int H, int W, int C, int R, int S, int stride,
                          int pad, int Ho, int Wo, int Kp, hipStream_t stream) {
  const int64_t per = (int64_t)H * W * C;
  if (per * B == 0) return hipSuccess;
  if (per >= kMaxItems || (int64_t)Ho * Wo * Kp >= kMaxItems) return hipErrorInvalidValue;
  const int vc = vec_for(C, dt == CS_BF16 ? 2 : 4);
  if (vc > 1 && Kp % vc != 0) return hipErrorInvalidValue;
  // chunk so both the dx items and the dcol rows a launch reads stay within 32-bit indices
  const int64_t per_col = (int64_t)Ho * Wo * Kp;
  const int cb = batch_chunk(B, per > per_col ? per : per_col);
  for (int b0 = 0; b0 < B; b0 += cb) {
    const int nb = B - b0 < cb ? B - b0 : cb;
    const int64_t xo = (int64_t)b0 * per, co = (int64_t)b0 * per_col;
    CS_NHWC_DISPATCH(dt, C, hipLaunchKernelGGL((col2im_kernel<T, V>), dim3(grid_for(nb * per / V)), dim3(256), 0,
                                               stream, (const T*)dcol + co, (T*)dx + xo, nb, H, W, C, R, S, stride,
                                               pad, Ho, Wo, Kp));
  }
  return hipGetLastError();
}
