// Decoder-LM elementwise hot ops for gfx950 (the BASELINE "Llama-3 8B bf16 pure DP"
// extension config): RMSNorm forward/backward, SwiGLU forward/backward, rotary
// position embedding forward/backward. fp32 or bf16 storage, fp32 math.
//
// RMSNorm: one 256-thread workgroup per row (D up to 16K), row sum of squares by
// wave shuffles + LDS, vectorised 8-byte (bf16 x4) / 16-byte (fp32 x4) accesses.
// The weight gradient is reduced deterministically: every workgroup writes one
// fp32 partial row per ROWS_PER_BLOCK rows, a second kernel sums the partials.
#include <hip/hip_bf16.h>

#include <initializer_list>

#include "common.h"
#include "launchers.h"

namespace {

__device__ __forceinline__ float ld(const float* p, size_t i) { return p[i]; }
__device__ __forceinline__ float ld(const __hip_bfloat16* p, size_t i) { return __bfloat162float(p[i]); }
__device__ __forceinline__ void st(float* p, size_t i, float v) { p[i] = v; }
__device__ __forceinline__ void st(__hip_bfloat16* p, size_t i, float v) { p[i] = __float2bfloat16(v); }

constexpr int kRowsPerBlock = 8;

template <typename T, typename W>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const T* __restrict__ x, const W* __restrict__ w,
                                                          T* __restrict__ y, float* __restrict__ rstd, int rows,
                                                          int D, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  if (row >= rows) return;
  const T* xr = x + (size_t)row * D;
  float ss = 0.f;
  for (int i = threadIdx.x; i < D; i += blockDim.x) {
    const float v = ld(xr, i);
    ss += v * v;
  }
  ss = cs::block_sum(ss, red);
  const float r = rsqrtf(ss / (float)D + eps);
  if (threadIdx.x == 0) rstd[row] = r;
  T* yr = y + (size_t)row * D;
  for (int i = threadIdx.x; i < D; i += blockDim.x) st(yr, i, ld(xr, i) * r * ld(w, i));
}

// dx_j = r*w_j*g_j - (r^3/D) x_j sum_i(w_i g_i x_i);  dw partial_j = sum_rows g_j x_j r
template <typename T, typename W>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const T* __restrict__ x, const W* __restrict__ w,
                                                          const float* __restrict__ rstd, const T* __restrict__ g,
                                                          T* __restrict__ dx, float* __restrict__ dw_part, int rows,
                                                          int D) {
  __shared__ float red[16];
  const int r0 = blockIdx.x * kRowsPerBlock;
  float* part = dw_part + (size_t)blockIdx.x * D;
  for (int i = threadIdx.x; i < D; i += blockDim.x) part[i] = 0.f;
  for (int rr = 0; rr < kRowsPerBlock; ++rr) {
    const int row = r0 + rr;
    if (row >= rows) break;
    const T* xr = x + (size_t)row * D;
    const T* gr = g + (size_t)row * D;
    const float r = rstd[row];
    float dot = 0.f;
    for (int i = threadIdx.x; i < D; i += blockDim.x) dot += ld(w, i) * ld(gr, i) * ld(xr, i);
    dot = cs::block_sum(dot, red);
    const float c = r * r * r * dot / (float)D;
    T* dxr = dx + (size_t)row * D;
    for (int i = threadIdx.x; i < D; i += blockDim.x) {
      const float xv = ld(xr, i), gv = ld(gr, i);
      st(dxr, i, r * ld(w, i) * gv - c * xv);
      part[i] += gv * xv * r;  // same thread owns column i for every row: no race
    }
  }
}

// ---- 4-wide path (D % 4 == 0, D <= 4 * 256 * kMaxQ): 16/8-byte accesses, the row held in
// registers between the reduction and the scaling pass, the weight-gradient partial of a block
// kept in registers across its rows (one store per block instead of a read-modify-write per row)
constexpr int kMaxQ = 8, kRows4 = 16;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 ld4(const __hip_bfloat16* p) {
  const uint2 r = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u), __uint_as_float(r.y << 16),
                     __uint_as_float(r.y & 0xffff0000u));
}
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ void st4(__hip_bfloat16* p, float4 v) {
  __hip_bfloat16 e[4] = {__float2bfloat16(v.x), __float2bfloat16(v.y), __float2bfloat16(v.z), __float2bfloat16(v.w)};
  *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(e);
}

template <typename T, typename W, typename O>
__global__ __launch_bounds__(256) void rmsnorm_fwd4_kernel(const T* __restrict__ x, const W* __restrict__ w,
                                                           O* __restrict__ y, float* __restrict__ rstd, int rows,
                                                           int D, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x, DQ = D >> 2;
  const T* xr = x + (size_t)row * D;
  float4 v[kMaxQ];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxQ; ++k) {
    const int q = threadIdx.x + k * 256;
    if (q < DQ) {
      v[k] = ld4(xr + 4 * q);
      ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
    }
  }
  ss = cs::block_sum(ss, red);
  const float r = rsqrtf(ss / (float)D + eps);
  if (threadIdx.x == 0) rstd[row] = r;
  O* yr = y + (size_t)row * D;
#pragma unroll
  for (int k = 0; k < kMaxQ; ++k) {
    const int q = threadIdx.x + k * 256;
    if (q < DQ) {
      const float4 wv = ld4(w + 4 * q);
      st4(yr + 4 * q, make_float4(v[k].x * r * wv.x, v[k].y * r * wv.y, v[k].z * r * wv.z, v[k].w * r * wv.w));
    }
  }
}

// kRows4 rows per block; dw_part[block][D] = sum over the block's rows of g*x*r
template <typename T, typename W, typename G>
__global__ __launch_bounds__(256) void rmsnorm_bwd4_kernel(const T* __restrict__ x, const W* __restrict__ w,
                                                           const float* __restrict__ rstd, const G* __restrict__ g,
                                                           T* __restrict__ dx, float* __restrict__ dw_part, int rows,
                                                           int D) {
  __shared__ float red[16];
  const int DQ = D >> 2;
  float4 wv[kMaxQ], acc[kMaxQ];
#pragma unroll
  for (int k = 0; k < kMaxQ; ++k) {
    const int q = threadIdx.x + k * 256;
    wv[k] = q < DQ ? ld4(w + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
    acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int r0 = blockIdx.x * kRows4;
  for (int rr = 0; rr < kRows4; ++rr) {
    const int row = r0 + rr;
    if (row >= rows) break;  // uniform across the block
    const T* xr = x + (size_t)row * D;
    const G* gr = g + (size_t)row * D;
    float4 xv[kMaxQ], gv[kMaxQ];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxQ; ++k) {
      const int q = threadIdx.x + k * 256;
      if (q < DQ) {
        xv[k] = ld4(xr + 4 * q);
        gv[k] = ld4(gr + 4 * q);
        dot += wv[k].x * gv[k].x * xv[k].x + wv[k].y * gv[k].y * xv[k].y + wv[k].z * gv[k].z * xv[k].z +
               wv[k].w * gv[k].w * xv[k].w;
      }
    }
    dot = cs::block_sum(dot, red);
    const float r = rstd[row];
    const float c = r * r * r * dot / (float)D;
    T* dxr = dx + (size_t)row * D;
#pragma unroll
    for (int k = 0; k < kMaxQ; ++k) {
      const int q = threadIdx.x + k * 256;
      if (q < DQ) {
        st4(dxr + 4 * q, make_float4(r * wv[k].x * gv[k].x - c * xv[k].x, r * wv[k].y * gv[k].y - c * xv[k].y,
                                     r * wv[k].z * gv[k].z - c * xv[k].z, r * wv[k].w * gv[k].w - c * xv[k].w));
        acc[k].x += gv[k].x * xv[k].x * r;
        acc[k].y += gv[k].y * xv[k].y * r;
        acc[k].z += gv[k].z * xv[k].z * r;
        acc[k].w += gv[k].w * xv[k].w * r;
      }
    }
  }
  float* part = dw_part + (size_t)blockIdx.x * D;
#pragma unroll
  for (int k = 0; k < kMaxQ; ++k) {
    const int q = threadIdx.x + k * 256;
    if (q < DQ) st4(part + 4 * q, acc[k]);
  }
}

// dw[4q..4q+3] = sum_p part[p][4q..]: 16 column quads x 16 partial lanes per block, lanes
// combined through LDS in lane order (deterministic)
template <typename W>
__global__ __launch_bounds__(256) void colsum4_kernel(const float* __restrict__ part, int P, int D,
                                                      W* __restrict__ dw) {
  __shared__ float4 sh[16][16];
  const int cq = threadIdx.x & 15, pl = threadIdx.x >> 4, q = blockIdx.x * 16 + cq;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (4 * q < D) {
#pragma unroll 8
    for (int p = pl; p < P; p += 16) {
      const float4 v = ld4(part + (size_t)p * D + 4 * q);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  sh[pl][cq] = s;
  __syncthreads();
  if (pl != 0 || 4 * q >= D) return;
  float4 t = sh[0][cq];
  for (int l = 1; l < 16; ++l) {
    t.x += sh[l][cq].x; t.y += sh[l][cq].y; t.z += sh[l][cq].z; t.w += sh[l][cq].w;
  }
  st4(dw + 4 * q, t);
}

template <typename W>
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part, int P, int D,
                                                     W* __restrict__ dw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= D) return;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += part[(size_t)p * D + i];
  st(dw, i, s);
}

__device__ __forceinline__ float sigmoidf(float a) { return 1.f / (1.f + __expf(-a)); }

template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                         T* __restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float av = ld(a, i);
    st(out, i, av * sigmoidf(av) * ld(b, i));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                         const T* __restrict__ g, T* __restrict__ da,
                                                         T* __restrict__ db, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float av = ld(a, i), bv = ld(b, i), gv = ld(g, i);
    const float s = sigmoidf(av);
    st(da, i, gv * bv * s * (1.f + av * (1.f - s)));
    st(db, i, gv * av * s);
  }
}

// 4-wide SwiGLU (8-byte bf16 / 16-byte fp32 accesses; n % 4 == 0, 16-byte aligned operands):
// the [tokens, 14336] gate/up pair of the Llama-3-8B MLP is a pure bandwidth pass
template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd4_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                          T* __restrict__ out, size_t n4) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 av = ld4(a + 4 * i), bv = ld4(b + 4 * i);
    st4(out + 4 * i, make_float4(av.x * sigmoidf(av.x) * bv.x, av.y * sigmoidf(av.y) * bv.y,
                                 av.z * sigmoidf(av.z) * bv.z, av.w * sigmoidf(av.w) * bv.w));
  }
}

__device__ __forceinline__ void swiglu_grad1(float a, float b, float g, float& da, float& db) {
  const float s = sigmoidf(a);
  da = g * b * s * (1.f + a * (1.f - s));
  db = g * a * s;
}

template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd4_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                          const T* __restrict__ g, T* __restrict__ da,
                                                          T* __restrict__ db, size_t n4) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 av = ld4(a + 4 * i), bv = ld4(b + 4 * i), gv = ld4(g + 4 * i);
    float4 x, y;
    swiglu_grad1(av.x, bv.x, gv.x, x.x, y.x);
    swiglu_grad1(av.y, bv.y, gv.y, x.y, y.y);
    swiglu_grad1(av.z, bv.z, gv.z, x.z, y.z);
    swiglu_grad1(av.w, bv.w, gv.w, x.w, y.w);
    st4(da + 4 * i, x);
    st4(db + 4 * i, y);
  }
}

bool aligned16(std::initializer_list<const void*> ps) {
  for (const void* p : ps)
    if (reinterpret_cast<uintptr_t>(p) % 16 != 0) return false;
  return true;
}

// x: [B, S, H, hd] contiguous, pairs (2j, 2j+1) rotated by angle (pos, j); sign = +1 fwd, -1 bwd
template <typename T>
__global__ __launch_bounds__(256) void rope_kernel(const T* __restrict__ x, const float* __restrict__ cosv,
                                                   const float* __restrict__ sinv, T* __restrict__ out, int S, int H,
                                                   int hd, size_t npairs, float sign) {
  const int half = hd >> 1;
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(p % half);
    const size_t rowi = p / half;  // (b, s, h)
    const int s = (int)((rowi / H) % S);
    const float c = cosv[(size_t)s * half + j], sn = sign * sinv[(size_t)s * half + j];
    const float x0 = ld(x, 2 * p), x1 = ld(x, 2 * p + 1);
    st(out, 2 * p, x0 * c - x1 * sn);
    st(out, 2 * p + 1, x0 * sn + x1 * c);
  }
}

int grid_for(size_t n) {
  size_t b = (n + 255) / 256;
  return (int)(b > 16384 ? 16384 : (b == 0 ? 1 : b));
}

// ---- softmax cross-entropy over bf16 / fp32 logits [R, V] (V % 8 == 0), mean over rows:
// forward = one read of the logits (online max / sum-exp per row: 8-element vectors, wave
// shuffles, then the 4 waves in order) -> per-row loss and log-sum-exp; backward = one more read
// and one write: dlogits = (softmax - onehot) * g / R, with the upstream scalar g read on device.
// Replaces the fp32 upcast + log_softmax + nll (and their backward) of nn.CrossEntropyLoss.
__device__ __forceinline__ void ms_combine(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) {
    m = m2;
    s = s2;
    return;
  }
  if (m2 > m) {
    s = s * __expf(m - m2) + s2;
    m = m2;
  } else {
    s += s2 * __expf(m2 - m);
  }
}

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&v)[8]) {
  const float4 a = ld4(p), b = ld4(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <typename T>
__global__ __launch_bounds__(256) void xent_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                       float* __restrict__ loss, float* __restrict__ lse, int V) {
  __shared__ float sm[4], ss[4];
  const int row = blockIdx.x;
  const T* x = logits + (size_t)row * V;
  float m = -INFINITY, s = 0.f;
  for (int i = threadIdx.x * 8; i < V; i += 256 * 8) {
    float v[8];
    ld8(x + i, v);
    float vm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) vm = fmaxf(vm, v[j]);
    float vs = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) vs += __expf(v[j] - vm);
    ms_combine(m, s, vm, vs);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float m2 = __shfl_xor(m, off, 64), s2 = __shfl_xor(s, off, 64);
    ms_combine(m, s, m2, s2);
  }
  if ((threadIdx.x & 63) == 0) {
    sm[threadIdx.x >> 6] = m;
    ss[threadIdx.x >> 6] = s;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  m = sm[0];
  s = ss[0];
  for (int w = 1; w < 4; ++w) ms_combine(m, s, sm[w], ss[w]);
  const float l = m + __logf(s);
  lse[row] = l;
  const int64_t t = tgt[row];
  loss[row] = (t >= 0 && t < V) ? l - ld(x, (size_t)t) : NAN;  // an out-of-range target poisons the loss
}

template <typename T>
__global__ __launch_bounds__(256) void xent_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                       const float* __restrict__ lse, const float* __restrict__ g,
                                                       float inv_n, T* __restrict__ dlogits, int V) {
  const int row = blockIdx.x;
  const T* x = logits + (size_t)row * V;
  T* d = dlogits + (size_t)row * V;
  const float l = lse[row], scale = g[0] * inv_n;
  const int64_t t = tgt[row];
  for (int i = threadIdx.x * 8; i < V; i += 256 * 8) {
    float v[8];
    ld8(x + i, v);
    float4 a, b;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (__expf(v[j] - l) - (i + j == t ? 1.f : 0.f)) * scale;
    a = make_float4(o[0], o[1], o[2], o[3]);
    b = make_float4(o[4], o[5], o[6], o[7]);
    st4(d + i, a);
    st4(d + i + 4, b);
  }
}

bool use4(int D) { return D % 4 == 0 && D / 4 <= 256 * kMaxQ; }

}  // namespace

int cs_rmsnorm_bwd_partials(int rows, int D) {
  return use4(D) ? (rows + kRows4 - 1) / kRows4 : (rows + kRowsPerBlock - 1) / kRowsPerBlock;
}

#define CS_DT_DISPATCH(dt, ...)                                         \
  do {                                                                  \
    if ((dt) == CS_F32) {                                               \
      using T = float;                                                  \
      __VA_ARGS__;                                                      \
    } else if ((dt) == CS_BF16) {                                       \
      using T = __hip_bfloat16;                                         \
      __VA_ARGS__;                                                      \
    } else {                                                            \
      return hipErrorInvalidValue;                                      \
    }                                                                   \
  } while (0)

#define CS_DT_DISPATCH2(dt, U, ...)                                    \
  do {                                                                  \
    if ((dt) == CS_F32) {                                               \
      using U = float;                                                  \
      __VA_ARGS__;                                                      \
    } else if ((dt) == CS_BF16) {                                       \
      using U = __hip_bfloat16;                                         \
      __VA_ARGS__;                                                      \
    } else {                                                            \
      return hipErrorInvalidValue;                                      \
    }                                                                   \
  } while (0)

hipError_t cs_rmsnorm_fwd(int dt, int wdt, int odt, const void* x, const void* w, void* y, float* rstd, int rows,
                          int D, float eps, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  if (use4(D)) {
    CS_DT_DISPATCH2(dt, T, CS_DT_DISPATCH2(wdt, Wt, CS_DT_DISPATCH2(odt, O,
        hipLaunchKernelGGL((rmsnorm_fwd4_kernel<T, Wt, O>), dim3(rows), dim3(256), 0, s, (const T*)x, (const Wt*)w,
                           (O*)y, rstd, rows, D, eps))));
    return hipGetLastError();
  }
  if (odt != dt) return hipErrorInvalidValue;  // the scalar path writes the input's dtype
  if (wdt == CS_F32) {
    CS_DT_DISPATCH(dt, hipLaunchKernelGGL((rmsnorm_fwd_kernel<T, float>), dim3(rows), dim3(256), 0, s,
                                          (const T*)x, (const float*)w, (T*)y, rstd, rows, D, eps));
  } else {
    CS_DT_DISPATCH(dt, hipLaunchKernelGGL((rmsnorm_fwd_kernel<T, __hip_bfloat16>), dim3(rows), dim3(256), 0, s,
                                          (const T*)x, (const __hip_bfloat16*)w, (T*)y, rstd, rows, D, eps));
  }
  return hipGetLastError();
}

hipError_t cs_rmsnorm_bwd(int dt, int wdt, int gdt, const void* x, const void* w, const float* rstd, const void* g,
                          void* dx, void* dw, float* part, int rows, int D, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  const int P = cs_rmsnorm_bwd_partials(rows, D);
  if (use4(D)) {
    CS_DT_DISPATCH2(dt, T, CS_DT_DISPATCH2(wdt, Wt, CS_DT_DISPATCH2(gdt, G,
        hipLaunchKernelGGL((rmsnorm_bwd4_kernel<T, Wt, G>), dim3(P), dim3(256), 0, s, (const T*)x, (const Wt*)w,
                           rstd, (const G*)g, (T*)dx, part, rows, D))));
    CS_DT_DISPATCH2(wdt, Wt, hipLaunchKernelGGL((colsum4_kernel<Wt>), dim3((D / 4 + 15) / 16), dim3(256), 0, s,
                                                part, P, D, (Wt*)dw));
    return hipGetLastError();
  }
  if (gdt != dt) return hipErrorInvalidValue;  // the scalar path reads the gradient in the input's dtype
  if (wdt == CS_F32) {
    CS_DT_DISPATCH(dt, hipLaunchKernelGGL((rmsnorm_bwd_kernel<T, float>), dim3(P), dim3(256), 0, s, (const T*)x,
                                          (const float*)w, rstd, (const T*)g, (T*)dx, part, rows, D));
    hipLaunchKernelGGL((colsum_kernel<float>), dim3((D + 255) / 256), dim3(256), 0, s, part, P, D, (float*)dw);
  } else {
    CS_DT_DISPATCH(dt, hipLaunchKernelGGL((rmsnorm_bwd_kernel<T, __hip_bfloat16>), dim3(P), dim3(256), 0, s,
                                          (const T*)x, (const __hip_bfloat16*)w, rstd, (const T*)g, (T*)dx, part,
                                          rows, D));
    hipLaunchKernelGGL((colsum_kernel<__hip_bfloat16>), dim3((D + 255) / 256), dim3(256), 0, s, part, P, D,
                       (__hip_bfloat16*)dw);
  }
  return hipGetLastError();
}

hipError_t cs_xent_fwd(int dt, const void* logits, const int64_t* tgt, float* loss, float* lse, int R, int V,
                       hipStream_t s) {
  if (R <= 0) return hipSuccess;
  if (V % 8 != 0) return hipErrorInvalidValue;
  CS_DT_DISPATCH(dt, hipLaunchKernelGGL((xent_fwd_kernel<T>), dim3(R), dim3(256), 0, s, (const T*)logits, tgt, loss,
                                        lse, V));
  return hipGetLastError();
}

hipError_t cs_xent_bwd(int dt, const void* logits, const int64_t* tgt, const float* lse, const float* g, float inv_n,
                       void* dlogits, int R, int V, hipStream_t s) {
  if (R <= 0) return hipSuccess;
  if (V % 8 != 0) return hipErrorInvalidValue;
  CS_DT_DISPATCH(dt, hipLaunchKernelGGL((xent_bwd_kernel<T>), dim3(R), dim3(256), 0, s, (const T*)logits, tgt, lse, g,
                                        inv_n, (T*)dlogits, V));
  return hipGetLastError();
}

hipError_t cs_swiglu_fwd(int dt, const void* a, const void* b, void* out, size_t n, hipStream_t s) {
  if (n % 4 == 0 && aligned16({a, b, out})) {
    CS_DT_DISPATCH(dt, hipLaunchKernelGGL((swiglu_fwd4_kernel<T>), dim3(grid_for(n / 4)), dim3(256), 0, s,
                                          (const T*)a, (const T*)b, (T*)out, n / 4));
    return hipGetLastError();
  }
  CS_DT_DISPATCH(dt, hipLaunchKernelGGL((swiglu_fwd_kernel<T>), dim3(grid_for(n)), dim3(256), 0, s, (const T*)a,
                                        (const T*)b, (T*)out, n));
  return hipGetLastError();
}

hipError_t cs_swiglu_bwd(int dt, const void* a, const void* b, const void* g, void* da, void* db, size_t n,
                         hipStream_t s) {
  if (n % 4 == 0 && aligned16({a, b, g, da, db})) {
    CS_DT_DISPATCH(dt, hipLaunchKernelGGL((swiglu_bwd4_kernel<T>), dim3(grid_for(n / 4)), dim3(256), 0, s,
                                          (const T*)a, (const T*)b, (const T*)g, (T*)da, (T*)db, n / 4));
    return hipGetLastError();
  }
  CS_DT_DISPATCH(dt, hipLaunchKernelGGL((swiglu_bwd_kernel<T>), dim3(grid_for(n)), dim3(256), 0, s, (const T*)a,
                                        (const T*)b, (const T*)g, (T*)da, (T*)db, n));
  return hipGetLastError();
}

hipError_t cs_rope(int dt, const void* x, const float* cosv, const float* sinv, void* out, int B, int S, int H, int hd,
                   int inverse, hipStream_t s) {
  if (hd & 1) return hipErrorInvalidValue;
  const size_t npairs = (size_t)B * S * H * (hd / 2);
  if (npairs == 0) return hipSuccess;
  CS_DT_DISPATCH(dt, hipLaunchKernelGGL((rope_kernel<T>), dim3(grid_for(npairs)), dim3(256), 0, s, (const T*)x, cosv,
                                        sinv, (T*)out, S, H, hd, npairs, inverse ? -1.f : 1.f));
  return hipGetLastError();
}
