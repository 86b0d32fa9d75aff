// Training BatchNorm2d (+ optional residual add, + optional ReLU) for NCHW activations in fp32
// or bf16 with fp32 parameters / statistics — the CNN extension config's hot memory-bound ops
// (ResNet-50, models/resnet.py; BASELINE.json "ResNet-50 on synthetic ImageNet-shape").
// Replaces MIOpen's BatchNorm forward/backward plus ATen's separate ReLU and residual-add
// passes (measured on MI355X, ResNet-50 bf16 B=128: BN 31 % and elementwise 10 % of the step,
// profiles/r2_resnet50_bf16_kernels.txt) with fused passes:
//   forward : stats (per (image-chunk, channel) block: shifted sums) -> finalize (C threads,
//             f64 combine, running-stat update, scale/shift) -> apply y = act(x*scale+shift+res)
//   backward: reduce (sum g, sum g*xhat with g = dy masked by the recomputed pre-activation)
//             -> finalize (dgamma, dbeta, coefficients) -> apply dx (+ dres = g)
// Each plane (n, c) is HW contiguous elements; vector width V (8, 4 or 1 elements) divides HW,
// so a vector never straddles two channels. Deterministic: fixed-shape reductions, no atomics.
#include <hip/hip_bf16.h>

#include "common.h"
#include "launchers.h"

namespace {

template <typename T>
struct Vec;
template <>
struct Vec<float> {
  __device__ static float ld(const float* p) { return *p; }
  __device__ static void st(float* p, float v) { *p = v; }
};
template <>
struct Vec<__hip_bfloat16> {
  __device__ static float ld(const __hip_bfloat16* p) { return __bfloat162float(*p); }
  __device__ static void st(__hip_bfloat16* p, float v) { *p = __float2bfloat16(v); }
};

// V consecutive elements of a plane through one (8/16/32-byte) access
template <typename T, int V>
__device__ __forceinline__ void load_v(const T* p, float (&v)[V]) {
  if constexpr (V == 1) {
    v[0] = Vec<T>::ld(p);
  } else {
    constexpr int BYTES = V * (int)sizeof(T);
    typedef unsigned u32v __attribute__((ext_vector_type(BYTES / 4)));
    const u32v raw = *reinterpret_cast<const u32v*>(p);
    const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = Vec<T>::ld(e + j);
  }
}
template <typename T, int V>
__device__ __forceinline__ void store_v(T* p, const float (&v)[V]) {
  if constexpr (V == 1) {
    Vec<T>::st(p, v[0]);
  } else {
    constexpr int BYTES = V * (int)sizeof(T);
    typedef unsigned u32v __attribute__((ext_vector_type(BYTES / 4)));
    u32v raw;
    T* e = reinterpret_cast<T*>(&raw);
#pragma unroll
    for (int j = 0; j < V; ++j) Vec<T>::st(e + j, v[j]);
    *reinterpret_cast<u32v*>(p) = raw;
  }
}

// the pre-activation, computed identically in the forward and in the backward's mask
__device__ __forceinline__ float preact(float x, float scale, float shift, float res) {
  return fmaf(x, scale, shift) + res;
}

__device__ __forceinline__ float block_sum256(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// block (p, c): images [p*npb, min(N, (p+1)*npb)) of channel c -> part[c][p] = {sum(x-K), sum((x-K)^2)}
// with K = the channel's first element (a shift that keeps the f32 sums well conditioned)
template <typename T, int V>
__global__ __launch_bounds__(256) void stats_kernel(const T* __restrict__ x, int N, int C, int HW, int npb,
                                                    float* __restrict__ part) {
  __shared__ float red[4];
  const int p = blockIdx.x, c = blockIdx.y, P = gridDim.x;
  const float K = Vec<T>::ld(x + (size_t)c * HW);
  const int n0 = p * npb, n1 = min(N, n0 + npb);
  const int per = HW / V, total = (n1 - n0) * per;
  float s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < total; i += 256) {
    const int n = n0 + i / per, e = (i % per) * V;
    float v[V];
    load_v<T, V>(x + ((size_t)n * C + c) * HW + e, v);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float d = v[j] - K;
      s1 += d;
      s2 = fmaf(d, d, s2);
    }
  }
  s1 = block_sum256(s1, red);
  s2 = block_sum256(s2, red);
  if (threadIdx.x == 0) {
    part[((size_t)c * P + p) * 2 + 0] = s1;
    part[((size_t)c * P + p) * 2 + 1] = s2;
  }
}

// one thread per channel: mean / biased var (normalisation), unbiased var (running stats)
template <typename T>
__global__ __launch_bounds__(256) void finalize_fwd_kernel(const T* __restrict__ x, const float* __restrict__ part,
                                                           int P, int C, int HW, double M, const float* __restrict__ w,
                                                           const float* __restrict__ b, float* __restrict__ rm,
                                                           float* __restrict__ rv, float momentum, float eps,
                                                           float* __restrict__ stat /* [4][C] */,
                                                           int64_t* __restrict__ nbt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt != nullptr) *nbt += 1;  // num_batches_tracked
  if (c >= C) return;
  double s1 = 0.0, s2 = 0.0;
  for (int p = 0; p < P; ++p) {
    s1 += (double)part[((size_t)c * P + p) * 2 + 0];
    s2 += (double)part[((size_t)c * P + p) * 2 + 1];
  }
  const double K = (double)Vec<T>::ld(x + (size_t)c * HW);
  const double dm = s1 / M;
  double var = s2 / M - dm * dm;
  if (var < 0.0) var = 0.0;
  const double mean = K + dm;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float scale = (w != nullptr ? w[c] : 1.f) * invstd;
  const float shift = (b != nullptr ? b[c] : 0.f) - (float)mean * scale;
  stat[c] = scale;
  stat[C + c] = shift;
  stat[2 * C + c] = (float)mean;
  stat[3 * C + c] = invstd;
  if (rm != nullptr) {
    const double unbiased = M > 1.0 ? var * M / (M - 1.0) : var;
    rm[c] = (1.f - momentum) * rm[c] + momentum * (float)mean;
    rv[c] = (1.f - momentum) * rv[c] + momentum * (float)unbiased;
  }
}

template <typename T, int V>
__global__ __launch_bounds__(256) void apply_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                        const float* __restrict__ stat, T* __restrict__ y, int C,
                                                        int HW, int64_t nvec, int relu) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int64_t e = i * V;
    const int c = (int)((e / HW) % C);
    const float sc = stat[c], sh = stat[C + c];
    float v[V], r[V];
    load_v<T, V>(x + e, v);
    if (res != nullptr) load_v<T, V>(res + e, r);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float z = preact(v[j], sc, sh, res != nullptr ? r[j] : 0.f);
      v[j] = relu && !(z > 0.f) ? 0.f : z;
    }
    store_v<T, V>(y + e, v);
  }
}

// g = dy masked by the recomputed pre-activation; part[c][p] = {sum g, sum g*xhat}
template <typename T, int V>
__global__ __launch_bounds__(256) void bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                         const T* __restrict__ res, const float* __restrict__ stat,
                                                         int N, int C, int HW, int npb, int relu,
                                                         float* __restrict__ part) {
  __shared__ float red[4];
  const int p = blockIdx.x, c = blockIdx.y, P = gridDim.x;
  const float sc = stat[c], sh = stat[C + c], mean = stat[2 * C + c], invstd = stat[3 * C + c];
  const int n0 = p * npb, n1 = min(N, n0 + npb);
  const int per = HW / V, total = (n1 - n0) * per;
  float sg = 0.f, sgx = 0.f;
  for (int i = threadIdx.x; i < total; i += 256) {
    const int n = n0 + i / per, e = (i % per) * V;
    const size_t off = ((size_t)n * C + c) * HW + e;
    float g[V], v[V], r[V];
    load_v<T, V>(dy + off, g);
    load_v<T, V>(x + off, v);
    if (relu && res != nullptr) load_v<T, V>(res + off, r);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      if (relu && !(preact(v[j], sc, sh, res != nullptr ? r[j] : 0.f) > 0.f)) g[j] = 0.f;
      sg += g[j];
      sgx = fmaf(g[j], (v[j] - mean) * invstd, sgx);
    }
  }
  sg = block_sum256(sg, red);
  sgx = block_sum256(sgx, red);
  if (threadIdx.x == 0) {
    part[((size_t)c * P + p) * 2 + 0] = sg;
    part[((size_t)c * P + p) * 2 + 1] = sgx;
  }
}

// dbeta = sum g, dgamma = sum g*xhat; coef[c] = {gamma*invstd, sum g / M, sum g*xhat / M}
__global__ __launch_bounds__(256) void finalize_bwd_kernel(const float* __restrict__ part, int P, int C, double M,
                                                           const float* __restrict__ w, const float* __restrict__ stat,
                                                           float* __restrict__ dw, float* __restrict__ db,
                                                           float* __restrict__ coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double sg = 0.0, sgx = 0.0;
  for (int p = 0; p < P; ++p) {
    sg += (double)part[((size_t)c * P + p) * 2 + 0];
    sgx += (double)part[((size_t)c * P + p) * 2 + 1];
  }
  if (dw != nullptr) dw[c] = (float)sgx;
  if (db != nullptr) db[c] = (float)sg;
  coef[c] = (w != nullptr ? w[c] : 1.f) * stat[3 * C + c];
  coef[C + c] = (float)(sg / M);
  coef[2 * C + c] = (float)(sgx / M);
}

template <typename T, int V>
__global__ __launch_bounds__(256) void apply_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                        const T* __restrict__ res, const float* __restrict__ stat,
                                                        const float* __restrict__ coef, T* __restrict__ dx,
                                                        T* __restrict__ dres, int C, int HW, int64_t nvec, int relu) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int64_t e = i * V;
    const int c = (int)((e / HW) % C);
    const float sc = stat[c], sh = stat[C + c], mean = stat[2 * C + c], invstd = stat[3 * C + c];
    const float k = coef[c], mg = coef[C + c], mgx = coef[2 * C + c];
    float g[V], v[V], r[V];
    load_v<T, V>(dy + e, g);
    load_v<T, V>(x + e, v);
    if (relu && res != nullptr) load_v<T, V>(res + e, r);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      if (relu && !(preact(v[j], sc, sh, res != nullptr ? r[j] : 0.f) > 0.f)) g[j] = 0.f;
      const float xhat = (v[j] - mean) * invstd;
      v[j] = k * (g[j] - mg - xhat * mgx);
    }
    store_v<T, V>(dx + e, v);
    if (dres != nullptr) store_v<T, V>(dres + e, g);
  }
}

int vec_width(int HW, int esize) {
  const int v16 = 16 / esize;  // elements per 16-byte access
  if (HW % v16 == 0) return v16;
  if (HW % 4 == 0) return 4;
  return 1;
}

int chunks(int N, int C) {
  int P = (2048 + C - 1) / C;
  return P < 1 ? 1 : (P > N ? N : P);
}

int apply_grid(int64_t nvec) {
  const int64_t b = (nvec + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}

template <typename T, int V>
void fwd_t(const void* x, const void* res, const float* w, const float* b, float* rm, float* rv, int64_t* nbt,
           float momentum, float eps, int relu, void* y, float* stat, float* part, int N, int C, int HW,
           hipStream_t st) {
  const int P = chunks(N, C), npb = (N + P - 1) / P;
  hipLaunchKernelGGL((stats_kernel<T, V>), dim3(P, C), dim3(256), 0, st, (const T*)x, N, C, HW, npb, part);
  hipLaunchKernelGGL(finalize_fwd_kernel<T>, dim3((C + 255) / 256), dim3(256), 0, st, (const T*)x, part, P, C, HW,
                     (double)N * HW, w, b, rm, rv, momentum, eps, stat, nbt);
  const int64_t nvec = (int64_t)N * C * HW / V;
  hipLaunchKernelGGL((apply_fwd_kernel<T, V>), dim3(apply_grid(nvec)), dim3(256), 0, st, (const T*)x, (const T*)res,
                     stat, (T*)y, C, HW, nvec, relu);
}

template <typename T, int V>
void bwd_t(const void* dy, const void* x, const void* res, const float* w, const float* stat, int relu, void* dx,
           void* dres, float* dw, float* db, float* coef, float* part, int N, int C, int HW, hipStream_t st) {
  const int P = chunks(N, C), npb = (N + P - 1) / P;
  hipLaunchKernelGGL((bwd_reduce_kernel<T, V>), dim3(P, C), dim3(256), 0, st, (const T*)dy, (const T*)x,
                     (const T*)res, stat, N, C, HW, npb, relu, part);
  hipLaunchKernelGGL(finalize_bwd_kernel, dim3((C + 255) / 256), dim3(256), 0, st, part, P, C, (double)N * HW, w,
                     stat, dw, db, coef);
  const int64_t nvec = (int64_t)N * C * HW / V;
  hipLaunchKernelGGL((apply_bwd_kernel<T, V>), dim3(apply_grid(nvec)), dim3(256), 0, st, (const T*)dy, (const T*)x,
                     (const T*)res, stat, coef, (T*)dx, (T*)dres, C, HW, nvec, relu);
}

}  // namespace

int cs_bn_nchw_partials(int N, int C) { return chunks(N, C) * C * 2; }

hipError_t cs_bn_nchw_fwd(int dt, const void* x, const void* res, const float* w, const float* b, float* rm, float* rv,
                          int64_t* nbt, float momentum, float eps, int relu, void* y, float* stat, float* part, int N,
                          int C, int HW, hipStream_t stream) {
  if ((int64_t)N * C * HW == 0) return hipSuccess;
  if (dt == CS_BF16) {
    const int V = vec_width(HW, 2);
    if (V == 8) fwd_t<__hip_bfloat16, 8>(x, res, w, b, rm, rv, nbt, momentum, eps, relu, y, stat, part, N, C, HW, stream);
    else if (V == 4) fwd_t<__hip_bfloat16, 4>(x, res, w, b, rm, rv, nbt, momentum, eps, relu, y, stat, part, N, C, HW, stream);
    else fwd_t<__hip_bfloat16, 1>(x, res, w, b, rm, rv, nbt, momentum, eps, relu, y, stat, part, N, C, HW, stream);
  } else {
    const int V = vec_width(HW, 4);
    if (V == 4) fwd_t<float, 4>(x, res, w, b, rm, rv, nbt, momentum, eps, relu, y, stat, part, N, C, HW, stream);
    else fwd_t<float, 1>(x, res, w, b, rm, rv, nbt, momentum, eps, relu, y, stat, part, N, C, HW, stream);
  }
  return hipGetLastError();
}

hipError_t cs_bn_nchw_bwd(int dt, const void* dy, const void* x, const void* res, const float* w, const float* stat,
                          int relu, void* dx, void* dres, float* dw, float* db, float* coef, float* part, int N, int C,
                          int HW, hipStream_t stream) {
  if ((int64_t)N * C * HW == 0) return hipSuccess;
  if (dt == CS_BF16) {
    const int V = vec_width(HW, 2);
    if (V == 8) bwd_t<__hip_bfloat16, 8>(dy, x, res, w, stat, relu, dx, dres, dw, db, coef, part, N, C, HW, stream);
    else if (V == 4) bwd_t<__hip_bfloat16, 4>(dy, x, res, w, stat, relu, dx, dres, dw, db, coef, part, N, C, HW, stream);
    else bwd_t<__hip_bfloat16, 1>(dy, x, res, w, stat, relu, dx, dres, dw, db, coef, part, N, C, HW, stream);
  } else {
    const int V = vec_width(HW, 4);
    if (V == 4) bwd_t<float, 4>(dy, x, res, w, stat, relu, dx, dres, dw, db, coef, part, N, C, HW, stream);
    else bwd_t<float, 1>(dy, x, res, w, stat, relu, dx, dres, dw, db, coef, part, N, C, HW, stream);
  }
  return hipGetLastError();
}
