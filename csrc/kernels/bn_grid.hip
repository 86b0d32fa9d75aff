// One-launch BatchNorm2d (+ReLU, + optional 2x2 max-pool) forward and backward, NHWC fp32, for
// the layers the single-block "fused" kernels (bn.hip) cannot serve — the reference block
// Conv -> BatchNorm2d -> ReLU(inplace) [-> MaxPool2d] (master/part1/model.py:16-25; SURVEY.md
// §2.2 N4-N7).
//
// Why: on the native step's critical path every BN layer cost 2 (forward: finalize, apply) or 3
// (backward: reduce, finalize, apply) launches of 5-9 us each, almost all launch/drain latency
// (measured per-queue timeline, profiles/r3_step_timeline.txt: 197 us of the 762 us main-queue
// time). Here each is ONE launch of P <= 256 blocks (one per CU at most, so every block is
// resident) whose phases meet at grid barriers:
//   backward: partial sums (the same block partition and order as bn.hip's reduce, so the
//             partials are bit-identical) | barrier | per-channel finalize, channels dealt over
//             the blocks, each summing the P partials in a fixed tree order | barrier | dZ apply;
//   forward:  per-channel finalize (Chan combine of the conv epilogue's tile partials, fixed
//             order) dealt over the blocks, running stats | barrier | normalize/ReLU/pool.
// Grid barrier (cdna_hip_programming.md §6 Guideline 16, placement-independent): every wave
// drains its stores, the block barriers, lane 0 releases at agent scope and takes a ticket;
// then polls the counter with memory-side atomics (an L2 of another XCD may hold a stale line)
// and acquires. Every spin is bounded (error word on timeout). The last block out resets the
// counters, so consecutive launches on one stream reuse them without a memset.
// `signal` (optional): a kernel stream link's counter bumped by block 0 as its first action —
// this launch starts only after the previous kernel on its stream completed and released, so
// that is the same "previous work done" edge as a separate link_signal launch, minus the launch.
#include <type_traits>

#include "bn_device.h"
#include "common.h"
#include "launchers.h"

namespace {

constexpr unsigned long long kSpinTicks = 2000000000ull;  // 20 s at the 100 MHz wall clock

__device__ __forceinline__ void link_bump(unsigned long long* signal) {
  if (signal != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_fetch_add(signal, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Counter layout (kBarInts ints, zeroed; every launch leaves it zeroed): barrier i owns
// [i * kBarStride, (i + 1) * kBarStride): 8 group counters 32 ints (128 B) apart, then the top
// counter at +256; the exit counter follows the last barrier.
constexpr int kBarStride = 288;

// all P blocks arrive; returns after every block's earlier global stores are visible.
// BARV 0: one counter, every block polls it with memory-side read-modify-writes (round-3 first
//         version: ~14 us per barrier at P = 256, measured — P RMWs serialise on one address).
// BARV 1: one counter for arrival, polled with agent-scope atomic loads.
// BARV 2: hierarchical arrival — block b counts into group (b & 7)'s counter (its own 128-B
//         line); the last of a group bumps the top counter, which the blocks poll with loads.
template <int BARV>
__device__ __forceinline__ void grid_barrier(unsigned* bar, int i, unsigned P, int* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* top = bar + i * kBarStride + 256;
    unsigned target = P;
    if (BARV == 2) {
      const unsigned g = blockIdx.x & 7u, gs = (P - g + 7u) >> 3;
      target = P < 8u ? P : 8u;
      // acq_rel: releases this block's stores and acquires the earlier arrivals' of its group,
      // so the group's last block releases all of them with its top bump
      const unsigned t = __hip_atomic_fetch_add(bar + i * kBarStride + g * 32, 1u, __ATOMIC_ACQ_REL,
                                                __HIP_MEMORY_SCOPE_AGENT);
      if (t == gs - 1u) __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const unsigned long long t0 = wall_clock64();
    unsigned zero = 0;
    asm volatile("" : "+v"(zero));  // a run-time 0: keeps the BARV 0 poll a memory-side read-modify-write
    for (;;) {
      const unsigned v = BARV == 0 ? __hip_atomic_fetch_add(top, zero, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : __hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v >= target) break;
      if (wall_clock64() - t0 > kSpinTicks) {
        if (err != nullptr) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(BARV == 0 ? 2 : 1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// the last block to finish resets the NB barriers' counters (every block is past every barrier)
__device__ __forceinline__ void grid_exit(unsigned* bar, int NB, unsigned P) {
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(bar + NB * kBarStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == P - 1) {
      for (int i = 0; i < NB; ++i) {
        for (int g = 0; g < 8; ++g) __hip_atomic_store(bar + i * kBarStride + g * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(bar + i * kBarStride + 256, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __hip_atomic_store(bar + NB * kBarStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

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

// fixed-order block reduction of K floats per thread (256 threads): wave butterfly, then the 4
// waves in order; result valid in thread 0
template <int K>
__device__ __forceinline__ void block_sum(float (&v)[K], float* lds) {
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = cs::wave_sum(v[k]);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) lds[wv * K + k] = v[k];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = lds[k] + lds[K + k] + lds[2 * K + k] + lds[3 * K + k];
}

// fixed-order Chan combine over 256 threads (butterfly within waves, then waves in order)
__device__ __forceinline__ void block_chan(float& n, float& m, float& M2, float* lds) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float nb = __shfl_xor(n, off, 64), mb = __shfl_xor(m, off, 64), M2b = __shfl_xor(M2, off, 64);
    chan_combine(n, m, M2, nb, mb, M2b);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
    lds[wv * 3] = n;
    lds[wv * 3 + 1] = m;
    lds[wv * 3 + 2] = M2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    n = m = M2 = 0.f;
    for (int w = 0; w < 4; ++w) chan_combine(n, m, M2, lds[w * 3], lds[w * 3 + 1], lds[w * 3 + 2]);
  }
}

__device__ __forceinline__ float4 bnrelu4(float4 y, float4 s, float4 t) {
  return make_float4(fmaxf(y.x * s.x + t.x, 0.f), fmaxf(y.y * s.y + t.y, 0.f), fmaxf(y.z * s.z + t.z, 0.f),
                     fmaxf(y.w * s.w + t.w, 0.f));
}

// ------------------------------------------------------------------ backward
template <bool POOL, int BARV>
__global__ __launch_bounds__(256) void bn_bwd_grid_kernel(CsBnGridBwd a) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // rows * C * 3 (phase 1), then scratch
  link_bump(a.signal);
  const unsigned P = gridDim.x;
  const int C = a.C;
  // phase 1: this block's partials part[b][C][3] — bn_red_body, the reduce launch's exact code
  const CsBnRed r{a.y, a.G, a.scale, a.shift, a.mean, a.invstd, a.part, a.gstride,
                  a.B, a.H, a.W, C, POOL ? 1 : 0, (int)P, a.gslabs};
  cs_bn::bn_red_body<POOL>(r, blockIdx.x, P, red);
  if (BARV >= 0) grid_barrier<BARV>(a.bar, 0, P, a.err);
  // phase 2: channels b, b + P, ...: sum the P partials (thread t holds p = t, t + 256, ...,
  // then a fixed tree), then the coefficients
  const int M = a.B * a.H * a.W;
  for (int c = blockIdx.x; c < C; c += P) {
    float v[3] = {0.f, 0.f, 0.f};
    for (int p = threadIdx.x; p < (int)P; p += 256) {
      const float* q = a.part + ((size_t)p * C + c) * 3;
      v[0] += q[0];
      v[1] += q[1];
      v[2] += q[2];
    }
    block_sum<3>(v, red);
    if (threadIdx.x == 0) {
      const float k1 = a.gamma[c] * a.invstd[c], k2 = v[0] / (float)M, k3 = v[1] / (float)M;
      if (a.dgamma) a.dgamma[c] = v[1];
      if (a.dbeta) a.dbeta[c] = v[0];
      if (a.dbias) a.dbias[c] = -k1 * k3 * v[2];
      a.coef[3 * c] = k1;
      a.coef[3 * c + 1] = k2;
      a.coef[3 * c + 2] = k3;
    }
  }
  if (BARV >= 0) grid_barrier<BARV>(a.bar, 1, P, a.err);
  // phase 3: dZ over this block's units (the apply pass of bn.hip, coefficients from global)
  const int C4 = C >> 2, rows = 256 / C4;
  const int cq = threadIdx.x % C4, rl = threadIdx.x / C4;
  const int units = POOL ? a.B * (a.H >> 1) * (a.W >> 1) : a.B * a.H * a.W;
  float dummy[3][4];
  if (rl < rows)
    for (int u = blockIdx.x * rows + rl; u < units; u += P * rows)
      cs_bn::bwd_visit<true, POOL>(a.y, a.G, a.B, a.H, a.W, C, cq, u, a.scale, a.shift, a.mean, a.invstd, a.coef, a.dz,
                                   dummy, a.gslabs, a.gstride);
  if (BARV >= 0) grid_exit(a.bar, 2, P);
}

// ------------------------------------------------------------------ forward
template <int BARV>
__global__ __launch_bounds__(256) void bn_fwd_grid_kernel(CsBnGridFwd a) {
  __shared__ float lds[16];
  link_bump(a.signal);
  const unsigned P = gridDim.x;
  const int C = a.C;
  float* scale = a.bnv;
  float* shift = a.bnv + C;
  // phase 1: channels b, b + P, ...: Chan-combine the T tile partials (thread t: tiles t, t + 256,
  // ... in order, then a fixed tree)
  for (int c = blockIdx.x; c < C; c += P) {
    float n = 0.f, m = 0.f, M2 = 0.f;
    for (int t = threadIdx.x; t < a.T; t += 256) {
      const float2 pm = *reinterpret_cast<const float2*>(a.part + ((size_t)t * C + c) * 2);
      chan_combine(n, m, M2, (float)((a.M - t * a.R) < a.R ? (a.M - t * a.R) : a.R), pm.x, pm.y);
    }
    block_chan(n, m, M2, lds);
    if (threadIdx.x == 0) {
      const float var = M2 / n, inv = 1.0f / sqrtf(var + a.eps);
      const float g = a.gamma[c], b = a.beta[c];
      scale[c] = g * inv;
      shift[c] = b - m * g * inv;
      a.bnv[2 * C + c] = m;
      a.bnv[3 * C + c] = inv;
      if (a.running_mean != nullptr) {
        const float unb = n > 1.f ? M2 / (n - 1.f) : var;
        a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * m;
        a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * unb;
      }
    }
  }
  if (a.nbt != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *a.nbt += 1;
  if (BARV >= 0) grid_barrier<BARV>(a.bar, 0, P, a.err);
  // phase 2: relu(y * scale + shift) (2x2 max with pooling), one thread per (unit, 4 channels)
  const int C4 = C >> 2;
  const int Ho = a.pool ? a.H >> 1 : a.H, Wo = a.pool ? a.W >> 1 : a.W;
  const int total = a.B * Ho * Wo * C4;
  const float4* y4 = reinterpret_cast<const float4*>(a.y);
  for (int t = blockIdx.x * 256 + threadIdx.x; t < total; t += P * 256) {
    const int cq = t % C4, pos = t / C4;
    const float4 s = reinterpret_cast<const float4*>(scale)[cq];
    const float4 sh = reinterpret_cast<const float4*>(shift)[cq];
    float4 o;
    if (!a.pool) {
      o = bnrelu4(y4[t], s, sh);
    } else {
      const int wo = pos % Wo, ho = (pos / Wo) % Ho, b = pos / (Wo * Ho);
      const size_t base = (((size_t)b * a.H + 2 * ho) * a.W + 2 * wo) * C4 + cq;
      const float4 a0 = bnrelu4(y4[base], s, sh), a1 = bnrelu4(y4[base + C4], s, sh);
      const float4 a2 = bnrelu4(y4[base + (size_t)a.W * C4], s, sh);
      const float4 a3 = bnrelu4(y4[base + (size_t)a.W * C4 + C4], s, sh);
      o = make_float4(fmaxf(fmaxf(a0.x, a1.x), fmaxf(a2.x, a3.x)), fmaxf(fmaxf(a0.y, a1.y), fmaxf(a2.y, a3.y)),
                      fmaxf(fmaxf(a0.z, a1.z), fmaxf(a2.z, a3.z)), fmaxf(fmaxf(a0.w, a1.w), fmaxf(a2.w, a3.w)));
    }
    reinterpret_cast<float4*>(a.out)[t] = o;
  }
  if (BARV >= 0) grid_exit(a.bar, 1, P);
}

}  // namespace

// experiment knobs (scripts/bn_grid_bench.py): CS_BN_GRID_PMUL = blocks per CU allowed for the
// forward (1..4), CS_BN_GRID_BARV = barrier version (0, 1, 2; -1 skips the barriers: wrong
// results, timing of the phases alone)
static int grid_pmul() {
  static const int v = [] {
    const char* e = getenv("CS_BN_GRID_PMUL");
    const int m = e ? atoi(e) : 1;
    return m < 1 ? 1 : (m > 4 ? 4 : m);
  }();
  return v;
}
static int grid_barv() {
  static const int v = [] {
    const char* e = getenv("CS_BN_GRID_BARV");
    const int b = e ? atoi(e) : 2;
    return b < -1 ? -1 : (b > 2 ? 2 : b);
  }();
  return v;
}

template <typename F>
static void with_barv(F&& f) {
  switch (grid_barv()) {
    case -1: f(std::integral_constant<int, -1>{}); break;
    case 0: f(std::integral_constant<int, 0>{}); break;
    case 1: f(std::integral_constant<int, 1>{}); break;
    default: f(std::integral_constant<int, 2>{}); break;
  }
}

int cs_bn_grid_fwd_blocks(int B, int H, int W, int C, int pool) {
  const int64_t total = (int64_t)B * (pool ? H / 2 : H) * (pool ? W / 2 : W) * (C / 4);
  int64_t p = (total + 255) / 256;
  if (p < C / 2) p = C / 2;  // at least half a block per channel for the finalize phase
  const int64_t cap = 256 * grid_pmul();
  return (int)(p > cap ? cap : (p < 1 ? 1 : p));
}

hipError_t cs_bn_grid_bwd(const CsBnGridBwd& a, hipStream_t stream) {
  if (a.C % 4 != 0 || a.C > 1024 || (a.pool && ((a.H | a.W) & 1)) || a.gslabs < 1 || a.bar == nullptr)
    return hipErrorInvalidValue;
  const int P = cs_bn_bwd_blocks(a.B, a.H, a.W, a.C, a.pool);  // <= 256: every block resident
  const size_t lds = (size_t)(256 / (a.C / 4)) * a.C * 3 * sizeof(float);
  with_barv([&](auto bv) {
    if (a.pool)
      hipLaunchKernelGGL((bn_bwd_grid_kernel<true, decltype(bv)::value>), dim3(P), dim3(256), lds, stream, a);
    else
      hipLaunchKernelGGL((bn_bwd_grid_kernel<false, decltype(bv)::value>), dim3(P), dim3(256), lds, stream, a);
  });
  return hipGetLastError();
}

hipError_t cs_bn_grid_fwd(const CsBnGridFwd& a, hipStream_t stream) {
  if (a.C % 4 != 0 || (a.pool && ((a.H | a.W) & 1)) || a.bar == nullptr || a.T < 1) return hipErrorInvalidValue;
  const int P = cs_bn_grid_fwd_blocks(a.B, a.H, a.W, a.C, a.pool);
  with_barv([&](auto bv) {
    hipLaunchKernelGGL((bn_fwd_grid_kernel<decltype(bv)::value>), dim3(P), dim3(256), 0, stream, a);
  });
  return hipGetLastError();
}
