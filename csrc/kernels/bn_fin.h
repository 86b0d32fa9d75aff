// Last-arriver BatchNorm finalize inside the launch that produces the statistics partials
// (the conv GEMM epilogue, or the split-K combine): the separate bn_finalize /
// bn_bwd_finalize launch (one kernel boundary + a latency-bound pass of ~5 us each on MI355X,
// profiles/r3_step_timeline_end.txt) disappears from the step.
//
// Hand-off (cdna_hip_programming.md §6 Guideline 16, the sc1 counter form; MI355X_MICROARCH.md
// § visibility, first row of the sc1 table): every partial is stored write-through (8-B agent
// atomic stores = global_store_dwordx2 sc1), every storing wave drains (vmcnt 0), the block
// barriers, ONE lane adds to the tile group's counter (agent scope); the block whose add comes
// last reads the partials with sc1 loads only (8-B agent atomic loads) — no release / acquire
// fence, no L2 writeback.
//
// Two levels, so no block combines more than 8 partials per thread: row tiles are grouped by
// G = 8 * (256 / NC); the last arriver of a group combines its tiles into a group partial
// (sc1 again) and takes a ticket on the column counter; the last group of a column combines
// the groups and writes the per-channel results. Every combine runs in a fixed order (tile
// slices by thread, then the slices in order), independent of which block arrives last:
// deterministic. The last arriver of each counter resets it, so the counters stay zeroed
// between launches (allocated zeroed by the engine).
//
// Partials: FWD (mean, M2) of R-row tiles, [T][C][2] (Chan combine, as bn.hip's finalize);
// BWD (sum g, sum g*xhat, sum xhat) of row tiles, [T][C][4] (plain sums, as bn_bwd_finalize).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "launchers.h"

namespace cs_fin {

typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ void st2(float* p, float a, float b) {
  const unsigned long long v =
      ((unsigned long long)__builtin_bit_cast(unsigned, b) << 32) | __builtin_bit_cast(unsigned, a);
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld2(const float* p) {
  const unsigned long long v =
      __hip_atomic_load((gu64*)const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float2(__builtin_bit_cast(float, (unsigned)v), __builtin_bit_cast(float, (unsigned)(v >> 32)));
}

// FWD partial of row tile t, channel c: (mean, M2)
__device__ __forceinline__ void put_stats(float* part, int C, int t, int c, float mean, float m2) {
  st2(part + ((size_t)t * C + c) * 2, mean, m2);
}
// BWD partial of row tile t, channel c: (sum g, sum g*xhat, sum xhat)
__device__ __forceinline__ void put_sums(float* part, int C, int t, int c, float s0, float s1, float s2) {
  st2(part + ((size_t)t * C + c) * 4, s0, s1);
  st2(part + ((size_t)t * C + c) * 4 + 2, s2, 0.f);
}

__device__ __forceinline__ void chan(float& n, float& m, float& M2, float nb, float mb, float M2b) {
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

struct St {
  float a, b, c, d;  // FWD: n, mean, M2; BWD: s0, s1, s2
};

// rows of the R-row tile t (or of a G-tile group when R = G * rows per tile) out of M
__device__ __forceinline__ float rows_of(int t, int R, int M) {
  const int r = M - t * R;
  return (float)(r < R ? r : R);
}

template <bool BWD>
__device__ __forceinline__ void add(St& s, const St& o) {
  if constexpr (BWD) {
    s.a += o.a; s.b += o.b; s.c += o.c;
  } else {
    chan(s.a, s.b, s.c, o.a, o.b, o.c);
  }
}

// one partial (tile or group) as a state: cnt rows (FWD only)
template <bool BWD>
__device__ __forceinline__ St load_state(const float* part, int C, int t, int c, float cnt) {
  St s;
  if constexpr (BWD) {
    const float2 x = ld2(part + ((size_t)t * C + c) * 4), y = ld2(part + ((size_t)t * C + c) * 4 + 2);
    s.a = x.x; s.b = x.y; s.c = y.x; s.d = 0.f;
  } else {
    const float2 x = ld2(part + ((size_t)t * C + c) * 2);
    s.a = cnt; s.b = x.x; s.c = x.y; s.d = 0.f;
  }
  return s;
}

// Combine partials t0, t0 + 1, ..., t1 - 1 of channels [c0, c0 + NC) (256 working threads:
// thread = slice * NC + channel, slice s takes t0 + s, t0 + s + TPC, ...; then the TPC slice
// states in slice order through LDS) -> the states of threads with slice 0. `trows` = rows per
// partial (FWD counts; the last partial may be short: rows_of with M).
template <bool BWD, int NC>
__device__ __forceinline__ St combine(const float* part, int C, int c0, int t0, int t1, int trows, int M,
                                      float* lds) {
  constexpr int TPC = 256 / NC;
  const int tid = threadIdx.x, c = tid % NC, s = tid / NC;
  St acc{0.f, 0.f, 0.f, 0.f};
  if (tid < 256 && c0 + c < C) {
    // 8 loads in flight before their combines (a dependent chain would wait one latency each)
    for (int b = t0 + s; b < t1; b += 8 * TPC) {
      St v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int t = b + j * TPC;
        v[j] = t < t1 ? load_state<BWD>(part, C, t, c0 + c, BWD ? 0.f : rows_of(t, trows, M))
                      : St{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) add<BWD>(acc, v[j]);
    }
  }
  if (TPC > 1) {
    if (tid < 256) {
      lds[(s * NC + c) * 4 + 0] = acc.a;
      lds[(s * NC + c) * 4 + 1] = acc.b;
      lds[(s * NC + c) * 4 + 2] = acc.c;
    }
    __syncthreads();
    if (s == 0 && tid < 256) {
      for (int q = 1; q < TPC; ++q) {
        const St o{lds[(q * NC + c) * 4], lds[(q * NC + c) * 4 + 1], lds[(q * NC + c) * 4 + 2], 0.f};
        add<BWD>(acc, o);
      }
    }
    __syncthreads();
  }
  return acc;
}

// per-channel result of the column's last block
template <bool BWD>
__device__ __forceinline__ void finish(const CsBnFin& f, int C, int c, const St& s) {
  if constexpr (BWD) {
    const float k1 = f.gamma[c] * f.invstd[c], k2 = s.a / (float)f.count, k3 = s.b / (float)f.count;
    if (f.dgamma) f.dgamma[c] = s.b;
    if (f.dbeta) f.dbeta[c] = s.a;
    if (f.dbias) f.dbias[c] = -k1 * k3 * s.c;
    f.coef[3 * c] = k1;
    f.coef[3 * c + 1] = k2;
    f.coef[3 * c + 2] = k3;
  } else {
    const float n = s.a, m = s.b, M2 = s.c;
    const float var = M2 / n, inv = 1.0f / sqrtf(var + f.eps);
    const float g = f.gamma[c], b = f.beta[c];
    f.bnv[c] = g * inv;
    f.bnv[C + c] = b - m * g * inv;
    f.bnv[2 * C + c] = m;
    f.bnv[3 * C + c] = inv;
    if (f.rmean != nullptr) {
      const float unb = n > 1.f ? M2 / (n - 1.f) : var;
      f.rmean[c] = (1.f - f.momentum) * f.rmean[c] + f.momentum * m;
      f.rvar[c] = (1.f - f.momentum) * f.rvar[c] + f.momentum * unb;
    }
  }
}

// tiles per level-1 group for NC channels per column tile
template <int NC>
constexpr int group_tiles() { return 8 * (256 / NC); }

// Called by EVERY thread of the block (barriers inside) after its partials of row tile `mt`
// for channels [c0, c0 + NC) (column tile nt) were stored with put_stats / put_sums.
// Memory ordering (why relaxed atomics are enough on gfx950): this is the write-through hand-off
// of MI355X_MICROARCH.md "Valid forms" (first table row) rather than a C++ release/acquire pair:
// (1) every partial is stored by an 8-byte agent-scope atomic store (put_stats / put_sums -> st2:
// `global_store_dwordx2 ... sc1`, write-through), (2) EVERY storing wave drains its stores with an inline-asm
// `s_waitcnt vmcnt(0)` (invisible to the compiler, so it cannot be dropped) before (3) the
// workgroup barrier, after which ONE lane does the agent-scope ticket add, and (4) the last
// arriver reads every partial back with 8-byte agent-scope atomic loads only (combine -> ld2: `sc1`
// loads, which bypass the reading CU's L1) — the guide's "{8-B agent atomics both sides}" form. The C++ memory model does not describe `sc1`, hence no ACQ_REL on the ticket;
// an ISA change that altered these cache semantics would need the agent release/acquire fences
// (cdna_hip_programming.md §6 Guideline 16). Opt-in path (CS_BN_FIN=1), fp64-parity tested.
// part: the partial array ([T][C][2] FWD, [T][C][4] BWD); C: channels; lds >= 1024 + 16 floats
// that no wave still reads.
template <bool BWD, int NC>
__device__ void arrive(const CsBnFin& f, const float* part, int C, int mt, int nt, int c0, float* lds) {
  constexpr int G = group_tiles<NC>();
  const int T = f.T, ng = (T + G - 1) / G, g = mt / G;
  int* cnt = f.cnt + (size_t)nt * (ng + 1);
  int* flag = reinterpret_cast<int*>(lds + 1024);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    const int in_g = (T - g * G) < G ? (T - g * G) : G;
    const int t = __hip_atomic_fetch_add(cnt + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == in_g - 1;
    if (last) __hip_atomic_store(cnt + g, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = last;
  }
  __syncthreads();
  const int last = flag[0];
  __syncthreads();  // flag read by every wave before lds is reused
  if (!last) return;
  const int tid = threadIdx.x, c = tid % NC, s = tid / NC;
  St v = combine<BWD, NC>(part, C, c0, g * G, (g + 1) * G < T ? (g + 1) * G : T, f.R, f.M, lds);
  if (ng > 1) {
    // level 2: publish this group's state, the column's last group combines the groups
    if (s == 0 && tid < 256 && c0 + c < C) {
      if constexpr (BWD) put_sums(f.grp, C, g, c0 + c, v.a, v.b, v.c);
      else put_stats(f.grp, C, g, c0 + c, v.b, v.c);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const int t = __hip_atomic_fetch_add(cnt + ng, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int l2 = t == ng - 1;
      if (l2) __hip_atomic_store(cnt + ng, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = l2;
    }
    __syncthreads();
    const int l2 = flag[0];
    __syncthreads();
    if (!l2) return;
    v = combine<BWD, NC>(f.grp, C, c0, 0, ng, G * f.R, f.M, lds);
  }
  if (s == 0 && tid < 256 && c0 + c < C) finish<BWD>(f, C, c0 + c, v);
  if constexpr (!BWD) {
    if (f.nbt != nullptr && nt == 0 && tid == 0) *f.nbt += 1;
  }
}

}  // namespace cs_fin
