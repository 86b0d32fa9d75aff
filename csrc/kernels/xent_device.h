// The classifier's per-column pass (xent.hip) as a per-wave device body, shared by its own launch
// and by the side stream's top-block weight-gradient launch, which carries it as extra workgroups
// (conv_gemm.hip, CsConvArgs::head): one definition, so both give the same bits.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "launchers.h"

namespace cs_head {

// head block hb of h.P = C * ceil(K / 64) + 1, run by one wave (lane = threadIdx.x & 63):
// hb < C * nkc: dW[j][k] = sum_b dl[b][j] feat[b][k] for one class j and 64 consecutive k (the
// b-loop unrolled so the loads pipeline); the last: db and the batch loss / correct count. Fixed
// summation order: deterministic.
__device__ __forceinline__ void cols_wave(const CsHeadCols& h, int hb, int lane) {
  const int B = h.B, K = h.K, C = h.C;
  const float* dl = h.ws;
  const float* rowloss = h.ws + (size_t)B * C;
  const float* rowcorr = rowloss + B;
  const int nkc = (K + 63) / 64;
  if (h.dW != nullptr && hb < C * nkc) {
    const int j = hb / nkc, k = (hb - j * nkc) * 64 + lane;
    if (k >= K) return;
    const float* feat = h.feat;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int b = 0;
    // 16 rows of loads in flight, then the adds in the 4-accumulator order of the loop below
    for (; b + 16 <= B; b += 16) {
      float d[16], f[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        d[i] = dl[(size_t)(b + i) * C + j];
        f[i] = feat[(size_t)(b + i) * K + k];
      }
#pragma unroll
      for (int i = 0; i < 16; i += 4) {
        s0 += d[i] * f[i];
        s1 += d[i + 1] * f[i + 1];
        s2 += d[i + 2] * f[i + 2];
        s3 += d[i + 3] * f[i + 3];
      }
    }
    for (; b + 4 <= B; b += 4) {
      s0 += dl[(size_t)b * C + j] * feat[(size_t)b * K + k];
      s1 += dl[(size_t)(b + 1) * C + j] * feat[(size_t)(b + 1) * K + k];
      s2 += dl[(size_t)(b + 2) * C + j] * feat[(size_t)(b + 2) * K + k];
      s3 += dl[(size_t)(b + 3) * C + j] * feat[(size_t)(b + 3) * K + k];
    }
    for (; b < B; ++b) s0 += dl[(size_t)b * C + j] * feat[(size_t)b * K + k];
    h.dW[(size_t)j * K + k] = (s0 + s1) + (s2 + s3);
    return;
  }
  float l = 0.f, c = 0.f;
  for (int r = lane; r < B; r += 64) {
    l += rowloss[r];
    c += rowcorr[r];
  }
  l = cs::wave_sum(l);
  c = cs::wave_sum(c);
  if (lane == 0) {
    if (h.loss_out) *h.loss_out = l / (float)B;
    if (h.correct_out) *h.correct_out = (int)(c + 0.5f);
  }
  if (h.db != nullptr && lane < C) {
    float acc = 0.f;
    for (int r = 0; r < B; ++r) acc += dl[(size_t)r * C + lane];
    h.db[lane] = acc;
  }
}

}  // namespace cs_head
