// Internal helpers shared by the VggEngine translation units (vgg_engine.cpp: the step;
// vgg_tiles.cpp: conv tile control and the autotune; vgg_bounds.cpp: the F3 operand bounds).
#pragma once
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <stdlib.h>

#include <stdexcept>
#include <string>

#include "runtime/vgg_engine.h"

namespace cs {
namespace vgg {

const float kMean[3] = {125.3f / 255.f, 123.0f / 255.f, 113.9f / 255.f};  // master/part1/part1.py:66-67
inline const float kStd[3] = {63.0f / 255.f, 62.1f / 255.f, 66.7f / 255.f};
constexpr float kBnMomentum = 0.1f, kBnEps = 1e-5f;
constexpr int64_t kWsElems = 16ll << 20;  // 64 MiB split-K workspace

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

// CS_DEBUG_SYNC=1: race/fault isolation mode — every launch is followed by a
// stream sync + error check (skipped while a hipGraph is being captured), so an async fault
// is reported at the kernel that caused it instead of at a later sync.
inline bool debug_sync() {
  static const bool on = [] {
    const char* e = getenv("CS_DEBUG_SYNC");
    return e != nullptr && atoi(e) != 0;
  }();
  return on;
}

inline void ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("VggEngine: ") + what + ": " + hipGetErrorString(e));
  if (debug_sync()) {
    hipStream_t s = cur_stream();
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusNone) {
      hipError_t e2 = hipStreamSynchronize(s);
      if (e2 == hipSuccess) e2 = hipGetLastError();
      if (e2 != hipSuccess)
        throw std::runtime_error(std::string("VggEngine [debug sync] after ") + what + ": " + hipGetErrorString(e2));
    }
  }
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

struct Dims {
  int64_t M, N, K;
};

inline Dims dims(const VggBlock& b, int mode, int64_t B) {
  const int64_t pix = B * b.H * b.H;
  if (mode == CS_CONV_FWD) return {pix, b.cout, 9ll * b.cin};
  if (mode == CS_CONV_DGRAD) return {pix, b.cin, 9ll * b.cout};
  return {b.cout, 9ll * b.cin, pix};
}

// the split count cs_conv_gemm will actually use (it re-balances K-steps per split)
inline int eff_splits(int64_t K, int splits, int bk) { return cs_conv_effective_splits((int)K, bk, splits); }

// default tile before autotune: ~2 waves of 256 CUs, >= 8 K-steps per split
inline ConvTile default_tile(const VggBlock& b, int mode, int64_t B) {
  const Dims d = dims(b, mode, B);
  ConvTile t;
  t.bm = 64;
  t.bn = 64;
  const int64_t tiles = cdiv(d.M, 64) * cdiv(d.N, 64);
  const int64_t ks = cdiv(d.K, 16);
  int s = 1;
  while (tiles * s < 512 && ks / (2 * s) >= 8 && (2 * s) * d.M * d.N <= kWsElems) s *= 2;
  t.bk = 16;
  t.splits = s;
  return t;
}


}  // namespace vgg
}  // namespace cs
