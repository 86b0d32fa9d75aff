// VggEngine, the F3 conv math's operand bounds (conv_gemm.hip "F3"; launchers.h CS_AMAX_*): which
// SGD launch produces which weight bound, the per-step rotation of the weight bounds, and the
// step / eval entry that re-measures, rotates and resets them.
#include "runtime/vgg_engine_util.h"

#include <algorithm>
#include <vector>

namespace cs {

using namespace vgg;

CsWeightBounds VggEngine::sgd_wb(int64_t off, int64_t n) {
  CsWeightBounds wb{};
  if (!f3_used_ || f3_probe_) return wb;
  // blocks >= 1 (block 0 never runs the F3 math); the conv weight tensor only (OHWI, float4 rows)
  for (int l = 1; l < (int)blocks_.size(); ++l) {
    const VggBlock& b = blocks_[l];
    const int64_t lo = std::max<int64_t>(b.w_off, off), hi = std::min<int64_t>(b.w_off + 9ll * b.cin * b.cout, off + n);
    if (lo >= hi) continue;
    TORCH_CHECK(wb.n < CS_WB_MAX && lo == b.w_off && hi == b.w_off + 9ll * b.cin * b.cout && (lo - off) % 4 == 0,
                "VggEngine: an SGD range must hold whole, float4-aligned conv weight tensors");
    wb.lo[wb.n] = lo - off;
    wb.hi[wb.n] = hi - off;
    wb.amax[wb.n] = amax_wnext(l);
    ++wb.n;
    w_pending_ |= 1u << l;
    if (sgd_deferring_) w_deferred_ |= 1u << l;
  }
  return wb;
}

void VggEngine::rotate_w(hipStream_t s, unsigned mask) {
  if (mask == 0) return;
  ok(cs_amax_rotate(amax_w(0), amax_wnext(0), mask, (int)blocks_.size(), s), "amax_rotate");
  w_pending_ &= ~mask;
  w_deferred_ &= ~mask;
}

void VggEngine::f3_refresh(hipStream_t s, bool zero_later) {
  rot_mask_ = 0;
  if (!f3_used_ || f3_probe_) return;
  const int L = (int)blocks_.size();
  if (w_dirty_) {
    // weights written outside the SGD (init, load, broadcast): measure them; drop pending bounds
    ok(hipMemsetAsync(amax_w(0), 0, (size_t)2 * L * CS_AMAX_SLOT * sizeof(float), s), "amax(w) reset");
    for (int l = 1; l < L; ++l) {
      const VggBlock& b = blocks_[l];
      ok(cs_amax(P(b.w_off), (int64_t)b.cout * 9 * b.cin, amax_w(l), s), "amax(w)");
    }
    w_dirty_ = false;
    w_pending_ = w_deferred_ = 0;
  }
  // deferred buckets' bounds wait for their join (forward_train), unless it already happened
  const unsigned rot = defer_comm_ == nullptr ? w_pending_ : (w_pending_ & ~w_deferred_);
  if (zero_later) {  // both ride the conv0 forward launch
    rot_mask_ = rot;
    w_pending_ &= ~rot;
    w_deferred_ &= ~rot;
    return;
  }
  rotate_w(s, rot);
  // x / dz bounds are per step: folded in by this step's BN apply / backward launches
  ok(hipMemsetAsync(amax_x(0), 0, (size_t)2 * L * CS_AMAX_SLOT * sizeof(float), s), "amax(x, dz) reset");
}

void VggEngine::set_f3_probe(bool on) {
  if (!on && f3_probe_) w_dirty_ = true;  // the real weight bounds were not kept: re-measure them
  f3_probe_ = on;
  if (on) amax_.fill_(1.0f);
}

}  // namespace cs
