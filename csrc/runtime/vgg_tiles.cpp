// VggEngine, conv tile control: set / get a GEMM's tile (shape, K-step, split-K, staging, math),
// run one conv GEMM of the step, and the per-GEMM autotune (HIP-event timed).
#include "runtime/vgg_engine_util.h"

#include <algorithm>
#include <vector>

namespace cs {

using namespace vgg;

void VggEngine::set_tile(int64_t block, int64_t mode, int64_t bm, int64_t bn, int64_t splits, int64_t bk,
                         int64_t stage) {
  TORCH_CHECK(block >= 0 && block < (int64_t)blocks_.size() && mode >= 0 && mode <= 2, "set_tile: index");
  TORCH_CHECK((bm == 64 || bm == 128) && (bn == 64 || bn == 128) && splits >= 1 && splits <= 1024, "set_tile: tile");
  const Dims d = dims(blocks_[block], (int)mode, Bmax_);
  const bool conv0_fwd = block == 0 && mode == CS_CONV_FWD && blocks_[0].cin == 4;
  TORCH_CHECK((bk == 16 || bk == 32 || bk == 64) && cs_conv_stage_ok((int)stage, (int)bm, (int)bn, (int)bk, conv0_fwd) &&
                  !(conv0_fwd && bk == 64),
              "set_tile: no kernel for stage ", stage, " with a ", bm, "x", bn, " tile and bk ", bk);
  // block 0's input has no producer-written bound (make_batch / the conv0 batch fold)
  TORCH_CHECK(!(stage & CS_STAGE_F3) || block > 0, "set_tile: the F3 conv math is for blocks >= 1");
  const int sp = eff_splits(d.K, (int)splits, (int)bk);
  TORCH_CHECK(sp == 1 || (int64_t)sp * d.M * d.N <= ws_elems_, "set_tile: split-K workspace too small");
  ConvTile& t = blocks_[block].tile[mode];
  t.bm = (int)bm;
  t.bn = (int)bn;
  t.splits = (int)splits;
  t.bk = (int)bk;
  t.stage = (int)stage;
  t.us = -1.f;
  update_f3_used();
}

void VggEngine::update_f3_used() {
  bool used = false;
  for (const VggBlock& b : blocks_)
    for (const ConvTile& t : b.tile) used = used || (t.stage & CS_STAGE_F3) != 0;
  if (used && !f3_used_) w_dirty_ = true;  // the weights' bounds were not kept while no tile needed them
  f3_used_ = used;
}

std::vector<int64_t> VggEngine::get_tile(int64_t block, int64_t mode) const {
  TORCH_CHECK(block >= 0 && block < (int64_t)blocks_.size() && mode >= 0 && mode <= 2, "get_tile: index");
  const ConvTile& t = blocks_[block].tile[mode];
  return {t.bm, t.bn, t.splits, t.bk, t.stage};
}

void VggEngine::run_conv(int64_t block, int64_t mode, int64_t B) {
  TORCH_CHECK(block >= 0 && block < (int64_t)blocks_.size() && mode >= 0 && mode <= 2, "run_conv: index");
  TORCH_CHECK(!(block == 0 && mode == CS_CONV_DGRAD), "run_conv: no dgrad for block 0");
  TORCH_CHECK(B > 0 && B <= Bmax_, "run_conv: B");
  conv((int)block, (int)mode, (int)B, blocks_[block].tile[mode], cur_stream(), mode == CS_CONV_FWD);
}

std::vector<double> VggEngine::autotune(int64_t B, int64_t iters) {
  TORCH_CHECK(B > 0 && B <= Bmax_ && iters >= 1, "autotune: args");
  hipStream_t s = cur_stream();
  hipEvent_t e0, e1;
  ok(hipEventCreate(&e0), "event");
  ok(hipEventCreate(&e1), "event");
  std::vector<double> best_us;
  const int split_opts[] = {1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 64, 128, 256};
  for (int l = 0; l < (int)blocks_.size(); ++l) {
    for (int mode = 0; mode < 3; ++mode) {
      if (l == 0 && mode == CS_CONV_DGRAD) {
        best_us.push_back(0.0);
        continue;
      }
      const Dims d = dims(blocks_[l], mode, B);
      ConvTile best = blocks_[l].tile[mode];
      float best_t = 1e30f;
      std::vector<std::vector<int>> seen;
      const bool conv0_fwd = l == 0 && mode == CS_CONV_FWD && blocks_[0].cin == 4;
      for (int stage : {(int)CS_STAGE_REGS, (int)CS_STAGE_LDS_DMA, (int)CS_STAGE_LDS_DMA_DEEP, (int)CS_STAGE_KG2,
                        (int)CS_STAGE_KG4, CS_STAGE_X6 | CS_STAGE_REGS, CS_STAGE_X6 | CS_STAGE_LDS_DMA,
                        CS_STAGE_X6 | CS_STAGE_LDS_DMA_DEEP, CS_STAGE_X6 | CS_STAGE_KG2, CS_STAGE_X6 | CS_STAGE_KG4,
                        CS_STAGE_X6S | CS_STAGE_REGS, CS_STAGE_X6S | CS_STAGE_KG2, CS_STAGE_X6S | CS_STAGE_KG4,
                        CS_STAGE_F3 | CS_STAGE_REGS, CS_STAGE_F3 | CS_STAGE_KG2, CS_STAGE_F3 | CS_STAGE_KG4,
                        CS_STAGE_BF16 | CS_STAGE_REGS, CS_STAGE_BF16 | CS_STAGE_KG2, CS_STAGE_BF16 | CS_STAGE_KG4})
      for (int bk : {16, 32, 64}) {
        // CS_CONV_MATH: 0 = f32 MFMA kernels only, 1 = the split maths only (X6, X6S, F3), 2 = all
        // of them (default), 3 = bf16 operands (reduced precision, opt-in; the padded conv0 forward
        // stays f32). F3 (scaled fp16 hi/lo) is not for block 0 (no producer-written input bound)
        const bool x6 = (stage & (CS_STAGE_X6 | CS_STAGE_X6S | CS_STAGE_F3)) != 0;
        const bool bf = (stage & CS_STAGE_BF16) != 0;
        if ((stage & CS_STAGE_F3) && l == 0) continue;
        if (math_ == 3) {
          if (!bf && !(conv0_fwd && stage == CS_STAGE_REGS)) continue;
        } else if (bf || (x6 && math_ == 0) || (!x6 && math_ == 1)) {
          continue;
        }
        if (bk == 64 && conv0_fwd) continue;
        const int64_t ks = cdiv(d.K, bk);
        for (int bm : {64, 128}) {
          for (int bn : {64, 128}) {
            if (!cs_conv_stage_ok(stage, bm, bn, bk, conv0_fwd)) continue;
            for (int sp : split_opts) {
              if (sp > 1 && ks / sp < 2) continue;
              const int e = eff_splits(d.K, sp, bk);
              if (e > 1 && (int64_t)e * d.M * d.N > ws_elems_) continue;
              std::vector<int> key = {bm, bn, bk, e, stage};
              if (std::find(seen.begin(), seen.end(), key) != seen.end()) continue;
              seen.push_back(key);
              ConvTile t;
              t.bm = bm;
              t.bn = bn;
              t.bk = bk;
              t.splits = sp;
              t.stage = stage;
              conv(l, mode, (int)B, t, s, mode == CS_CONV_FWD);  // warm
              ok(hipEventRecord(e0, s), "record");
              for (int64_t i = 0; i < iters; ++i) conv(l, mode, (int)B, t, s, mode == CS_CONV_FWD);
              ok(hipEventRecord(e1, s), "record");
              ok(hipEventSynchronize(e1), "sync");
              float ms = 0.f;
              ok(hipEventElapsedTime(&ms, e0, e1), "elapsed");
              const float us = 1000.f * ms / (float)iters;
              if (us < best_t) {
                best_t = us;
                best = t;
              }
            }
          }
        }
      }
      best.us = best_t;
      blocks_[l].tile[mode] = best;
      best_us.push_back(best_t);
    }
  }
  update_f3_used();
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return best_us;
}

}  // namespace cs
