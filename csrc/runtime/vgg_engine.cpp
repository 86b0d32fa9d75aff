#include "runtime/vgg_engine.h"

#include "runtime/markers.h"
#include "runtime/vgg_engine_util.h"

#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <stdexcept>
#include <string>

namespace cs {

using namespace vgg;

VggEngine::VggEngine(int64_t Bmax, std::vector<int64_t> desc, std::vector<int64_t> offs,
                     std::vector<int64_t> buf_offs, int64_t feat, int64_t ncls, torch::Tensor params,
                     torch::Tensor grads, torch::Tensor mom, torch::Tensor bufs, torch::Tensor nbt)
    : Bmax_(Bmax), feat_(feat), ncls_(ncls), params_(params), grads_(grads), mom_(mom), bufs_(bufs), nbt_(nbt) {
  TORCH_CHECK(desc.size() % 4 == 0 && !desc.empty(), "VggEngine: desc must be 4 ints per block");
  const int64_t L = desc.size() / 4;
  TORCH_CHECK((int64_t)offs.size() == 4 * L + 2 && (int64_t)buf_offs.size() == 2 * L, "VggEngine: offsets");
  TORCH_CHECK(Bmax > 0 && Bmax <= 2048, "VggEngine: 0 < Bmax <= 2048");
  TORCH_CHECK(ncls > 0 && ncls <= 16, "VggEngine: <= 16 classes (fused head)");
  for (auto* t : {&params_, &grads_, &mom_, &bufs_}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->dim() == 1,
                "VggEngine: flat buffers must be contiguous 1-D float32 GPU tensors");
  }
  TORCH_CHECK(params_.numel() == grads_.numel() && params_.numel() == mom_.numel(), "VggEngine: flat sizes");
  TORCH_CHECK(nbt_.is_cuda() && nbt_.scalar_type() == at::kLong && nbt_.numel() == L, "VggEngine: nbt int64 [L]");
  const auto fo = params_.options();
  const int64_t P = params_.numel();
  int64_t gmax = 0, dzmax = 0, partmax = 0, cmax = 0;
  blocks_.resize(L);
  for (int64_t l = 0; l < L; ++l) {
    VggBlock& b = blocks_[l];
    b.cin = desc[4 * l];
    b.cout = desc[4 * l + 1];
    b.H = desc[4 * l + 2];
    b.pool = desc[4 * l + 3] ? 1 : 0;
    TORCH_CHECK(b.H >= 1 && (b.H & (b.H - 1)) == 0 && (b.cin & (b.cin - 1)) == 0 && (b.cout & (b.cout - 1)) == 0 &&
                    b.cout >= 64 && b.cout <= 1024 && b.cin >= 4,
                "VggEngine: block ", l, " needs power-of-two H/cin/cout, cin>=4, 64<=cout<=1024");
    TORCH_CHECK(l == 0 || b.cin >= 64, "VggEngine: only block 0 may have a padded (4-channel) input");
    if (l > 0) {
      const VggBlock& p = blocks_[l - 1];
      TORCH_CHECK(p.cout == b.cin && (p.pool ? p.H / 2 : p.H) == b.H, "VggEngine: blocks ", l - 1, "->", l,
                  " do not chain");
    }
    b.w_off = offs[4 * l];
    b.b_off = offs[4 * l + 1];
    b.g_off = offs[4 * l + 2];
    b.be_off = offs[4 * l + 3];
    b.rm_off = buf_offs[2 * l];
    b.rv_off = buf_offs[2 * l + 1];
    const int64_t wn = (l == 0 && b.cin == 4) ? b.cout * 27 : b.cout * 9 * b.cin;
    for (int64_t o : {b.w_off, b.b_off, b.g_off, b.be_off})
      TORCH_CHECK(o % 4 == 0 && o >= 0, "VggEngine: tensor offsets must be 16-B aligned");
    TORCH_CHECK(b.w_off + wn <= P && b.b_off + b.cout <= P && b.g_off + b.cout <= P && b.be_off + b.cout <= P,
                "VggEngine: block ", l, " exceeds the flat buffer");
    TORCH_CHECK(b.rm_off + b.cout <= bufs_.numel() && b.rv_off + b.cout <= bufs_.numel(), "VggEngine: bufs");
    const int64_t pix = Bmax * b.H * b.H;
    b.x = torch::zeros({Bmax, b.H, b.H, b.cin}, fo);
    b.y = torch::zeros({pix, b.cout}, fo);
    b.stats = torch::zeros({cdiv(pix, CS_SPLITK_STAT_ROWS), b.cout, 2}, fo);
    b.bn = torch::zeros({4, b.cout}, fo);
    const int64_t ho = b.pool ? b.H / 2 : b.H;
    gmax = std::max(gmax, Bmax * ho * ho * b.cout);
    dzmax = std::max(dzmax, pix * b.cout);
    partmax = std::max<int64_t>(partmax, (int64_t)cs_bn_bwd_blocks(Bmax, b.H, b.H, b.cout, b.pool) * b.cout * 3);
    // block l-1's BN-backward partials out of block l's data gradient: [row tiles][cin][3]
    if (l > 0) partmax = std::max<int64_t>(partmax, cdiv(pix, CS_SPLITK_STAT_ROWS) * b.cin * 3);
    cmax = std::max<int64_t>(cmax, b.cout);
    for (int m = 0; m < 3; ++m) b.tile[m] = default_tile(b, m, Bmax);
  }
  const VggBlock& last = blocks_.back();
  TORCH_CHECK((last.pool ? last.H / 2 : last.H) == 1 && last.cout == feat, "VggEngine: last block must end at 1x1x",
              feat);
  fc_w_ = offs[4 * L];
  fc_b_ = offs[4 * L + 1];
  TORCH_CHECK(fc_w_ % 4 == 0 && fc_w_ + ncls * feat <= P && fc_b_ + ncls <= P, "VggEngine: fc offsets");
  const auto lo = torch::TensorOptions().dtype(at::kLong).device(params_.device());
  idx_ = torch::zeros({Bmax}, lo);
  ylab_ = torch::zeros({Bmax}, lo);
  pred_ = torch::zeros({Bmax}, lo);
  loss_ = torch::zeros({}, fo);
  correct_ = torch::zeros({}, fo.dtype(at::kInt));
  logits_ = torch::zeros({Bmax, ncls}, fo);
  gbuf_[0] = torch::zeros({gmax}, fo);
  gbuf_[1] = torch::zeros({gmax}, fo);
  feats_ = torch::zeros({Bmax * feat}, fo);
  dz_[0] = torch::zeros({dzmax}, fo);
  dz_[1] = torch::zeros({dzmax}, fo);
  ws_elems_ = kWsElems;
  ws_ = torch::zeros({ws_elems_}, fo);
  ws_w_ = torch::zeros({ws_elems_}, fo);
  side_ = reserved_side_stream();  // process-wide, created early (device_comm.h)
  dz_link_ = std::make_unique<StreamLink>();
  wg_link_ = std::make_unique<StreamLink>();
  for (const VggBlock& b : blocks_) dz_blk_.push_back(torch::zeros({Bmax * b.H * b.H * b.cout}, fo));
  if (const char* e = getenv("CS_OVERLAP_WGRAD")) overlap_ = atoi(e) != 0;
  // CS_ENGINE_OFF: comma list of default-on schedule features to turn off for a cross-process A/B
  // (one switch instead of one per feature): conv0_direct, conv0_bn_fold, conv0_sgd_fold,
  // conv0_batch_fold, head_bn_fold, side_sgd_tail, sgd_tail, bn_fused
  if (const char* e = getenv("CS_ENGINE_OFF")) {
    const std::string off = std::string(",") + e + ",";
    auto has = [&](const char* n) { return off.find(std::string(",") + n + ",") != std::string::npos; };
    if (has("conv0_direct")) conv0_direct_ = false;
    if (has("conv0_bn_fold")) conv0_bn_fold_ = false;
    if (has("conv0_sgd_fold")) conv0_sgd_fold_ = false;
    if (has("conv0_batch_fold")) conv0_batch_fold_ = false;
    if (has("head_bn_fold")) head_bn_fold_ = false;
    if (has("side_sgd_tail")) side_sgd_tail_ = false;
    if (has("sgd_tail")) sgd_tail_on_ = false;
    if (has("bn_fused")) bn_fused_rows_ = 0;
  }
  // per-block parameter ranges for the per-block SGD: the backward-ready layout puts fc first,
  // then blocks L-1..0, each {w, bias, gamma, beta} inside [w_off, next block's w_off)
  {
    bool contiguous = fc_w_ + ncls * feat <= blocks_[L - 1].w_off && fc_b_ + ncls <= blocks_[L - 1].w_off;
    for (int64_t l = 0; l < L && contiguous; ++l) {
      const VggBlock& b = blocks_[l];
      const int64_t lo = l == L - 1 ? 0 : b.w_off;
      const int64_t hi = l == 0 ? P : blocks_[l - 1].w_off;
      const int64_t wn = (l == 0 && b.cin == 4) ? b.cout * 27 : b.cout * 9 * b.cin;
      contiguous = l == 0 || blocks_[l - 1].w_off > b.w_off;  // blocks laid out last -> first
      for (int64_t o : {b.b_off, b.g_off, b.be_off}) contiguous = contiguous && o >= b.w_off && o + b.cout <= hi;
      contiguous = contiguous && b.w_off + wn <= hi;
      blk_range_.emplace_back(lo, hi - lo);
    }
    if (!contiguous) blk_range_.clear();
  }
  if (const char* e = getenv("CS_CONV_MATH")) math_ = atoi(e);
  if (const char* e = getenv("CS_DEBUG_SKIP")) debug_skip_ = atoi(e);
  TORCH_CHECK(L <= 32 && L <= CS_WB_MAX + 1, "VggEngine: at most ", CS_WB_MAX + 1, " blocks (F3 weight-bound tables)");
  amax_ = torch::zeros({4 * L * CS_AMAX_SLOT}, fo);
  bn_part_ = torch::zeros({partmax}, fo);
  bn_coef_ = torch::zeros({cmax * 3}, fo);
  bn_eval_ = torch::zeros({2, cmax}, fo);
  TORCH_CHECK(feat % 4 == 0, "VggEngine: feature size must be a multiple of 4");
  head_ws_ = torch::zeros({cs_linear_xent_ws((int)Bmax, (int)ncls)}, fo);
}

torch::Tensor VggEngine::tensor(int64_t block, const std::string& name) const {
  if (name == "g0") return gbuf_[0];
  if (name == "g1") return gbuf_[1];
  if (name == "dz") return dz_[block & 1];
  TORCH_CHECK(block >= 0 && block < (int64_t)blocks_.size(), "tensor: block index");
  if (name == "dz_blk") return dz_blk_[block];  // the overlapped backward's per-block dZ
  const VggBlock& b = blocks_[block];
  if (name == "x") return b.x;
  if (name == "y") return b.y;
  if (name == "bn") return b.bn;
  if (name == "stats") return b.stats;
  TORCH_CHECK(false, "tensor: unknown name ", name);
  return b.x;
}

void VggEngine::set_data(int64_t slot, torch::Tensor data, torch::Tensor labels, torch::Tensor aug) {
  TORCH_CHECK(slot == 0 || slot == 1, "set_data: slot 0 (train) or 1 (eval)");
  TORCH_CHECK(data.is_cuda() && data.scalar_type() == at::kByte && data.dim() == 4 && data.size(1) == 32 &&
                  data.size(2) == 32 && data.size(3) == 3 && data.is_contiguous(),
              "set_data: data must be contiguous uint8 [N,32,32,3] on the GPU");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.numel() == data.size(0),
              "set_data: labels int64 [N]");
  TORCH_CHECK(aug.is_cuda() && aug.scalar_type() == at::kInt && aug.dim() == 2 && aug.size(0) == data.size(0) &&
                  aug.size(1) == 3 && aug.is_contiguous(),
              "set_data: aug int32 [N,3]");
  data_[slot] = data;
  labels_[slot] = labels.contiguous();
  aug_[slot] = aug;
}

CsConvArgs VggEngine::conv_args(int l, int mode, int B, bool with_stats, float* ws, float* dz) {
  VggBlock& b = blocks_[l];
  const int L = (int)blocks_.size();
  CsConvArgs a{};
  a.B = B;
  a.H = b.H;
  a.W = b.H;
  a.Cin = b.cin;
  a.Cout = b.cout;
  a.w_oihw = (l == 0 && b.cin == 4) ? 1 : 0;
  a.ws = ws != nullptr ? ws : ws_.data_ptr<float>();
  if (dz == nullptr) dz = dz_[0].data_ptr<float>();
  if (mode == CS_CONV_FWD) {
    a.x = b.x.data_ptr<float>();
    a.w = P(b.w_off);
    a.bias = P(b.b_off);
    a.out = b.y.data_ptr<float>();
    a.stats = with_stats ? b.stats.data_ptr<float>() : nullptr;
    a.amax_a = amax_x(l);
    a.amax_b = amax_w(l);
  } else if (mode == CS_CONV_DGRAD) {
    TORCH_CHECK(l > 0, "VggEngine: no dgrad for block 0");
    a.dz = dz;
    a.w = P(b.w_off);
    a.out = gbuf_[(L - l) % 2].data_ptr<float>();
    a.amax_a = amax_dz(l);
    a.amax_b = amax_w(l);
  } else {
    a.x = b.x.data_ptr<float>();
    a.dz = dz;
    a.out = G(b.w_off);
    a.amax_a = amax_dz(l);
    a.amax_b = amax_x(l);
  }
  return a;
}

void VggEngine::conv(int l, int mode, int B, const ConvTile& t, hipStream_t s, bool with_stats, float* ws,
                     float* dz, const CsBnRed* ered, const CsSgdTail* sgd) {
  VggBlock& b = blocks_[l];
  CsConvArgs a = conv_args(l, mode, B, with_stats, ws, dz);
  if (ered != nullptr) {
    TORCH_CHECK(mode == CS_CONV_DGRAD, "VggEngine: BN partials ride a data gradient");
    a.ered = *ered;
  }
  if (sgd != nullptr) a.sgd = *sgd;
  const Dims d = dims(b, mode, B);
  const int sp = eff_splits(d.K, t.splits, t.bk);
  TORCH_CHECK(sp == 1 || (int64_t)sp * d.M * d.N <= ws_elems_, "VggEngine: split-K workspace too small");
  ok(cs_conv_gemm(a, mode, t.bm, t.bn, t.bk, t.splits, s, t.stage), "conv_gemm");
}

bool VggEngine::bn_fused(int l, int64_t B) const {
  const VggBlock& b = blocks_[l];
  return B * b.H * b.H <= bn_fused_rows_ && b.cout % 16 == 0;
}

CsSgdTail VggEngine::sgd_tail_args(int64_t block) {
  CsSgdTail t{};
  const int64_t off = blk_range_[block].first, n = blk_range_[block].second;
  if (n <= 0 || off % 4 != 0) return t;  // float4 rows (otherwise a launch of its own takes it)
  t.p = P(off);
  t.g = G(off);
  t.m = mom_.data_ptr<float>() + off;
  t.n = n;
  t.lr = (float)hp_[0];
  t.mom = (float)hp_[1];
  t.wd = (float)hp_[2];
  t.damp = (float)hp_[3];
  t.first = sgd_first_ ? 1 : 0;
  t.wb = sgd_wb(off, n);
  return t;
}

CsBnRed VggEngine::ered_args(int l, int B) {
  VggBlock& c = blocks_[l - 1];
  float* cb = c.bn.data_ptr<float>();
  CsBnRed r{};
  r.y = c.y.data_ptr<float>();
  r.scale = cb;
  r.shift = cb + c.cout;
  r.mean = cb + 2 * c.cout;
  r.invstd = cb + 3 * c.cout;
  r.part = bn_part_.data_ptr<float>();
  r.B = B;
  r.H = r.W = (int)c.H;
  r.C = (int)c.cout;
  r.pool = c.pool;
  // P = row tiles of block l's data gradient (M = B * H_l * W_l rows)
  const ConvTile& t = blocks_[l].tile[CS_CONV_DGRAD];
  const Dims d = dims(blocks_[l], CS_CONV_DGRAD, B);
  r.P = (int)cdiv(d.M, cs_conv_ered_rows((int)d.K, t.bm, t.bk, t.splits));
  TORCH_CHECK((int64_t)r.P * c.cout * 4 <= bn_part_.numel(), "VggEngine: BN partial buffer");
  return r;
}

bool VggEngine::side_ok(hipStream_t s) const { return overlap_ && side_ != nullptr && !stream_capturing(s); }

void VggEngine::flush_signal(hipStream_t s) {
  if (pending_sig_ == nullptr) return;
  ok(cs_link_signal(pending_sig_, s), "link signal");
  pending_sig_ = nullptr;
}

void VggEngine::flush_side_sgd() {
  // the SGD of the last block whose weight gradient forked, not yet carried by a later one
  if (side_sgd_pending_ < 0) return;
  sgd_on(side_, blk_range_[side_sgd_pending_].first, blk_range_[side_sgd_pending_].second, false);
  wg_link_->signal(side_);
  side_sgd_pending_ = -1;
}

void VggEngine::join_side(hipStream_t s) {
  flush_side_sgd();
  flush_signal(s);  // the side stream may be waiting for it: never wait on side before it is out
  wg_link_->wait(s);
}

void VggEngine::forward_train(int64_t B) {
  TORCH_CHECK(B > 0 && B <= Bmax_, "forward_train: 0 < B <= Bmax");
  TORCH_CHECK(data_[0].defined(), "forward_train: set_data(0, ...) first");
  hipStream_t s = cur_stream();
  const int L = (int)blocks_.size();
  red_pending_ = -1;
  flush_signal(s);
  // the per-step bounds are reset by the conv0 forward launch when it runs first (no extra launch)
  const bool zero_in_conv0 = conv0_direct_ok(B) && !(debug_skip_ & 8);
  f3_refresh(s, zero_in_conv0);
  // one launch: sampler index (device cursor into the epoch permutation, or idx_ when no
  // permutation is set), label gather, crop/flip/normalize into block 0's NHWC input
  const bool use_perm = perm_len_ > 0;
  // with the direct block-0 kernels the batch is built inside conv0's forward (one launch fewer at
  // the head of the chain; CS_CONV0_BATCH_FOLD=0 keeps make_batch)
  const bool batch_fold = conv0_batch_fold_ && conv0_direct_ok(B) && !(debug_skip_ & 8);
  CsBatchSrc bsrc{data_[0].data_ptr<uint8_t>(), labels_[0].data_ptr<int64_t>(),
                  use_perm ? perm_.data_ptr<int64_t>() : nullptr, use_perm ? cursor_.data_ptr<int64_t>() : nullptr,
                  (int)Bmax_, use_perm ? nullptr : idx_.data_ptr<int64_t>(), aug_[0].data_ptr<int32_t>(),
                  blocks_[0].x.data_ptr<float>(), idx_.data_ptr<int64_t>(), ylab_.data_ptr<int64_t>(),
                  {kMean[0], kMean[1], kMean[2]}, {1.0f / kStd[0], 1.0f / kStd[1], 1.0f / kStd[2]}};
  if (!batch_fold)
    ok(cs_make_batch(data_[0].data_ptr<uint8_t>(), labels_[0].data_ptr<int64_t>(),
                     use_perm ? perm_.data_ptr<int64_t>() : nullptr, use_perm ? cursor_.data_ptr<int64_t>() : nullptr,
                     (int)Bmax_, use_perm ? nullptr : idx_.data_ptr<int64_t>(), aug_[0].data_ptr<int32_t>(),
                     blocks_[0].x.data_ptr<float>(), idx_.data_ptr<int64_t>(), ylab_.data_ptr<int64_t>(), (int)B,
                     kMean, kStd, s),
       "make_batch");
  float* bufs = bufs_.data_ptr<float>();
  CsHeadBn head_bn{nullptr, nullptr, nullptr};
  for (int l = 0; l < L; ++l) {
    VggBlock& b = blocks_[l];
    const ConvTile& t = b.tile[CS_CONV_FWD];
    float* bn = b.bn.data_ptr<float>();
    if (l == defer_block_) join_deferred(s);  // the previous step's deferred buckets wrote these weights
    if ((w_deferred_ >> l) & 1u) {  // ... and their bounds (the join above, or an earlier join_lag)
      join_deferred(s);
      rotate_w(s, w_deferred_);
    }
    float* out = (l + 1 < L) ? blocks_[l + 1].x.data_ptr<float>() : feats_.data_ptr<float>();
    if (!(debug_skip_ & 8)) {
      const int64_t M = B * b.H * b.H;
      int rows;
      if (l == 0 && conv0_direct_ok(B)) {
        ok(cs_conv0_fwd(b.x.data_ptr<float>(), P(b.w_off), P(b.b_off), b.y.data_ptr<float>(), b.stats.data_ptr<float>(),
                        (int)B, b.H, b.H, b.cout, s, batch_fold ? &bsrc : nullptr, bounds_to_zero(), 2 * L,
                        rot_mask_ ? amax_w(0) : nullptr, amax_wnext(0), rot_mask_),
           "conv0_fwd");
        rows = cs_conv0_tile_rows();
      } else {
        conv(l, CS_CONV_FWD, (int)B, t, s, true);
        rows = cs_conv_stat_rows(9 * b.cin, t.bm, t.bk, t.splits);
      }
      const int T = (int)cdiv(M, rows);
      ok(cs_bn_finalize(b.stats.data_ptr<float>(), T, rows, (int)M, b.cout, P(b.g_off),
                        P(b.be_off), bufs + b.rm_off, bufs + b.rv_off, nbt_.data_ptr<int64_t>() + l, kBnMomentum,
                        kBnEps, bn, bn + b.cout, bn + 2 * b.cout, bn + 3 * b.cout, s),
         "bn_finalize");
    } else {
      conv(l, CS_CONV_FWD, (int)B, t, s, true);
    }
    if (l + 1 == L && head_bn_fold_ && b.pool && b.H == 2 && b.cout == feat_ && !(debug_skip_ & 4)) {
      // the last block's normalize/ReLU/pool runs inside the classifier's row pass (below)
      head_bn = CsHeadBn{b.y.data_ptr<float>(), bn, bn + b.cout};
      continue;
    }
    if (!(debug_skip_ & 4))
    ok(cs_bn_apply(b.y.data_ptr<float>(), bn, bn + b.cout, out, (int)B, b.H, b.H, b.cout, b.pool, s,
                   l + 1 < L ? x_amax_out(l + 1) : nullptr),
       "bn_apply");
  }
  // classifier + loss: dfeat -> gbuf_[0]. Inside the overlapped step the per-column pass (dW, db,
  // loss, accuracy: only the SGD and the host read them) forks to the side stream, off the
  // critical chain that continues with dfeat (the top block's BN backward)
  const bool fork = in_step_ && side_ok(s);
  ok(cs_linear_xent(feats_.data_ptr<float>(), P(fc_w_), P(fc_b_), ylab_.data_ptr<int64_t>(), (int)B, (int)feat_,
                    (int)ncls_, 1.0f, loss_.data_ptr<float>(), correct_.data_ptr<int>(), logits_.data_ptr<float>(),
                    G(fc_w_), G(fc_b_), gbuf_[0].data_ptr<float>(), pred_.data_ptr<int64_t>(), head_ws_.data_ptr<float>(), s,
                    fork ? 1 : 0, head_bn.y != nullptr ? &head_bn : nullptr),
     "linear_xent");
  if (fork) {
    pending_sig_ = dz_link_->defer();  // rides the top block's BN backward launch
    dz_link_->wait(side_);
    ok(cs_linear_xent(feats_.data_ptr<float>(), P(fc_w_), P(fc_b_), ylab_.data_ptr<int64_t>(), (int)B, (int)feat_,
                      (int)ncls_, 1.0f, loss_.data_ptr<float>(), correct_.data_ptr<int>(), logits_.data_ptr<float>(),
                      G(fc_w_), G(fc_b_), nullptr, pred_.data_ptr<int64_t>(), head_ws_.data_ptr<float>(), side_, 2),
       "linear_xent(cols)");
    wg_link_->signal(side_);
  }
}

void VggEngine::backward(int64_t hi, int64_t lo, int64_t B, bool join) {
  const int L = (int)blocks_.size();
  TORCH_CHECK(0 <= lo && lo <= hi && hi < L, "backward: need 0 <= lo <= hi < num_blocks");
  TORCH_CHECK(B > 0 && B <= Bmax_, "backward: 0 < B <= Bmax");
  hipStream_t s = cur_stream();
  const bool ovl = side_ok(s);
  for (int l = (int)hi; l >= (int)lo; --l) {
    VggBlock& b = blocks_[l];
    float* bn = b.bn.data_ptr<float>();
    // overlapped: every block has its own dz buffer (no WAR wait on a side wgrad still reading it)
    float* dz = ovl ? dz_blk_[l].data_ptr<float>() : dz_[l & 1].data_ptr<float>();
    const float* Gin = gbuf_[(L - 1 - l) % 2].data_ptr<float>();
    // ---- BN (+ReLU, +pool) backward of block l -> dz (the deferred side-stream signal of block
    // l+1's fork rides its first launch)
    if (debug_skip_ & 16) {
      flush_signal(s);
    } else if (red_pending_ == l && l == 0 && conv0_bn_fold_ && b.pool && conv0_direct_ok(B)) {
      // block 0: only the finalize here; the apply runs inside the weight gradient (conv0_wgrad)
      ok(cs_bn_bwd_finalize(bn_part_.data_ptr<float>(), red_P_, b.cout, (int)(B * b.H * b.H), P(b.g_off),
                            bn + 3 * b.cout, bn_coef_.data_ptr<float>(), G(b.g_off), G(b.be_off), G(b.b_off), s,
                            pending_sig_),
         "bn_bwd_finalize");
      pending_sig_ = nullptr;
      conv0_bn_G_ = Gin;
    } else if (red_pending_ == l) {
      // the partial sums ran inside block l+1's data-gradient launch: finalize + apply
      ok(cs_bn_bwd_tail(b.y.data_ptr<float>(), Gin, (int)B, b.H, b.H, b.cout, b.pool, bn, bn + b.cout,
                        bn + 2 * b.cout, bn + 3 * b.cout, P(b.g_off), bn_part_.data_ptr<float>(), red_P_,
                        bn_coef_.data_ptr<float>(), G(b.g_off), G(b.be_off), G(b.b_off), dz, s, pending_sig_,
                        dz_amax_out(l)),
         "bn_bwd_tail");
      pending_sig_ = nullptr;
    } else if (bn_fused(l, B)) {  // reduce + finalize + apply in one launch (the top block)
      ok(cs_bn_fused_bwd(b.y.data_ptr<float>(), Gin, (int)B, b.H, b.H, b.cout, b.pool, bn, P(b.g_off),
                         bn_coef_.data_ptr<float>(), G(b.g_off), G(b.be_off), G(b.b_off), dz, s, pending_sig_,
                         dz_amax_out(l)),
         "bn_fused_bwd");
      pending_sig_ = nullptr;
    } else {
      flush_signal(s);
      ok(cs_bn_bwd(b.y.data_ptr<float>(), Gin, (int)B, b.H, b.H, b.cout, b.pool, bn, bn + b.cout,
                   bn + 2 * b.cout, bn + 3 * b.cout, P(b.g_off), bn_part_.data_ptr<float>(),
                   bn_coef_.data_ptr<float>(), G(b.g_off), G(b.be_off), G(b.b_off), dz, s, dz_amax_out(l)),
         "bn_bwd");
    }
    red_pending_ = -1;
    // ---- weight and data gradients of block l; block l-1's BN-backward partials ride the data
    // gradient (measured against the BN backward's own reduce pass next to the side stream:
    // +0.2-0.7 %, profiles/r4_ab_bn_epi_red.txt)
    const bool er = l > 0;
    CsBnRed erv{};
    if (er) erv = ered_args(l, (int)B);
    if (ovl) {
      if (l > 0) {
        // the data gradient keeps the whole chip on the critical chain; the weight gradient forks
        // to the side stream after it and fills the chip while the main stream runs the
        // latency-bound BN kernels (and the split-K combine) of the block below
        conv(l, CS_CONV_DGRAD, (int)B, b.tile[CS_CONV_DGRAD], s, false, nullptr, dz, &erv);
        pending_sig_ = dz_link_->defer();
        fork_wgrad(l, B);
      } else {
        // block 0's weight gradient is the step's last GEMM: nothing left to overlap it with, so it
        // runs here (the main split-K workspace is free: no data gradient for block 0)
        const bool sgd_done = conv0_wgrad(B, s, dz, bwd_sgd_);
        if (bwd_sgd_ && !sgd_done) sgd_on(s, blk_range_[0].first, blk_range_[0].second, true);
      }
    } else {
      // block l+1's SGD rides this weight-gradient launch (its BN backward and data gradient ran)
      CsSgdTail tail{};
      if (sgd_tail_ && l + 1 < L) {
        tail = sgd_tail_args(l + 1);
        if (tail.n == 0) sgd_on(s, blk_range_[l + 1].first, blk_range_[l + 1].second, false);
      }
      if (l == 0 && conv0_direct_ok(B)) {
        if (tail.n > 0) sgd_on(s, blk_range_[l + 1].first, blk_range_[l + 1].second, false);
        conv0_wgrad(B, s, dz);
      } else {
        conv(l, CS_CONV_WGRAD, (int)B, b.tile[CS_CONV_WGRAD], s, false, ws_w_.data_ptr<float>(), dz, nullptr,
             tail.n > 0 ? &tail : nullptr);
      }
      if (l > 0) conv(l, CS_CONV_DGRAD, (int)B, b.tile[CS_CONV_DGRAD], s, false, nullptr, dz, &erv);
    }
    if (er) {
      red_pending_ = l - 1;
      red_P_ = erv.P;
    }
  }
  if (join) {
    flush_signal(s);
    if (ovl) join_side(s);
  }
}

bool VggEngine::conv0_direct_ok(int64_t B) const {
  const VggBlock& b = blocks_[0];
  return conv0_direct_ && b.cin == 4 && b.cout == 64 && b.H == 32 &&
         cs_conv0_wgrad_part_floats((int)B, b.H, b.H) <= (size_t)ws_elems_;
}

bool VggEngine::conv0_wgrad(int64_t B, hipStream_t s, float* dz, bool with_sgd) {
  VggBlock& b = blocks_[0];
  if (!conv0_direct_ok(B)) {
    conv(0, CS_CONV_WGRAD, (int)B, b.tile[CS_CONV_WGRAD], s, false, ws_.data_ptr<float>(), dz);
    return false;
  }
  CsSgdTail sgd{};
  int w_rel = 0;
  int64_t* counter = nullptr;
  if (with_sgd && conv0_sgd_fold_ && !blk_range_.empty()) {
    sgd = sgd_tail_args(0);
    w_rel = (int)(b.w_off - blk_range_[0].first);
    if (w_rel < 0 || w_rel + 27 * b.cout > sgd.n) sgd.n = 0;
    counter = perm_len_ > 0 ? cursor_.data_ptr<int64_t>() : nullptr;
  }
  const CsSgdTail* sp = sgd.n > 0 ? &sgd : nullptr;
  if (conv0_bn_G_ != nullptr) {  // block 0's BN-backward apply folded in (dz is not written)
    const float* bn = b.bn.data_ptr<float>();
    const float* Gin = conv0_bn_G_;
    conv0_bn_G_ = nullptr;
    ok(cs_conv0_wgrad_bn(b.x.data_ptr<float>(), b.y.data_ptr<float>(), Gin, bn, bn + b.cout, bn + 2 * b.cout,
                         bn + 3 * b.cout, bn_coef_.data_ptr<float>(), ws_.data_ptr<float>(), G(b.w_off), (int)B, b.H,
                         b.H, b.cout, s, sp, w_rel, counter),
       "conv0_wgrad_bn");
    return sp != nullptr;
  }
  ok(cs_conv0_wgrad(b.x.data_ptr<float>(), dz, ws_.data_ptr<float>(), G(b.w_off), (int)B, b.H, b.H, b.cout, s, sp,
                    w_rel, counter),
     "conv0_wgrad");
  return sp != nullptr;
}

void VggEngine::join_lag() { join_deferred(cur_stream()); }

void VggEngine::join_deferred(hipStream_t s) {
  if (defer_comm_ == nullptr) return;
  if (!(debug_skip_ & 64)) defer_comm_->join(s);
  defer_comm_ = nullptr;
  defer_block_ = -1;
}

void VggEngine::fork_wgrad(int l, int64_t B) {
  // the side stream waits for the deferred signal just issued (it rides a main-stream launch), then
  // block l's weight gradient into its own dz buffer's consumer, its SGD, and the join signal
  VggBlock& b = blocks_[l];
  float* dz = dz_blk_[l].data_ptr<float>();
  dz_link_->wait(side_);
  // the previous fork's SGD (its gradient is final: its weight gradient ran before on this stream)
  // rides this weight gradient's launch as extra workgroups; block l's own SGD waits for the next
  // fork or the join (block l's dgrad — the last reader of its weights — ran before the fork)
  CsSgdTail tail{};
  if (side_sgd_pending_ >= 0) {
    tail = side_sgd_tail_ ? sgd_tail_args(side_sgd_pending_) : CsSgdTail{};
    if (tail.n == 0) sgd_on(side_, blk_range_[side_sgd_pending_].first, blk_range_[side_sgd_pending_].second, false);
    side_sgd_pending_ = -1;
  }
  if (!(debug_skip_ & 32)) {
    conv(l, CS_CONV_WGRAD, (int)B, b.tile[CS_CONV_WGRAD], side_, false, ws_w_.data_ptr<float>(), dz, nullptr,
         tail.n > 0 ? &tail : nullptr);
  } else if (tail.n > 0) {
    sgd_on(side_, tail.p - P(0), tail.n, false);
  }
  if (bwd_sgd_) side_sgd_pending_ = l;
  wg_link_->signal(side_);
}

std::string VggEngine::link_error() const {
  std::string e = dz_link_ ? dz_link_->error() : std::string();
  if (e.empty() && wg_link_) e = wg_link_->error();
  return e;
}

VggEngine::~VggEngine() {
  for (auto e : tev_) hipEventDestroy(e);
}

void VggEngine::sgd_on(hipStream_t st, int64_t off, int64_t n, bool cursor) {
  if (n == 0) return;
  const CsWeightBounds wb = sgd_wb(off, n);
  ok(cs_sgd_flat(P(off), G(off), mom_.data_ptr<float>() + off, n, (float)hp_[0], (float)hp_[1], (float)hp_[2],
                 (float)hp_[3], 1.0f, sgd_first_ ? 1 : 0, st,
                 cursor && perm_len_ > 0 ? cursor_.data_ptr<int64_t>() : nullptr, &wb),
     "sgd_flat(block)");
}

void VggEngine::sgd(double lr, double momentum, double wd, double dampening, int64_t off, int64_t n) {
  TORCH_CHECK(off >= 0 && n >= 0 && off + n <= params_.numel(), "sgd: range");
  if (n == 0) return;
  const CsWeightBounds wb = sgd_wb(off, n);
  // first step (set_sgd_first): buf = d, torch's clone — with dampening 0 bit-equal to the
  // 0*mom + (1-damp)*d of later steps. The step's one optimizer launch also advances the
  // device-side batch cursor
  ok(cs_sgd_flat(P(off), G(off), mom_.data_ptr<float>() + off, n, (float)lr, (float)momentum, (float)wd,
                 (float)dampening, 1.0f, sgd_first_ ? 1 : 0, cur_stream(),
                 perm_len_ > 0 ? cursor_.data_ptr<int64_t>() : nullptr, &wb),
     "sgd_flat");
  sgd_first_ = false;
}

void VggEngine::set_perm(torch::Tensor perm) {
  TORCH_CHECK(data_[0].defined(), "set_perm: set_data(0, ...) first");
  TORCH_CHECK(perm.scalar_type() == at::kLong && perm.dim() == 1 && perm.numel() > 0, "set_perm: int64 [n] indices");
  const int64_t n = perm.numel();
  TORCH_CHECK(n <= data_[0].size(0) + Bmax_, "set_perm: permutation longer than the dataset");
  if (!perm_.defined()) {
    // fixed capacity (graph-captured kernels keep the pointer): dataset size + one batch of slack
    perm_ = torch::zeros({data_[0].size(0) + Bmax_}, params_.options().dtype(at::kLong));
    cursor_ = torch::zeros({1}, params_.options().dtype(at::kLong));
  }
  perm_.narrow(0, 0, n).copy_(perm.to(perm_.device()), /*non_blocking=*/false);
  cursor_.zero_();
  perm_len_ = n;
}

void VggEngine::set_timing(bool on) {
  timing_ = on;
  if (on && tev_.empty()) {
    tev_.resize(32);
    for (auto& e : tev_) ok(hipEventCreate(&e), "timing event");
  }
}

void VggEngine::mark(const char* phase) {
  if (!timing_ || tn_ >= tev_.size()) return;
  ok(hipEventRecord(tev_[tn_], cur_stream()), "timing record");
  if (tn_ > 0) {
    if (tnames_.size() < tn_) tnames_.resize(tn_);
    tnames_[tn_ - 1] = phase;
  }
  ++tn_;
}

std::vector<std::pair<std::string, double>> VggEngine::phase_times() {
  std::vector<std::pair<std::string, double>> out;
  if (tn_ < 2) return out;
  ok(hipEventSynchronize(tev_[tn_ - 1]), "timing sync");
  double total = 0.0;
  for (size_t i = 1; i < tn_; ++i) {
    float ms = 0.f;
    ok(hipEventElapsedTime(&ms, tev_[i - 1], tev_[i]), "elapsed");
    out.emplace_back(tnames_[i - 1], (double)ms);
    total += ms;
  }
  out.emplace_back("step", total);
  return out;
}

void VggEngine::forward_eval(int64_t B) {
  TORCH_CHECK(B > 0 && B <= Bmax_, "forward_eval: 0 < B <= Bmax");
  TORCH_CHECK(data_[1].defined(), "forward_eval: set_data(1, ...) first");
  join_lag();
  hipStream_t s = cur_stream();
  const int L = (int)blocks_.size();
  f3_refresh(s);
  ok(cs_gather_labels(labels_[1].data_ptr<int64_t>(), idx_.data_ptr<int64_t>(), ylab_.data_ptr<int64_t>(), (int)B, s),
     "gather_labels");
  ok(cs_augment(data_[1].data_ptr<uint8_t>(), idx_.data_ptr<int64_t>(), aug_[1].data_ptr<int32_t>(),
                blocks_[0].x.data_ptr<float>(), (int)B, 1, blocks_[0].cin, kMean, kStd, s),
     "augment");
  float* sc = bn_eval_.data_ptr<float>();
  float* sh = sc + bn_eval_.size(1);
  float* bufs = bufs_.data_ptr<float>();
  for (int l = 0; l < L; ++l) {
    VggBlock& b = blocks_[l];
    if (l == 0 && conv0_direct_ok(B))
      ok(cs_conv0_fwd(b.x.data_ptr<float>(), P(b.w_off), P(b.b_off), b.y.data_ptr<float>(), nullptr, (int)B, b.H, b.H,
                      b.cout, s),
         "conv0_fwd");
    else
      conv(l, CS_CONV_FWD, (int)B, b.tile[CS_CONV_FWD], s, false);
    ok(cs_bn_eval_coeffs(P(b.g_off), P(b.be_off), bufs + b.rm_off, bufs + b.rv_off, b.cout, kBnEps, sc, sh, s),
       "bn_eval_coeffs");
    float* out = (l + 1 < L) ? blocks_[l + 1].x.data_ptr<float>() : feats_.data_ptr<float>();
    ok(cs_bn_apply(b.y.data_ptr<float>(), sc, sh, out, (int)B, b.H, b.H, b.cout, b.pool, s,
                   l + 1 < L ? x_amax_out(l + 1) : nullptr),
       "bn_apply");
  }
  ok(cs_linear_xent(feats_.data_ptr<float>(), P(fc_w_), P(fc_b_), ylab_.data_ptr<int64_t>(), (int)B, (int)feat_,
                    (int)ncls_, 1.0f, loss_.data_ptr<float>(), correct_.data_ptr<int>(), logits_.data_ptr<float>(),
                    nullptr, nullptr, nullptr, pred_.data_ptr<int64_t>(), head_ws_.data_ptr<float>(), s),
     "linear_xent");
}

void VggEngine::step(int64_t B, DeviceComm* comm, const std::vector<int64_t>& bucket_blocks,
                     const std::vector<int64_t>& bucket_ranges, bool broadcast_buffers, double lr, double momentum,
                     double wd, double dampening) {
  try {
    step_impl(B, comm, bucket_blocks, bucket_ranges, broadcast_buffers, lr, momentum, wd, dampening);
  } catch (...) {
    // a launch failed with a deferred link signal pending: bump it now, so the side stream's wait
    // does not spin to the link timeout behind a kernel that will never run
    if (pending_sig_ != nullptr) {
      (void)cs_link_signal(pending_sig_, cur_stream());
      pending_sig_ = nullptr;
    }
    in_step_ = false;
    throw;
  }
}

void VggEngine::step_impl(int64_t B, DeviceComm* comm, const std::vector<int64_t>& bucket_blocks,
                          const std::vector<int64_t>& bucket_ranges, bool broadcast_buffers, double lr,
                          double momentum, double wd, double dampening) {
  const int64_t L = (int64_t)blocks_.size();
  const size_t nb = bucket_blocks.size();
  TORCH_CHECK(nb >= 1 && bucket_ranges.size() == 2 * nb && bucket_blocks.back() == 0, "step: bucket plan");
  hipStream_t s = cur_stream();
  // the caller passes a communicator only when the step is data-parallel (a one-rank
  // communicator too: the CS_COMM_PROBE measurement and the ProbeComm ordering test)
  const bool dp = comm != nullptr;
  // deferred buckets: never inside a graph capture (the wait would have to cross graph launches),
  // and a previous step's deferral on another communicator (or none) is waited for here
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  ok(hipStreamIsCapturing(s, &cap), "hipStreamIsCapturing");
  const bool capturing = cap != hipStreamCaptureStatusNone;
  // a join inside a capture would wait on a stream that is not captured (the dependency could be
  // dropped): the caller joins before capturing (NativeTrainer._capture -> join_lag)
  TORCH_CHECK(!(capturing && defer_comm_ != nullptr),
              "VggEngine::step: deferred buckets pending while capturing a graph; call join_lag() first");
  if (defer_comm_ != nullptr && defer_comm_ != comm) join_deferred(s);
  std::vector<size_t> deferred;
  tn_ = 0;
  Range step_range("cs.step");
  mark("start");
  in_step_ = true;
  {
    Range r("cs.forward");
    forward_train(B);
  }
  mark("forward");
  hp_[0] = lr;
  hp_[1] = momentum;
  hp_[2] = wd;
  hp_[3] = dampening;
  // data-parallel: each bucket's SGD runs on the comm stream right behind its all-reduce (every
  // reader of the bucket's weights — its blocks' data gradients — was enqueued before the fork);
  // the buckets must tile the flat buffer
  bool comm_sgd = dp;
  for (size_t k = 0, at = 0; k < nb && comm_sgd; ++k) {
    comm_sgd = bucket_ranges[2 * k] == (int64_t)at;
    at += bucket_ranges[2 * k + 1];
    if (k + 1 == nb) comm_sgd = comm_sgd && (int64_t)at == params_.numel();
  }
  // world 1: overlapped — block l's SGD right behind its weight gradient on the side stream (block
  // 0's, with the batch cursor, on this stream); serial — block l+1's SGD rides block l's
  // weight-gradient launch
  const bool ovl = side_ok(s);
  bwd_sgd_ = ovl && !dp && !blk_range_.empty();

  sgd_tail_ = !ovl && sgd_tail_on_ && !dp && !blk_range_.empty();
  int64_t hi = L - 1;
  for (size_t k = 0; k < nb; ++k) {
    const int64_t lo = bucket_blocks[k];
    TORCH_CHECK(lo <= hi, "step: bucket blocks must decrease");
    static const char* kBwdR[] = {"cs.backward.bucket0", "cs.backward.bucket1", "cs.backward.bucket2",
                                  "cs.backward.bucket3", "cs.backward.bucket4", "cs.backward.bucket5",
                                  "cs.backward.bucket6", "cs.backward.bucket7"};
    Range bwd_range(k < 8 ? kBwdR[k] : "cs.backward.bucket8+");
    backward(hi, lo, B, /*join=*/false);
    bwd_range.end();
    static const char* kBwd[] = {"backward_bucket0", "backward_bucket1", "backward_bucket2", "backward_bucket3",
                                 "backward_bucket4", "backward_bucket5", "backward_bucket6", "backward_bucket7"};
    mark(k < 8 ? kBwd[k] : "backward_bucket8+");
    hi = lo - 1;
    if (!dp) continue;
    if (comm_sgd && !capturing && k + 1 < nb &&
        std::find(comm_defer_.begin(), comm_defer_.end(), (int64_t)k) != comm_defer_.end()) {
      deferred.push_back(k);  // enqueued after the last bucket (below)
      if (broadcast_buffers && k == 0) {
        // no all-reduce of bucket 0 ahead of it to order it after this forward: the broadcast forks
        comm->broadcast(bufs_.data_ptr<float>(), bufs_.numel(), ncclFloat32, 0, s, /*fork=*/true);
        comm->broadcast(nbt_.data_ptr<int64_t>(), nbt_.numel(), ncclInt64, 0, s, /*fork=*/false);
      }
      continue;
    }
    {
      // the bucket is complete once its last weight gradient is: the all-reduce forks from there
      // (the side stream when overlapped; the bucket holding block 0, whose weight gradient ran on
      // this stream, joins the side stream first) and overlaps the rest of the backward
      Range r("cs.allreduce.enqueue");
      hipStream_t src = s;
      if (ovl && lo == 0) {
        join_side(s);
      } else if (ovl) {
        src = side_;
        // a host-blocking communicator (staged) runs the collective inside this call: the deferred
        // signal its fork waits behind must be out first
        if (comm->host_blocking()) flush_signal(s);
      }
      comm->all_reduce(G(bucket_ranges[2 * k]), bucket_ranges[2 * k + 1], ncclFloat32, ncclAvg, src,
                       /*fork=*/!(debug_skip_ & 2));
    }
    if (broadcast_buffers && k == 0) {
      // DDP broadcast_buffers (rank 0's BN running stats before every training forward), issued
      // for the NEXT forward right behind the first bucket: this forward has produced the
      // buffers, nothing touches them until the next forward, and the step's closing join
      // orders them before it (step 0 is covered by the construction-time broadcast)
      comm->broadcast(bufs_.data_ptr<float>(), bufs_.numel(), ncclFloat32, 0, s, /*fork=*/false);
      comm->broadcast(nbt_.data_ptr<int64_t>(), nbt_.numel(), ncclInt64, 0, s, /*fork=*/false);
    }
    if (comm_sgd) sgd_on(comm->stream(), bucket_ranges[2 * k], bucket_ranges[2 * k + 1], k + 1 == nb);
  }
  {
    Range r("cs.comm.join");
    flush_signal(s);
    if (ovl) join_side(s);
    if (dp && !(debug_skip_ & 1)) comm->join(s);
    if (!deferred.empty()) {
      // every weight gradient is complete on this stream (joined above): the deferred buckets fork
      // from here, behind the last bucket on the comm stream; the next forward joins them
      for (size_t k : deferred) {
        comm->all_reduce(G(bucket_ranges[2 * k]), bucket_ranges[2 * k + 1], ncclFloat32, ncclAvg, s, /*fork=*/true);
        sgd_deferring_ = true;
        sgd_on(comm->stream(), bucket_ranges[2 * k], bucket_ranges[2 * k + 1], false);
        sgd_deferring_ = false;
        const int lo = (int)bucket_blocks[k];
        defer_block_ = defer_block_ < 0 ? lo : std::min(defer_block_, lo);
      }
      defer_comm_ = comm;
    }
  }
  mark("allreduce_wait");
  {
    Range r("cs.sgd");
    if (sgd_tail_) {
      // blocks 1.. rode the weight-gradient launches; block 0 (+ the cursor) here
      sgd_on(s, blk_range_[0].first, blk_range_[0].second, true);
    } else if (!comm_sgd && !bwd_sgd_) {
      sgd(lr, momentum, wd, dampening, 0, params_.numel());
    }
    sgd_first_ = false;
    sgd_tail_ = false;
    bwd_sgd_ = false;
    in_step_ = false;
  }
  mark("sgd");
}

}  // namespace cs
