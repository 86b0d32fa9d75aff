// Native VGG training engine: a hand-scheduled forward/backward (no autograd) over
// flat parameter / gradient / momentum buffers, every op a gfx950 HIP kernel.
//
// Replaces, for the reference's whole hot loop (master/part1/part1.py:31-38 and
// its part2/part3 variants): the torchvision batch pipeline, nn.Sequential VGG
// forward (master/part1/model.py:42-46), CrossEntropyLoss, autograd backward,
// the gradient synchronisation of part2a/2b/3 and optimizer.step().
//
// Layout (set by the Python side, runtime/engine.py):
//  * flat buffers hold tensors in BACKWARD-READY order — fc1.{weight,bias}, then
//    the conv blocks from last to first, each {conv.weight (OHWI; conv0 OIHW),
//    conv.bias, bn.weight, bn.bias} — every tensor 256-B aligned, so a gradient
//    bucket is one contiguous range that is complete as soon as the backward of
//    its last block has run;
//  * activations NHWC; conv0's input padded to 4 channels (one float4 / pixel);
//  * per block: conv input x, conv output y (pre-BN, kept for BN/ReLU/pool
//    backward recompute), BN tile partials (from the conv epilogue), BN coeffs.
// Every method enqueues on the caller's current HIP stream and never syncs the
// host, so a whole step (or any bucket segment of it) can be captured as a graph.
//
// Kernel boundaries of one training step: a block's forward is conv [+ split-K combine] (BN tile
// statistics from the epilogue) + BN finalize + apply (ReLU, pool); its backward is BN finalize +
// apply (the partial sums come from the data-gradient epilogue of the block above) + data
// gradient on the main stream, and the weight gradient + SGD on the side stream.
#pragma once
#include <torch/extension.h>

#include <memory>
#include <vector>

#include "kernels/launchers.h"
#include "runtime/device_comm.h"

namespace cs {

struct ConvTile {
  int bm = 64, bn = 64, splits = 1, bk = 16;
  int stage = CS_STAGE_REGS;  // operand staging: registers + ds_write, or LDS-DMA ring (bk 32)
  float us = -1.f;  // measured time of the chosen config (autotune), -1 = untuned
};

struct VggBlock {
  int cin = 0, cout = 0, H = 0, pool = 0;  // cin = 4 for the padded conv0
  int64_t w_off = 0, b_off = 0, g_off = 0, be_off = 0, rm_off = 0, rv_off = 0;
  ConvTile tile[3];
  torch::Tensor x;      // [Bmax, H, H, cin]
  torch::Tensor y;      // [Bmax*H*H, cout]
  torch::Tensor stats;  // [ceil(Bmax*H*H/16), cout, 2] BN (mean, M2) partials per row tile
  torch::Tensor bn;     // [4, cout]: scale, shift, mean, invstd
};

class VggEngine {
 public:
  // desc: 4 ints per block (cin, cout, H, pool); offs: 4 per block (w, b, gamma, beta) + (fc_w, fc_b);
  // buf_offs: 2 per block (running_mean, running_var) into `bufs`.
  VggEngine(int64_t Bmax, std::vector<int64_t> desc, std::vector<int64_t> offs, std::vector<int64_t> buf_offs,
            int64_t feat, int64_t ncls, torch::Tensor params, torch::Tensor grads, torch::Tensor mom,
            torch::Tensor bufs, torch::Tensor nbt);

  // slot 0 = train, 1 = eval. data uint8 [N,32,32,3], labels int64 [N], aug int32 [N,3] (dy, dx, flip)
  void set_data(int64_t slot, torch::Tensor data, torch::Tensor labels, torch::Tensor aug);
  torch::Tensor idx() const { return idx_; }
  // epoch sampling order for the training forward: batch k = perm[k*Bmax ...]; resets the device
  // cursor, which the step's SGD launch advances (no per-step host copy)
  void set_perm(torch::Tensor perm);
  torch::Tensor cursor() const { return cursor_; }
  torch::Tensor loss() const { return loss_; }
  torch::Tensor correct() const { return correct_; }
  torch::Tensor logits() const { return logits_; }
  int64_t num_blocks() const { return (int64_t)blocks_.size(); }
  // debug/test access: "x" (block input), "y" (conv output), "bn" ([4,C] scale/shift/mean/invstd), "stats",
  // "g0"/"g1" (gradient ping-pong), "dz"
  torch::Tensor tensor(int64_t block, const std::string& name) const;

  // augment + conv/BN/ReLU/pool chain + fused linear/xent fwd+bwd (train) for B <= Bmax samples
  void forward_train(int64_t B);
  // backward of blocks hi..lo (inclusive, hi >= lo), writing their gradients into `grads`.
  // Overlapped (default, not while a graph is captured): block l's weight gradient runs on the
  // side stream once block l's data gradient is done, beside the BN backward and data gradient
  // of the blocks below on the caller's stream; join = true makes the caller's stream wait for
  // the side stream before returning.
  void backward(int64_t hi, int64_t lo, int64_t B, bool join = true);
  // weight gradients on the side stream (default on); off = the serial backward
  void set_overlap(bool on) { overlap_ = on; }
  // SGD (momentum, weight decay, dampening) on [off, off+n) of the flat buffers
  void sgd(double lr, double momentum, double wd, double dampening, int64_t off, int64_t n);
  void set_bn_fused_rows(int64_t r) { bn_fused_rows_ = r; }
  // torch.optim.SGD's first step sets buf = d (no dampening): the next step's SGD launches
  // use first = 1 (only matters with dampening != 0); cleared once that step's SGD is enqueued
  void set_sgd_first(bool on) { sgd_first_ = on; }
  // world-1 serial step: block l+1's SGD rides block l's weight-gradient launch (default on)
  void set_sgd_tail(bool on) { sgd_tail_on_ = on; }
  // test-only ordering faults for the ProbeComm test's negative control (tests must see a
  // mismatch): bit 0 = step() skips the closing join, bit 1 = its all-reduces skip the fork
  // measurement / negative-control switches (WRONG numbers when set; never in a product run):
  // 1 skip the comm join, 2 no comm fork (ordering-test controls); ablation upper bounds of a
  // fusion (what the step would save if a launch class were free): 4 forward bn_apply,
  // 8 forward bn_finalize, 16 backward BN (finalize + apply), 32 side-stream weight-gradient GEMMs;
  // 64 the next forward skips its wait for deferred buckets (ordering-test control).
  // CS_DEBUG_SKIP sets the mask at construction.
  void set_debug_skip(int64_t mask) { debug_skip_ = (int)mask; }
  // Default-on schedule features, each a setter for the bitwise tests and one name in
  // CS_ENGINE_OFF (constructor) for cross-process A/Bs:
  // block 0's convolution (3 -> 64) as the direct conv0.hip kernels instead of the implicit GEMM
  // (forward + BN tile statistics, weight gradient): conv0_direct
  void set_conv0_direct(bool on) { conv0_direct_ = on; }
  // with the direct kernels, block 0's BN-backward apply folded into its weight gradient (dZ of
  // block 0 never written): conv0_bn_fold
  void set_conv0_bn_fold(bool on) { conv0_bn_fold_ = on; }
  // ... and block 0's SGD step (+ batch cursor) into the weight gradient's final sum (world 1,
  // overlapped backward): conv0_sgd_fold
  void set_conv0_sgd_fold(bool on) { conv0_sgd_fold_ = on; }
  // ... and the training batch (make_batch) into the conv0 forward's input halo: conv0_batch_fold
  void set_conv0_batch_fold(bool on) { conv0_batch_fold_ = on; }
  // the last block's BN + ReLU + max-pool inside the classifier's row pass: head_bn_fold
  void set_head_bn_fold(bool on) { head_bn_fold_ = on; }
  // side stream: block l+1's SGD as extra workgroups of block l's weight-gradient launch: side_sgd_tail
  void set_side_sgd_tail(bool on) { side_sgd_tail_ = on; }
  bool conv0_direct(int64_t B) const { return conv0_direct_ok(B); }
  // the current stream waits for deferred buckets' all-reduce + SGD (set_comm_defer, below): every
  // host read of the parameters goes through here
  void join_lag();
  // Data-parallel steps: the buckets listed (bucket indices, never the last one) have their
  // all-reduce + SGD enqueued on the comm stream AFTER the last bucket's, and the step's closing
  // join covers only the others; the next step's forward waits for them right before the conv of
  // their lowest block. The bottom blocks' buckets — produced last by the backward, needed first by
  // the next forward — then no longer queue behind a large top bucket, whose collective instead
  // overlaps the next forward's lower blocks. join_lag() waits for them (eval, host reads).
  void set_comm_defer(std::vector<int64_t> buckets) { comm_defer_ = std::move(buckets); }
  std::vector<int64_t> comm_defer() const { return comm_defer_; }
  bool defer_pending() const { return defer_comm_ != nullptr; }
  // measurement only (WRONG numbers): every operand bound of the F3 conv math reads 1.0 and no
  // producer writes one — prices the F3 GEMMs in the step before the bounds are produced
  void set_f3_probe(bool on);
  // the parameters were rewritten outside the engine's SGD (load, broadcast, init): the next step
  // re-measures the weights' bounds for the F3 conv math
  void params_changed() { w_dirty_ = true; }
  torch::Tensor amax() const { return amax_; }
  // conv autotune candidates (CS_CONV_MATH): 0 f32, 1 x6, 2 f32 + x6 (default), 3 bf16 operands
  void set_math(int64_t m) {
    TORCH_CHECK(m >= 0 && m <= 3, "set_math: 0..3");
    math_ = (int)m;
  }
  // eval forward (running stats): loss (mean over the batch) -> loss(), correct count -> correct()
  void forward_eval(int64_t B);

  // whole step in C++: forward, bucketed backward with (optional) all-reduce(avg) of each
  // bucket on `comm` (RcclComm on a multi-GPU job; StagedComm / ProbeComm in tests: any
  // DeviceComm, device_comm.h) as soon as it is complete, SGD. comm == nullptr: no DP. bucket_blocks[k] = lowest block of
  // bucket k (buckets cover blocks from the top), bucket_ranges = (off, n) per bucket.
  // SGD: world 1 — block l+1's update rides block l's weight-gradient launch (block 0's, with
  // the batch cursor, closes the step); data-parallel — each bucket's update runs on the comm
  // stream right behind its all-reduce, overlapping the rest of the backward.
  void step(int64_t B, DeviceComm* comm, const std::vector<int64_t>& bucket_blocks,
            const std::vector<int64_t>& bucket_ranges, bool broadcast_buffers, double lr, double momentum,
            double wd, double dampening);

  void step_impl(int64_t B, DeviceComm* comm, const std::vector<int64_t>& bucket_blocks,
                 const std::vector<int64_t>& bucket_ranges, bool broadcast_buffers, double lr, double momentum,
                 double wd, double dampening);

  // Phase timing (opt-in): timing events on the compute stream at the step's phase
  // boundaries (forward, each gradient bucket's backward, waiting for the all-reduces, SGD);
  // phase_times() synchronizes and returns the last step's phases in ms. Off by default: an event
  // record on the compute stream costs a few us of launch gap on this stack.
  void set_timing(bool on);
  std::vector<std::pair<std::string, double>> phase_times();

  // error of the side-stream weight-gradient links (dz_link_ main -> side, wg_link_ side -> main):
  // a wait that timed out or was released by abort_links() ran its consumer unordered, so the
  // wgrad / SGD ordering of the steps since can no longer be trusted ("" when healthy)
  std::string link_error() const;

  // conv tile control: mode 0 fwd / 1 dgrad / 2 wgrad
  void set_tile(int64_t block, int64_t mode, int64_t bm, int64_t bn, int64_t splits, int64_t bk = 16,
                int64_t stage = 0);
  // -> {bm, bn, splits, bk, stage}
  std::vector<int64_t> get_tile(int64_t block, int64_t mode) const;
  // time every candidate (bm, bn in {64,128}, bk in {16,32}, split-K, register or LDS-DMA
  // staging) per (block, mode) with HIP events and keep the fastest
  std::vector<double> autotune(int64_t B, int64_t iters);
  // run a single conv GEMM of the training step (for profiling / tests)
  void run_conv(int64_t block, int64_t mode, int64_t B);

 private:
  void conv(int l, int mode, int B, const ConvTile& t, hipStream_t s, bool with_stats, float* ws = nullptr,
            float* dz = nullptr, const CsBnRed* ered = nullptr, const CsSgdTail* sgd = nullptr);
  CsConvArgs conv_args(int l, int mode, int B, bool with_stats, float* ws, float* dz);
  // single-launch BN backward (reduce + finalize + apply) for the top block when it has at most
  // bn_fused_rows_ rows (B*H*W)
  bool bn_fused(int l, int64_t B) const;
  // Block l-1's BN-backward partial sums are computed where block l's data gradient is finished
  // (the dgrad GEMM's epilogue, or its split-K combine: CsConvArgs::ered): the BN backward of
  // block l-1 is then finalize + apply.
  CsBnRed ered_args(int l, int B);
  int red_pending_ = -1;  // block whose BN-backward partials are already in place
  int red_P_ = 0;         // ... as red_P_ row-tile partials (bn_part_; the separate finalize reads them)
  // ---- side-stream weight gradients (overlap_): kernel stream links (device_comm.h) main -> side
  // "dz(l) ready" and side -> main "weight gradients done", one dz buffer per block (the side
  // stream may still read dz(l) while the main stream writes dz(l-2)); the main -> side signal
  // rides the next main-stream launch (StreamLink::defer) instead of a launch of its own
  bool overlap_ = true;
  hipStream_t side_ = nullptr;
  std::unique_ptr<StreamLink> dz_link_, wg_link_;
  std::vector<torch::Tensor> dz_blk_;
  unsigned long long* pending_sig_ = nullptr;
  bool bwd_sgd_ = false;  // set by step() (world 1, overlapped): block l's SGD behind its wgrad on the side stream
  bool in_step_ = false;  // inside step(): the head's per-column pass forks to the side stream
  torch::Tensor feats_;   // [Bmax, feat]: the last block's output, the classifier's input
  bool side_ok(hipStream_t s) const;  // overlap on and `s` not capturing a graph
  void flush_signal(hipStream_t s);   // launch a pending deferred signal as its own kernel
  void join_side(hipStream_t s);      // `s` waits for every side-stream kernel enqueued so far
  float* P(int64_t off) { return params_.data_ptr<float>() + off; }
  float* G(int64_t off) { return grads_.data_ptr<float>() + off; }
  int64_t Bmax_, feat_, ncls_;
  std::vector<VggBlock> blocks_;
  int64_t fc_w_ = 0, fc_b_ = 0;
  torch::Tensor params_, grads_, mom_, bufs_, nbt_;
  torch::Tensor data_[2], labels_[2], aug_[2];
  torch::Tensor idx_, ylab_, loss_, correct_, logits_, pred_;
  torch::Tensor perm_, cursor_;
  int64_t perm_len_ = 0;
  // gbuf_: gradient ping-pong; ws_ / ws_w_: split-K slabs of the data / weight gradient (distinct:
  // the side stream's weight gradient runs beside the next data gradient); bn_part_: BN-backward partials
  torch::Tensor gbuf_[2], dz_[2], ws_, ws_w_, bn_part_, bn_coef_, bn_eval_, head_ws_;
  // F3 operand bounds, CS_AMAX_SLOT floats per slot: x of block l (slot l), dz of block l (L + l),
  // weights of block l (2L + l)
  torch::Tensor amax_;
  bool f3_probe_ = false;
  float* amax_x(int l) { return amax_.data_ptr<float>() + (int64_t)l * CS_AMAX_SLOT; }
  float* amax_dz(int l) { return amax_.data_ptr<float>() + (int64_t)(blocks_.size() + l) * CS_AMAX_SLOT; }
  // weight bounds, exact per conv weight tensor: the GEMMs read the current slot (2L + l); every
  // SGD launch that rewrites block l's weights folds their new absolute maximum into the next slot
  // (3L + l), whatever its range (CsWeightBounds); the step's first launch makes next current
  // (cs_amax_rotate, folded into the conv0 forward) — for deferred buckets right before their block
  float* amax_w(int l) { return amax_.data_ptr<float>() + (int64_t)(2 * blocks_.size() + l) * CS_AMAX_SLOT; }
  float* amax_wnext(int l) { return amax_.data_ptr<float>() + (int64_t)(3 * blocks_.size() + l) * CS_AMAX_SLOT; }
  unsigned w_pending_ = 0;     // blocks whose next weight bound an enqueued SGD launch is producing
  unsigned w_deferred_ = 0;    // ... of those, the deferred buckets' (rotated after their join)
  bool sgd_deferring_ = false; // step(): the SGD launches being enqueued belong to deferred buckets
  void rotate_w(hipStream_t s, unsigned mask);
  bool f3_used_ = false;  // some conv tile runs the F3 math: the producers publish the bounds
  void update_f3_used();
  bool w_dirty_ = true;   // the weights changed outside an SGD launch: re-measure their bounds
  float* x_amax_out(int l) { return f3_used_ && !f3_probe_ ? amax_x(l) : nullptr; }
  float* dz_amax_out(int l) { return f3_used_ && !f3_probe_ ? amax_dz(l) : nullptr; }
  // the step's / eval's entry: weight bounds re-measured if dirty, else the last step's rotated in
  // (all but deferred buckets'); x / dz bounds zeroed — or, zero_later, both by the conv0 forward,
  // whose launch then takes bounds_to_zero() / rot_mask_
  void f3_refresh(hipStream_t s, bool zero_later = false);
  float* bounds_to_zero() { return f3_used_ && !f3_probe_ ? amax_x(0) : nullptr; }
  unsigned rot_mask_ = 0;  // the weight-bound rotation the conv0 forward folds in (zero_later)
  CsWeightBounds sgd_wb(int64_t off, int64_t n);  // the weight bounds an SGD launch over [off, off + n) produces
  int64_t ws_elems_ = 0;
  int math_ = 2;  // conv autotune candidates: 0 f32 MFMA, 1 split-bf16 X6, 2 both (CS_CONV_MATH)
  // 0 disables (CS_ENGINE_OFF=bn_fused). Measured on MI355X at B=64 (img/s): 0 -> 71.46k, 256 (blocks 6-7)
  // -> 71.64k, 1024 -> 69.85k, 4096 -> 63.07k: one block per 16 channels serialises too many rows
  int64_t bn_fused_rows_ = 256;
  bool sgd_tail_on_ = true;
  bool sgd_tail_ = false;  // set by step() for the step in flight (world 1)
  bool sgd_first_ = false;
  int debug_skip_ = 0;
  // block l's weight gradient (+ the previous fork's SGD as tail workgroups) on the side stream,
  // behind the deferred signal the next main-stream launch carries
  void fork_wgrad(int l, int64_t B);
  bool conv0_direct_ = true;
  bool conv0_direct_ok(int64_t B) const;
  // with_sgd: block 0's SGD step (+ the batch cursor) rides the weight gradient's final sum when the
  // direct kernels run; returns whether it did (else the caller launches the SGD)
  bool conv0_wgrad(int64_t B, hipStream_t s, float* dz, bool with_sgd = false);
  // block 0's BN-backward apply runs inside its weight gradient (cs_conv0_wgrad_bn): set by the BN
  // step of block 0 (only its finalize launched), consumed by conv0_wgrad
  const float* conv0_bn_G_ = nullptr;
  bool conv0_bn_fold_ = true;
  bool conv0_sgd_fold_ = true;
  bool conv0_batch_fold_ = true;
  bool head_bn_fold_ = true;
  bool side_sgd_tail_ = true;
  int side_sgd_pending_ = -1;  // block whose side-stream SGD has not been enqueued yet
  void flush_side_sgd();
  std::vector<int64_t> comm_defer_;
  DeviceComm* defer_comm_ = nullptr;  // deferred buckets enqueued on this communicator, not waited for
  int defer_block_ = -1;              // the next forward waits before this block's conv
  void join_deferred(hipStream_t s);
  double hp_[4] = {0, 0, 0, 0};  // lr, momentum, wd, dampening of the step in flight
  std::vector<std::pair<int64_t, int64_t>> blk_range_;  // block l's [off, off + n) (block L-1 from 0: fc)
  CsSgdTail sgd_tail_args(int64_t block);
  void sgd_on(hipStream_t st, int64_t off, int64_t n, bool cursor);
  bool timing_ = false;
  std::vector<hipEvent_t> tev_;          // timing events (created on demand)
  std::vector<std::string> tnames_;      // phase ending at tev_[i + 1]
  size_t tn_ = 0;                        // events recorded in the last step
  void mark(const char* phase);           // record the next timing event (timing_ only)

 public:
  ~VggEngine();
  VggEngine(const VggEngine&) = delete;
  VggEngine& operator=(const VggEngine&) = delete;
};

}  // namespace cs
