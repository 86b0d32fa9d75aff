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
  bool use_dual = true;  // backward wgrad + dgrad as one launch (if both tiles allow; autotuned)
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
  // With overlap_wgrad the weight-gradient GEMM of block l > 0 runs on a low-priority side
  // stream once block l's data gradient is enqueued, beside the rest of the backward; block
  // 0's (the last GEMM of the step, nothing left to overlap) stays on the caller's stream.
  // join = true makes the caller's stream wait for the side stream before returning.
  void backward(int64_t hi, int64_t lo, int64_t B, bool join = true);
  void set_overlap_wgrad(bool on);
  bool side_wgrad(hipStream_t s) const;  // overlap on and `s` not capturing a graph
  void join_side(hipStream_t s);          // `s` waits for every side-stream weight gradient so far
  // join_side also waits on an event recorded with a SYSTEM-scope release on the side stream:
  // needed when a consumer outside the device's kernels reads the weight gradients (gloo's
  // device-to-host copy of an all-reduce issued from Python; see join_side)
  void set_sys_join(bool on);
  // "" unless a side-stream link wait timed out (device_comm.h StreamLink: bounded waits)
  std::string link_error() const;
  void set_fixup(bool on) { fixup_ = on; }
  void set_epi_red(bool on) { epi_red_ = on; }
  void set_dual(bool on) { dual_ = on; }
  void set_bn_fused_rows(int64_t r) { bn_fused_rows_ = r; }
  bool block_dual(int64_t l) const { return blocks_.at(l).use_dual; }
  void set_block_dual(int64_t l, bool on) { blocks_.at(l).use_dual = on; }
  // SGD (momentum, weight decay, dampening) on [off, off+n) of the flat buffers
  void sgd(double lr, double momentum, double wd, double dampening, int64_t off, int64_t n);
  // SGD of one gradient bucket [off, off+n) (blocks >= lo_block) on the optimizer stream, overlapped
  // with the rest of the backward: it waits for everything enqueued on the current stream (block
  // lo_block's data gradient is the last reader of its weights) and, with a communicator, for the
  // bucket's all-reduce already enqueued on the comm stream. advance_cursor: the step's last
  // bucket moves the device-side batch cursor. join_opt() makes the current stream wait for it.
  void sgd_bucket(DeviceComm* comm, int64_t lo_block, int64_t off, int64_t n, double lr, double momentum, double wd,
                  double dampening, bool advance_cursor);
  void join_opt();
  void set_sgd_overlap(bool on) { sgd_overlap_ = on; }
  void set_sgd_side(bool on) { sgd_side_ = on; }
  // torch.optim.SGD's first step sets buf = d (no dampening): the next step's SGD launches
  // use first = 1 (only matters with dampening != 0); cleared once that step's SGD is enqueued
  void set_sgd_first(bool on) { sgd_first_ = on; }
  // test-only ordering faults for the ProbeComm test's negative control (tests must see a
  // mismatch): bit 0 = step() skips the join before SGD, bit 1 = its all-reduces skip the fork
  void set_debug_skip(int64_t mask) { debug_skip_ = (int)mask; }
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
  void step(int64_t B, DeviceComm* comm, const std::vector<int64_t>& bucket_blocks,
            const std::vector<int64_t>& bucket_ranges, bool broadcast_buffers, double lr, double momentum,
            double wd, double dampening);

  // Phase timing (opt-in): timing events on the compute stream at the step's phase
  // boundaries (forward, each gradient bucket's backward, waiting for the all-reduces, SGD);
  // phase_times() synchronizes and returns the last step's phases in ms. Off by default: an event
  // record on the compute stream costs a few us of launch gap on this stack.
  void set_timing(bool on);
  std::vector<std::pair<std::string, double>> phase_times();

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
            float* dz = nullptr, bool keep_slabs = false, const CsBnRed* red = nullptr,
            const CsBnRed* ered = nullptr, const CsSgdTail* sgd = nullptr, const CsSplitkTail* ktail = nullptr);
  // Serial step: block l's split-K weight-gradient combine rides block l's data-gradient launch as
  // appended blocks (the GEMMs are independent; the combined gradient's first reader is block l's
  // SGD, later) — one launch fewer per split-K weight gradient. Opt-in (CS_KTAIL=1): bit-equal, but
  // measured 83.7k vs 84.1k img/s (profiles/r3_overlap_ab.txt) — the appended slab-summing blocks
  // share the CUs with the data gradient on the critical chain.
  bool ktail_on_ = false;
  CsSplitkTail pend_ktail_{};
  // Block l-1's BN-backward partial sums computed where block l's data gradient is finished —
  // in the dgrad GEMM's epilogue, or in its split-K combine (CsConvArgs::ered) — instead of a
  // reduce launch re-reading G and y; the BN backward of block l-1 is then finalize + apply,
  // with the deferred side-stream signal riding the finalize launch (CS_BN_EPI_RED=0 disables).
  // Only with the three-launch BN path (bn_path_ 0), no in-launch combine and no kept slabs.
  bool epi_red_ = true;
  bool epi_red_ok(int l, int64_t B) const;  // block l's dgrad can carry block l-1's partials
  CsBnRed epi_red_args(int l, int B);       // ... and their arguments (part = bn_part_)
  // Backward order dgrad(l) -> wgrad(l) with block l-1's BN partial-sum pass appended to the
  // wgrad launch (extra blocks dispatched after the GEMM tiles, filling its tail): one launch
  // per block fewer on the critical chain, bit-identical partials (CS_FUSE_BN_RED=0 disables)
  bool fuse_red_ = true;
  int red_pending_ = -1;  // block whose BN partials already sit in bn_part_ (from red_P_ blocks)
  int red_P_ = 0;
  CsConvArgs conv_args(int l, int mode, int B, bool with_stats, float* ws, float* dz);
  // block l's wgrad + dgrad as one launch (both 64x64 register-staged tiles)
  bool dual_ok(int l) const;
  // single-launch BN forward / backward for layers with at most bn_fused_rows_ rows (B*H*W)
  bool bn_fused(int l, int64_t B) const;
  void conv_dual(int l, int B, hipStream_t s, float* dz, const CsBnRed* ered = nullptr);
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
  torch::Tensor gbuf_[2], dz_[2], ws_, ws_side_, bn_part_, bn_coef_, bn_eval_, head_ws_;
  int64_t ws_elems_ = 0;
  torch::Tensor counters_;  // split-K tile tickets, [3 * L][tiles_max_] int32
  int64_t tiles_max_ = 1;
  // in-launch split-K combine where it fits (the last block of a tile sums the slabs in z order;
  // CS_CONV_FIXUP=1 enables). Off by measurement: round 2 64.8k vs 69.1k img/s; round 3, same
  // box, 74.6k / 73.9k (on) vs 78.8k (off). (A first round-3 A/B showed it faster — 96.9k vs
  // 92.3k — because the K-group kernels skipped the combine altogether: neither the in-launch
  // combine nor the reduce launch ran, fixed in conv_common.h and covered by the KG fixup tests.)
  bool fixup_ = false;
  bool dual_ = true;
  // CS_BN_FUSED_ROWS; 0 disables. Measured on MI355X at B=64 (img/s): 0 -> 71.46k, 256 (blocks 6-7)
  // -> 71.64k, 1024 -> 69.85k, 4096 -> 63.07k: one block per 16 channels serialises too many rows
  // BN launches (CS_BN_PATH): 1 = forward finalize+apply in one row-chunked launch, backward
  // chunk partials + finalize-in-apply (two launches); 0 = the separate finalize launches.
  // 0 by measurement (MI355X, B=64): 80.7k img/s vs 77.1k — the channel-sliced blocks of the
  // folded launches stream NHWC rows as 64-B pieces and repeat the finalize in every block,
  // which costs more than the launch they save (e.g. block 0 forward 27.8 us vs 4.9 + 5.2 us)
  // 2 = one-launch grid-barrier BN forward / backward (bn_grid.hip) for the layers the
  // single-block fused kernels do not serve. Measured round 3 (profiles/r3_bn_grid_barrier.txt):
  // the phases alone beat the split launches by 1-2 us per layer, but each in-kernel grid barrier
  // costs ~10-14 us on MI355X (256 blocks over 8 XCDs; hierarchical arrival + load polling still
  // ~10 us), so the step is slower: 69.6k (2) vs 90.6k (0) img/s. Kept opt-in.
  int bn_path_ = 0;
  torch::Tensor grid_bar_;     // zeroed grid-barrier counters of the BN kernels (main stream)
  int* grid_err_ = nullptr;    // host-mapped: a grid barrier timed out
  // a dz-link signal deferred into the next main-stream kernel (StreamLink::defer), or nullptr
  unsigned long long* pending_sig_ = nullptr;
  bool defer_signals_ = true;  // CS_DEFER_SIGNALS=0: every link signal as its own launch
  void flush_signal(hipStream_t s);  // launch a pending deferred signal as its own kernel
  // set by step(): a signal still pending at the end of one bucket's backward() rides the first
  // launch of the next bucket's (with layer-aligned buckets every backward() call is one block,
  // so flushing there put every signal on a launch of its own); step() flushes before any wait
  bool in_step_ = false;
  // World-1 serial step: split-K weight gradients (blocks > 0, <= 32 slabs) leave their slabs in
  // keep_ws_ and the step's one SGD launch sums them (z order: bit-equal) while it updates —
  // no combine launch, no gradient round trip (CS_SGD_SLABS=1 enables). Off with a
  // communicator (the all-reduce needs the combined gradient) and outside step(). Opt-in
  // (CS_SGD_SLABS=1): measured even on MI355X (82.3-82.8k vs 82.8-83.6k img/s) — the SGD pass
  // then walks each range's slabs one float4 at a time, which costs what the saved launches did.
  bool sgd_slabs_on_ = false;
  // World-1 serial step: block l+1's SGD rides block l's weight-gradient GEMM launch as appended
  // blocks (its parameters' last readers — block l+1's BN backward and data gradient — are done),
  // in the GEMM's tail instead of one 9.2M-parameter pass at the end of the step; block 0's update
  // (and the cursor) stays a launch of its own (CS_SGD_TAIL=0 disables)
  bool sgd_tail_on_ = true;
  bool sgd_tail_ = false;  // set by step() for the step in flight
  CsSgdTail sgd_tail_args(int64_t block);
  bool keep_wg_ = false;     // set by step() for the step in flight
  torch::Tensor keep_ws_;
  int64_t keep_used_ = 0;
  CsSgdSlabs sgd_slabs_{};
  // CS_KEEP_SLABS=1: split-K data gradients leave their slabs in ws_ and the next BN backward
  // sums them (z order, bit-equal) while it reads G, instead of a separate combine launch.
  // Off: measured equal on MI355X (81.8-82.0k vs 82.0-82.1k img/s) — both BN passes then read
  // every slab, which costs what the saved launch did. g_slabs_ / g_stride_ describe where the
  // gradient of the block below currently lives (1 = gbuf_)
  bool keep_slabs_ = false;
  int g_slabs_ = 1;
  int64_t g_stride_ = 0;
  int math_ = 2;  // conv autotune candidates: 0 f32 MFMA, 1 split-bf16 X6, 2 both (CS_CONV_MATH)
  int64_t bn_fused_rows_ = 256;  // horizontal wgrad+dgrad fusion in backward (CS_CONV_DUAL=0 disables)
  hipStream_t side_ = nullptr;
  bool overlap_wgrad_ = false;
  bool sys_join_ = false;
  hipEvent_t sys_ev_ = nullptr;
  // per-bucket SGD on opt_ overlapping the backward of the blocks below (CS_SGD_OVERLAP=1 enables).
  // Off: measured on MI355X (B=64, full-step hipGraph) 66.0-66.6k img/s with it vs 81.2k without —
  // the graph's cross-stream fork/join edges cost far more than the 28 us SGD they hide
  hipStream_t opt_ = nullptr;
  bool sgd_overlap_ = false;
  bool sgd_first_ = false;
  int debug_skip_ = 0;
  std::vector<hipEvent_t> ev_opt_;  // pool: main-stream / comm-stream marks per bucket, opt done
  size_t next_opt_ev_ = 0;
  hipEvent_t opt_event();
  bool timing_ = false;
  std::vector<hipEvent_t> tev_;          // timing events (created on demand)
  std::vector<std::string> tnames_;      // phase ending at tev_[i + 1]
  size_t tn_ = 0;                        // events recorded in the last step
  void mark(const char* phase);           // record the next timing event (timing_ only)
  // side-stream weight gradients (CS_OVERLAP_WGRAD=1): kernel stream links (device_comm.h),
  // main -> side "dz(l) ready" and side -> main "weight gradients done", and one dz buffer
  // per block
  std::unique_ptr<StreamLink> dz_link_, wg_link_;
  bool wgrad_after_dgrad_ = true;  // fork point of the side wgrad (CS_WGRAD_AFTER_DGRAD=0: before dgrad)
  std::vector<torch::Tensor> dz_blk_;
  // SGD behind the weight gradients (CS_SGD_SIDE=0 disables; needs overlap_wgrad, the
  // dgrad-first fork and a block-contiguous flat layout): at world 1 each block's parameters
  // are updated on the side stream right after its weight gradient (block 0's on the main
  // stream), with a communicator each bucket's SGD runs on the comm stream right behind its
  // all-reduce — the 28 us optimizer pass leaves the end of the step. Bit-identical: every
  // element gets the same update, only its launch differs.
  bool sgd_side_ = true;
  bool bwd_sgd_ = false;  // set by step(): backward() issues the per-block SGD
  double hp_[4] = {0, 0, 0, 0};  // lr, momentum, wd, dampening of the step in flight
  std::vector<std::pair<int64_t, int64_t>> blk_range_;  // block l's [off, off + n) (block L-1 from 0: fc)
  void sgd_on(hipStream_t st, int64_t off, int64_t n, bool cursor);

 public:
  ~VggEngine();
  VggEngine(const VggEngine&) = delete;
  VggEngine& operator=(const VggEngine&) = delete;
};

}  // namespace cs
