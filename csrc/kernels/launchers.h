// Host-side launch API of the gfx950 kernels (raw pointers + stream; no torch headers,
// so every .hip compiles in seconds and the kernels are reusable from the C++ runtime).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct CsTensorEntry {
  float* p;
  float* g;
  float* m;
  int64_t n;
  uint16_t* shadow;  // optional bf16 copy of p, rewritten by the update (the bf16 GEMMs' operand)
};

// data pipeline
hipError_t cs_augment(const uint8_t* data, const int64_t* idx, const int32_t* params, float* out, int B, int nhwc,
                      int cstride, const float* mean, const float* std_, hipStream_t stream);
hipError_t cs_gather_labels(const int64_t* labels, const int64_t* idx, int64_t* out, int B, hipStream_t stream);
// engine batch: sample = perm[*cursor * stride + b] (or idx_in[b] when perm is null) -> NHWC x4 input, idx_out, labels
hipError_t cs_make_batch(const uint8_t* data, const int64_t* labels, const int64_t* perm, const int64_t* cursor,
                         int stride, const int64_t* idx_in, const int32_t* params, float* out, int64_t* idx_out,
                         int64_t* ylab, int B, const float* mean, const float* std_, hipStream_t stream);

// optimizer
// counter (optional): incremented once by the launch (the engine's device-side step cursor)
// The F3 conv math's weight bounds, produced by the SGD launch that writes the weights: up to
// CS_WB_MAX conv-weight intervals [lo, hi) (element offsets relative to the launch's range start),
// each with the CS_AMAX_SLOT bound the absolute maximum of its updated elements is folded into. Each
// element counts for the interval that holds it, so the bounds are exact per weight tensor whatever
// the SGD launch's range (a block, a bucket, the whole buffer). n == 0: none.
#define CS_WB_MAX 16
struct CsWeightBounds {
  int64_t lo[CS_WB_MAX], hi[CS_WB_MAX];
  float* amax[CS_WB_MAX];
  int n;
};
// the absolute maximum of x[0, n) folded (atomic max) into one CS_AMAX_SLOT bound
hipError_t cs_amax(const float* x, int64_t n, float* amax, hipStream_t stream);
// F3 weight bounds of the blocks in `mask`: cur = next, next = 0 (CS_AMAX_SLOT slots, block l at l)
hipError_t cs_amax_rotate(float* cur, float* next, unsigned mask, int L, hipStream_t stream);
hipError_t cs_sgd_flat(float* p, const float* g, float* m, int64_t n, float lr, float mom, float wd, float damp,
                       float scale, int first, hipStream_t stream, int64_t* counter = nullptr,
                       const CsWeightBounds* wb = nullptr);
// faithful sync modes on flat gradients (flat_ops.hip): dst = mean over `rows` rows of src [rows][n];
// g = g + t, then / div when div > 0
hipError_t cs_rows_mean(float* src, int rows, int64_t n, float* dst, int bcast, hipStream_t stream);
hipError_t cs_accumulate(float* g, const float* t, int64_t n, float div, hipStream_t stream);
// bf16 gradient transport: to_bf16 = 1: fp32 src -> bf16 dst (round to nearest even); 0: bf16 -> fp32
hipError_t cs_cast_grad(const void* src, void* dst, int64_t n, int to_bf16, hipStream_t stream);
hipError_t cs_sgd_multi(const CsTensorEntry* tab_dev, int ntens, const int64_t* chunk_start_dev, int nchunks,
                        float lr, float mom, float wd, float damp, float scale, int first, hipStream_t stream);

// classifier head
// bn (optional, part 0 / 1): the features are the last VGG block's BatchNorm + ReLU + 2x2 max-pool of
// its pre-BN output y [B][2][2][K] (scale / shift per channel), computed in the row pass (bn_apply's
// arithmetic and max order: the same bits) and written to feat for the column pass
// the classifier's per-column pass (dW, db, loss, correct count) as data (P = C*ceil(K/64)+1
// wave-sized pieces)
struct CsHeadCols {
  const float* feat;
  int B, K, C;
  const float* ws;
  float* dW;
  float* db;
  float* loss_out;
  int* correct_out;
  int P;
};
inline int cs_head_cols_pieces(int K, int C) { return C * ((K + 63) / 64) + 1; }
struct CsHeadBn {
  const float* y;
  const float* scale;
  const float* shift;
};
hipError_t cs_linear_xent(const float* feat, const float* W, const float* bias, const int64_t* labels, int B, int K,
                          int C, float gscale, float* loss_out, int* correct_out, float* logits_out, float* dW,
                          float* db, float* dfeat, int64_t* pred_out, float* ws, hipStream_t stream, int part = 0,
                          const CsHeadBn* bn = nullptr);
// part: 0 both launches; 1 the per-row pass (logits, prediction, dlogits -> ws, dfeat); 2 the
// per-column pass (dW, db, loss, correct count from ws and feat) — run after part 1 (ws)
inline int64_t cs_linear_xent_ws(int B, int C) { return (int64_t)B * (C + 2); }
hipError_t cs_softmax_xent(const float* logits, const int64_t* labels, int B, int C, float gscale, float* loss_out,
                           float* dlogits, int* correct_out, hipStream_t stream);

// ---------------------------------------------------------------- conv (implicit GEMM, fp32 MFMA)
enum { CS_CONV_FWD = 0, CS_CONV_DGRAD = 1, CS_CONV_WGRAD = 2 };
// operand absolute-maximum bounds (the F3 conv math's scales) are kept as CS_AMAX_SHARDS shards,
// each the atomic max of the producer workgroups with blockIdx % CS_AMAX_SHARDS == shard (one atomic
// per workgroup, shards CS_AMAX_STRIDE floats = one 128-byte line apart: no hot word or line), and
// the bound is the largest shard; a slot is CS_AMAX_SLOT floats
#define CS_AMAX_SHARDS 64
#define CS_AMAX_STRIDE 32
#define CS_AMAX_SLOT (CS_AMAX_SHARDS * CS_AMAX_STRIDE)

// One BN-backward partial-sum pass (bn.hip "reduce"): y, incoming gradient G, the forward's
// scale/shift/mean/invstd, partials out part [P][C][3]. P == 0: none.
struct CsBnRed {
  const float *y, *G, *scale, *shift, *mean, *invstd;
  float* part;
  int B, H, W, C, pool, P;
};

// An SGD update of one parameter range carried by extra blocks appended to a GEMM launch (after
// its tiles, like CsBnRed): P blocks (the launcher sizes it when n > 0); n == 0: none.
struct CsSgdTail {
  float* p;
  const float* g;
  float* m;
  int64_t n;
  float lr, mom, wd, damp;
  int first, P;
  CsWeightBounds wb;  // optional (wb.n == 0): the weights' bounds for the F3 conv math
};

// BatchNorm finalize by the last-arriving block of the launch that produces the statistics
// partials (bn_fin.h): FWD with CsConvArgs::stats (scale / shift / mean / invstd -> bnv [4][C],
// running stats, num_batches_tracked), BWD with CsConvArgs::ered (coef [C][3], dgamma, dbeta,
// dbias; ered.part is then [T][C][4]). cnt == null: off (the separate finalize launch runs).
struct CsBnFin {
  int* cnt;    // zeroed ticket counters, >= cs_bn_fin_ints(...) ints (left zeroed by the launch)
  float* grp;  // level-1 group partials, >= cs_bn_fin_grp_floats(...) floats
  int T, R, M;  // row tiles of the partials, rows per tile, rows (the last tile may be short)
  int count;    // BWD: elements per channel of the BN layer (full resolution) for the means
  const float *gamma, *beta, *invstd;  // invstd: BWD (the forward's)
  float *rmean, *rvar;                 // FWD running stats (may be null)
  int64_t* nbt;                        // FWD (may be null)
  float momentum, eps;
  float* bnv;                          // FWD out [4][C]
  float *coef, *dgamma, *dbeta, *dbias;  // BWD out (dgamma / dbeta / dbias may be null)
};
// tickets and group-partial floats a launch needs for T row tiles of C channels in column
// tiles of nc channels (64 or 128)
inline int cs_bn_fin_groups(int T, int nc) { return (T + 8 * (256 / nc) - 1) / (8 * (256 / nc)); }
inline int cs_bn_fin_ints(int T, int C, int nc) { return ((C + nc - 1) / nc) * (cs_bn_fin_groups(T, nc) + 1); }
inline int64_t cs_bn_fin_grp_floats(int T, int C, int nc) { return (int64_t)cs_bn_fin_groups(T, nc) * C * 4; }

struct CsConvArgs {
  const float* x;     // FWD / WGRAD: conv input, NHWC [B,H,W,Cin] (Cin = 4 for the padded conv0 input)
  const float* w;     // FWD / DGRAD: weights, OHWI [Cout][9][Cin]; conv0 (w_oihw=1): OIHW [Cout][3][9]
  const float* dz;    // DGRAD / WGRAD: gradient w.r.t. conv output, NHWC [B,H,W,Cout]
  const float* bias;  // FWD: [Cout] or null
  float* out;         // FWD: y [M][Cout]; DGRAD: dx [M][Cin]; WGRAD: dW (OHWI, or OIHW for conv0)
  float* ws;          // split-K slabs [splits][M][N] (required when splits > 1)
  float* stats;       // FWD: per-row-tile BN partials [tiles][Cout][2] = (mean, M2); may be null
  int B, H, W, Cin, Cout;
  int w_oihw;
  // DGRAD: the BN-backward partial sums of the block below (whose output gradient this GEMM
  // produces), taken from the finished output values where they are still in registers — the
  // GEMM epilogue, or the split-K combine — instead of a separate reduce pass over G and y.
  // Uses y, scale, shift, mean, invstd, pool and part ([row tiles][N][3], row tiles of BM rows,
  // or CS_SPLITK_STAT_ROWS behind the split-K combine: cs_conv_ered_rows); part == null: none
  CsBnRed ered;
  // an independent SGD update appended to the launch (the serial world-1 step: block l+1's
  // parameters, whose last reader has run, ride block l's weight-gradient GEMM)
  CsSgdTail sgd;
  // CS_STAGE_F3: device pointers to CS_AMAX_SLOT bounds (largest shard) of |A| / |B| (the
  // GEMM's A operand: FWD x, DGRAD / WGRAD dz; B: FWD / DGRAD w, WGRAD x); each sets its operand's
  // power-of-two scale
  const float* amax_a;
  const float* amax_b;
  // FWD (with stats) / DGRAD (with ered): the BN finalize by the launch's last-arriving block
  // (or the split-K combine's); fin.cnt == null: off
  CsBnFin fin;
  // filled by the launcher:
  int lgH, lgW, lgCin, lgCout, M, N, K, ksteps_per_split, total_ksteps;
};

void cs_conv_fill_dims(CsConvArgs* a, int mode);

// VGG block 0 (3 -> 64 channels, 32 x 32, input padded to 4 channels NHWC, OIHW weights) as direct
// f32 kernels (conv0.hip). fwd: y [pix][64] (+bias) and, when stats != null, the BatchNorm tile
// statistics [pix / cs_conv0_tile_rows()][64][2] = (mean, M2); wgrad: dW (OIHW [64][27]) through
// `part` scratch of cs_conv0_wgrad_part_floats() floats (fixed-order sum: deterministic)
// the training batch itself (augment.hip make_batch's job) as conv0's input source: sample index
// (device cursor into the permutation, or idx_in), label gather, RandomCrop(32, 4) + HFlip +
// Normalize of the uint8 images straight into the conv's LDS halo; the block-0 input x_out
// (for the weight gradient) is written as make_batch writes it
struct CsBatchSrc {
  const uint8_t* data;
  const int64_t* labels;
  const int64_t* perm;
  const int64_t* cursor;
  int stride;
  const int64_t* idx_in;
  const int32_t* params;
  float* x_out;
  int64_t* idx_out;
  int64_t* ylab;
  float m[3], inv[3];
};
int cs_conv0_tile_rows();
size_t cs_conv0_wgrad_part_floats(int B, int H, int W);
// zero_bounds (optional): zero_slots F3 operand bounds (CS_AMAX_SLOT apart) this launch resets;
// rot_cur / rot_next / rot_mask (optional): the weight-bound rotation of cs_amax_rotate, folded in
hipError_t cs_conv0_fwd(const float* x, const float* w, const float* bias, float* y, float* stats, int B, int H,
                        int W, int Cout, hipStream_t stream, const CsBatchSrc* batch = nullptr,
                        float* zero_bounds = nullptr, int zero_slots = 0, float* rot_cur = nullptr,
                        float* rot_next = nullptr, unsigned rot_mask = 0);
// sgd (optional): block 0's parameter range, whose SGD step then rides the fixed-order sum (dW at
// w_rel within the range; the range's other gradients must be final; counter: the batch cursor)
hipError_t cs_conv0_wgrad(const float* x, const float* dz, float* part, float* dw, int B, int H, int W, int Cout,
                          hipStream_t stream, const CsSgdTail* sgd = nullptr, int w_rel = 0,
                          int64_t* counter = nullptr);
// the same weight gradient with block 0's BN (+ReLU, 2x2 max-pool) backward apply folded in: dZ is
// computed in LDS from y (pre-BN conv output), G (gradient of the pooled output), the forward's
// scale/shift/mean/invstd and the backward finalize's coef [C][3] (cs_bn_bwd_finalize) — the
// same bits as cs_bn_bwd_tail's dZ, never written to memory
hipError_t cs_conv0_wgrad_bn(const float* x, const float* y, const float* G, const float* scale, const float* shift,
                             const float* mean, const float* invstd, const float* coef, float* part, float* dw, int B,
                             int H, int W, int Cout, hipStream_t stream, const CsSgdTail* sgd = nullptr,
                             int w_rel = 0, int64_t* counter = nullptr);
// bm, bn in {64, 128}; bk in {16, 32}; splits >= 1 (split-K over blockIdx.z + deterministic reduce).
// FWD stats tiles have `bm` rows when splits == 1 and CS_SPLITK_STAT_ROWS rows otherwise.
#define CS_SPLITK_STAT_ROWS 16
// stage: CS_STAGE_REGS (global -> registers -> ds_write, padded LDS) or CS_STAGE_LDS_DMA(_DEEP)
// (buffer_load ... lds into a 3- (5-) deep ring of swizzled images; bk = 32, not conv0's fwd;
// the deep ring only where 5 images fit the 160 KiB LDS)
// CS_STAGE_KG2 / KG4: register staging with 2 / 4 K-groups of 4 waves per block (bk >= 32 / 64)
// | CS_STAGE_X6: the same staging with fp32-accurate split-bf16 math (3 bf16 pieces per
// operand, 6 v_mfma_f32_32x32x16_bf16 per 32x32x16 product; conv_gemm.hip "X6")
// | CS_STAGE_X6S: X6 math with the split done once at the LDS store into bf16 planes (register
// staging / K-groups only; bk 64 only with 64x64 tiles)
// | CS_STAGE_BF16: operands rounded to bf16 at the LDS store, one bf16 MFMA, f32 accumulate
// (reduced precision: only for the engine's opt-in bf16 mode, never picked by the f32 autotune)
// | CS_STAGE_F3: fp32-class split into two fp16 planes of the power-of-two-scaled operand (scales
// from CsConvArgs::amax_a / amax_b, required), 3 v_mfma_f32_32x32x16_f16 per product (conv_gemm.hip "F3")
enum { CS_STAGE_REGS = 0, CS_STAGE_LDS_DMA = 1, CS_STAGE_LDS_DMA_DEEP = 2, CS_STAGE_KG2 = 3, CS_STAGE_KG4 = 4,
       CS_STAGE_X6 = 8, CS_STAGE_X6S = 16, CS_STAGE_BF16 = 32, CS_STAGE_F3 = 64 };
// whether a (stage, tile, bk) combination has a kernel
bool cs_conv_stage_ok(int stage, int bm, int bn, int bk, bool conv0_fwd);
hipError_t cs_conv_gemm(CsConvArgs a, int mode, int bm, int bn, int bk, int splits, hipStream_t stream,
                        int stage = CS_STAGE_REGS);
// deterministic split-K combine of `splits` fp32 slabs in a.ws (dims filled): sum in split order
// (+bias and BN tile statistics of CS_SPLITK_STAT_ROWS rows for FWD; conv0's OIHW scatter for WGRAD)
hipError_t cs_conv_splitk_reduce(const CsConvArgs& a, int mode, int splits, hipStream_t stream);
// the split count cs_conv_gemm actually launches (K-steps re-balanced over splits)
int cs_conv_effective_splits(int K, int bk, int splits);
// FWD statistics tile height for a launch (bm, or CS_SPLITK_STAT_ROWS behind the reduce kernel)
int cs_conv_stat_rows(int K, int bm, int bk, int splits);
// rows per BN-backward partial of a DGRAD launch carrying `ered` (bm, or CS_SPLITK_STAT_ROWS
// when split-K: the combine launch computes them)
int cs_conv_ered_rows(int K, int bm, int bk, int splits);

// ---------------------------------------------------------------- BatchNorm + ReLU (+ 2x2 max-pool), NHWC
hipError_t cs_bn_finalize(const float* part, int T, int R, int M, int C, const float* gamma, const float* beta,
                          float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps,
                          float* scale, float* shift, float* save_mean, float* save_invstd, hipStream_t stream);
hipError_t cs_bn_eval_coeffs(const float* gamma, const float* beta, const float* rm, const float* rv, int C, float eps,
                             float* scale, float* shift, hipStream_t stream);
// amax (optional): a CS_AMAX_SLOT bound the output's absolute maximum is atomically folded into
// (the F3 conv math's operand bound); the same for dz in the BN-backward launchers below
hipError_t cs_bn_apply(const float* y, const float* scale, const float* shift, float* out, int B, int H, int W, int C,
                       int pool, hipStream_t stream, float* amax = nullptr);
int cs_bn_bwd_blocks(int B, int H, int W, int C, int pool);
// part: [cs_bn_bwd_blocks][C][3] scratch; coef: [C][3] scratch; dgamma/dbeta/dbias may be null.
// LDS bytes the BN-backward reduce body needs (C channels)
inline size_t cs_bn_red_lds(int C) { return (size_t)(256 / (C / 4)) * C * 3 * sizeof(float); }
// finalize + apply of the BN backward when the reduce already ran (part from P blocks, e.g.
// appended to the weight-gradient GEMM launch of the block above, or P row tiles of the data-
// gradient GEMM that produced G: CsConvArgs::ered); signal: optional stream-link counter the
// finalize launch bumps when it starts
hipError_t cs_bn_bwd_tail(const float* y, const float* G, int B, int H, int W, int C, int pool, const float* scale,
                          const float* shift, const float* mean, const float* invstd, const float* gamma,
                          const float* part, int P, float* coef, float* dgamma, float* dbeta, float* dbias, float* dz,
                          hipStream_t stream, unsigned long long* signal = nullptr, float* amax = nullptr);
// the finalize half of cs_bn_bwd_tail alone (coef, dgamma / dbeta / dbias), for a consumer that
// applies the backward itself (cs_conv0_wgrad_bn)
hipError_t cs_bn_bwd_finalize(const float* part, int P, int C, int M, const float* gamma, const float* invstd,
                              float* coef, float* dgamma, float* dbeta, float* dbias, hipStream_t stream,
                              unsigned long long* signal = nullptr);
hipError_t cs_bn_bwd(const float* y, const float* G, int B, int H, int W, int C, int pool, const float* scale,
                     const float* shift, const float* mean, const float* invstd, const float* gamma, float* part,
                     float* coef, float* dgamma, float* dbeta, float* dbias, float* dz, hipStream_t stream,
                     float* amax = nullptr);

// single-launch BN for small layers (one block per 16 channels owns all their rows):
// forward = finalize (tile partials -> bnv [4][C] = scale, shift, mean, invstd + running stats)
// + normalize/ReLU(/pool); backward = reduce + finalize + apply (coef [C][3] scratch)
hipError_t cs_bn_fused_fwd(const float* part, int T, int R, int M, int C, const float* gamma, const float* beta,
                           float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps,
                           float* bnv, const float* y, float* out, int B, int H, int W, int pool, hipStream_t stream);
hipError_t cs_bn_fused_bwd(const float* y, const float* G, int B, int H, int W, int C, int pool, const float* bnv,
                           const float* gamma, float* coef, float* dgamma, float* dbeta, float* dbias, float* dz,
                           hipStream_t stream, unsigned long long* signal = nullptr, float* amax = nullptr);
// finalize + apply of the BN backward in ONE launch when the reduce already ran (the data-gradient
// epilogue's P row-tile partials [P][C][3], CsConvArgs::ered): grid (C/16, row chunks), every block
// finalizes its 16 channels from the P partials (the same fixed-order sum in every block), block row
// 0 publishes coef / dgamma / dbeta / dbias, each block applies dZ to its chunk of rows — the
// backward twin of cs_bn_fused_fwd (one launch boundary fewer than cs_bn_bwd_tail)
hipError_t cs_bn_bwd_tail_fused(const float* y, const float* G, int B, int H, int W, int C, int pool, const float* bnv,
                                const float* gamma, const float* part, int P, float* coef, float* dgamma, float* dbeta,
                                float* dbias, float* dz, hipStream_t stream, unsigned long long* signal = nullptr);
// the BN backward's apply pass alone (dZ from G, y and the finalized coef [C][3]): the finalize
// ran as the last-arriver tail of the data-gradient launch that produced G (CsConvArgs::fin)
hipError_t cs_bn_bwd_apply(const float* y, const float* G, int B, int H, int W, int C, int pool, const float* scale,
                           const float* shift, const float* mean, const float* invstd, const float* coef, float* dz,
                           hipStream_t stream, unsigned long long* signal = nullptr);

// ---------------------------------------------------------------- ordering-probe communicator (comm_probe.hip)
enum { CS_SCRAMBLE_F32 = 0, CS_SCRAMBLE_I64 = 1, CS_SCRAMBLE_I32 = 2 };
// a bounded (<= 0.1 s) busy wait of `us` microseconds on `stream`
// ctas > 0: that many busy 256-thread workgroups (an RCCL collective's CTA footprint) instead
// of one sleeping wave; sink: 256 floats never written in practice
hipError_t cs_comm_spin(double us, hipStream_t stream, int ctas = 0, float* sink = nullptr);
// exact invertible scramble: floats x2 (inverse x0.5), integers +1 (inverse -1)
hipError_t cs_comm_scramble(void* buf, int64_t n, int kind, int inverse, hipStream_t stream);

// ---------------------------------------------------------------- stream links (stream_link.hip)
// signal: count += 1 on `stream`; wait: *expect += delta, then poll until count >= *expect.
// The wait ends early only when the host sets *abort (host-mapped; *err = 2) or after timeout_s
// (*err = 1; the engine sets it to the communicator timeout, so the step watchdog fires
// first). count / expect: device memory, zeroed; err / abort: host-mapped.
hipError_t cs_link_signal(unsigned long long* count, hipStream_t stream);
hipError_t cs_link_wait(const unsigned long long* count, unsigned long long* expect, int* err, const int* abort,
                        double timeout_s, hipStream_t stream, unsigned long long delta = 1);

// Diagnostic shader-clock sampler (clock_probe.hip; scripts/ramp_clock.py): out holds
// max_samples + 1 pairs (s_memrealtime, s_memtime), 0-terminated when stopped early; stop and
// slots: device memory, zeroed. Not used by the engine.
hipError_t cs_clock_sampler(unsigned long long* out, int max_samples, int* stop, hipStream_t stream);
hipError_t cs_clock_stamp(unsigned long long* slots, int i, hipStream_t stream);
hipError_t cs_clock_stop(int* stop, hipStream_t stream);

// ---------------------------------------------------------------- decoder-LM elementwise ops (lm.hip)
enum { CS_F32 = 0, CS_BF16 = 1 };
int cs_rmsnorm_bwd_partials(int rows, int D);
// y has dtype odt (e.g. bf16 out of an fp32 residual stream under autocast; odt != dt needs D % 4 == 0)
hipError_t cs_rmsnorm_fwd(int dt, int wdt, int odt, const void* x, const void* w, void* y, float* rstd, int rows,
                          int D, float eps, hipStream_t s);
// part: [cs_rmsnorm_bwd_partials(rows, D)][D] fp32 scratch; dw has the weight's dtype, g dtype gdt, dx x's
hipError_t cs_rmsnorm_bwd(int dt, int wdt, int gdt, const void* x, const void* w, const float* rstd, const void* g,
                          void* dx, void* dw, float* part, int rows, int D, hipStream_t s);
// softmax cross-entropy, logits [R, V] fp32/bf16 with V % 8 == 0, targets in [0, V): per-row loss and
// log-sum-exp; backward dlogits = (softmax - onehot) * g[0] * inv_n in the logits' dtype
hipError_t cs_xent_fwd(int dt, const void* logits, const int64_t* tgt, float* loss, float* lse, int R, int V,
                       hipStream_t s);
hipError_t cs_xent_bwd(int dt, const void* logits, const int64_t* tgt, const float* lse, const float* g, float inv_n,
                       void* dlogits, int R, int V, hipStream_t s);
hipError_t cs_swiglu_fwd(int dt, const void* a, const void* b, void* out, size_t n, hipStream_t s);
hipError_t cs_swiglu_bwd(int dt, const void* a, const void* b, const void* g, void* da, void* db, size_t n,
                         hipStream_t s);
// x/out: [B, S, H, hd] contiguous; cos/sin: [S, hd/2] fp32; inverse rotates by -angle (backward)
// causal / full grouped-query flash attention, bf16 [B, S, H, D] (attention.hip); lse: f32 [B, Hq, S]
// base-2 row log-sum-exp of the scaled scores; delta: f32 [B, Hq, S] scratch of the backward
hipError_t cs_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int Hq, int Hkv,
                       int D, float scale, int causal, hipStream_t stream);
hipError_t cs_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                       float* delta, void* dq, void* dk, void* dv, int B, int S, int Hq, int Hkv, int D, float scale,
                       int causal, hipStream_t stream);
// training BatchNorm2d (+ residual add, + ReLU) on NCHW fp32 / bf16 activations (bn_nchw.hip).
// stat: f32 [4, C] = scale, shift, mean, invstd (written by the forward, read by the backward);
// part: f32 scratch of cs_bn_nchw_partials(N, C) floats; coef: f32 [3, C] scratch (backward).
// rm / rv (running stats, updated with `momentum`; nbt += 1), w / b, res, dres, dw, db, nbt may be null.
int cs_bn_nchw_partials(int N, int C);
hipError_t cs_bn_nchw_fwd(int dt, const void* x, const void* res, const float* w, const float* b, float* rm, float* rv,
                          int64_t* nbt, float momentum, float eps, int relu, void* y, float* stat, float* part, int N,
                          int C, int HW, hipStream_t stream);
hipError_t cs_bn_nchw_bwd(int dt, const void* dy, const void* x, const void* res, const float* w, const float* stat,
                          int relu, void* dx, void* dres, float* dw, float* db, float* coef, float* part, int N, int C,
                          int HW, hipStream_t stream);
// 3x3 / stride 2 / pad 1 max-pool on NCHW planes (pool_nchw.hip); pos: uint8 winning window
// position per output (0..8), consumed by the gather-style backward
hipError_t cs_maxpool3s2_fwd(int dt, const void* x, void* y, unsigned char* pos, int64_t planes, int H, int W, int Ho,
                             int Wo, hipStream_t stream);
hipError_t cs_maxpool3s2_bwd(int dt, const void* dy, const unsigned char* pos, void* dx, int64_t planes, int H, int W,
                             int Ho, int Wo, hipStream_t stream);
// bf16 GEMM on the matrix cores (gemm_bf16.hip): C[M, N] (=, +=) sum_k A(m, k) B(n, k), fp32
// accumulate. A is stored K-major ([M][K], row stride lda) or M-major ([K][M]); B K-major ([N][K])
// or N-major ([K][N]). out_mode 0: C bf16, 1: C fp32, 2: C fp32 +=, 3: C bf16 +=. Needs 16-byte aligned
// operands, lda / ldb % 8 == 0, K % 8 == 0 for a K-major operand, N, ldc % 4 == 0.
// splits > 1 (out_mode 1 only): split s of the reduction writes the fp32 slab C + s * slab
// (elements), to be summed by cs_slab_sum; cs_gemm_bf16_splits gives the default count.
// forward product with BatchNorm statistics of its bf16 output C[M, N] (A, B K-major, out bf16):
// stats[tile row t][N][2] = (mean, M2) of the bf16 values of rows [256 t, 256 t + 256)
hipError_t cs_gemm_bf16_bn_stats(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M,
                                 int N, int K, float* stats, hipStream_t stream);
int cs_gemm_bf16_splits(int M, int N, int K);
hipError_t cs_gemm_bf16(int a_kmajor, const void* A, int64_t lda, int b_kmajor, const void* B, int64_t ldb, void* C,
                        int64_t ldc, int M, int N, int K, int out_mode, int splits, int64_t slab, hipStream_t stream);
hipError_t cs_rope(int dt, const void* x, const float* cosv, const float* sinv, void* out, int B, int S, int H, int hd,
                   int inverse, hipStream_t s);
// channels-last (NHWC) CNN kernels (cnn_nhwc.hip), fp32 / bf16 activations, M = B*H*W rows of C.
// BatchNorm: stat / coef / part exactly as the NCHW kernels above (part: cs_bn_nhwc_partials floats).
// mask (optional, M*C/V bytes, V = cs_bn_nhwc_vec): the forward writes each V-channel vector's
// pre-activation > 0 bits; the backward then takes the ReLU mask from it instead of recomputing it
// from x and the residual (one activation-sized read fewer per pass for a residual BatchNorm).
int cs_bn_nhwc_partials(int64_t M, int C, int dt);
int cs_bn_nhwc_vec(int C, int dt);
hipError_t cs_bn_nhwc_fwd(int dt, const void* x, const void* res, const float* w, const float* b, float* rm, float* rv,
                          int64_t* nbt, float momentum, float eps, int relu, void* y, float* stat, float* part,
                          int64_t M, int C, hipStream_t stream, unsigned char* mask = nullptr);
// the same from per-tile (mean, M2) partials of R-row tiles ([T][C][2], cs_gemm_bf16_bn_stats)
// instead of a statistics pass over x: finalize (Chan, f64, fixed order) + apply
hipError_t cs_bn_nhwc_fwd_tiles(int dt, const void* x, const void* res, const float* w, const float* b, float* rm,
                                float* rv, int64_t* nbt, float momentum, float eps, int relu, void* y, float* stat,
                                const float* tiles, int T, int R, int64_t M, int C, hipStream_t stream,
                                unsigned char* mask);
hipError_t cs_bn_nhwc_bwd(int dt, const void* dy, const void* x, const void* res, const float* w, const float* stat,
                          int relu, void* dx, void* dres, float* dw, float* db, float* coef, float* part, int64_t M,
                          int C, hipStream_t stream, const unsigned char* mask = nullptr,
                          const unsigned char* pool_pos = nullptr, int H = 0, int W = 0, int Ho = 0, int Wo = 0);
// (pool_pos: the BatchNorm's output was 3x3/2 max-pooled (cs_maxpool3s2_nhwc_fwd's window positions
// for the [B, Ho, Wo, C] output; x is [B, H, W, C]) and dy is the pooled gradient — the pool's
// backward gather is fused into both BatchNorm backward passes)
// stat (optional, a BatchNorm's [4][C] from cs_bn_nhwc_fwd with y == nullptr = statistics only):
// pool relu(BN(x)) — the BatchNorm apply fused into the pool's window loads
hipError_t cs_maxpool3s2_nhwc_fwd(int dt, const void* x, void* y, unsigned char* pos, int B, int H, int W, int C,
                                  int Ho, int Wo, hipStream_t stream, const float* stat = nullptr);
hipError_t cs_maxpool3s2_nhwc_bwd(int dt, const void* dy, const unsigned char* pos, void* dx, int B, int H, int W,
                                  int C, int Ho, int Wo, hipStream_t stream);
// bf16 NHWC implicit-GEMM convolution (conv_nhwc.hip; C, Co % 32 == 0, any R x S / stride / pad):
// FWD y[B,Ho,Wo,Co] = conv(x, w [Co][R][S][C]); DGRAD dx = y-shaped dy through wt [C][R][S][Co]
// (the weight transposed by the caller), written to y; WGRAD: split-K fp32 slabs in dw
// ([splits][Co][R*S*C], cs_conv_nhwc_splits) summed in split order into dw_out [Co][R*S*C] fp32.
struct CsConvNhwcArgs {
  const void* x;   // FWD / WGRAD: bf16 [B, H, W, C]
  const void* w;   // FWD: bf16 [Co][R][S][C]; DGRAD: bf16 [C][R][S][Co]
  const void* dy;  // DGRAD / WGRAD: bf16 [B, Ho, Wo, Co]
  void* y;         // FWD: y; DGRAD: dx (bf16 [B, H, W, C])
  float* dw;       // WGRAD: slab workspace
  float* dw_out;   // WGRAD: fp32 [Co][R*S*C]
  int B, H, W, C, Co, R, S, st, pad;
  // filled by the launcher
  int Ho, Wo, M, N, K, ksteps, ksteps_per_split;
};
// out[n] = deterministic sum of part[z][n] over z < splits (fp32; n % 4 == 0)
hipError_t cs_slab_sum(const float* part, int splits, int64_t n, float* out, hipStream_t stream);
int cs_conv_nhwc_splits(int mode, int B, int H, int W, int C, int Co, int R, int S, int st, int pad);
hipError_t cs_conv_nhwc(int mode, const CsConvNhwcArgs& a, int splits, hipStream_t stream);
// col: [B*Ho*Wo, Kp], columns (r*S + s)*C + c, zero for k >= R*S*C; col2im is its adjoint (gather)
hipError_t cs_im2col_nhwc(int dt, const void* x, void* col, int B, int H, int W, int C, int R, int S, int stride,
                          int pad, int Ho, int Wo, int Kp, hipStream_t stream);
hipError_t cs_col2im_nhwc(int dt, const void* dcol, void* dx, int B, int H, int W, int C, int R, int S, int stride,
                          int pad, int Ho, int Wo, int Kp, hipStream_t stream);
