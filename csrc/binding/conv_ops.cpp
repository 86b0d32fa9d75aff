// torch bindings: implicit-GEMM conv (fwd / dgrad / wgrad) and the fused BN kernels.
// All shapes are validated on the host before any launch.
#include "binding/torch_util.h"
#include "kernels/launchers.h"

namespace {

using csb::cur_stream;
using csb::DevGuard;

const float* cptr(const c10::optional<torch::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}
float* mptr(const c10::optional<torch::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}

void check_t(const c10::optional<torch::Tensor>& t, int64_t numel, const char* name) {
  if (!t.has_value() || !t->defined()) return;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous(), name,
              ": must be a contiguous float32 GPU tensor");
  TORCH_CHECK(t->numel() >= numel, name, ": has ", t->numel(), " elements, kernel needs ", numel);
}

bool pow2(int64_t v) { return v > 0 && (v & (v - 1)) == 0; }

// returns the number of rows per FWD statistics tile
int64_t conv_gemm(int64_t mode, c10::optional<torch::Tensor> x, c10::optional<torch::Tensor> w,
                  c10::optional<torch::Tensor> dz, c10::optional<torch::Tensor> bias, torch::Tensor out,
                  c10::optional<torch::Tensor> ws, c10::optional<torch::Tensor> stats, int64_t B, int64_t H, int64_t W,
                  int64_t Cin, int64_t Cout, bool w_oihw, int64_t bm, int64_t bn, int64_t splits, int64_t bk,
                  c10::optional<torch::Tensor> counters, int64_t stage) {
  TORCH_CHECK(mode >= 0 && mode <= 2, "conv_gemm: bad mode");
  TORCH_CHECK(pow2(H) && pow2(W) && pow2(Cin) && pow2(Cout) && Cin >= 4 && Cout >= 64 && B > 0,
              "conv_gemm: H, W, Cin, Cout must be powers of two (Cin>=4, Cout>=64)");
  TORCH_CHECK((bm == 64 || bm == 128) && (bn == 64 || bn == 128) && (bk == 16 || bk == 32 || bk == 64) && splits >= 1,
              "conv_gemm: bad tiling");
  TORCH_CHECK(!w_oihw || Cin == 4, "conv_gemm: OIHW weights only for the padded conv0 (Cin=4)");
  if (mode == CS_CONV_DGRAD) TORCH_CHECK(Cin >= 64 && !w_oihw, "conv_gemm: dgrad needs Cin >= 64");
  const int64_t pix = B * H * W;
  const int64_t wnum = w_oihw ? Cout * 27 : Cout * 9 * Cin;
  CsConvArgs a{};
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.w_oihw = w_oihw ? 1 : 0;
  cs_conv_fill_dims(&a, (int)mode);
  if (mode == CS_CONV_FWD) {
    TORCH_CHECK(x.has_value() && w.has_value(), "conv fwd needs x and w");
    check_t(x, pix * Cin, "x"); check_t(w, wnum, "w"); check_t(bias, Cout, "bias");
    check_t(out, pix * Cout, "out");
    const int64_t R = cs_conv_stat_rows(9 * Cin, bm, bn, bk, splits, counters.has_value());
    check_t(stats, ((pix + R - 1) / R) * Cout * 2, "stats");
  } else if (mode == CS_CONV_DGRAD) {
    TORCH_CHECK(dz.has_value() && w.has_value(), "conv dgrad needs dz and w");
    check_t(dz, pix * Cout, "dz"); check_t(w, wnum, "w"); check_t(out, pix * Cin, "out");
  } else {
    TORCH_CHECK(dz.has_value() && x.has_value(), "conv wgrad needs dz and x");
    check_t(dz, pix * Cout, "dz"); check_t(x, pix * Cin, "x"); check_t(out, wnum, "out");
  }
  const int64_t sp = cs_conv_effective_splits(a.K, bk, splits);
  if (sp > 1) {
    TORCH_CHECK(ws.has_value() && ws->defined(), "conv_gemm: split-K needs a workspace");
    check_t(ws, sp * (int64_t)a.M * a.N, "ws");
  }
  const int64_t ntiles = ((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
  if (counters.has_value()) {
    TORCH_CHECK(counters->is_cuda() && counters->scalar_type() == at::kInt && counters->is_contiguous() &&
                    counters->numel() >= ntiles,
                "conv_gemm: counters must be a zeroed contiguous int32 GPU tensor with >= ", ntiles, " elements");
    a.counters = counters->data_ptr<int>();
  }
  DevGuard g(out.device());
  a.x = cptr(x); a.w = cptr(w); a.dz = cptr(dz); a.bias = cptr(bias);
  a.out = out.data_ptr<float>(); a.ws = mptr(ws); a.stats = mptr(stats);
  TORCH_CHECK(cs_conv_stage_ok((int)stage, (int)bm, (int)bn, (int)bk, w_oihw && mode == CS_CONV_FWD) &&
                  !(bk == 64 && w_oihw && mode == CS_CONV_FWD),
              "conv_gemm: no kernel for stage ", stage, " / ", bm, "x", bn, " / bk ", bk);
  CS_LAUNCH(cs_conv_gemm(a, (int)mode, (int)bm, (int)bn, (int)bk, (int)splits, cur_stream(), (int)stage));
  return cs_conv_stat_rows(a.K, bm, bn, bk, splits, counters.has_value());
}

// P3 operand: contiguous bfloat16 [n/8, 3, 8] chunks (h, m, l per 8 elements, split3)
const uint16_t* planes(const c10::optional<torch::Tensor>& t, int64_t need, int64_t& ps, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->numel() >= 3 * need,
              name, ": must be a contiguous bfloat16 GPU tensor of >= 3 x ", need, " elements (P3 chunks, split3)");
  ps = need;
  return reinterpret_cast<const uint16_t*>(t->data_ptr<at::BFloat16>());
}

// pre-split ("XP") conv GEMM: operands as bf16 planes [3][n] (split3); returns FWD stats rows
int64_t conv_gemm_xp(int64_t mode, c10::optional<torch::Tensor> x3, c10::optional<torch::Tensor> w3,
                     c10::optional<torch::Tensor> dz3, c10::optional<torch::Tensor> bias, torch::Tensor out,
                     c10::optional<torch::Tensor> ws, c10::optional<torch::Tensor> stats, int64_t B, int64_t H,
                     int64_t W, int64_t Cin, int64_t Cout, int64_t bm, int64_t bn, int64_t splits, int64_t bk,
                     int64_t kg, int64_t nb) {
  TORCH_CHECK(mode >= 0 && mode <= 2, "conv_gemm_xp: bad mode");
  TORCH_CHECK(pow2(H) && pow2(W) && pow2(Cin) && pow2(Cout) && Cin >= 64 && Cout >= 64 && B > 0,
              "conv_gemm_xp: H, W, Cin, Cout powers of two, Cin/Cout >= 64");
  TORCH_CHECK(cs_conv_xp_ok((int)bm, (int)bn, (int)bk, (int)kg, (int)nb) && splits >= 1,
              "conv_gemm_xp: no kernel for ", bm, "x", bn, " bk ", bk, " kg ", kg, " nb ", nb);
  const int64_t pix = B * H * W, wnum = Cout * 9 * Cin;
  CsConvArgs a{};
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout;
  cs_conv_fill_dims(&a, (int)mode);
  if (mode != CS_CONV_DGRAD) {
    TORCH_CHECK(x3.has_value(), "conv_gemm_xp: needs x3");
    a.x3 = planes(x3, pix * Cin, a.x3s, "x3");
  }
  if (mode != CS_CONV_WGRAD) {
    TORCH_CHECK(w3.has_value(), "conv_gemm_xp: needs w3");
    a.w3 = planes(w3, wnum, a.w3s, "w3");
  }
  if (mode != CS_CONV_FWD) {
    TORCH_CHECK(dz3.has_value(), "conv_gemm_xp: needs dz3");
    a.dz3 = planes(dz3, pix * Cout, a.dz3s, "dz3");
  }
  check_t(bias, Cout, "bias");
  check_t(out, mode == CS_CONV_FWD ? pix * Cout : (mode == CS_CONV_DGRAD ? pix * Cin : wnum), "out");
  const int64_t R = cs_conv_stat_rows(a.K, bm, bn, bk, splits, false);
  if (mode == CS_CONV_FWD) check_t(stats, ((pix + R - 1) / R) * Cout * 2, "stats");
  const int64_t sp = cs_conv_effective_splits(a.K, bk, splits);
  if (sp > 1) {
    TORCH_CHECK(ws.has_value() && ws->defined(), "conv_gemm_xp: split-K needs a workspace");
    check_t(ws, sp * (int64_t)a.M * a.N, "ws");
  }
  DevGuard g(out.device());
  a.bias = cptr(bias);
  a.out = out.data_ptr<float>(); a.ws = mptr(ws); a.stats = mode == CS_CONV_FWD ? mptr(stats) : nullptr;
  CS_LAUNCH(cs_conv_xp(a, (int)mode, (int)bm, (int)bn, (int)bk, (int)splits, (int)kg, (int)nb, cur_stream()));
  return R;
}

void split3(torch::Tensor x, torch::Tensor out) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.numel() % 8 == 0,
              "split3: x must be a contiguous float32 GPU tensor with numel % 8 == 0");
  int64_t ps = 0;
  const uint16_t* o = planes(out, x.numel(), ps, "out");
  DevGuard g(x.device());
  CS_LAUNCH(cs_split3(x.data_ptr<float>(), const_cast<uint16_t*>(o), x.numel(), cur_stream()));
}

void bn_finalize(torch::Tensor part, int64_t T, int64_t R, int64_t M, torch::Tensor gamma, torch::Tensor beta,
                 c10::optional<torch::Tensor> running_mean, c10::optional<torch::Tensor> running_var,
                 c10::optional<torch::Tensor> nbt, double momentum, double eps, torch::Tensor scale,
                 torch::Tensor shift, torch::Tensor save_mean, torch::Tensor save_invstd) {
  const int64_t C = gamma.numel();
  check_t(part, T * C * 2, "part");
  TORCH_CHECK(T == (M + R - 1) / R, "bn_finalize: T must be ceil(M/R)");
  for (auto* t : {&beta, &scale, &shift, &save_mean, &save_invstd}) check_t(*t, C, "bn vec");
  check_t(running_mean, C, "running_mean"); check_t(running_var, C, "running_var");
  int64_t* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    TORCH_CHECK(nbt->scalar_type() == at::kLong && nbt->is_cuda(), "num_batches_tracked must be int64 GPU");
    nb = nbt->data_ptr<int64_t>();
  }
  DevGuard g(part.device());
  CS_LAUNCH(cs_bn_finalize(part.data_ptr<float>(), T, R, M, C, gamma.data_ptr<float>(), beta.data_ptr<float>(),
                           mptr(running_mean), mptr(running_var), nb, (float)momentum, (float)eps,
                           scale.data_ptr<float>(), shift.data_ptr<float>(), save_mean.data_ptr<float>(),
                           save_invstd.data_ptr<float>(), cur_stream()));
}

void bn_eval_coeffs(torch::Tensor gamma, torch::Tensor beta, torch::Tensor rm, torch::Tensor rv, double eps,
                    torch::Tensor scale, torch::Tensor shift) {
  const int64_t C = gamma.numel();
  for (auto* t : {&beta, &rm, &rv, &scale, &shift}) check_t(*t, C, "bn vec");
  DevGuard g(gamma.device());
  CS_LAUNCH(cs_bn_eval_coeffs(gamma.data_ptr<float>(), beta.data_ptr<float>(), rm.data_ptr<float>(),
                              rv.data_ptr<float>(), C, (float)eps, scale.data_ptr<float>(), shift.data_ptr<float>(),
                              cur_stream()));
}

void bn_apply(torch::Tensor y, torch::Tensor scale, torch::Tensor shift, torch::Tensor out, int64_t B, int64_t H,
              int64_t W, int64_t C, bool pool) {
  TORCH_CHECK(C % 4 == 0 && (!pool || (H % 2 == 0 && W % 2 == 0)), "bn_apply: shape");
  check_t(y, B * H * W * C, "y"); check_t(scale, C, "scale"); check_t(shift, C, "shift");
  check_t(out, B * (pool ? H / 2 : H) * (pool ? W / 2 : W) * C, "out");
  DevGuard g(y.device());
  CS_LAUNCH(cs_bn_apply(y.data_ptr<float>(), scale.data_ptr<float>(), shift.data_ptr<float>(), out.data_ptr<float>(),
                        B, H, W, C, pool ? 1 : 0, cur_stream()));
}

int64_t bn_bwd_blocks(int64_t B, int64_t H, int64_t W, int64_t C, bool pool) {
  return cs_bn_bwd_blocks(B, H, W, C, pool ? 1 : 0);
}

void bn_bwd(torch::Tensor y, torch::Tensor G, int64_t B, int64_t H, int64_t W, int64_t C, bool pool,
            torch::Tensor scale, torch::Tensor shift, torch::Tensor mean, torch::Tensor invstd, torch::Tensor gamma,
            torch::Tensor part, torch::Tensor coef, c10::optional<torch::Tensor> dgamma,
            c10::optional<torch::Tensor> dbeta, c10::optional<torch::Tensor> dbias, torch::Tensor dz) {
  TORCH_CHECK(C % 4 == 0 && C <= 1024 && (!pool || (H % 2 == 0 && W % 2 == 0)), "bn_bwd: shape");
  check_t(y, B * H * W * C, "y");
  check_t(G, B * (pool ? H / 2 : H) * (pool ? W / 2 : W) * C, "G");
  for (auto* t : {&scale, &shift, &mean, &invstd, &gamma}) check_t(*t, C, "bn vec");
  check_t(part, (int64_t)cs_bn_bwd_blocks(B, H, W, C, pool) * C * 3, "part");
  check_t(coef, C * 3, "coef");
  check_t(dgamma, C, "dgamma"); check_t(dbeta, C, "dbeta"); check_t(dbias, C, "dbias");
  check_t(dz, B * H * W * C, "dz");
  DevGuard g(y.device());
  CS_LAUNCH(cs_bn_bwd(y.data_ptr<float>(), G.data_ptr<float>(), B, H, W, C, pool ? 1 : 0, scale.data_ptr<float>(),
                      shift.data_ptr<float>(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                      gamma.data_ptr<float>(), part.data_ptr<float>(), coef.data_ptr<float>(), mptr(dgamma),
                      mptr(dbeta), mptr(dbias), dz.data_ptr<float>(), cur_stream()));
}

void bn_fused_fwd(torch::Tensor part, int64_t T, int64_t R, int64_t M, torch::Tensor gamma, torch::Tensor beta,
                  c10::optional<torch::Tensor> running_mean, c10::optional<torch::Tensor> running_var,
                  c10::optional<torch::Tensor> nbt, double momentum, double eps, torch::Tensor bnv, torch::Tensor y,
                  torch::Tensor out, int64_t B, int64_t H, int64_t W, bool pool) {
  const int64_t C = gamma.numel();
  TORCH_CHECK(C % 16 == 0 && (!pool || (H % 2 == 0 && W % 2 == 0)) && M == B * H * W && T == (M + R - 1) / R,
              "bn_fused_fwd: shape");
  check_t(part, T * C * 2, "part"); check_t(beta, C, "beta"); check_t(bnv, 4 * C, "bnv");
  check_t(running_mean, C, "running_mean"); check_t(running_var, C, "running_var");
  check_t(y, M * C, "y"); check_t(out, B * (pool ? H / 2 : H) * (pool ? W / 2 : W) * C, "out");
  if (nbt.has_value()) TORCH_CHECK(nbt->scalar_type() == at::kLong && nbt->is_cuda(), "nbt: int64 GPU scalar");
  DevGuard g(y.device());
  CS_LAUNCH(cs_bn_fused_fwd(part.data_ptr<float>(), T, R, M, C, gamma.data_ptr<float>(), beta.data_ptr<float>(),
                            mptr(running_mean), mptr(running_var),
                            nbt.has_value() ? nbt->data_ptr<int64_t>() : nullptr, (float)momentum, (float)eps,
                            bnv.data_ptr<float>(), y.data_ptr<float>(), out.data_ptr<float>(), B, H, W, pool ? 1 : 0,
                            cur_stream()));
}

// one-launch grid-barrier BN (bn_grid.hip); bar: zeroed int32 counters (>= kCsBnGridBarInts), left zeroed
void bn_grid_fwd(torch::Tensor part, int64_t T, int64_t R, int64_t M, torch::Tensor gamma, torch::Tensor beta,
                 c10::optional<torch::Tensor> running_mean, c10::optional<torch::Tensor> running_var,
                 c10::optional<torch::Tensor> nbt, double momentum, double eps, torch::Tensor bnv, torch::Tensor y,
                 torch::Tensor out, int64_t B, int64_t H, int64_t W, bool pool, torch::Tensor bar) {
  const int64_t C = gamma.numel();
  TORCH_CHECK(C % 4 == 0 && (!pool || (H % 2 == 0 && W % 2 == 0)) && M == B * H * W && T == (M + R - 1) / R,
              "bn_grid_fwd: shape");
  check_t(part, T * C * 2, "part"); check_t(beta, C, "beta"); check_t(bnv, 4 * C, "bnv");
  check_t(running_mean, C, "running_mean"); check_t(running_var, C, "running_var");
  check_t(y, M * C, "y"); check_t(out, B * (pool ? H / 2 : H) * (pool ? W / 2 : W) * C, "out");
  TORCH_CHECK(bar.is_cuda() && bar.scalar_type() == at::kInt && bar.numel() >= kCsBnGridBarInts, "bn_grid: bar int32 [>= kCsBnGridBarInts]");
  if (nbt.has_value()) TORCH_CHECK(nbt->scalar_type() == at::kLong && nbt->is_cuda(), "nbt: int64 GPU scalar");
  CsBnGridFwd g{};
  g.part = part.data_ptr<float>(); g.gamma = gamma.data_ptr<float>(); g.beta = beta.data_ptr<float>();
  g.y = y.data_ptr<float>(); g.running_mean = mptr(running_mean); g.running_var = mptr(running_var);
  g.bnv = bnv.data_ptr<float>(); g.out = out.data_ptr<float>();
  g.nbt = nbt.has_value() ? nbt->data_ptr<int64_t>() : nullptr;
  g.momentum = (float)momentum; g.eps = (float)eps;
  g.T = T; g.R = R; g.M = M; g.B = B; g.H = H; g.W = W; g.C = C; g.pool = pool ? 1 : 0;
  g.bar = reinterpret_cast<unsigned*>(bar.data_ptr<int>());
  DevGuard dg(y.device());
  CS_LAUNCH(cs_bn_grid_fwd(g, cur_stream()));
}

void bn_grid_bwd(torch::Tensor y, torch::Tensor G, int64_t B, int64_t H, int64_t W, int64_t C, bool pool,
                 torch::Tensor bnv, torch::Tensor gamma, torch::Tensor part, torch::Tensor coef,
                 c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta,
                 c10::optional<torch::Tensor> dbias, torch::Tensor dz, torch::Tensor bar) {
  TORCH_CHECK(C % 4 == 0 && C <= 1024 && (!pool || (H % 2 == 0 && W % 2 == 0)), "bn_grid_bwd: shape");
  check_t(y, B * H * W * C, "y");
  check_t(G, B * (pool ? H / 2 : H) * (pool ? W / 2 : W) * C, "G");
  check_t(bnv, 4 * C, "bnv"); check_t(gamma, C, "gamma"); check_t(coef, 3 * C, "coef");
  check_t(part, (int64_t)cs_bn_bwd_blocks(B, H, W, C, pool) * C * 3, "part");
  check_t(dgamma, C, "dgamma"); check_t(dbeta, C, "dbeta"); check_t(dbias, C, "dbias");
  check_t(dz, B * H * W * C, "dz");
  TORCH_CHECK(bar.is_cuda() && bar.scalar_type() == at::kInt && bar.numel() >= kCsBnGridBarInts, "bn_grid: bar int32 [>= kCsBnGridBarInts]");
  CsBnGridBwd g{};
  const float* bv = bnv.data_ptr<float>();
  g.y = y.data_ptr<float>(); g.G = G.data_ptr<float>();
  g.scale = bv; g.shift = bv + C; g.mean = bv + 2 * C; g.invstd = bv + 3 * C; g.gamma = gamma.data_ptr<float>();
  g.part = part.data_ptr<float>(); g.coef = coef.data_ptr<float>();
  g.dgamma = mptr(dgamma); g.dbeta = mptr(dbeta); g.dbias = mptr(dbias); g.dz = dz.data_ptr<float>();
  g.B = B; g.H = H; g.W = W; g.C = C; g.pool = pool ? 1 : 0; g.gslabs = 1;
  g.bar = reinterpret_cast<unsigned*>(bar.data_ptr<int>());
  DevGuard dg(y.device());
  CS_LAUNCH(cs_bn_grid_bwd(g, cur_stream()));
}

void bn_fused_bwd(torch::Tensor y, torch::Tensor G, int64_t B, int64_t H, int64_t W, int64_t C, bool pool,
                  torch::Tensor bnv, torch::Tensor gamma, torch::Tensor coef, c10::optional<torch::Tensor> dgamma,
                  c10::optional<torch::Tensor> dbeta, c10::optional<torch::Tensor> dbias, torch::Tensor dz) {
  TORCH_CHECK(C % 16 == 0 && (!pool || (H % 2 == 0 && W % 2 == 0)), "bn_fused_bwd: shape");
  check_t(y, B * H * W * C, "y");
  check_t(G, B * (pool ? H / 2 : H) * (pool ? W / 2 : W) * C, "G");
  check_t(bnv, 4 * C, "bnv"); check_t(gamma, C, "gamma"); check_t(coef, 3 * C, "coef");
  check_t(dgamma, C, "dgamma"); check_t(dbeta, C, "dbeta"); check_t(dbias, C, "dbias");
  check_t(dz, B * H * W * C, "dz");
  DevGuard g(y.device());
  CS_LAUNCH(cs_bn_fused_bwd(y.data_ptr<float>(), G.data_ptr<float>(), B, H, W, C, pool ? 1 : 0, bnv.data_ptr<float>(),
                            gamma.data_ptr<float>(), coef.data_ptr<float>(), mptr(dgamma), mptr(dbeta), mptr(dbias),
                            dz.data_ptr<float>(), cur_stream()));
}

void bn_bwd2(torch::Tensor y, torch::Tensor G, int64_t B, int64_t H, int64_t W, int64_t C, bool pool,
             torch::Tensor bnv, torch::Tensor gamma, torch::Tensor part, c10::optional<torch::Tensor> dgamma,
             c10::optional<torch::Tensor> dbeta, c10::optional<torch::Tensor> dbias, torch::Tensor dz) {
  TORCH_CHECK(C % 16 == 0 && C <= 1024 && (!pool || (H % 2 == 0 && W % 2 == 0)), "bn_bwd2: shape");
  check_t(y, B * H * W * C, "y");
  check_t(G, B * (pool ? H / 2 : H) * (pool ? W / 2 : W) * C, "G");
  check_t(bnv, 4 * C, "bnv"); check_t(gamma, C, "gamma");
  check_t(part, (int64_t)cs_bn_bwd_chunks(B, H, W, C, pool) * C * 3, "part");
  check_t(dgamma, C, "dgamma"); check_t(dbeta, C, "dbeta"); check_t(dbias, C, "dbias");
  check_t(dz, B * H * W * C, "dz");
  DevGuard g(y.device());
  CS_LAUNCH(cs_bn_bwd2(y.data_ptr<float>(), G.data_ptr<float>(), B, H, W, C, pool ? 1 : 0, bnv.data_ptr<float>(),
                       gamma.data_ptr<float>(), part.data_ptr<float>(), mptr(dgamma), mptr(dbeta), mptr(dbias),
                       dz.data_ptr<float>(), cur_stream()));
}

}  // namespace

void register_conv_ops(pybind11::module& m) {
  m.def("bn_bwd2", &bn_bwd2, "two-launch BN backward: chunk partials, then finalize folded into the apply");
  m.def("bn_bwd_chunks", [](int64_t B, int64_t H, int64_t W, int64_t C, bool pool) {
    return cs_bn_bwd_chunks(B, H, W, C, pool ? 1 : 0);
  });
  m.def("bn_fused_fwd", &bn_fused_fwd, "single-launch BN finalize + normalize/ReLU(/pool) (small layers)");
  m.def("bn_grid_fwd", &bn_grid_fwd, "one-launch grid-barrier BN finalize + normalize/ReLU(/pool)");
  m.def("bn_grid_bwd", &bn_grid_bwd, "one-launch grid-barrier BN backward: partials | finalize | apply");
  m.def("bn_fused_bwd", &bn_fused_bwd, "single-launch BN backward: reduce + finalize + apply (small layers)");
  m.def("conv_gemm", &conv_gemm, "implicit-GEMM 3x3 conv (mode 0 fwd / 1 dgrad / 2 wgrad), fp32 MFMA",
        py::arg("mode"), py::arg("x"), py::arg("w"), py::arg("dz"), py::arg("bias"), py::arg("out"), py::arg("ws"),
        py::arg("stats"), py::arg("B"), py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("Cout"),
        py::arg("w_oihw"), py::arg("bm"), py::arg("bn"), py::arg("splits"), py::arg("bk") = 16,
        py::arg("counters") = py::none(), py::arg("stage") = 0);
  m.def("conv_stage_ok", [](int64_t stage, int64_t bm, int64_t bn, int64_t bk, bool conv0_fwd) {
    return cs_conv_stage_ok((int)stage, (int)bm, (int)bn, (int)bk, conv0_fwd) && !(bk == 64 && conv0_fwd);
  }, "whether a conv GEMM (staging, tile, K-step) variant exists");
  m.def("conv_stat_rows", [](int64_t K, int64_t bm, int64_t bn, int64_t bk, int64_t splits, bool counters) {
    return cs_conv_stat_rows((int)K, (int)bm, (int)bn, (int)bk, (int)splits, counters);
  }, "FWD BN-statistics tile height of a conv_gemm launch");
  m.def("conv_gemm_xp", &conv_gemm_xp, "pre-split (bf16 planes) implicit-GEMM 3x3 conv, six-product split-bf16 MFMA",
        py::arg("mode"), py::arg("x3"), py::arg("w3"), py::arg("dz3"), py::arg("bias"), py::arg("out"), py::arg("ws"),
        py::arg("stats"), py::arg("B"), py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("Cout"), py::arg("bm"),
        py::arg("bn"), py::arg("splits"), py::arg("bk"), py::arg("kg"), py::arg("nb") = 0);
  m.def("conv_xp_ok", [](int64_t bm, int64_t bn, int64_t bk, int64_t kg, int64_t nb) {
    return cs_conv_xp_ok((int)bm, (int)bn, (int)bk, (int)kg, (int)nb);
  }, "whether a pre-split conv GEMM variant exists", py::arg("bm"), py::arg("bn"), py::arg("bk"), py::arg("kg"),
        py::arg("nb") = 0);
  m.def("split3", &split3, "fp32 -> P3 bf16 chunks [n/8][3][8] (h, m, l: x = h + m + l to 2^-26)");
  m.def("bn_finalize", &bn_finalize);
  m.def("bn_eval_coeffs", &bn_eval_coeffs);
  m.def("bn_apply", &bn_apply);
  m.def("bn_bwd_blocks", &bn_bwd_blocks);
  m.def("bn_bwd", &bn_bwd);
}
