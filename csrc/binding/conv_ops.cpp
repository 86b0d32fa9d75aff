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
                  int64_t stage, c10::optional<torch::Tensor> fin_cnt, c10::optional<torch::Tensor> fin_grp,
                  c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta,
                  c10::optional<torch::Tensor> running_mean, c10::optional<torch::Tensor> running_var,
                  c10::optional<torch::Tensor> bnv, double momentum, double eps, c10::optional<torch::Tensor> amax_a,
                  c10::optional<torch::Tensor> amax_b) {
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
    const int64_t R = cs_conv_stat_rows(9 * Cin, bm, bk, splits);
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
  if (fin_cnt.has_value() && fin_cnt->defined()) {
    // FWD BatchNorm finalize by the launch's last-arriving block (bn_fin.h): bnv [4][Cout] out
    TORCH_CHECK(mode == CS_CONV_FWD && stats.has_value() && gamma.has_value() && beta.has_value() && bnv.has_value(),
                "conv_gemm: the in-launch BN finalize needs FWD, stats, gamma, beta and bnv");
    const int R = cs_conv_stat_rows(a.K, bm, bk, splits), T = (a.M + R - 1) / R, nc = sp > 1 ? 64 : bn;
    TORCH_CHECK(fin_cnt->is_cuda() && fin_cnt->scalar_type() == at::kInt && fin_cnt->is_contiguous() &&
                    fin_cnt->numel() >= cs_bn_fin_ints(T, Cout, nc),
                "conv_gemm: fin_cnt must be a zeroed int32 GPU tensor of >= ", cs_bn_fin_ints(T, Cout, nc), " ints");
    TORCH_CHECK(fin_grp.has_value(), "conv_gemm: fin_grp needed");
    check_t(fin_grp, cs_bn_fin_grp_floats(T, Cout, nc), "fin_grp");
    check_t(gamma, Cout, "gamma"); check_t(beta, Cout, "beta"); check_t(bnv, 4 * Cout, "bnv");
    check_t(running_mean, Cout, "running_mean"); check_t(running_var, Cout, "running_var");
    a.fin.cnt = fin_cnt->data_ptr<int>();
    a.fin.grp = fin_grp->data_ptr<float>();
    a.fin.T = T; a.fin.R = R; a.fin.M = a.M;
    a.fin.gamma = cptr(gamma); a.fin.beta = cptr(beta);
    a.fin.rmean = mptr(running_mean); a.fin.rvar = mptr(running_var);
    a.fin.momentum = (float)momentum; a.fin.eps = (float)eps;
    a.fin.bnv = mptr(bnv);
  }
  DevGuard g(out.device());
  a.x = cptr(x); a.w = cptr(w); a.dz = cptr(dz); a.bias = cptr(bias);
  a.out = out.data_ptr<float>(); a.ws = mptr(ws); a.stats = mptr(stats);
  // CS_STAGE_F3: GPU tensors of CS_AMAX_SLOT floats whose shards bound |A| / |B| (the scales' source)
  check_t(amax_a, CS_AMAX_SLOT, "amax_a"); check_t(amax_b, CS_AMAX_SLOT, "amax_b");
  a.amax_a = cptr(amax_a); a.amax_b = cptr(amax_b);
  TORCH_CHECK(!(stage & CS_STAGE_F3) || (a.amax_a != nullptr && a.amax_b != nullptr),
              "conv_gemm: the F3 stage needs amax_a and amax_b");
  TORCH_CHECK(cs_conv_stage_ok((int)stage, (int)bm, (int)bn, (int)bk, w_oihw && mode == CS_CONV_FWD) &&
                  !(bk == 64 && w_oihw && mode == CS_CONV_FWD),
              "conv_gemm: no kernel for stage ", stage, " / ", bm, "x", bn, " / bk ", bk);
  CS_LAUNCH(cs_conv_gemm(a, (int)mode, (int)bm, (int)bn, (int)bk, (int)splits, cur_stream(), (int)stage));
  return cs_conv_stat_rows(a.K, bm, bk, splits);
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

}  // namespace

void register_conv_ops(pybind11::module& m) {
  m.def("bn_fused_fwd", &bn_fused_fwd, "single-launch BN finalize + normalize/ReLU(/pool) (small layers)");
  m.def("bn_fused_bwd", &bn_fused_bwd, "single-launch BN backward: reduce + finalize + apply (small layers)");
  m.def("conv_gemm", &conv_gemm, "implicit-GEMM 3x3 conv (mode 0 fwd / 1 dgrad / 2 wgrad), fp32 MFMA",
        py::arg("mode"), py::arg("x"), py::arg("w"), py::arg("dz"), py::arg("bias"), py::arg("out"), py::arg("ws"),
        py::arg("stats"), py::arg("B"), py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("Cout"),
        py::arg("w_oihw"), py::arg("bm"), py::arg("bn"), py::arg("splits"), py::arg("bk") = 16,
        py::arg("stage") = 0, py::arg("fin_cnt") = py::none(), py::arg("fin_grp") = py::none(),
        py::arg("gamma") = py::none(), py::arg("beta") = py::none(), py::arg("running_mean") = py::none(),
        py::arg("running_var") = py::none(), py::arg("bnv") = py::none(), py::arg("momentum") = 0.1,
        py::arg("eps") = 1e-5, py::arg("amax_a") = py::none(), py::arg("amax_b") = py::none());
  m.def("bn_fin_sizes", [](int64_t T, int64_t C, int64_t nc) {
    return std::vector<int64_t>{cs_bn_fin_ints((int)T, (int)C, (int)nc), cs_bn_fin_grp_floats((int)T, (int)C, (int)nc)};
  }, "(ticket ints, group-partial floats) of an in-launch BN finalize over T row tiles, C channels, nc-wide column tiles");
  m.def("conv_stage_ok", [](int64_t stage, int64_t bm, int64_t bn, int64_t bk, bool conv0_fwd) {
    return cs_conv_stage_ok((int)stage, (int)bm, (int)bn, (int)bk, conv0_fwd) && !(bk == 64 && conv0_fwd);
  }, "whether a conv GEMM (staging, tile, K-step) variant exists");
  m.def("conv_effective_splits", [](int64_t K, int64_t bk, int64_t splits) {
    return cs_conv_effective_splits((int)K, (int)bk, (int)splits);
  }, "the split-K count a conv_gemm launch actually uses");
  m.def("conv_stat_rows", [](int64_t K, int64_t bm, int64_t bk, int64_t splits) {
    return cs_conv_stat_rows((int)K, (int)bm, (int)bk, (int)splits);
  }, "FWD BN-statistics tile height of a conv_gemm launch");
  m.def(
      "conv0_fwd",
      [](torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> bias, bool with_stats) {
        // x [B, 32, 32, 4] NHWC (channel 3 unused), w OIHW [64, 3, 3, 3] -> y [B*32*32, 64] (+ stats)
        TORCH_CHECK(x.dim() == 4 && x.size(1) == 32 && x.size(2) == 32 && x.size(3) == 4, "conv0_fwd: x [B,32,32,4]");
        check_t(x, x.numel(), "x");
        check_t(w, 64 * 27, "w");
        check_t(bias, 64, "bias");
        DevGuard g(x.device());
        const int64_t B = x.size(0), pix = B * 1024;
        auto y = torch::empty({pix, 64}, x.options());
        torch::Tensor st = with_stats ? torch::empty({pix / cs_conv0_tile_rows(), 64, 2}, x.options()) : torch::Tensor();
        CS_LAUNCH(cs_conv0_fwd(x.data_ptr<float>(), w.data_ptr<float>(), cptr(bias), y.data_ptr<float>(),
                               with_stats ? st.data_ptr<float>() : nullptr, (int)B, 32, 32, 64, cur_stream()));
        return std::vector<torch::Tensor>{y, st};
      },
      "VGG block 0's 3x3 conv (3 -> 64) as the direct f32 kernel (+ BN tile statistics)");
  m.def(
      "conv0_wgrad",
      [](torch::Tensor x, torch::Tensor dz) {
        TORCH_CHECK(x.dim() == 4 && x.size(1) == 32 && x.size(2) == 32 && x.size(3) == 4, "conv0_wgrad: x [B,32,32,4]");
        const int64_t B = x.size(0), pix = B * 1024;
        check_t(x, x.numel(), "x");
        check_t(dz, pix * 64, "dz");
        DevGuard g(x.device());
        auto part = torch::empty({(int64_t)cs_conv0_wgrad_part_floats((int)B, 32, 32)}, x.options());
        auto dw = torch::empty({64, 3, 3, 3}, x.options());
        CS_LAUNCH(cs_conv0_wgrad(x.data_ptr<float>(), dz.data_ptr<float>(), part.data_ptr<float>(), dw.data_ptr<float>(),
                                 (int)B, 32, 32, 64, cur_stream()));
        return dw;
      },
      "VGG block 0's weight gradient (OIHW) as the direct f32 kernels (fixed-order sum)");
  m.def(
      "conv0_wgrad_bn",
      [](torch::Tensor x, torch::Tensor y, torch::Tensor G, torch::Tensor scale, torch::Tensor shift,
         torch::Tensor mean, torch::Tensor invstd, torch::Tensor coef) {
        TORCH_CHECK(x.dim() == 4 && x.size(1) == 32 && x.size(2) == 32 && x.size(3) == 4, "conv0_wgrad_bn: x [B,32,32,4]");
        const int64_t B = x.size(0), pix = B * 1024;
        check_t(x, x.numel(), "x");
        check_t(y, pix * 64, "y");
        check_t(G, pix / 4 * 64, "G");
        for (auto* t : {&scale, &shift, &mean, &invstd}) check_t(*t, 64, "bn vec");
        check_t(coef, 64 * 3, "coef");
        DevGuard g(x.device());
        auto part = torch::empty({(int64_t)cs_conv0_wgrad_part_floats((int)B, 32, 32)}, x.options());
        auto dw = torch::empty({64, 3, 3, 3}, x.options());
        CS_LAUNCH(cs_conv0_wgrad_bn(x.data_ptr<float>(), y.data_ptr<float>(), G.data_ptr<float>(),
                                    scale.data_ptr<float>(), shift.data_ptr<float>(), mean.data_ptr<float>(),
                                    invstd.data_ptr<float>(), coef.data_ptr<float>(), part.data_ptr<float>(),
                                    dw.data_ptr<float>(), (int)B, 32, 32, 64, cur_stream()));
        return dw;
      },
      "VGG block 0's weight gradient with its BN (+ReLU, 2x2 max-pool) backward apply folded in");
  m.def("bn_finalize", &bn_finalize);
  m.def("bn_eval_coeffs", &bn_eval_coeffs);
  m.def("bn_apply", &bn_apply);
  m.def("bn_bwd_blocks", &bn_bwd_blocks);
  m.def("bn_bwd", &bn_bwd);
}
