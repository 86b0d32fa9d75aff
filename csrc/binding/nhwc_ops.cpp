// torch bindings of the channels-last CNN kernels (csrc/kernels/cnn_nhwc.hip). Activations are
// contiguous [B, H, W, C] fp32 / bf16 GPU tensors; shapes, dtypes and the vector-width
// preconditions are validated here, before any launch.
#include "binding/torch_util.h"
#include "kernels/launchers.h"

namespace {

using csb::cur_stream;
using csb::DevGuard;

int act_dt(const torch::Tensor& t, const char* who) {
  if (t.scalar_type() == at::kFloat) return CS_F32;
  if (t.scalar_type() == at::kBFloat16) return CS_BF16;
  TORCH_CHECK(false, who, ": activations must be float32 or bfloat16, got ", t.scalar_type());
  return -1;
}

void check_nhwc(const torch::Tensor& t, const char* who) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.dim() == 4, who, ": expected a contiguous [B, H, W, C] GPU tensor");
}

void check_like(const torch::Tensor& t, const torch::Tensor& like, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.sizes() == like.sizes() && t.scalar_type() == like.scalar_type(),
              n, " must be a contiguous [B, H, W, C] GPU tensor shaped and typed like x");
}

void check_param(const c10::optional<torch::Tensor>& t, int64_t C, const char* n) {
  if (!t.has_value() || !t->defined()) return;
  TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == at::kFloat && t->numel() == C, n,
              " must be a contiguous float32 GPU tensor of C elements");
}

template <typename T>
T* opt_ptr(const c10::optional<torch::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<T>() : nullptr;
}

// bf16 NHWC implicit-GEMM convolution (conv_nhwc.hip). mode 0: a = x [B,H,W,C], b = w
// [Co,R,S,C] -> y [B,Ho,Wo,Co]; mode 1: a = dy [B,Ho,Wo,Co], b = wt [C,R,S,Co] -> dx [B,H,W,C]
// (H, W given); mode 2: a = dy, b = x -> fp32 dW [Co, R*S*C]
torch::Tensor conv_nhwc_bf16(int64_t mode, torch::Tensor a, torch::Tensor b, int64_t R, int64_t S, int64_t stride,
                             int64_t pad, int64_t H, int64_t W) {
  TORCH_CHECK(mode >= 0 && mode <= 2, "conv_nhwc_bf16: mode 0 fwd, 1 dgrad, 2 wgrad");
  for (const auto* t : {&a, &b})
    TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == at::kBFloat16 && t->dim() == 4,
                "conv_nhwc_bf16: operands must be contiguous 4-D bfloat16 GPU tensors");
  TORCH_CHECK(R >= 1 && S >= 1 && stride >= 1 && pad >= 0, "conv_nhwc_bf16: geometry");
  CsConvNhwcArgs p{};
  p.R = (int)R;
  p.S = (int)S;
  p.st = (int)stride;
  p.pad = (int)pad;
  DevGuard g(a.device());
  torch::Tensor out, ws;
  if (mode == 0) {
    p.B = (int)a.size(0), p.H = (int)a.size(1), p.W = (int)a.size(2), p.C = (int)a.size(3), p.Co = (int)b.size(0);
    // the 4-channel stem: kernel rows padded to 8 taps, weight [Co, R, 8, 4]
    TORCH_CHECK(b.size(1) == R && b.size(2) == (p.C == 4 ? 8 : S) && b.size(3) == p.C,
                "conv_nhwc_bf16: weight [Co, R, S, C] ([Co, R, 8, 4] for a 4-channel input)");
    const int64_t Ho = (p.H + 2 * pad - R) / stride + 1, Wo = (p.W + 2 * pad - S) / stride + 1;
    out = torch::empty({p.B, Ho, Wo, p.Co}, a.options());
    p.x = a.data_ptr();
    p.w = b.data_ptr();
    p.y = out.data_ptr();
  } else if (mode == 1) {
    p.B = (int)a.size(0), p.H = (int)H, p.W = (int)W, p.Co = (int)a.size(3), p.C = (int)b.size(0);
    TORCH_CHECK(b.size(1) == R && b.size(2) == S && b.size(3) == p.Co, "conv_nhwc_bf16: transposed weight [C, R, S, Co]");
    TORCH_CHECK(a.size(1) == (H + 2 * pad - R) / stride + 1 && a.size(2) == (W + 2 * pad - S) / stride + 1,
                "conv_nhwc_bf16: dy spatial size does not match H, W");
    out = torch::empty({p.B, H, W, p.C}, a.options());
    p.dy = a.data_ptr();
    p.w = b.data_ptr();
    p.y = out.data_ptr();
  } else {
    p.B = (int)b.size(0), p.H = (int)b.size(1), p.W = (int)b.size(2), p.C = (int)b.size(3), p.Co = (int)a.size(3);
    TORCH_CHECK(a.size(0) == p.B && a.size(1) == (p.H + 2 * pad - R) / stride + 1 &&
                    a.size(2) == (p.W + 2 * pad - S) / stride + 1,
                "conv_nhwc_bf16: dy / x shapes");
    const int sp = cs_conv_nhwc_splits(2, p.B, p.H, p.W, p.C, p.Co, p.R, p.S, p.st, p.pad);
    const int64_t kc = p.C == 4 ? R * 32 : R * S * p.C;  // (r, s < 8, c < 4) columns for the stem
    ws = torch::empty({(int64_t)sp * p.Co * kc}, a.options().dtype(at::kFloat));
    out = torch::empty({p.Co, kc}, a.options().dtype(at::kFloat));
    p.dy = a.data_ptr();
    p.x = b.data_ptr();
    p.dw = ws.data_ptr<float>();
    p.dw_out = out.data_ptr<float>();
    CS_LAUNCH(cs_conv_nhwc(2, p, sp, cur_stream()));
    return out;
  }
  CS_LAUNCH(cs_conv_nhwc((int)mode, p, 1, cur_stream()));
  return out;
}

// [S, ...] fp32 partials -> their sum over dim 0 (fixed order: deterministic)
torch::Tensor slab_sum(torch::Tensor part) {
  TORCH_CHECK(part.is_cuda() && part.is_contiguous() && part.scalar_type() == at::kFloat && part.dim() >= 2,
              "slab_sum: contiguous fp32 [S, ...] GPU tensor");
  const int64_t S = part.size(0), n = part.numel() / std::max<int64_t>(S, 1);
  TORCH_CHECK(S >= 1 && n % 4 == 0, "slab_sum: the slab size must be a multiple of 4");
  DevGuard g(part.device());
  auto out = torch::empty(part.sizes().slice(1), part.options());
  CS_LAUNCH(cs_slab_sum(part.data_ptr<float>(), (int)S, n, out.data_ptr<float>(), cur_stream()));
  return out;
}

// -> {y, stat [4, C] = scale, shift, mean, invstd, ReLU mask (with_mask; else undefined)}
std::vector<torch::Tensor> bn_nhwc_fwd(torch::Tensor x, c10::optional<torch::Tensor> res,
                                       c10::optional<torch::Tensor> w, c10::optional<torch::Tensor> b,
                                       c10::optional<torch::Tensor> rm, c10::optional<torch::Tensor> rv,
                                       c10::optional<torch::Tensor> nbt, double momentum, double eps, bool relu,
                                       bool with_mask, c10::optional<torch::Tensor> tiles, int64_t tile_rows) {
  check_nhwc(x, "bn_nhwc_fwd");
  const int dt = act_dt(x, "bn_nhwc_fwd");
  const int64_t C = x.size(3), M = x.numel() / C;
  TORCH_CHECK(M > 0 && C > 0, "bn_nhwc_fwd: empty input");
  const bool has_res = res.has_value() && res->defined();
  if (has_res) check_like(*res, x, "res");
  check_param(w, C, "weight");
  check_param(b, C, "bias");
  check_param(rm, C, "running_mean");
  check_param(rv, C, "running_var");
  TORCH_CHECK(rm.has_value() == rv.has_value(), "bn_nhwc_fwd: running mean and var go together");
  if (nbt.has_value())
    TORCH_CHECK(nbt->is_cuda() && nbt->scalar_type() == at::kLong && nbt->numel() == 1, "bn_nhwc_fwd: num_batches_tracked");
  DevGuard g(x.device());
  auto fo = x.options().dtype(at::kFloat);
  auto y = torch::empty_like(x);
  auto stat = torch::empty({4, C}, fo);
  torch::Tensor mask;
  if (with_mask) mask = torch::empty({M * C / cs_bn_nhwc_vec((int)C, dt)}, x.options().dtype(at::kByte));
  if (tiles.has_value() && tiles->defined()) {
    // statistics already computed per row tile by the producing GEMM (mm_bf16_bn_stats)
    TORCH_CHECK(tiles->is_cuda() && tiles->scalar_type() == at::kFloat && tiles->is_contiguous() && tiles->dim() == 3 &&
                    tiles->size(1) == C && tiles->size(2) == 2 && tile_rows > 0 &&
                    tiles->size(0) == (M + tile_rows - 1) / tile_rows,
                "bn_nhwc_fwd: tiles must be fp32 [ceil(M / tile_rows), C, 2] (mean, M2) partials of x");
    CS_LAUNCH(cs_bn_nhwc_fwd_tiles(dt, x.data_ptr(), has_res ? res->data_ptr() : nullptr, opt_ptr<float>(w),
                                   opt_ptr<float>(b), opt_ptr<float>(rm), opt_ptr<float>(rv), opt_ptr<int64_t>(nbt),
                                   (float)momentum, (float)eps, relu ? 1 : 0, y.data_ptr(), stat.data_ptr<float>(),
                                   tiles->data_ptr<float>(), (int)tiles->size(0), (int)tile_rows, M, (int)C,
                                   cur_stream(), with_mask ? mask.data_ptr<uint8_t>() : nullptr));
    return {y, stat, mask};
  }
  auto part = torch::empty({cs_bn_nhwc_partials(M, (int)C, dt)}, fo);
  CS_LAUNCH(cs_bn_nhwc_fwd(dt, x.data_ptr(), has_res ? res->data_ptr() : nullptr, opt_ptr<float>(w), opt_ptr<float>(b),
                           opt_ptr<float>(rm), opt_ptr<float>(rv), opt_ptr<int64_t>(nbt), (float)momentum, (float)eps,
                           relu ? 1 : 0, y.data_ptr(), stat.data_ptr<float>(), part.data_ptr<float>(), M, (int)C,
                           cur_stream(), with_mask ? mask.data_ptr<uint8_t>() : nullptr));
  return {y, stat, mask};
}

// -> {dx, dres (or undefined), dweight, dbias}
std::vector<torch::Tensor> bn_nhwc_bwd(torch::Tensor dy, torch::Tensor x, c10::optional<torch::Tensor> res,
                                       c10::optional<torch::Tensor> w, torch::Tensor stat, bool relu, bool need_dres,
                                       c10::optional<torch::Tensor> mask) {
  check_nhwc(x, "bn_nhwc_bwd");
  const int dt = act_dt(x, "bn_nhwc_bwd");
  check_like(dy, x, "dy");
  const bool has_res = res.has_value() && res->defined();
  if (has_res) check_like(*res, x, "res");
  const int64_t C = x.size(3), M = x.numel() / C;
  check_param(w, C, "weight");
  TORCH_CHECK(stat.is_cuda() && stat.scalar_type() == at::kFloat && stat.numel() == 4 * C, "bn_nhwc_bwd: stat");
  const bool has_mask = mask.has_value() && mask->defined();
  if (has_mask)
    TORCH_CHECK(relu && mask->is_cuda() && mask->scalar_type() == at::kByte &&
                    mask->numel() == M * C / cs_bn_nhwc_vec((int)C, dt),
                "bn_nhwc_bwd: mask from bn_nhwc_fwd(with_mask=True) of this activation");
  DevGuard g(x.device());
  auto fo = x.options().dtype(at::kFloat);
  auto dx = torch::empty_like(x);
  torch::Tensor dres = need_dres ? torch::empty_like(x) : torch::Tensor();
  auto dw = torch::empty({C}, fo), db = torch::empty({C}, fo);
  auto coef = torch::empty({3, C}, fo);
  auto part = torch::empty({cs_bn_nhwc_partials(M, (int)C, dt)}, fo);
  CS_LAUNCH(cs_bn_nhwc_bwd(dt, dy.data_ptr(), x.data_ptr(), has_res ? res->data_ptr() : nullptr, opt_ptr<float>(w),
                           stat.data_ptr<float>(), relu ? 1 : 0, dx.data_ptr(), need_dres ? dres.data_ptr() : nullptr,
                           dw.data_ptr<float>(), db.data_ptr<float>(), coef.data_ptr<float>(), part.data_ptr<float>(),
                           M, (int)C, cur_stream(), has_mask ? mask->data_ptr<uint8_t>() : nullptr));
  return {dx, dres, dw, db};
}

// training BatchNorm2d + ReLU + 3x3/2 pad-1 max-pool (the ResNet stem) -> {y (pooled), pos, stat}:
// statistics as bn_nhwc_fwd, then the pool applies BN + ReLU to its window loads (no full-size output)
std::vector<torch::Tensor> bn_relu_maxpool_nhwc_fwd(torch::Tensor x, c10::optional<torch::Tensor> w,
                                                    c10::optional<torch::Tensor> b, c10::optional<torch::Tensor> rm,
                                                    c10::optional<torch::Tensor> rv, c10::optional<torch::Tensor> nbt,
                                                    double momentum, double eps) {
  check_nhwc(x, "bn_relu_maxpool_nhwc_fwd");
  const int dt = act_dt(x, "bn_relu_maxpool_nhwc_fwd");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), M = x.numel() / C;
  TORCH_CHECK(M > 0 && C > 0, "bn_relu_maxpool_nhwc_fwd: empty input");
  check_param(w, C, "weight");
  check_param(b, C, "bias");
  check_param(rm, C, "running_mean");
  check_param(rv, C, "running_var");
  TORCH_CHECK(rm.has_value() == rv.has_value(), "bn_relu_maxpool_nhwc_fwd: running mean and var go together");
  if (nbt.has_value())
    TORCH_CHECK(nbt->is_cuda() && nbt->scalar_type() == at::kLong && nbt->numel() == 1,
                "bn_relu_maxpool_nhwc_fwd: num_batches_tracked");
  DevGuard g(x.device());
  auto fo = x.options().dtype(at::kFloat);
  auto stat = torch::empty({4, C}, fo);
  auto part = torch::empty({cs_bn_nhwc_partials(M, (int)C, dt)}, fo);
  CS_LAUNCH(cs_bn_nhwc_fwd(dt, x.data_ptr(), nullptr, opt_ptr<float>(w), opt_ptr<float>(b), opt_ptr<float>(rm),
                           opt_ptr<float>(rv), opt_ptr<int64_t>(nbt), (float)momentum, (float)eps, 1, nullptr,
                           stat.data_ptr<float>(), part.data_ptr<float>(), M, (int)C, cur_stream()));
  const int64_t Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  auto y = torch::empty({B, Ho, Wo, C}, x.options());
  auto pos = torch::empty({B, Ho, Wo, C}, x.options().dtype(at::kByte));
  CS_LAUNCH(cs_maxpool3s2_nhwc_fwd(dt, x.data_ptr(), y.data_ptr(), pos.data_ptr<uint8_t>(), (int)B, (int)H, (int)W,
                                   (int)C, (int)Ho, (int)Wo, cur_stream(), stat.data_ptr<float>()));
  return {y, pos, stat};
}

// 3x3 / 2 pad-1 max-pool -> {y, pos (uint8 window position per output element)}
std::vector<torch::Tensor> maxpool3s2_nhwc_fwd(torch::Tensor x) {
  check_nhwc(x, "maxpool3s2_nhwc_fwd");
  const int dt = act_dt(x, "maxpool3s2_nhwc_fwd");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  DevGuard g(x.device());
  auto y = torch::empty({B, Ho, Wo, C}, x.options());
  auto pos = torch::empty({B, Ho, Wo, C}, x.options().dtype(at::kByte));
  CS_LAUNCH(cs_maxpool3s2_nhwc_fwd(dt, x.data_ptr(), y.data_ptr(), pos.data_ptr<uint8_t>(), (int)B, (int)H, (int)W,
                                   (int)C, (int)Ho, (int)Wo, cur_stream()));
  return {y, pos};
}

torch::Tensor maxpool3s2_nhwc_bwd(torch::Tensor dy, torch::Tensor pos, int64_t H, int64_t W) {
  check_nhwc(dy, "maxpool3s2_nhwc_bwd");
  const int dt = act_dt(dy, "maxpool3s2_nhwc_bwd");
  TORCH_CHECK(pos.sizes() == dy.sizes() && pos.scalar_type() == at::kByte && pos.is_contiguous(),
              "maxpool3s2_nhwc_bwd: pos must match dy");
  TORCH_CHECK(dy.size(1) == (H - 1) / 2 + 1 && dy.size(2) == (W - 1) / 2 + 1, "maxpool3s2_nhwc_bwd: input size");
  DevGuard g(dy.device());
  auto dx = torch::empty({dy.size(0), H, W, dy.size(3)}, dy.options());
  CS_LAUNCH(cs_maxpool3s2_nhwc_bwd(dt, dy.data_ptr(), pos.data_ptr<uint8_t>(), dx.data_ptr(), (int)dy.size(0), (int)H,
                                   (int)W, (int)dy.size(3), (int)dy.size(1), (int)dy.size(2), cur_stream()));
  return dx;
}

int vec_of(int64_t C, int dt) {
  const int v16 = dt == CS_BF16 ? 8 : 4;
  if (C % v16 == 0) return v16;
  return C % 4 == 0 ? 4 : 1;
}

// x [B, H, W, C] -> col [B*Ho*Wo, Kp] (Kp >= R*S*C, a multiple of the channel vector width)
torch::Tensor im2col_nhwc(torch::Tensor x, int64_t R, int64_t S, int64_t stride, int64_t pad, int64_t Kp) {
  check_nhwc(x, "im2col_nhwc");
  const int dt = act_dt(x, "im2col_nhwc");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(R > 0 && S > 0 && stride > 0 && pad >= 0 && Kp >= R * S * C && Kp % vec_of(C, dt) == 0,
              "im2col_nhwc: bad geometry");
  const int64_t Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "im2col_nhwc: empty output");
  DevGuard g(x.device());
  auto col = torch::empty({B * Ho * Wo, Kp}, x.options());
  CS_LAUNCH(cs_im2col_nhwc(dt, x.data_ptr(), col.data_ptr(), (int)B, (int)H, (int)W, (int)C, (int)R, (int)S,
                           (int)stride, (int)pad, (int)Ho, (int)Wo, (int)Kp, cur_stream()));
  return col;
}

// dcol [B*Ho*Wo, Kp] -> dx [B, H, W, C] (the adjoint of im2col_nhwc)
torch::Tensor col2im_nhwc(torch::Tensor dcol, int64_t B, int64_t H, int64_t W, int64_t C, int64_t R, int64_t S,
                          int64_t stride, int64_t pad) {
  TORCH_CHECK(dcol.is_cuda() && dcol.is_contiguous() && dcol.dim() == 2, "col2im_nhwc: dcol must be a contiguous 2-D GPU tensor");
  const int dt = act_dt(dcol, "col2im_nhwc");
  const int64_t Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1, Kp = dcol.size(1);
  TORCH_CHECK(R > 0 && S > 0 && stride > 0 && pad >= 0 && Ho > 0 && Wo > 0, "col2im_nhwc: bad geometry");
  TORCH_CHECK(dcol.size(0) == B * Ho * Wo && Kp >= R * S * C && Kp % vec_of(C, dt) == 0, "col2im_nhwc: dcol shape");
  DevGuard g(dcol.device());
  auto dx = torch::empty({B, H, W, C}, dcol.options());
  CS_LAUNCH(cs_col2im_nhwc(dt, dcol.data_ptr(), dx.data_ptr(), (int)B, (int)H, (int)W, (int)C, (int)R, (int)S,
                           (int)stride, (int)pad, (int)Ho, (int)Wo, (int)Kp, cur_stream()));
  return dx;
}

}  // namespace

void register_nhwc_ops(pybind11::module& m) {
  m.def("conv_nhwc_bf16", &conv_nhwc_bf16,
        "bf16 NHWC implicit-GEMM conv: mode 0 fwd (a=x, b=w[Co,R,S,C]) -> y; 1 dgrad (a=dy, b=wt[C,R,S,Co]) -> dx; "
        "2 wgrad (a=dy, b=x) -> fp32 dW [Co, R*S*C]; a 4-channel x (the stem, S <= 8) uses kernel rows padded "
        "to 8 taps: weight [Co, R, 8, 4], dW [Co, R*32]");
  m.def("slab_sum", &slab_sum, "sum of fp32 partial slabs over dim 0, deterministic");
  m.def("bn_nhwc_fwd", &bn_nhwc_fwd, "training BatchNorm2d (+residual) (+ReLU), NHWC fp32/bf16 -> (y, stat, mask)",
        pybind11::arg("x"), pybind11::arg("res"), pybind11::arg("w"), pybind11::arg("b"), pybind11::arg("rm"), pybind11::arg("rv"), pybind11::arg("nbt"),
        pybind11::arg("momentum"), pybind11::arg("eps"), pybind11::arg("relu"), pybind11::arg("with_mask") = false,
        pybind11::arg("tiles") = c10::nullopt, pybind11::arg("tile_rows") = 256);
  m.def("bn_nhwc_bwd", &bn_nhwc_bwd, "its backward -> (dx, dres, dweight, dbias); mask: the forward's ReLU mask",
        pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("res"), pybind11::arg("w"), pybind11::arg("stat"), pybind11::arg("relu"),
        pybind11::arg("need_dres"), pybind11::arg("mask") = pybind11::none());
  m.def("bn_relu_maxpool_nhwc_fwd", &bn_relu_maxpool_nhwc_fwd,
        "training BatchNorm2d + ReLU + 3x3/2 max-pool, NHWC, the apply fused into the pool -> (y, pos, stat)");
  m.def("maxpool3s2_nhwc_fwd", &maxpool3s2_nhwc_fwd, "3x3/2 pad-1 max-pool, NHWC -> (y, window position)");
  m.def("maxpool3s2_nhwc_bwd", &maxpool3s2_nhwc_bwd, "its gather-style backward");
  m.def("im2col_nhwc", &im2col_nhwc, "NHWC im2col -> [B*Ho*Wo, Kp], columns (r, s, c)");
  m.def("col2im_nhwc", &col2im_nhwc, "adjoint of im2col_nhwc (gather, deterministic)");
}
