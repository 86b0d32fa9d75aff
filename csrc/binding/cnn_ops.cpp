// torch bindings of the CNN-extension kernels (csrc/kernels/bn_nchw.hip): fused training
// BatchNorm2d (+ residual add, + ReLU) on NCHW activations; shapes/dtypes validated on the host.
#include "binding/torch_util.h"
#include "kernels/launchers.h"

namespace {

using csb::cur_stream;
using csb::DevGuard;

int act_dt(const torch::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return CS_F32;
  if (t.scalar_type() == at::kBFloat16) return CS_BF16;
  TORCH_CHECK(false, "bn_act: activations must be float32 or bfloat16, got ", t.scalar_type());
  return -1;
}

void check_act(const torch::Tensor& t, const torch::Tensor& like, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.sizes() == like.sizes() && t.scalar_type() == like.scalar_type(),
              n, " must be a contiguous NCHW GPU tensor shaped and typed like x");
}

void check_param(const torch::Tensor& t, int64_t C, const char* n) {
  if (!t.defined()) return;
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kFloat && t.numel() == C, n,
              " must be a contiguous float32 GPU tensor of C elements");
}

template <typename T>
T* opt_ptr(const c10::optional<torch::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<T>() : nullptr;
}

// -> {y, stat [4, C]}
std::vector<torch::Tensor> bn_act_fwd(torch::Tensor x, c10::optional<torch::Tensor> res, c10::optional<torch::Tensor> w,
                                      c10::optional<torch::Tensor> b, c10::optional<torch::Tensor> rm,
                                      c10::optional<torch::Tensor> rv, c10::optional<torch::Tensor> nbt, double momentum,
                                      double eps, bool relu) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4, "bn_act: x must be a contiguous NCHW GPU tensor");
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  if (res.has_value() && res->defined()) check_act(*res, x, "res");
  for (auto* t : {&w, &b, &rm, &rv})
    if (t->has_value()) check_param(**t, C, "bn parameter");
  TORCH_CHECK(rm.has_value() == rv.has_value(), "bn_act: running mean and var go together");
  if (nbt.has_value())
    TORCH_CHECK(nbt->is_cuda() && nbt->scalar_type() == at::kLong && nbt->numel() == 1, "bn_act: num_batches_tracked");
  TORCH_CHECK(N * HW > 0, "bn_act: empty batch");
  DevGuard g(x.device());
  auto fo = x.options().dtype(at::kFloat);
  auto y = torch::empty_like(x);
  auto stat = torch::empty({4, C}, fo);
  auto part = torch::empty({cs_bn_nchw_partials((int)N, (int)C)}, fo);
  CS_LAUNCH(cs_bn_nchw_fwd(act_dt(x), x.data_ptr(), res.has_value() && res->defined() ? res->data_ptr() : nullptr,
                           opt_ptr<float>(w), opt_ptr<float>(b), opt_ptr<float>(rm), opt_ptr<float>(rv),
                           opt_ptr<int64_t>(nbt), (float)momentum, (float)eps, relu ? 1 : 0, y.data_ptr(), stat.data_ptr<float>(),
                           part.data_ptr<float>(), (int)N, (int)C, (int)HW, cur_stream()));
  return {y, stat};
}

// -> {dx, dres (or undefined), dw, db}
std::vector<torch::Tensor> bn_act_bwd(torch::Tensor dy, torch::Tensor x, c10::optional<torch::Tensor> res,
                                      c10::optional<torch::Tensor> w, torch::Tensor stat, bool relu, bool need_dres) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4, "bn_act_bwd: x must be a contiguous NCHW GPU tensor");
  check_act(dy, x, "dy");
  const bool has_res = res.has_value() && res->defined();
  if (has_res) check_act(*res, x, "res");
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  if (w.has_value()) check_param(*w, C, "weight");
  TORCH_CHECK(stat.is_cuda() && stat.scalar_type() == at::kFloat && stat.numel() == 4 * C, "bn_act_bwd: stat");
  DevGuard g(x.device());
  auto fo = x.options().dtype(at::kFloat);
  auto dx = torch::empty_like(x);
  torch::Tensor dres = need_dres ? torch::empty_like(x) : torch::Tensor();
  auto dw = torch::empty({C}, fo), db = torch::empty({C}, fo);
  auto coef = torch::empty({3, C}, fo);
  auto part = torch::empty({cs_bn_nchw_partials((int)N, (int)C)}, fo);
  CS_LAUNCH(cs_bn_nchw_bwd(act_dt(x), dy.data_ptr(), x.data_ptr(), has_res ? res->data_ptr() : nullptr,
                           opt_ptr<float>(w), stat.data_ptr<float>(), relu ? 1 : 0, dx.data_ptr(),
                           need_dres ? dres.data_ptr() : nullptr, dw.data_ptr<float>(), db.data_ptr<float>(),
                           coef.data_ptr<float>(), part.data_ptr<float>(), (int)N, (int)C, (int)HW, cur_stream()));
  return {dx, dres, dw, db};
}

// 3x3/2 max-pool, padding 1: -> {y, pos (uint8 window position)}
std::vector<torch::Tensor> maxpool3s2_fwd(torch::Tensor x) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4, "maxpool3s2: x must be a contiguous NCHW GPU tensor");
  const int64_t H = x.size(2), W = x.size(3), Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  DevGuard g(x.device());
  auto y = torch::empty({x.size(0), x.size(1), Ho, Wo}, x.options());
  auto pos = torch::empty({x.size(0), x.size(1), Ho, Wo}, x.options().dtype(at::kByte));
  CS_LAUNCH(cs_maxpool3s2_fwd(act_dt(x), x.data_ptr(), y.data_ptr(), pos.data_ptr<uint8_t>(), x.size(0) * x.size(1),
                              (int)H, (int)W, (int)Ho, (int)Wo, cur_stream()));
  return {y, pos};
}

torch::Tensor maxpool3s2_bwd(torch::Tensor dy, torch::Tensor pos, int64_t H, int64_t W) {
  TORCH_CHECK(dy.is_cuda() && dy.is_contiguous() && dy.dim() == 4 && pos.sizes() == dy.sizes() &&
                  pos.scalar_type() == at::kByte && pos.is_contiguous(), "maxpool3s2_bwd: dy / pos");
  TORCH_CHECK(dy.size(2) == (H - 1) / 2 + 1 && dy.size(3) == (W - 1) / 2 + 1, "maxpool3s2_bwd: input size");
  DevGuard g(dy.device());
  auto dx = torch::empty({dy.size(0), dy.size(1), H, W}, dy.options());
  CS_LAUNCH(cs_maxpool3s2_bwd(act_dt(dy), dy.data_ptr(), pos.data_ptr<uint8_t>(), dx.data_ptr(), dy.size(0) * dy.size(1),
                              (int)H, (int)W, (int)dy.size(2), (int)dy.size(3), cur_stream()));
  return dx;
}

}  // namespace

void register_cnn_ops(pybind11::module& m) {
  m.def("bn_act_fwd", &bn_act_fwd, "fused training BatchNorm2d (+residual) (+ReLU), NCHW fp32/bf16 -> (y, stat)");
  m.def("bn_act_bwd", &bn_act_bwd, "its backward -> (dx, dres, dweight, dbias)");
  m.def("maxpool3s2_fwd", &maxpool3s2_fwd, "3x3/2 pad-1 max-pool, NCHW -> (y, window position)");
  m.def("maxpool3s2_bwd", &maxpool3s2_bwd, "its gather-style backward");
}
