// torch bindings for the gfx950 kernels (module name: cs744_pytorch_distributed_tutorial_amd._C).
// Every op checks device/dtype/shape on the host BEFORE launching, so a bad call
// fails loudly in Python instead of faulting the GPU.
#include "binding/torch_util.h"
#include "kernels/launchers.h"

namespace {

using csb::cur_stream;
using csb::DevGuard;

const float kMean[3] = {125.3f / 255.f, 123.0f / 255.f, 113.9f / 255.f};
const float kStd[3] = {63.0f / 255.f, 62.1f / 255.f, 66.7f / 255.f};

torch::Tensor augment(torch::Tensor data, torch::Tensor idx, torch::Tensor params, bool nhwc, int64_t cstride) {
  CS_CHECK_CUDA(data); CS_CHECK_CUDA(idx); CS_CHECK_CUDA(params);
  TORCH_CHECK(data.scalar_type() == at::kByte && data.dim() == 4 && data.size(1) == 32 && data.size(2) == 32 &&
              data.size(3) == 3, "data must be uint8 [N,32,32,3]");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.dim() == 1, "idx must be int64 [B]");
  TORCH_CHECK(params.scalar_type() == at::kInt && params.dim() == 2 && params.size(1) == 3 &&
              params.size(0) == data.size(0), "params must be int32 [N,3]");
  CS_CHECK_CONTIG(data); CS_CHECK_CONTIG(idx); CS_CHECK_CONTIG(params);
  TORCH_CHECK(cstride == 3 || cstride == 4, "cstride must be 3 or 4");
  const int64_t B = idx.size(0);
  // bounds check of the gather indices on the host side of the call (cheap: B values)
  if (B > 0) {
    auto mm = at::aminmax(idx);
    TORCH_CHECK(std::get<0>(mm).item<int64_t>() >= 0 && std::get<1>(mm).item<int64_t>() < data.size(0),
                "augment: index out of range");
  }
  DevGuard g(data.device());
  auto out = nhwc ? torch::empty({B, 32, 32, cstride}, data.options().dtype(at::kFloat))
                  : torch::empty({B, 3, 32, 32}, data.options().dtype(at::kFloat));
  CS_LAUNCH(cs_augment(data.data_ptr<uint8_t>(), idx.data_ptr<int64_t>(), params.data_ptr<int32_t>(),
                       out.data_ptr<float>(), (int)B, nhwc ? 1 : 0, (int)cstride, kMean, kStd, cur_stream()));
  return out;
}

void sgd_flat(torch::Tensor p, torch::Tensor g, torch::Tensor m, double lr, double mom, double wd, double damp,
              double scale, bool first) {
  for (auto* t : {&p, &g, &m}) { CS_CHECK_CUDA(*t); CS_CHECK_F32(*t); CS_CHECK_CONTIG(*t); }
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel(), "sgd_flat: size mismatch");
  DevGuard gd(p.device());
  CS_LAUNCH(cs_sgd_flat(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), p.numel(), (float)lr,
                        (float)mom, (float)wd, (float)damp, (float)scale, first ? 1 : 0, cur_stream()));
}

// Builds the device table {p,g,m,n} + chunk prefix once per distinct pointer set; returns it
// as an int64 tensor the caller caches. Layout: [ntens*4 entries | ntens chunk starts | nchunks].
// shadows (optional): per parameter a bf16 tensor of the same layout that the update rewrites
// with the new value, or an empty tensor for none
torch::Tensor sgd_multi_table(std::vector<torch::Tensor> ps, std::vector<torch::Tensor> gs,
                              std::vector<torch::Tensor> ms, c10::optional<std::vector<torch::Tensor>> shadows) {
  TORCH_CHECK(ps.size() == gs.size() && ps.size() == ms.size() && !ps.empty(), "sgd_multi_table: list sizes");
  TORCH_CHECK(!shadows.has_value() || shadows->size() == ps.size(), "sgd_multi_table: shadow list size");
  const int64_t nt = ps.size();
  auto host = torch::empty({nt * 5 + nt + 1}, torch::kLong);
  int64_t* h = host.data_ptr<int64_t>();
  int64_t chunks = 0;
  for (int64_t i = 0; i < nt; ++i) {
    // the update is elementwise: any dense layout works as long as p, g and m share it
    // (channels_last conv weights of the CNN models are dense but not "contiguous")
    for (auto* t : {&ps[i], &gs[i], &ms[i]}) {
      CS_CHECK_CUDA(*t); CS_CHECK_F32(*t);
      TORCH_CHECK(t->is_non_overlapping_and_dense(), "sgd_multi_table: tensors must be dense");
    }
    TORCH_CHECK(ps[i].strides() == gs[i].strides() && ps[i].strides() == ms[i].strides(),
                "sgd_multi_table: param, grad and momentum must share one memory layout");
    TORCH_CHECK(ps[i].numel() == gs[i].numel() && ps[i].numel() == ms[i].numel(), "sgd_multi_table: numel");
    int64_t sh = 0;
    if (shadows.has_value() && (*shadows)[i].numel() > 0) {
      const auto& t = (*shadows)[i];
      CS_CHECK_CUDA(t);
      TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.numel() == ps[i].numel() && t.strides() == ps[i].strides(),
                  "sgd_multi_table: a shadow must be a bf16 tensor laid out like its parameter");
      sh = (int64_t)t.data_ptr();
    }
    h[i * 5 + 0] = (int64_t)ps[i].data_ptr<float>();
    h[i * 5 + 1] = (int64_t)gs[i].data_ptr<float>();
    h[i * 5 + 2] = (int64_t)ms[i].data_ptr<float>();
    h[i * 5 + 3] = ps[i].numel();
    h[i * 5 + 4] = sh;
    h[nt * 5 + i] = chunks;
    chunks += (ps[i].numel() + 4095) / 4096;
  }
  h[nt * 6] = chunks;
  return host.to(ps[0].device());
}

void sgd_multi(torch::Tensor table, int64_t ntens, int64_t nchunks, double lr, double mom, double wd, double damp,
               double scale, bool first) {
  CS_CHECK_CUDA(table);
  TORCH_CHECK(table.scalar_type() == at::kLong && table.numel() == ntens * 6 + 1, "sgd_multi: bad table");
  static_assert(sizeof(CsTensorEntry) == 5 * sizeof(int64_t), "CsTensorEntry: five 8-byte fields");
  DevGuard gd(table.device());
  const int64_t* t = table.data_ptr<int64_t>();
  CS_LAUNCH(cs_sgd_multi(reinterpret_cast<const CsTensorEntry*>(t), (int)ntens, t + ntens * 5, (int)nchunks,
                         (float)lr, (float)mom, (float)wd, (float)damp, (float)scale, first ? 1 : 0, cur_stream()));
}

// part2a root combine: dst[n] = mean over rows of src[rows * n] (rank order)
// (bcast: the mean is also written over every row of src)
void rows_mean(torch::Tensor src, int64_t rows, torch::Tensor dst, bool bcast) {
  for (auto* t : {&src, &dst}) { CS_CHECK_CUDA(*t); CS_CHECK_F32(*t); CS_CHECK_CONTIG(*t); }
  TORCH_CHECK(rows >= 1 && src.numel() == rows * dst.numel(), "rows_mean: src must hold rows * dst.numel()");
  DevGuard gd(dst.device());
  CS_LAUNCH(cs_rows_mean(src.data_ptr<float>(), (int)rows, dst.numel(), dst.data_ptr<float>(), bcast ? 1 : 0,
                         cur_stream()));
}

// part2a_extra root combine: g += t (then g /= div when div > 0)
void cast_grad(torch::Tensor src, torch::Tensor dst) {
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.is_contiguous() && dst.is_contiguous() &&
                  src.numel() == dst.numel(),
              "cast_grad: contiguous GPU tensors of equal size");
  const bool to_bf16 = src.scalar_type() == at::kFloat && dst.scalar_type() == at::kBFloat16;
  TORCH_CHECK(to_bf16 || (src.scalar_type() == at::kBFloat16 && dst.scalar_type() == at::kFloat),
              "cast_grad: float32 -> bfloat16 or bfloat16 -> float32");
  DevGuard g(src.device());
  CS_LAUNCH(cs_cast_grad(src.data_ptr(), dst.data_ptr(), src.numel(), to_bf16 ? 1 : 0, cur_stream()));
}

void accumulate(torch::Tensor g, torch::Tensor t, double div) {
  for (auto* x : {&g, &t}) { CS_CHECK_CUDA(*x); CS_CHECK_F32(*x); CS_CHECK_CONTIG(*x); }
  TORCH_CHECK(g.numel() == t.numel(), "accumulate: size mismatch");
  DevGuard gd(g.device());
  CS_LAUNCH(cs_accumulate(g.data_ptr<float>(), t.data_ptr<float>(), g.numel(), (float)div, cur_stream()));
}

std::vector<torch::Tensor> linear_xent(torch::Tensor feat, torch::Tensor W, torch::Tensor bias, torch::Tensor labels,
                                       double gscale, bool backward) {
  for (auto* t : {&feat, &W, &bias}) { CS_CHECK_CUDA(*t); CS_CHECK_F32(*t); CS_CHECK_CONTIG(*t); }
  CS_CHECK_CUDA(labels);
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.dim() == 1, "labels int64 [B]");
  TORCH_CHECK(feat.dim() == 2 && W.dim() == 2 && bias.dim() == 1 && feat.size(1) == W.size(1) &&
              W.size(0) == bias.size(0) && labels.size(0) == feat.size(0), "linear_xent: shapes");
  const int B = feat.size(0), K = feat.size(1), C = W.size(0);
  TORCH_CHECK(C <= 16 && K % 4 == 0, "linear_xent: C <= 16 and K % 4 == 0");
  DevGuard gd(feat.device());
  auto loss = torch::empty({}, feat.options());
  auto correct = torch::empty({}, feat.options().dtype(at::kInt));
  auto logits = torch::empty({B, C}, feat.options());
  auto pred = torch::empty({B}, feat.options().dtype(at::kLong));
  auto ws = torch::empty({cs_linear_xent_ws(B, C)}, feat.options());
  torch::Tensor dW, db, dfeat;
  if (backward) {
    dW = torch::empty_like(W);
    db = torch::empty_like(bias);
    dfeat = torch::empty_like(feat);
  }
  CS_LAUNCH(cs_linear_xent(feat.data_ptr<float>(), W.data_ptr<float>(), bias.data_ptr<float>(),
                           labels.data_ptr<int64_t>(), B, K, C, (float)gscale, loss.data_ptr<float>(),
                           correct.data_ptr<int>(), logits.data_ptr<float>(),
                           backward ? dW.data_ptr<float>() : nullptr, backward ? db.data_ptr<float>() : nullptr,
                           backward ? dfeat.data_ptr<float>() : nullptr, pred.data_ptr<int64_t>(),
                           ws.data_ptr<float>(), cur_stream()));
  if (backward) return {loss, correct, logits, dW, db, dfeat, pred};
  return {loss, correct, logits, pred};
}

std::vector<torch::Tensor> softmax_xent(torch::Tensor logits, torch::Tensor labels, double gscale) {
  CS_CHECK_CUDA(logits); CS_CHECK_F32(logits); CS_CHECK_CONTIG(logits); CS_CHECK_CUDA(labels);
  TORCH_CHECK(logits.dim() == 2 && labels.dim() == 1 && labels.size(0) == logits.size(0) &&
              labels.scalar_type() == at::kLong, "softmax_xent: shapes");
  TORCH_CHECK(logits.size(1) <= 16, "softmax_xent: C <= 16");
  DevGuard gd(logits.device());
  auto loss = torch::empty({}, logits.options());
  auto dl = torch::empty_like(logits);
  auto correct = torch::empty({}, logits.options().dtype(at::kInt));
  CS_LAUNCH(cs_softmax_xent(logits.data_ptr<float>(), labels.data_ptr<int64_t>(), logits.size(0), logits.size(1),
                            (float)gscale, loss.data_ptr<float>(), dl.data_ptr<float>(), correct.data_ptr<int>(),
                            cur_stream()));
  return {loss, dl, correct};
}

}  // namespace

void register_conv_ops(pybind11::module& m);
void register_runtime(pybind11::module& m);
void register_lm_ops(pybind11::module& m);
void register_cnn_ops(pybind11::module& m);
void register_nhwc_ops(pybind11::module& m);

PYBIND11_MODULE(_C, m) {
  m.doc() = "gfx950 (MI355X) kernels + native runtime for cs744_pytorch_distributed_tutorial_amd";
  m.def("augment", &augment, "fused CIFAR gather+crop+flip+normalize");
  m.def("sgd_flat", &sgd_flat, "fused SGD on flat buffers");
  m.def("sgd_multi_table", &sgd_multi_table, "build the multi-tensor SGD table", pybind11::arg("ps"), pybind11::arg("gs"),
        pybind11::arg("ms"), pybind11::arg("shadows") = pybind11::none());
  m.def("sgd_multi", &sgd_multi, "multi-tensor fused SGD");
  m.def("rows_mean", &rows_mean, "mean over the rows of a [rows, n] buffer (part2a root)", pybind11::arg("src"),
        pybind11::arg("rows"), pybind11::arg("dst"), pybind11::arg("bcast") = false);
  m.def("accumulate", &accumulate, "g += t, optionally then g /= div (part2a_extra root)");
  m.def("cast_grad", &cast_grad, "gradient bucket fp32 <-> bf16 (bf16 gradient transport of the DDP)");
  m.def("linear_xent", &linear_xent, "fused Linear + softmax cross-entropy fwd(+bwd)");
  m.def("softmax_xent", &softmax_xent, "softmax cross-entropy fwd+bwd");
  register_conv_ops(m);
  register_runtime(m);
  register_lm_ops(m);
  register_cnn_ops(m);
  register_nhwc_ops(m);
}
