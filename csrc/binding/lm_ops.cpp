// torch bindings of the decoder-LM kernels (csrc/kernels/lm.hip); shapes/dtypes validated on the host.
#include "binding/torch_util.h"
#include "kernels/launchers.h"

namespace {

using csb::cur_stream;
using csb::DevGuard;

int dt_of(const torch::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return CS_F32;
  if (t.scalar_type() == at::kBFloat16) return CS_BF16;
  TORCH_CHECK(false, "LM kernels support float32 / bfloat16, got ", t.scalar_type());
  return -1;
}

void check(const torch::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), n, " must be a contiguous GPU tensor");
}

// out_bf16: write y in bf16 whatever x's dtype (the fp32 residual stream feeding bf16 GEMMs)
std::vector<torch::Tensor> rmsnorm_fwd(torch::Tensor x, torch::Tensor w, double eps, bool out_bf16) {
  check(x, "x"); check(w, "w");
  const int64_t D = w.numel();
  TORCH_CHECK(x.size(-1) == D, "rmsnorm: last dim must match the weight");
  TORCH_CHECK(!out_bf16 || x.scalar_type() == at::kBFloat16 || D % 4 == 0, "rmsnorm: bf16 output of fp32 input needs D % 4 == 0");
  const int64_t rows = x.numel() / D;
  DevGuard g(x.device());
  auto y = out_bf16 ? torch::empty_like(x, x.options().dtype(at::kBFloat16)) : torch::empty_like(x);
  auto rstd = torch::empty({rows}, x.options().dtype(at::kFloat));
  CS_LAUNCH(cs_rmsnorm_fwd(dt_of(x), dt_of(w), dt_of(y), x.data_ptr(), w.data_ptr(), y.data_ptr(),
                           rstd.data_ptr<float>(), (int)rows, (int)D, (float)eps, cur_stream()));
  return {y, rstd};
}

std::vector<torch::Tensor> rmsnorm_bwd(torch::Tensor x, torch::Tensor w, torch::Tensor rstd, torch::Tensor gy) {
  check(x, "x"); check(w, "w"); check(rstd, "rstd"); check(gy, "gy");
  const int64_t D = w.numel(), rows = x.numel() / D;
  TORCH_CHECK(gy.sizes() == x.sizes() && rstd.numel() == rows, "rmsnorm_bwd: shapes");
  TORCH_CHECK(gy.scalar_type() == x.scalar_type() || D % 4 == 0, "rmsnorm_bwd: mixed dtypes need D % 4 == 0");
  DevGuard g(x.device());
  auto dx = torch::empty_like(x);
  auto dw = torch::empty_like(w);
  auto part = torch::empty({(int64_t)cs_rmsnorm_bwd_partials((int)rows, (int)D), D}, x.options().dtype(at::kFloat));
  CS_LAUNCH(cs_rmsnorm_bwd(dt_of(x), dt_of(w), dt_of(gy), x.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(),
                           gy.data_ptr(), dx.data_ptr(), dw.data_ptr(), part.data_ptr<float>(), (int)rows, (int)D,
                           cur_stream()));
  return {dx, dw};
}

// logits [R, V], targets [R] int64 -> {loss_rows [R] f32, lse [R] f32}
std::vector<torch::Tensor> xent_fwd(torch::Tensor logits, torch::Tensor tgt) {
  check(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.size(1) % 8 == 0, "xent: logits [R, V] with V % 8 == 0");
  TORCH_CHECK(tgt.is_cuda() && tgt.is_contiguous() && tgt.scalar_type() == at::kLong && tgt.numel() == logits.size(0),
              "xent: targets [R] int64");
  DevGuard g(logits.device());
  auto fo = logits.options().dtype(at::kFloat);
  auto loss = torch::empty({logits.size(0)}, fo), lse = torch::empty({logits.size(0)}, fo);
  CS_LAUNCH(cs_xent_fwd(dt_of(logits), logits.data_ptr(), tgt.data_ptr<int64_t>(), loss.data_ptr<float>(),
                        lse.data_ptr<float>(), (int)logits.size(0), (int)logits.size(1), cur_stream()));
  return {loss, lse};
}

torch::Tensor xent_bwd(torch::Tensor logits, torch::Tensor tgt, torch::Tensor lse, torch::Tensor gscale, double inv_n) {
  check(logits, "logits");
  check(lse, "lse");
  TORCH_CHECK(logits.dim() == 2 && logits.size(1) % 8 == 0 && lse.numel() == logits.size(0), "xent_bwd: shapes");
  TORCH_CHECK(tgt.is_cuda() && tgt.scalar_type() == at::kLong && tgt.numel() == logits.size(0), "xent_bwd: targets");
  TORCH_CHECK(gscale.is_cuda() && gscale.scalar_type() == at::kFloat && gscale.numel() == 1, "xent_bwd: g");
  DevGuard g(logits.device());
  auto d = torch::empty_like(logits);
  CS_LAUNCH(cs_xent_bwd(dt_of(logits), logits.data_ptr(), tgt.data_ptr<int64_t>(), lse.data_ptr<float>(),
                        gscale.data_ptr<float>(), (float)inv_n, d.data_ptr(), (int)logits.size(0), (int)logits.size(1),
                        cur_stream()));
  return d;
}

torch::Tensor swiglu_fwd(torch::Tensor a, torch::Tensor b) {
  check(a, "a"); check(b, "b");
  TORCH_CHECK(a.sizes() == b.sizes() && a.scalar_type() == b.scalar_type(), "swiglu: a/b mismatch");
  DevGuard g(a.device());
  auto out = torch::empty_like(a);
  CS_LAUNCH(cs_swiglu_fwd(dt_of(a), a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), cur_stream()));
  return out;
}

std::vector<torch::Tensor> swiglu_bwd(torch::Tensor a, torch::Tensor b, torch::Tensor gy) {
  check(a, "a"); check(b, "b"); check(gy, "gy");
  TORCH_CHECK(a.sizes() == b.sizes() && gy.sizes() == a.sizes() && gy.scalar_type() == a.scalar_type(),
              "swiglu_bwd: shapes");
  DevGuard g(a.device());
  auto da = torch::empty_like(a);
  auto db = torch::empty_like(b);
  CS_LAUNCH(cs_swiglu_bwd(dt_of(a), a.data_ptr(), b.data_ptr(), gy.data_ptr(), da.data_ptr(), db.data_ptr(),
                          a.numel(), cur_stream()));
  return {da, db};
}

torch::Tensor rope(torch::Tensor x, torch::Tensor cosv, torch::Tensor sinv, bool inverse) {
  check(x, "x"); check(cosv, "cos"); check(sinv, "sin");
  TORCH_CHECK(x.dim() == 4, "rope: x must be [B, S, H, head_dim]");
  const int64_t B = x.size(0), S = x.size(1), H = x.size(2), hd = x.size(3);
  TORCH_CHECK(hd % 2 == 0 && cosv.scalar_type() == at::kFloat && sinv.scalar_type() == at::kFloat &&
                  cosv.numel() == S * hd / 2 && sinv.numel() == S * hd / 2,
              "rope: cos/sin must be fp32 [S, head_dim/2]");
  DevGuard g(x.device());
  auto out = torch::empty_like(x);
  CS_LAUNCH(cs_rope(dt_of(x), x.data_ptr(), cosv.data_ptr<float>(), sinv.data_ptr<float>(), out.data_ptr(), (int)B,
                    (int)S, (int)H, (int)hd, inverse ? 1 : 0, cur_stream()));
  return out;
}

// q [B, S, Hq, D], k/v [B, S, Hkv, D] bf16 contiguous -> {o [B, S, Hq, D], lse f32 [B, Hq, S]}
void attn_check(const torch::Tensor& q, const torch::Tensor& k, const torch::Tensor& v) {
  for (auto* t : {&q, &k, &v}) {
    check(*t, "attention input");
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->dim() == 4, "attention: bf16 [B, S, H, D] tensors");
  }
  TORCH_CHECK(k.sizes() == v.sizes() && q.size(0) == k.size(0) && q.size(1) == k.size(1) && q.size(3) == k.size(3),
              "attention: q/k/v shapes");
  TORCH_CHECK(q.size(3) == 64 || q.size(3) == 128, "attention: head dim 64 or 128");
  TORCH_CHECK(q.size(2) % k.size(2) == 0, "attention: query heads must be a multiple of kv heads");
}

std::vector<torch::Tensor> attn_fwd(torch::Tensor q, torch::Tensor k, torch::Tensor v, double scale, bool causal) {
  attn_check(q, k, v);
  DevGuard g(q.device());
  auto o = torch::empty_like(q);
  auto lse = torch::empty({q.size(0), q.size(2), q.size(1)}, q.options().dtype(at::kFloat));
  CS_LAUNCH(cs_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), q.size(0),
                        q.size(1), q.size(2), k.size(2), q.size(3), (float)scale, causal ? 1 : 0, cur_stream()));
  return {o, lse};
}

std::vector<torch::Tensor> attn_bwd(torch::Tensor q, torch::Tensor k, torch::Tensor v, torch::Tensor o,
                                    torch::Tensor lse, torch::Tensor dout, double scale, bool causal) {
  attn_check(q, k, v);
  check(o, "o"); check(dout, "dout"); check(lse, "lse");
  TORCH_CHECK(o.sizes() == q.sizes() && dout.sizes() == q.sizes() && o.scalar_type() == at::kBFloat16 &&
                  dout.scalar_type() == at::kBFloat16, "attn_bwd: o / dout must match q");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.numel() == q.size(0) * q.size(2) * q.size(1), "attn_bwd: lse");
  DevGuard g(q.device());
  auto dq = torch::empty_like(q), dk = torch::empty_like(k), dv = torch::empty_like(v);
  auto delta = torch::empty_like(lse);
  CS_LAUNCH(cs_attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(),
                        delta.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), q.size(0), q.size(1),
                        q.size(2), k.size(2), q.size(3), (float)scale, causal ? 1 : 0, cur_stream()));
  return {dq, dk, dv};
}

// C = a @ b on the bf16 matrix cores (gemm_bf16.hip). a: [M, K], b: [K, N], bf16, each with unit
// stride along one of its two dimensions (so x @ w.t(), dy @ w and dy.t() @ x all run without a
// copy); out: a new bf16 (out_f32 false) or fp32 [M, N] tensor, or `acc` [M, N] += a @ b (fp32, or
// bf16: summed in fp32 with one rounding).
// splits: reduction splits of an fp32 result (-1: cs_gemm_bf16_splits), summed in fixed order.
bool mode_bf16_acc(const c10::optional<torch::Tensor>& acc) {
  return acc.has_value() && acc->scalar_type() == at::kBFloat16;
}

torch::Tensor mm_bf16(torch::Tensor a, torch::Tensor b, bool out_f32, c10::optional<torch::Tensor> acc,
                      int64_t splits) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.dim() == 2 && b.dim() == 2, "mm_bf16: 2-D GPU tensors");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16, "mm_bf16: bf16 operands");
  TORCH_CHECK(a.size(1) == b.size(0), "mm_bf16: inner dimensions differ");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(1);
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31), "mm_bf16: dimension too large");
  int ak, bk;
  int64_t lda, ldb;
  if (a.stride(1) == 1) { ak = 1; lda = a.stride(0); }
  else if (a.stride(0) == 1) { ak = 0; lda = a.stride(1); }
  else TORCH_CHECK(false, "mm_bf16: a needs a unit stride");
  if (b.stride(0) == 1) { bk = 1; ldb = b.stride(1); }
  else if (b.stride(1) == 1) { bk = 0; ldb = b.stride(0); }
  else TORCH_CHECK(false, "mm_bf16: b needs a unit stride");
  DevGuard g(a.device());
  if (M == 0 || N == 0 || K == 0) {
    // empty reduction: torch.mm semantics (zeros; an accumulator is returned unchanged) without a
    // launch — the kernel would return hipSuccess and leave a fresh output uninitialised
    if (acc.has_value()) return *acc;
    return torch::zeros({M, N}, a.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  }
  torch::Tensor c;
  int mode;
  // fp32 results of a reduction too long for the output's tile count are split over K into slabs
  int S = splits >= 0 ? (int)splits : cs_gemm_bf16_splits((int)M, (int)N, (int)K);
  if ((!out_f32 && !acc.has_value()) || mode_bf16_acc(acc)) S = 1;
  TORCH_CHECK(S >= 1 && S <= 256, "mm_bf16: splits out of range");
  if (acc.has_value()) {
    c = *acc;
    TORCH_CHECK(c.is_cuda() && (c.scalar_type() == at::kFloat || c.scalar_type() == at::kBFloat16) && c.dim() == 2 &&
                    c.size(0) == M && c.size(1) == N && c.stride(1) == 1,
                "mm_bf16: acc must be fp32 or bf16 [M, N] with unit column stride");
    mode = c.scalar_type() == at::kFloat ? 2 : 3;
  } else {
    c = torch::empty({M, N}, a.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
    mode = out_f32 ? 1 : 0;
  }
  if (S > 1) {
    auto part = torch::empty({S + (mode == 2 ? 1 : 0), M, N}, a.options().dtype(at::kFloat));
    CS_LAUNCH(cs_gemm_bf16(ak, a.data_ptr(), lda, bk, b.data_ptr(), ldb, part.data_ptr(), N, (int)M, (int)N, (int)K, 1,
                           S, M * N, cur_stream()));
    if (mode == 2) part[S].copy_(c);  // the accumulator joins the fixed-order sum as the last slab
    if (c.is_contiguous()) {
      CS_LAUNCH(cs_slab_sum(part.data_ptr<float>(), (int)part.size(0), M * N, c.data_ptr<float>(), cur_stream()));
    } else {
      auto sum = torch::empty({M, N}, part.options());
      CS_LAUNCH(cs_slab_sum(part.data_ptr<float>(), (int)part.size(0), M * N, sum.data_ptr<float>(), cur_stream()));
      c.copy_(sum);
    }
    return c;
  }
  CS_LAUNCH(cs_gemm_bf16(ak, a.data_ptr(), lda, bk, b.data_ptr(), ldb, c.data_ptr(), c.stride(0), (int)M, (int)N,
                         (int)K, mode, 1, 0, cur_stream()));
  return c;
}

// y = a @ b (bf16, a [M, K] K-major, b [K, N] with unit stride along K) plus the BatchNorm
// statistics of y per 256-row tile: {y, tiles [ceil(M / 256), N, 2] = (mean, M2)}
std::vector<torch::Tensor> mm_bf16_bn_stats(torch::Tensor a, torch::Tensor b) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.dim() == 2 && b.dim() == 2 && a.scalar_type() == at::kBFloat16 &&
                  b.scalar_type() == at::kBFloat16, "mm_bf16_bn_stats: 2-D bf16 GPU tensors");
  TORCH_CHECK(a.size(1) == b.size(0) && a.stride(1) == 1 && b.stride(0) == 1,
              "mm_bf16_bn_stats: a [M, K] and b [K, N], both with unit stride along K");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(1);
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31), "mm_bf16_bn_stats: dimension too large");
  DevGuard g(a.device());
  auto y = torch::empty({M, N}, a.options());
  auto tiles = torch::empty({(M + 255) / 256, N, 2}, a.options().dtype(at::kFloat));
  CS_LAUNCH(cs_gemm_bf16_bn_stats(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(1), y.data_ptr(), N, (int)M,
                                  (int)N, (int)K, tiles.data_ptr<float>(), cur_stream()));
  return {y, tiles};
}

}  // namespace

void register_lm_ops(pybind11::module& m) {
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("xent_fwd", &xent_fwd, "softmax cross-entropy rows -> (loss, lse)");
  m.def("xent_bwd", &xent_bwd, "its backward -> dlogits");
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("rope", &rope);
  m.def("attn_fwd", &attn_fwd, "flash attention forward (bf16 [B,S,H,D], GQA, causal)");
  m.def("attn_bwd", &attn_bwd, "flash attention backward -> dq, dk, dv");
  m.def("mm_bf16", &mm_bf16, "C = a @ b on the bf16 matrix cores", pybind11::arg("a"), pybind11::arg("b"),
        pybind11::arg("out_f32") = false, pybind11::arg("acc") = c10::nullopt, pybind11::arg("splits") = -1);
  m.def("mm_bf16_bn_stats", &mm_bf16_bn_stats, "a @ b (bf16) plus per-256-row-tile BatchNorm (mean, M2) of the result");
}
