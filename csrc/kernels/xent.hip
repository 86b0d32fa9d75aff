// Fused classifier head: fc1 (Linear 512->10, master/part1/model.py:40,45) +
// CrossEntropyLoss(mean) (master/part1/part1.py:94) forward AND backward, plus the
// eval argmax/accuracy count (master/part2b/part2b.py:64-65) — SURVEY.md §2.2 N8/N9/N13.
//
// The head is tiny (B x 10 x 512), so one 512-thread workgroup does everything with
// the logits / dlogits in LDS: no intermediate tensor ever touches HBM and the five
// ATen kernels of the reference (addmm, log_softmax, nll, their backwards, argmax)
// become one launch. The loss is written as a device scalar so the training loop
// never syncs the host (the loss is read only every 20 iterations).
#include "common.h"
#include "launchers.h"

namespace {

constexpr int kThreads = 512;
constexpr int kMaxC = 16;

// logits[b][j] = bias[j] + <feat[b], W[j]>   (one wave per (b, j) pair)
__device__ void head_forward(const float* __restrict__ feat, const float* __restrict__ W,
                             const float* __restrict__ bias, int B, int K, int C, float* lg) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int pr = wid; pr < B * C; pr += nw) {
    const int b = pr / C, j = pr - b * C;
    const float* f = feat + (size_t)b * K;
    const float* w = W + (size_t)j * K;
    float acc = 0.f;
    for (int k = lane; k < K; k += 64) acc += f[k] * w[k];
    acc = cs::wave_sum(acc);
    if (lane == 0) lg[pr] = acc + (bias ? bias[j] : 0.f);
  }
}

// per-sample softmax-xent: loss partial, dlogits (mean reduction), argmax correctness
__device__ void head_loss(const float* lg, const int64_t* __restrict__ labels, int B, int C, float gscale,
                          float* dlg, float* red, float* loss_out, int* correct_out, float* logits_out,
                          int64_t* pred_out) {
  float lsum = 0.f;
  int corr = 0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const float* x = lg + b * C;
    float mx = x[0];
    int am = 0;
    for (int j = 1; j < C; ++j)
      if (x[j] > mx) { mx = x[j]; am = j; }
    float se = 0.f;
    for (int j = 0; j < C; ++j) se += expf(x[j] - mx);
    const float lse = logf(se);
    const int y = (int)labels[b];
    lsum += (mx + lse) - x[y];
    corr += (am == y);
    if (pred_out) pred_out[b] = am;
    if (logits_out)
      for (int j = 0; j < C; ++j) logits_out[b * C + j] = x[j];
    if (dlg) {
      const float inv = gscale / (float)B;
      for (int j = 0; j < C; ++j) {
        const float p = expf(x[j] - mx - lse);
        dlg[b * C + j] = (p - (j == y ? 1.f : 0.f)) * inv;
      }
    }
  }
  const float tot = cs::block_sum(lsum, red);
  const float ctot = cs::block_sum((float)corr, red);
  if (threadIdx.x == 0) {
    if (loss_out) *loss_out = tot / (float)B;
    if (correct_out) *correct_out = (int)(ctot + 0.5f);
  }
}

__global__ __launch_bounds__(kThreads) void linear_xent_kernel(
    const float* __restrict__ feat, const float* __restrict__ W, const float* __restrict__ bias,
    const int64_t* __restrict__ labels, int B, int K, int C, float gscale, float* __restrict__ loss_out,
    int* __restrict__ correct_out, float* __restrict__ logits_out, float* __restrict__ dW,
    float* __restrict__ db, float* __restrict__ dfeat, int64_t* __restrict__ pred_out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* lg = smem;              // [B*C]
  float* dlg = smem + B * C;     // [B*C]
  float* red = dlg + B * C;      // [16]
  head_forward(feat, W, bias, B, K, C, lg);
  __syncthreads();
  const bool bwd = dW != nullptr;
  head_loss(lg, labels, B, C, gscale, bwd ? dlg : nullptr, red, loss_out, correct_out, logits_out, pred_out);
  __syncthreads();
  if (!bwd) return;
  // dW[j][k] = sum_b dlg[b][j] * feat[b][k];  db[j] = sum_b dlg[b][j]
  for (int e = threadIdx.x; e < C * K; e += blockDim.x) {
    const int j = e / K, k = e - j * K;
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += dlg[b * C + j] * feat[(size_t)b * K + k];
    dW[e] = acc;
  }
  if (threadIdx.x < (unsigned)C) {
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += dlg[b * C + threadIdx.x];
    db[threadIdx.x] = acc;
  }
  // dfeat[b][k] = sum_j dlg[b][j] * W[j][k]
  if (dfeat) {
    for (int e = threadIdx.x; e < B * K; e += blockDim.x) {
      const int b = e / K, k = e - b * K;
      float acc = 0.f;
      for (int j = 0; j < C; ++j) acc += dlg[b * C + j] * W[(size_t)j * K + k];
      dfeat[e] = acc;
    }
  }
}

__global__ __launch_bounds__(kThreads) void softmax_xent_kernel(const float* __restrict__ logits,
                                                                const int64_t* __restrict__ labels, int B, int C,
                                                                float gscale, float* __restrict__ loss_out,
                                                                float* __restrict__ dlogits,
                                                                int* __restrict__ correct_out) {
  __shared__ float red[16];
  head_loss(logits, labels, B, C, gscale, dlogits, red, loss_out, correct_out, nullptr, nullptr);
}

}  // namespace

hipError_t cs_linear_xent(const float* feat, const float* W, const float* bias, const int64_t* labels, int B, int K,
                          int C, float gscale, float* loss_out, int* correct_out, float* logits_out, float* dW,
                          float* db, float* dfeat, int64_t* pred_out, hipStream_t stream) {
  if (C > kMaxC || B <= 0) return hipErrorInvalidValue;
  const size_t lds = (size_t)(2 * B * C + 16) * sizeof(float);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(linear_xent_kernel, dim3(1), dim3(kThreads), lds, stream, feat, W, bias, labels, B, K, C, gscale,
                     loss_out, correct_out, logits_out, dW, db, dfeat, pred_out);
  return hipGetLastError();
}

hipError_t cs_softmax_xent(const float* logits, const int64_t* labels, int B, int C, float gscale, float* loss_out,
                           float* dlogits, int* correct_out, hipStream_t stream) {
  if (C > kMaxC || B <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(1), dim3(kThreads), 0, stream, logits, labels, B, C, gscale, loss_out,
                     dlogits, correct_out);
  return hipGetLastError();
}
