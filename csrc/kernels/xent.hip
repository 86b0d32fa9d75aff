// Fused classifier head: fc1 (Linear 512->10, master/part1/model.py:40,45) +
// CrossEntropyLoss(mean) (master/part1/part1.py:94) forward AND backward, plus the
// eval argmax/accuracy count (master/part2b/part2b.py:64-65) — SURVEY.md §2.2 N8/N9/N13.
//
// Two launches replace the reference's five ATen kernels (addmm, log_softmax, nll,
// their backwards, argmax): a row pass (one wave per sample: logits, softmax, loss,
// argmax and dfeat from registers) and a column pass (dW / db / batch loss), both
// with fixed summation order. `ws` holds dl [B][C] + per-sample loss/correct. The loss is written as a device scalar so the training loop
// never syncs the host (the loss is read only every 20 iterations).
#include "common.h"
#include "launchers.h"
#include "xent_device.h"

namespace {

constexpr int kThreads = 512;
constexpr int kMaxC = 16;

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

// Row pass: one wave per sample. Each lane holds K/256 float4 slices of the
// sample's features and of every W row, so the C logits, the softmax, the
// per-sample loss/argmax AND dfeat[b] = sum_j dl[b][j] W[j] come out of
// registers; dl is staged in `ws` for the column pass. CT = compile-time class count
// (10 for CIFAR-10: every class loop and cross-lane sum is unrolled and interleaved),
// 0 = runtime C <= kMaxC.
// feature float4 k of a row: read, or (bn.y != null) the last block's BN + ReLU + 2x2 max-pool of
// its pre-BN output [2][2][K] (bn.hip bn_apply's arithmetic and max order), written back to feat
__device__ __forceinline__ float4 bnrelu4h(float4 y, float4 s, float4 t) {
  return make_float4(fmaxf(y.x * s.x + t.x, 0.f), fmaxf(y.y * s.y + t.y, 0.f), fmaxf(y.z * s.z + t.z, 0.f),
                     fmaxf(y.w * s.w + t.w, 0.f));
}
__device__ __forceinline__ float4 head_feat(float4* f4, const CsHeadBn& bn, int row, int K4, int k) {
  if (bn.y == nullptr) return f4[k];
  const float4* y4 = reinterpret_cast<const float4*>(bn.y) + (size_t)row * 4 * K4 + k;
  const float4 s = reinterpret_cast<const float4*>(bn.scale)[k], t = reinterpret_cast<const float4*>(bn.shift)[k];
  const float4 a0 = bnrelu4h(y4[0], s, t), a1 = bnrelu4h(y4[K4], s, t);
  const float4 a2 = bnrelu4h(y4[2 * K4], s, t), a3 = bnrelu4h(y4[3 * K4], s, t);
  const float4 r = make_float4(fmaxf(fmaxf(a0.x, a1.x), fmaxf(a2.x, a3.x)), fmaxf(fmaxf(a0.y, a1.y), fmaxf(a2.y, a3.y)),
                               fmaxf(fmaxf(a0.z, a1.z), fmaxf(a2.z, a3.z)), fmaxf(fmaxf(a0.w, a1.w), fmaxf(a2.w, a3.w)));
  f4[k] = r;
  return r;
}

template <int CT>
__global__ __launch_bounds__(256) void head_rows_kernel(float* __restrict__ feat, const float* __restrict__ W,
                                                        const float* __restrict__ bias,
                                                        const int64_t* __restrict__ labels, int B, int K, int C,
                                                        float gscale, float* __restrict__ ws,
                                                        float* __restrict__ logits_out, int64_t* __restrict__ pred_out,
                                                        float* __restrict__ dfeat, CsHeadBn bn) {
  constexpr int NC = CT ? CT : kMaxC;
  if (CT) C = CT;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const int K4 = K >> 2;
  float4* f4 = reinterpret_cast<float4*>(feat) + (size_t)row * K4;
  const float4* w4 = reinterpret_cast<const float4*>(W);
  // label and bias loaded up front: their latency overlaps the dot products
  const int y = (int)labels[row];
  float bj[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) bj[j] = (bias && j < C) ? bias[j] : 0.f;
  float acc[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) acc[j] = 0.f;
  // compile-time class count and K <= 512 (VGG's 512 features): the lane's W slices stay in
  // registers for the dfeat pass (no second, dependent W read); same summation order
  constexpr int KIT = 2;
  const bool cached = CT != 0 && K4 <= 64 * KIT;
  float4 wc[CT ? KIT : 1][CT ? NC : 1];
  if constexpr (CT != 0) {
    if (cached) {
#pragma unroll
      for (int it = 0; it < KIT; ++it) {
        const int k = lane + 64 * it;
        if (k < K4) {
          const float4 f = head_feat(f4, bn, row, K4, k);
#pragma unroll
          for (int j = 0; j < NC; ++j) {
            wc[it][j] = w4[(size_t)j * K4 + k];
            acc[j] += f.x * wc[it][j].x + f.y * wc[it][j].y + f.z * wc[it][j].z + f.w * wc[it][j].w;
          }
        }
      }
    }
  }
  if (!cached) {
    for (int k = lane; k < K4; k += 64) {
      const float4 f = head_feat(f4, bn, row, K4, k);
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        if (j < C) {
          const float4 w = w4[(size_t)j * K4 + k];
          acc[j] += f.x * w.x + f.y * w.y + f.z * w.z + f.w * w.w;
        }
      }
    }
  }
  float mx = -INFINITY;
  int am = 0;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    if (j < C) {
      acc[j] = cs::wave_sum(acc[j]) + bj[j];
      if (acc[j] > mx) { mx = acc[j]; am = j; }
    }
  }
  float se = 0.f;
#pragma unroll
  for (int j = 0; j < NC; ++j)
    if (j < C) se += expf(acc[j] - mx);
  const float lse = logf(se);
  float xy = 0.f;
#pragma unroll
  for (int j = 0; j < NC; ++j)
    if (j == y) xy = acc[j];
  float* dl = ws;                      // [B][C]
  float* rowloss = ws + (size_t)B * C;  // [B]
  float* rowcorr = rowloss + B;         // [B]
  if (lane == 0) {
    rowloss[row] = (mx + lse) - xy;
    rowcorr[row] = (am == y) ? 1.f : 0.f;
    if (pred_out) pred_out[row] = am;
  }
  if (logits_out && lane < C) {
#pragma unroll
    for (int j = 0; j < NC; ++j)
      if (j == lane) logits_out[(size_t)row * C + j] = acc[j];
  }
  if (dfeat == nullptr) return;
  const float inv = gscale / (float)B;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    if (j < C) {
      acc[j] = (expf(acc[j] - mx - lse) - (j == y ? 1.f : 0.f)) * inv;
      if (lane == j) dl[(size_t)row * C + j] = acc[j];
    }
  }
  float4* d4 = reinterpret_cast<float4*>(dfeat) + (size_t)row * K4;
  if constexpr (CT != 0) {
    if (cached) {
#pragma unroll
      for (int it = 0; it < KIT; ++it) {
        const int k = lane + 64 * it;
        if (k < K4) {
          float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int j = 0; j < NC; ++j) {
            o.x += acc[j] * wc[it][j].x; o.y += acc[j] * wc[it][j].y;
            o.z += acc[j] * wc[it][j].z; o.w += acc[j] * wc[it][j].w;
          }
          d4[k] = o;
        }
      }
      return;
    }
  }
  for (int k = lane; k < K4; k += 64) {
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      if (j < C) {
        const float4 w = w4[(size_t)j * K4 + k];
        o.x += acc[j] * w.x; o.y += acc[j] * w.y; o.z += acc[j] * w.z; o.w += acc[j] * w.w;
      }
    }
    d4[k] = o;
  }
}

// Column pass: one 64-thread block per piece of cs_head::cols_wave (xent_device.h)
__global__ __launch_bounds__(64) void head_cols_kernel(CsHeadCols h) { cs_head::cols_wave(h, blockIdx.x, threadIdx.x); }

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
                          float* db, float* dfeat, int64_t* pred_out, float* ws, hipStream_t stream, int part,
                          const CsHeadBn* bn) {
  if (C > kMaxC || C < 1 || B <= 0 || (K & 3) != 0 || ws == nullptr || part < 0 || part > 2) return hipErrorInvalidValue;
  const CsHeadBn hb = bn != nullptr ? *bn : CsHeadBn{nullptr, nullptr, nullptr};
  float* fw = const_cast<float*>(feat);  // written only when the row pass builds the features (bn)
  if (part == 2) goto cols;
  if (C == 10)
    hipLaunchKernelGGL(head_rows_kernel<10>, dim3((B + 3) / 4), dim3(256), 0, stream, fw, W, bias, labels, B, K, C,
                       gscale, ws, logits_out, pred_out, dfeat, hb);
  else
    hipLaunchKernelGGL(head_rows_kernel<0>, dim3((B + 3) / 4), dim3(256), 0, stream, fw, W, bias, labels, B, K, C,
                       gscale, ws, logits_out, pred_out, dfeat, hb);
  if (part == 1) return hipGetLastError();
cols:
  const bool bwd = dW != nullptr && db != nullptr && (dfeat != nullptr || part == 2);
  const CsHeadCols h{feat, B, K, C, ws, bwd ? dW : nullptr, bwd ? db : nullptr, loss_out, correct_out,
                     bwd ? cs_head_cols_pieces(K, C) : 1};
  hipLaunchKernelGGL(head_cols_kernel, dim3(h.P), dim3(64), 0, stream, h);
  return hipGetLastError();
}

hipError_t cs_softmax_xent(const float* logits, const int64_t* labels, int B, int C, float gscale, float* loss_out,
                           float* dlogits, int* correct_out, hipStream_t stream) {
  if (C > kMaxC || B <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(1), dim3(kThreads), 0, stream, logits, labels, B, C, gscale, loss_out,
                     dlogits, correct_out);
  return hipGetLastError();
}
