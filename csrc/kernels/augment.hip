// Fused CIFAR batch construction: gather by sampler index + RandomCrop(32, pad 4)
// + RandomHorizontalFlip + ToTensor (/255) + Normalize(mean, std), in one pass
// from the HBM-resident uint8 dataset (reference transforms:
// master/part1/part1.py:66-77).
//
// One thread per output pixel; the 3 channels of a pixel are written together.
// Output layouts: NCHW fp32 (module path) or NHWC with a channel stride of 3 or 4
// (the native engine pads to 4 channels so conv0 loads one float4 per pixel).
#include "common.h"
#include "launchers.h"

namespace {

struct Norm {
  float m[3], inv[3];
};

__global__ __launch_bounds__(256) void augment_kernel(const uint8_t* __restrict__ data,
                                                      const int64_t* __restrict__ idx,
                                                      const int32_t* __restrict__ params,
                                                      float* __restrict__ out, int B, int nhwc,
                                                      int cstride, Norm nm) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * 1024) return;
  const int b = t >> 10, y = (t >> 5) & 31, x = t & 31;
  const int64_t s = idx[b];
  const int dy = params[s * 3 + 0], dx = params[s * 3 + 1], fl = params[s * 3 + 2];
  const int sx = fl ? (31 - x) : x;
  const int py = y + dy - 4, px = sx + dx - 4;  // coordinates in the un-padded image
  float v[3] = {0.f, 0.f, 0.f};
  if (py >= 0 && py < 32 && px >= 0 && px < 32) {
    const uint8_t* p = data + ((s * 32 + py) * 32 + px) * 3;
    v[0] = p[0];
    v[1] = p[1];
    v[2] = p[2];
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) v[c] = (v[c] / 255.0f - nm.m[c]) * nm.inv[c];
  if (nhwc) {
    float* o = out + (size_t)t * cstride;
    o[0] = v[0];
    o[1] = v[1];
    o[2] = v[2];
    if (cstride == 4) o[3] = 0.f;
  } else {
    float* o = out + (size_t)b * 3072 + y * 32 + x;
    o[0] = v[0];
    o[1024] = v[1];
    o[2048] = v[2];
  }
}

}  // namespace

hipError_t cs_augment(const uint8_t* data, const int64_t* idx, const int32_t* params, float* out, int B,
                      int nhwc, int cstride, const float* mean, const float* std_, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  Norm nm;
  for (int c = 0; c < 3; ++c) {
    nm.m[c] = mean[c];
    nm.inv[c] = 1.0f / std_[c];
  }
  const int n = B * 1024;
  hipLaunchKernelGGL(augment_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, data, idx, params, out, B, nhwc,
                     cstride, nm);
  return hipGetLastError();
}

namespace {
// The native engine's whole batch step in one launch: sample s = perm[cursor * stride + b]
// (the rank's DistributedSampler order for the epoch, with a device-side step cursor that
// the SGD kernel advances — so a replayed step graph needs no host-side index copy), or
// s = idx[b] when perm is null; then RandomCrop/HFlip/Normalize into NHWC (channel stride
// 4) and, once per sample, idx_out[b] = s and the label gather.
__global__ __launch_bounds__(256) void make_batch_kernel(const uint8_t* __restrict__ data,
                                                         const int64_t* __restrict__ labels,
                                                         const int64_t* __restrict__ perm,
                                                         const int64_t* __restrict__ cursor, int stride,
                                                         const int64_t* __restrict__ idx_in,
                                                         const int32_t* __restrict__ params, float* __restrict__ out,
                                                         int64_t* __restrict__ idx_out, int64_t* __restrict__ ylab,
                                                         int B, Norm nm) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * 1024) return;
  const int b = t >> 10, y = (t >> 5) & 31, x = t & 31;
  const int64_t s = perm != nullptr ? perm[*cursor * stride + b] : idx_in[b];
  if ((t & 1023) == 0) {
    idx_out[b] = s;
    ylab[b] = labels[s];
  }
  const int dy = params[s * 3 + 0], dx = params[s * 3 + 1], fl = params[s * 3 + 2];
  const int sx = fl ? (31 - x) : x;
  const int py = y + dy - 4, px = sx + dx - 4;
  float v[3] = {0.f, 0.f, 0.f};
  if (py >= 0 && py < 32 && px >= 0 && px < 32) {
    const uint8_t* p = data + ((s * 32 + py) * 32 + px) * 3;
    v[0] = p[0];
    v[1] = p[1];
    v[2] = p[2];
  }
  float4 o;
  o.x = (v[0] / 255.0f - nm.m[0]) * nm.inv[0];
  o.y = (v[1] / 255.0f - nm.m[1]) * nm.inv[1];
  o.z = (v[2] / 255.0f - nm.m[2]) * nm.inv[2];
  o.w = 0.f;
  reinterpret_cast<float4*>(out)[t] = o;
}

__global__ void gather_labels_kernel(const int64_t* __restrict__ labels, const int64_t* __restrict__ idx,
                                     int64_t* __restrict__ out, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) out[b] = labels[idx[b]];
}
}  // namespace

hipError_t cs_gather_labels(const int64_t* labels, const int64_t* idx, int64_t* out, int B, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_labels_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, labels, idx, out, B);
  return hipGetLastError();
}

hipError_t cs_make_batch(const uint8_t* data, const int64_t* labels, const int64_t* perm, const int64_t* cursor,
                         int stride, const int64_t* idx_in, const int32_t* params, float* out, int64_t* idx_out,
                         int64_t* ylab, int B, const float* mean, const float* std_, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  if ((perm == nullptr) == (idx_in == nullptr) || (perm != nullptr && cursor == nullptr)) return hipErrorInvalidValue;
  Norm nm;
  for (int c = 0; c < 3; ++c) {
    nm.m[c] = mean[c];
    nm.inv[c] = 1.0f / std_[c];
  }
  const int n = B * 1024;
  hipLaunchKernelGGL(make_batch_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, data, labels, perm, cursor,
                     stride, idx_in, params, out, idx_out, ylab, B, nm);
  return hipGetLastError();
}
