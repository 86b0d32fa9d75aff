// VGG block 0: the 3 -> 64 channel 3x3 convolution (nn.Conv2d(3, 64, 3, padding=1) at
// master/part1/model.py:18-23, the first layer of every VGG cfg) as DIRECT f32 kernels instead of
// the implicit GEMM. Its GEMM is (pixels x 64) with K = 27: far too shallow for the MFMA tiles
// (1024 blocks of 64 x 64 with a 2-step K loop, ~12 us for 0.23 GFLOP), and its weight gradient
// (64 x 27 outputs reduced over every pixel) needed 256 split-K slabs + a fold + a combine. Both
// are bandwidth-shaped: one pass over the activations.
//
//  * conv0_fwd: 256 pixels per workgroup (8 image rows), one pixel per thread, all 64 output
//    channels in registers: the 10 x 34 x 4 input halo tile and the weights ([27][64], transposed:
//    every lane reads the same word -> LDS broadcast) in LDS, 27 x 64 exact-f32 FMAs per pixel, y
//    (+bias) stored as 16 float4 per thread (256 contiguous bytes per pixel). The BatchNorm tile
//    statistics of the 256 rows — per channel mean, then M2 = sum (y - mean)^2 around it (two
//    passes, no cancellation) — come out of the same registers: a 6-stage reduce-scatter
//    butterfly over the wave (lane l ends with channel l's wave sum), then the 4 waves in order
//    through LDS. Fixed order everywhere: deterministic.
//  * conv0_wgrad_part: 256 pixels per workgroup: dz tile [256][64] and the input halo in LDS,
//    thread = (output channel, slice of the 27 (ci, tap) columns), partial dW [64][27] per
//    workgroup (OIHW order);  conv0_wgrad_sum: the partials summed in a fixed order (4 slices
//    per column, then the slices in order) -> dW (OIHW [64][3][3][3]).
#include "common.h"
#include "launchers.h"

namespace {

constexpr int kPix = 256;  // pixels per workgroup (= threads)
constexpr int kCo = 64;

// input halo tile of image rows [h0 - 1, h0 + rows + 1) x columns [-1, W + 1) x 4 channels, zeros
// outside the image (conv padding 1); W = 32 (CIFAR)
template <int ROWS>
__device__ __forceinline__ void load_halo(const float* __restrict__ x, int b, int h0, int H, float* xs) {
  constexpr int W = 32, WP = W + 2, N = (ROWS + 2) * WP;  // float4 cells
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const int r = i / WP, c = i - r * WP;
    const int h = h0 - 1 + r, w = c - 1;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W)
      v = *reinterpret_cast<const float4*>(x + (((size_t)b * H + h) * W + w) * 4);
    *reinterpret_cast<float4*>(xs + 4 * i) = v;
  }
}

// reduce-scatter of 64 per-lane values over the wave: lane l returns sum over lanes of v[l]
// (6 stages: at stage s each lane keeps the half of its remaining channels selected by lane bit
// 5 - s and adds the partner's copy of it; the surviving index equals the lane)
__device__ __forceinline__ float wave_reduce_scatter64(float (&v)[kCo]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int half = 32 >> s;  // channels kept after this stage
    const bool hi = (lane >> (5 - s)) & 1;
#pragma unroll
    for (int j = 0; j < half; ++j) {
      const float mine = hi ? v[j + half] : v[j];
      const float give = hi ? v[j] : v[j + half];
      v[j] = mine + __shfl_xor(give, half, 64);
    }
  }
  return v[0];
}

__global__ __launch_bounds__(kPix) void conv0_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ bias, float* __restrict__ y,
                                                         float* __restrict__ stats, int H) {
  constexpr int W = 32, ROWS = kPix / W, WP = W + 2;
  __shared__ float wt[27 * kCo];            // [k = ci*9 + tap][co]
  __shared__ float xs[(ROWS + 2) * WP * 4];  // halo tile
  __shared__ float red[4 * kCo];
  const int tid = threadIdx.x;
  const int m0 = blockIdx.x * kPix;  // first pixel (NHWC row) of the tile
  const int b = m0 / (H * W), h0 = (m0 / W) % H;
  for (int i = tid; i < 27 * kCo; i += kPix) {
    const int co = i / 27, k = i - co * 27;
    wt[k * kCo + co] = w[i];  // OIHW [64][3][3][3] -> [27][64]
  }
  load_halo<ROWS>(x, b, h0, H, xs);
  float acc[kCo];
#pragma unroll
  for (int c = 0; c < kCo; ++c) acc[c] = bias != nullptr ? bias[c] : 0.f;
  __syncthreads();
  const int r = tid / W, cpx = tid % W;
#pragma unroll 1
  for (int tap = 0; tap < 9; ++tap) {
    const int dh = tap / 3, dw = tap % 3;
    const float4 xv = *reinterpret_cast<const float4*>(xs + 4 * ((r + dh) * WP + cpx + dw));
    const float xin[3] = {xv.x, xv.y, xv.z};
#pragma unroll
    for (int ci = 0; ci < 3; ++ci) {
      const float* wr = wt + (ci * 9 + tap) * kCo;
#pragma unroll
      for (int c = 0; c < kCo; c += 4) {
        const float4 wv = *reinterpret_cast<const float4*>(wr + c);
        acc[c] = fmaf(xin[ci], wv.x, acc[c]);
        acc[c + 1] = fmaf(xin[ci], wv.y, acc[c + 1]);
        acc[c + 2] = fmaf(xin[ci], wv.z, acc[c + 2]);
        acc[c + 3] = fmaf(xin[ci], wv.w, acc[c + 3]);
      }
    }
  }
  float4* yo = reinterpret_cast<float4*>(y + (size_t)(m0 + tid) * kCo);
#pragma unroll
  for (int c = 0; c < kCo; c += 4) yo[c / 4] = make_float4(acc[c], acc[c + 1], acc[c + 2], acc[c + 3]);
  if (stats == nullptr) return;
  // ---- tile statistics over the 256 pixels, per channel
  const int lane = tid & 63, wv = tid >> 6;
  float t[kCo];
#pragma unroll
  for (int c = 0; c < kCo; ++c) t[c] = acc[c];
  const float ws = wave_reduce_scatter64(t);  // lane = channel
  red[wv * kCo + lane] = ws;
  __syncthreads();
  __shared__ float mean_sh[kCo];
  if (tid < kCo) mean_sh[tid] = (((red[tid] + red[kCo + tid]) + red[2 * kCo + tid]) + red[3 * kCo + tid]) / (float)kPix;
  __syncthreads();
#pragma unroll
  for (int c = 0; c < kCo; ++c) {
    const float d = acc[c] - mean_sh[c];
    t[c] = d * d;
  }
  const float wq = wave_reduce_scatter64(t);
  __syncthreads();  // every wave read its first-pass sums
  red[wv * kCo + lane] = wq;
  __syncthreads();
  if (tid < kCo) {
    const float m2 = ((red[tid] + red[kCo + tid]) + red[2 * kCo + tid]) + red[3 * kCo + tid];
    *reinterpret_cast<float2*>(stats + ((size_t)blockIdx.x * kCo + tid) * 2) = make_float2(mean_sh[tid], m2);
  }
}

// partial dW of 256 pixels: thread (co = tid & 63, slice = tid >> 6) sums columns k = slice + 4j
__global__ __launch_bounds__(kPix) void conv0_wgrad_part_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ dz,
                                                                float* __restrict__ part, int H) {
  constexpr int W = 32, ROWS = kPix / W, WP = W + 2;
  __shared__ float xs[(ROWS + 2) * WP * 4];
  __shared__ float dzs[kPix * (kCo + 1)];  // +1: the per-pixel column reads are conflict-free
  const int tid = threadIdx.x;
  const int m0 = blockIdx.x * kPix;
  const int b = m0 / (H * W), h0 = (m0 / W) % H;
  load_halo<ROWS>(x, b, h0, H, xs);
  for (int i = tid; i < kPix * kCo / 4; i += kPix) {
    const float4 v = reinterpret_cast<const float4*>(dz + (size_t)m0 * kCo)[i];
    const int p = (4 * i) / kCo, c = (4 * i) % kCo;
    float* d = dzs + p * (kCo + 1) + c;
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
  __syncthreads();
  const int co = tid & 63, sl = tid >> 6;
  float acc[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int p = 0; p < kPix; ++p) {
    const float g = dzs[p * (kCo + 1) + co];
    const int r = p / W, cpx = p % W;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int k = sl + 4 * j;  // k = ci * 9 + tap
      if (k < 27) {
        const int ci = k / 9, tap = k - 9 * ci;
        acc[j] = fmaf(g, xs[4 * ((r + tap / 3) * WP + cpx + tap % 3) + ci], acc[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int k = sl + 4 * j;
    if (k < 27) part[(size_t)blockIdx.x * 27 * kCo + co * 27 + k] = acc[j];
  }
}

// dW[i] = sum over the nb partials in order: block = 64 columns x 4 row slices, slice s sums rows
// s, s + 4, ... (8 loads in flight), then the 4 slices in order
__global__ __launch_bounds__(256) void conv0_wgrad_sum_kernel(const float* __restrict__ part, int nb,
                                                             float* __restrict__ dw) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), sl = threadIdx.x >> 6;
  constexpr int NC = 27 * kCo;
  float s = 0.f;
  if (col < NC) {
    for (int r0 = sl; r0 < nb; r0 += 4 * 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = r0 + 4 * j;
        v[j] = r < nb ? part[(size_t)r * NC + col] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
  }
  red[sl][threadIdx.x & 63] = s;
  __syncthreads();
  if (sl == 0 && col < NC) dw[col] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

}  // namespace

int cs_conv0_tile_rows() { return kPix; }

size_t cs_conv0_wgrad_part_floats(int B, int H, int W) {
  return (size_t)((B * H * W) / kPix) * 27 * kCo;
}

hipError_t cs_conv0_fwd(const float* x, const float* w, const float* bias, float* y, float* stats, int B, int H,
                        int W, int Cout, hipStream_t stream) {
  if (W != 32 || Cout != kCo || (B * H * W) % kPix != 0 || (H * W) % kPix != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(conv0_fwd_kernel, dim3((B * H * W) / kPix), dim3(kPix), 0, stream, x, w, bias, y, stats, H);
  return hipGetLastError();
}

hipError_t cs_conv0_wgrad(const float* x, const float* dz, float* part, float* dw, int B, int H, int W, int Cout,
                          hipStream_t stream) {
  if (W != 32 || Cout != kCo || (B * H * W) % kPix != 0 || (H * W) % kPix != 0) return hipErrorInvalidValue;
  const int nb = (B * H * W) / kPix;
  hipLaunchKernelGGL(conv0_wgrad_part_kernel, dim3(nb), dim3(kPix), 0, stream, x, dz, part, H);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  hipLaunchKernelGGL(conv0_wgrad_sum_kernel, dim3((27 * kCo + 63) / 64), dim3(256), 0, stream, part, nb, dw);
  return hipGetLastError();
}
