// VGG block 0: the 3 -> 64 channel 3x3 convolution (nn.Conv2d(3, 64, 3, padding=1) at
// master/part1/model.py:18-23, the first layer of every VGG cfg) as DEDICATED f32 MFMA kernels
// instead of the general implicit GEMM. Its GEMM is (pixels x 64) with K = 27: far too shallow for
// the LDS-staged GEMM tiles (a 2-step K loop behind a full tile load, ~12 us for 0.23 GFLOP), and
// its weight gradient (64 x 27 outputs reduced over every pixel) needed 256 split-K slabs + a fold +
// a combine. Here both are one pass over the activations, on v_mfma_f32_32x32x2_f32 (exact f32,
// a k-ordered fmaf chain): the operands come straight from registers, the only LDS traffic is a
// 4 B/lane read of the input halo per MFMA pair. (Two earlier VALU versions were bound by LDS data
// return — a broadcast ds_read_b128 still returns 1 KiB per wave — and by scalar-load latency.)
//
//  * conv0_fwd: 128 pixels (4 image rows) per workgroup, wave w = image row w of the tile: 32 pixels
//    (MFMA rows) x 64 channels (2 MFMA column tiles), K = 27 padded to 28 in 14 steps of 2. B = the
//    weights, 28 registers loaded once per lane; A = the pixel's 3 x 3 x 3 input window from a
//    channel-planar LDS halo. The BatchNorm tile statistics of the 128 rows come out of the
//    accumulators (lane = channel): per channel mean, then M2 = sum (y - mean)^2 around it (two
//    passes, no cancellation); waves combined in order: deterministic.
//  * conv0_wgrad_part: 128 pixels per workgroup, wave = 32 pixels, dW[co][k] =
//    sum_p dz[p][co] x_p[k]: A = dz (M = output channels, K = pixels, loaded up front, coalesced),
//    B = the input windows (N = the 27 (ci, tap) columns) from the LDS halo. The 4 waves' tiles
//    are summed in order into one [64][27] partial per workgroup (OIHW order); conv0_wgrad_sum: the
//    partials summed in a fixed order -> dW.
//  Folds (each bit-equal to the separate launch it replaces; vgg_engine.cpp chooses them):
//    conv0_fwd<BATCH> builds the training batch in its halo load (make_batch's sampler index, label
//    gather and crop/flip/normalize of the uint8 images); conv0_wgrad_bn_part computes block 0's
//    BN-backward dZ in LDS instead of reading it; conv0_wgrad_sum can apply block 0's SGD step.
#include "common.h"
#include "launchers.h"
#include "sgd_device.h"

namespace {

constexpr int kCo = 64;
constexpr int kPix = 128;  // pixels per workgroup (4 image rows) = BN statistics tile rows
constexpr int kCols = 27 * kCo;
constexpr int kW = 32, kWP = kW + 2, kRows = kPix / kW, kPlane = (kRows + 2) * kWP;

typedef float f32x16 __attribute__((ext_vector_type(16)));

// input halo of image rows [h0 - 1, h0 + kRows + 1) x columns [-1, W + 1), channel-planar
// (xs[ci][row][col], ci < 3), zeros outside the image (conv padding 1); W = 32 (CIFAR)
__device__ __forceinline__ void load_halo_planar(const float* __restrict__ x, int b, int h0, int H, float* xs) {
  for (int i = threadIdx.x; i < kPlane; i += blockDim.x) {
    const int r = i / kWP, c = i - r * kWP;
    const int h = h0 - 1 + r, w = c - 1;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)kW)
      v = *reinterpret_cast<const float4*>(x + (((size_t)b * H + h) * kW + w) * 4);
    xs[i] = v.x;
    xs[kPlane + i] = v.y;
    xs[2 * kPlane + i] = v.z;
  }
}

// the same halo computed from the uint8 training images (make_batch's arithmetic: crop offsets and
// flip of the sample, (v / 255 - mean) / std), writing the tile's own rows to the block-0 input
__device__ __forceinline__ void load_halo_batch(const CsBatchSrc& src, int b, int h0, int H, int m0, float* xs) {
  const int64_t smp = src.perm != nullptr ? src.perm[*src.cursor * src.stride + b] : src.idx_in[b];
  if (m0 % (H * kW) == 0 && threadIdx.x == 0) {
    src.idx_out[b] = smp;
    src.ylab[b] = src.labels[smp];
  }
  const int dy = src.params[smp * 3 + 0], dx = src.params[smp * 3 + 1], fl = src.params[smp * 3 + 2];
  for (int i = threadIdx.x; i < kPlane; i += blockDim.x) {
    const int r = i / kWP, c = i - r * kWP;
    const int h = h0 - 1 + r, w = c - 1;
    float v[3] = {0.f, 0.f, 0.f};
    if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)kW) {
      const int sx = fl ? (31 - w) : w;
      const int py = h + dy - 4, px = sx + dx - 4;
      float u[3] = {0.f, 0.f, 0.f};
      if (py >= 0 && py < 32 && px >= 0 && px < 32) {
        const uint8_t* p = src.data + ((smp * 32 + py) * 32 + px) * 3;
        u[0] = p[0];
        u[1] = p[1];
        u[2] = p[2];
      }
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) v[ci] = (u[ci] / 255.0f - src.m[ci]) * src.inv[ci];
      if (r >= 1 && r <= kRows)
        *reinterpret_cast<float4*>(src.x_out + (((size_t)b * H + h) * kW + w) * 4) = make_float4(v[0], v[1], v[2], 0.f);
    }
    xs[i] = v[0];
    xs[kPlane + i] = v[1];
    xs[2 * kPlane + i] = v[2];
  }
}

// halo offset of column k = ci * 9 + tap of the (row 0, column 0) pixel's window
__host__ __device__ constexpr int win_off(int k) { return (k / 9) * kPlane + ((k % 9) / 3) * kWP + (k % 9) % 3; }

template <bool BATCH>
__global__ __launch_bounds__(256) void conv0_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, float* __restrict__ y,
                                                        float* __restrict__ stats, int H, CsBatchSrc src,
                                                        float* __restrict__ zero_bounds, int zero_slots,
                                                        float* __restrict__ rot_cur, float* __restrict__ rot_next,
                                                        unsigned rot_mask) {
  // the step's first launch also resets the F3 conv math's per-step operand bounds (one word per
  // shard, launchers.h CS_AMAX_*), which this step's BN launches then fold into, and makes the
  // weight bounds the last step's SGD launches produced current (cs_amax_rotate)
  {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const size_t o = (size_t)(i / CS_AMAX_SHARDS) * CS_AMAX_SLOT + (i % CS_AMAX_SHARDS) * CS_AMAX_STRIDE;
    if (zero_bounds != nullptr && i < zero_slots * CS_AMAX_SHARDS) zero_bounds[o] = 0.f;
    if (rot_cur != nullptr && i < 32 * CS_AMAX_SHARDS && ((rot_mask >> (i / CS_AMAX_SHARDS)) & 1u)) {
      rot_cur[o] = rot_next[o];
      rot_next[o] = 0.f;
    }
  }
  __shared__ float xs[3 * kPlane];
  __shared__ float red[4][kCo];
  __shared__ float mean_sh[kCo];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // image row of the tile
  const int m0 = blockIdx.x * kPix;
  const int b = m0 / (H * kW), h0 = (m0 / kW) % H;
  const int j = lane & 31, kh = lane >> 5;  // MFMA operand lane map: row/column j, k-half kh
  // B = weights [k][channel]: lane (k = 2s + kh, channel nt * 32 + j), k = 27 is padding
  float bw[2][14];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int st = 0; st < 14; ++st) {
      const int k = 2 * st + kh;
      bw[nt][st] = k < 27 ? w[(nt * 32 + j) * 27 + k] : 0.f;
    }
  f32x16 acc[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const float bv = bias != nullptr ? bias[nt * 32 + j] : 0.f;  // C column = channel nt * 32 + j
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[nt][g] = bv;
  }
  if constexpr (BATCH)
    load_halo_batch(src, b, h0, H, m0, xs);
  else
    load_halo_planar(x, b, h0, H, xs);
  __syncthreads();
  // A = windows [pixel j of image row wv][k]
  const float* xw = xs + wv * kWP + j;
#pragma unroll
  for (int st = 0; st < 14; ++st) {
    const int off = kh ? win_off(2 * st + 1) : win_off(2 * st);
    const float a = (2 * st + kh < 27) ? xw[off] : 0.f;
    acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bw[0][st], acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bw[1][st], acc[1], 0, 0, 0);
  }
  // D: lane (channel nt * 32 + j), register g = pixel (g & 3) + 8 (g >> 2) + 4 kh of the row;
  // each store instruction covers two full 128-byte channel runs
  float* yr = y + (size_t)(m0 + wv * kW) * kCo + j;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int g = 0; g < 16; ++g) yr[(size_t)((g & 3) + 8 * (g >> 2) + 4 * kh) * kCo + nt * 32] = acc[nt][g];
  if (stats == nullptr) return;
  // ---- tile statistics: lane sums its 16 pixels, + the other k-half (lane ^ 32), waves in order
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += acc[nt][g];
    t += __shfl_xor(t, 32);
    if (kh == 0) red[wv][nt * 32 + j] = t;
  }
  __syncthreads();
  if (tid < kCo) mean_sh[tid] = (((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid]) / (float)kPix;
  __syncthreads();
  float m2p[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const float mu = mean_sh[nt * 32 + j];
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const float d = acc[nt][g] - mu;
      t = fmaf(d, d, t);
    }
    m2p[nt] = t + __shfl_xor(t, 32);
  }
  __syncthreads();  // every wave read red before it is reused
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
    if (kh == 0) red[wv][nt * 32 + j] = m2p[nt];
  __syncthreads();
  if (tid < kCo) {
    const float m2 = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
    *reinterpret_cast<float2*>(stats + ((size_t)blockIdx.x * kCo + tid) * 2) = make_float2(mean_sh[tid], m2);
  }
}

__global__ __launch_bounds__(256) void conv0_wgrad_part_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ dz,
                                                               float* __restrict__ part, int H) {
  __shared__ float xs[3 * kPlane];
  __shared__ float red[4][kCols];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // image row of the tile
  const int m0 = blockIdx.x * kPix;
  const int b = m0 / (H * kW), h0 = (m0 / kW) % H;
  const int j = lane & 31, kh = lane >> 5;
  // A = dz^T [channel mt * 32 + j][pixel 2s + kh of the wave's row]: 32 coalesced loads, up front
  const float* dzp = dz + (size_t)(m0 + wv * kW + kh) * kCo + j;
  float ga[2][16];
#pragma unroll
  for (int st = 0; st < 16; ++st)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) ga[mt][st] = dzp[(size_t)(2 * st) * kCo + mt * 32];
  load_halo_planar(x, b, h0, H, xs);
  __syncthreads();
  // B = windows [pixel][column j = ci * 9 + tap]; columns 27..31 are zero
  const bool col_ok = j < 27;
  const float* xw = xs + wv * kWP + kh + (col_ok ? (j / 9) * kPlane + ((j % 9) / 3) * kWP + (j % 9) % 3 : 0);
  f32x16 acc[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[mt][g] = 0.f;
#pragma unroll
  for (int st = 0; st < 16; ++st) {
    const float bv = col_ok ? xw[2 * st] : 0.f;
    acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(ga[0][st], bv, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(ga[1][st], bv, acc[1], 0, 0, 0);
  }
  // D: lane (column j), register g = channel mt * 32 + (g & 3) + 8 (g >> 2) + 4 kh; the waves'
  // tiles summed in order through LDS into one [64][27] partial
  if (col_ok) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int g = 0; g < 16; ++g) red[wv][(mt * 32 + (g & 3) + 8 * (g >> 2) + 4 * kh) * 27 + j] = acc[mt][g];
  }
  __syncthreads();
  for (int e = tid; e < kCols; e += 256)
    part[(size_t)blockIdx.x * kCols + e] = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
}

// The same partial dW with block 0's BatchNorm backward folded in (dZ is never written to memory):
// the block first turns its 128 pixels' incoming gradient into dZ in LDS — G is the gradient of
// the 2x2-pooled output, so each unit is one pooling window x 4 channels: recompute relu(bn(y)),
// route G to the window's first maximum (if positive), dZ = k1 (g - k2 - x_hat k3) — the very
// expression and decisions of bn_device.h bwd_visit, so dZ has the same bits — then runs the MFMA
// loop with the A operand read from that tile. The tile's 4 image rows are 2 pooling rows.
constexpr int kDZP = kCo + 4;  // dZ tile pitch: lanes j read consecutive channels, k-halves 68 apart
__global__ __launch_bounds__(256) void conv0_wgrad_bn_part_kernel(
    const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ G,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ coef, float* __restrict__ part, int H) {
  __shared__ float xs[3 * kPlane];
  __shared__ float dzs[kPix * kDZP];  // reused as the waves' [4][64 * 27] partial tiles at the end
  static_assert(4 * kCols <= kPix * kDZP, "partial tiles alias the dZ tile");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = blockIdx.x * kPix;
  const int b = m0 / (H * kW), h0 = (m0 / kW) % H;
  const int j = lane & 31, kh = lane >> 5;
  load_halo_planar(x, b, h0, H, xs);
  // ---- dZ tile: 2 pooling rows x 16 windows x 16 channel quads = 512 units, 2 per thread
  constexpr int C4 = kCo / 4, Wo = kW / 2;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int u = tid + 256 * it;
    const int cq = u % C4, win = u / C4, pr = win / Wo, pc = win % Wo;
    const int ug = (b * (H / 2) + h0 / 2 + pr) * Wo + pc;  // pooled position
    const float4 g4 = reinterpret_cast<const float4*>(G)[(size_t)ug * C4 + cq];
    const float4 s4 = reinterpret_cast<const float4*>(scale)[cq], t4 = reinterpret_cast<const float4*>(shift)[cq];
    const float4 mu4 = reinterpret_cast<const float4*>(mean)[cq], is4 = reinterpret_cast<const float4*>(invstd)[cq];
    const float4 c0 = reinterpret_cast<const float4*>(coef)[3 * cq], c1 = reinterpret_cast<const float4*>(coef)[3 * cq + 1],
                 c2 = reinterpret_cast<const float4*>(coef)[3 * cq + 2];
    const float gin[4] = {g4.x, g4.y, g4.z, g4.w}, sc[4] = {s4.x, s4.y, s4.z, s4.w}, sh[4] = {t4.x, t4.y, t4.z, t4.w};
    const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, is[4] = {is4.x, is4.y, is4.z, is4.w};
    const float cf[12] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c2.x, c2.y, c2.z, c2.w};
    int px[4];  // tile pixels of the window in bwd_visit's order: (0,0) (0,1) (1,0) (1,1)
#pragma unroll
    for (int p = 0; p < 4; ++p) px[p] = (2 * pr + (p >> 1)) * kW + 2 * pc + (p & 1);
    float yv[4][4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const float4 v = reinterpret_cast<const float4*>(y)[(size_t)(m0 + px[p]) * C4 + cq];
      yv[p][0] = v.x; yv[p][1] = v.y; yv[p][2] = v.z; yv[p][3] = v.w;
    }
    float out[4][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float z[4];
      int am = 0;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        z[p] = fmaxf(yv[p][q] * sc[q] + sh[q], 0.f);
        if (p > 0 && z[p] > z[am]) am = p;
      }
      const float k1 = cf[3 * q], k2 = cf[3 * q + 1], k3 = cf[3 * q + 2];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float g = (p == am && z[p] > 0.f) ? gin[q] : 0.f;
        const float xh = (yv[p][q] - mu[q]) * is[q];
        out[p][q] = k1 * (g - k2 - xh * k3);
      }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p)
      *reinterpret_cast<float4*>(dzs + px[p] * kDZP + 4 * cq) = make_float4(out[p][0], out[p][1], out[p][2], out[p][3]);
  }
  __syncthreads();
  // ---- A = dZ^T [channel mt * 32 + j][pixel 2s + kh of the wave's row], from the LDS tile
  const float* dzp = dzs + (wv * kW + kh) * kDZP + j;
  const bool col_ok = j < 27;
  const float* xw = xs + wv * kWP + kh + (col_ok ? (j / 9) * kPlane + ((j % 9) / 3) * kWP + (j % 9) % 3 : 0);
  f32x16 acc[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[mt][g] = 0.f;
#pragma unroll
  for (int st = 0; st < 16; ++st) {
    const float bv = col_ok ? xw[2 * st] : 0.f;
    const float a0 = dzp[2 * st * kDZP], a1 = dzp[2 * st * kDZP + 32];
    acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bv, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bv, acc[1], 0, 0, 0);
  }
  __syncthreads();  // every wave's dZ reads are done: the tile becomes the partial buffer
  float* red = dzs;
  if (col_ok) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int g = 0; g < 16; ++g) red[wv * kCols + (mt * 32 + (g & 3) + 8 * (g >> 2) + 4 * kh) * 27 + j] = acc[mt][g];
  }
  __syncthreads();
  for (int e = tid; e < kCols; e += 256)
    part[(size_t)blockIdx.x * kCols + e] = ((red[e] + red[kCols + e]) + red[2 * kCols + e]) + red[3 * kCols + e];
}

// dW[i] = sum over the nb partials in a fixed order: workgroup = 16 columns x 16 row slices, slice s
// sums rows s, s + 16, ... (16 loads in flight), then the 16 slices in order. With an SGD range
// (sgd.n > 0: block 0's parameters, dW at w_rel within it) each finished column also takes its
// SGD step here, and one extra workgroup updates the range's other parameters (their gradients
// are final) and bumps the batch cursor: the step's last separate optimizer launch disappears
// (the same cs_sgd::step1 on the same values as the flat pass: bit-equal)
__global__ __launch_bounds__(256) void conv0_wgrad_sum_kernel(const float* __restrict__ part, int nb,
                                                             float* __restrict__ dw, CsSgdTail sgd, int w_rel,
                                                             int64_t* __restrict__ counter) {
  constexpr int NCB = (kCols + 15) / 16;  // column workgroups
  if ((int)blockIdx.x == NCB) {           // the range's other parameters + the cursor
    if (counter != nullptr && threadIdx.x == 0) *counter += 1;
    for (int64_t i = threadIdx.x; i < sgd.n; i += 256) {
      if (i >= w_rel && i < w_rel + kCols) continue;
      float pv = sgd.p[i], mv = sgd.first ? 0.f : sgd.m[i];
      cs_sgd::step1(pv, sgd.g[i], mv, sgd.lr, sgd.mom, sgd.wd, sgd.damp, 1.0f, sgd.first);
      sgd.p[i] = pv;
      if (sgd.mom != 0.f) sgd.m[i] = mv;
    }
    return;
  }
  __shared__ float red[16][16];
  const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + cl;
  float s = 0.f;
  if (col < kCols) {
    for (int r0 = sl; r0 < nb; r0 += 16 * 16) {
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int r = r0 + 16 * j;
        v[j] = r < nb ? part[(size_t)r * kCols + col] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) s += v[j];
    }
  }
  red[sl][cl] = s;
  __syncthreads();
  if (sl == 0 && col < kCols) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) t += red[j][cl];
    dw[col] = t;
    if (sgd.n > 0) {
      const int64_t i = w_rel + col;
      float pv = sgd.p[i], mv = sgd.first ? 0.f : sgd.m[i];
      cs_sgd::step1(pv, t, mv, sgd.lr, sgd.mom, sgd.wd, sgd.damp, 1.0f, sgd.first);
      sgd.p[i] = pv;
      if (sgd.mom != 0.f) sgd.m[i] = mv;
    }
  }
}

}  // namespace

int cs_conv0_tile_rows() { return kPix; }

size_t cs_conv0_wgrad_part_floats(int B, int H, int W) {
  return (size_t)((B * H * W) / kPix) * kCols;
}

hipError_t cs_conv0_fwd(const float* x, const float* w, const float* bias, float* y, float* stats, int B, int H,
                        int W, int Cout, hipStream_t stream, const CsBatchSrc* batch, float* zero_bounds,
                        int zero_slots, float* rot_cur, float* rot_next, unsigned rot_mask) {
  if (W != 32 || Cout != kCo || (H * W) % kPix != 0) return hipErrorInvalidValue;
  if ((zero_bounds != nullptr && (int64_t)zero_slots * CS_AMAX_SHARDS > (int64_t)(B * H * W) / kPix * 256) ||
      (rot_cur != nullptr && 32 * CS_AMAX_SHARDS > (int64_t)(B * H * W) / kPix * 256))
    return hipErrorInvalidValue;
  if (batch != nullptr) {
    if (H != 32 || (batch->perm == nullptr) == (batch->idx_in == nullptr) ||
        (batch->perm != nullptr && batch->cursor == nullptr))
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(conv0_fwd_kernel<true>, dim3((B * H * W) / kPix), dim3(256), 0, stream, nullptr, w, bias, y,
                       stats, H, *batch, zero_bounds, zero_slots, rot_cur, rot_next, rot_mask);
  } else {
    hipLaunchKernelGGL(conv0_fwd_kernel<false>, dim3((B * H * W) / kPix), dim3(256), 0, stream, x, w, bias, y, stats,
                       H, CsBatchSrc{}, zero_bounds, zero_slots, rot_cur, rot_next, rot_mask);
  }
  return hipGetLastError();
}

static hipError_t conv0_sum(const float* part, int nb, float* dw, const CsSgdTail* sgd, int w_rel,
                            int64_t* counter, hipStream_t stream) {
  CsSgdTail t{};
  if (sgd != nullptr) {
    if (sgd->n < w_rel + kCols || w_rel < 0) return hipErrorInvalidValue;
    t = *sgd;
  }
  const int ncb = (kCols + 15) / 16;
  hipLaunchKernelGGL(conv0_wgrad_sum_kernel, dim3(ncb + (t.n > 0 ? 1 : 0)), dim3(256), 0, stream, part, nb, dw, t,
                     w_rel, t.n > 0 ? counter : nullptr);
  return hipGetLastError();
}

hipError_t cs_conv0_wgrad(const float* x, const float* dz, float* part, float* dw, int B, int H, int W, int Cout,
                          hipStream_t stream, const CsSgdTail* sgd, int w_rel, int64_t* counter) {
  if (W != 32 || Cout != kCo || (H * W) % kPix != 0) return hipErrorInvalidValue;
  const int nb = (B * H * W) / kPix;
  hipLaunchKernelGGL(conv0_wgrad_part_kernel, dim3(nb), dim3(256), 0, stream, x, dz, part, H);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  return conv0_sum(part, nb, dw, sgd, w_rel, counter, stream);
}

hipError_t cs_conv0_wgrad_bn(const float* x, const float* y, const float* G, const float* scale, const float* shift,
                             const float* mean, const float* invstd, const float* coef, float* part, float* dw, int B,
                             int H, int W, int Cout, hipStream_t stream, const CsSgdTail* sgd, int w_rel,
                             int64_t* counter) {
  if (W != 32 || Cout != kCo || (H * W) % kPix != 0 || H % 4 != 0) return hipErrorInvalidValue;
  const int nb = (B * H * W) / kPix;
  hipLaunchKernelGGL(conv0_wgrad_bn_part_kernel, dim3(nb), dim3(256), 0, stream, x, y, G, scale, shift, mean, invstd,
                     coef, part, H);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  return conv0_sum(part, nb, dw, sgd, w_rel, counter, stream);
}
