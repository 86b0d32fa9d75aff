// bf16 NHWC convolution as implicit GEMM on CDNA4 bf16 MFMA (v_mfma_f32_32x32x16_bf16, f32
// accumulate) for the ResNet family's channels-last path — any R x S kernel, stride and padding,
// C and Cout multiples of 32. Replaces the im2col gather + library GEMM (+ col2im) of
// ops/cnn_nhwc.py for those convolutions: the patch matrix is never written to memory, each
// K-step gathers its rows straight from the activation (the 3x3 taps re-read from L2).
// (Reference layer: nn.Conv2d of torchvision's ResNet, BASELINE.json config 4)
//
//   FWD  : y [M = B*Ho*Wo][N = Co]  = A . W^T,  A[m][k] = x[b, oh*st-pad+r, ow*st-pad+s, c]
//   DGRAD: dx[M = B*H*W][N = C]     = A . Wt^T, A[m][k] = dy[b, (ih+pad-r)/st, (iw+pad-s)/st, co]
//          (zero unless both divide), Wt = W as [C][R][S][Co] (the caller's transpose)
//   WGRAD: dW[M = Co][N = R*S*C]    = dy^T . im2col(x) over K = B*Ho*Wo pixels, split-K into
//          fp32 partial slabs [splits][Co][R*S*C], summed in split order by conv_nhwc_reduce
//   k = (r, s, c) with c fastest (FWD / WGRAD), (r, s, co) for DGRAD; a 32-wide K-step never
//   crosses a tap (C, Cout % 32 == 0), so its tap is wave-uniform.
//   C4 (the stem: 4-channel image, FWD / WGRAD only): the taps of a kernel row are padded to 8, so
//   k = (r, s < 8, c < 4), K = R*32 and a K-step is one kernel row r; a 16-byte chunk is two
//   adjacent taps = two 8-byte pixel loads, each with its own bounds check (the weight's taps
//   s >= S are zero; WGRAD's columns for them are computed and dropped by the caller).
//
// Tiling: 256 threads = 4 waves (2 x 2), block tile 128 x BN (BN 64 / 128), K-step 32, wave tile
// 64 x BN/2 of 32x32 MFMA tiles. Global -> registers (next K-step's loads in flight during this
// one's MFMAs) -> LDS double buffer, one barrier per K-step. Operands whose K runs along rows
// (K-contiguous: FWD/DGRAD A and B) sit in LDS as [row][32 + 8]; pixel-major WGRAD operands
// (K-major) as [k][cols + 32] and reach the MFMA through ds_read_b64_tr_b16 (the gfx950
// transpose read). Every global access goes through a buffer descriptor: padding and
// out-of-range elements get an offset past the range and load zeros / drop stores — no branches.
#include <algorithm>

#include "common.h"
#include "launchers.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int kOOB = 0x7ffffff0;
constexpr int BK = 32;

__device__ __forceinline__ rsrc_t rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 bload16(rsrc_t r, int off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ uint2 bload8(rsrc_t r, int off) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
// two 4-channel pixels (iw, iw + 1) of image row (b*H + ih): 16 bytes, each half bounds-checked
__device__ __forceinline__ uint4 pix_pair(rsrc_t r, bool okr, int rowbase, int iw, int W) {
  const int o = (rowbase * W + iw) * 8;
  const uint2 lo = bload8(r, okr && (unsigned)iw < (unsigned)W ? o : kOOB);
  const uint2 hi = bload8(r, okr && (unsigned)(iw + 1) < (unsigned)W ? o + 8 : kOOB);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

template <int MODE>
struct Ops {  // which operands are K-contiguous in memory (A_G, B_KC) and in their LDS image (A_KC, B_KC)
  // (WGRAD's A, dy^T, arrives pixel-major and is transposed on its way into a K-contiguous image:
  // 8 two-byte LDS stores per chunk; the pixel-major image + transpose read is the B path)
  static constexpr bool A_G = MODE != CS_CONV_WGRAD, A_KC = true, B_KC = MODE != CS_CONV_WGRAD;
};

template <int BM_, int BN, int MODE>
struct Geo {
  static constexpr int BM = BM_, NT = 256;
  static constexpr bool A_G = Ops<MODE>::A_G, A_KC = Ops<MODE>::A_KC, B_KC = Ops<MODE>::B_KC;
  // LDS images in bf16 elements: K-contiguous [rows][BK + 8], K-major [BK][cols + 32]
  static constexpr int PA = A_KC ? BK + 8 : BM + 32, PB = B_KC ? BK + 8 : BN + 32;
  static constexpr int A_EL = A_KC ? BM * PA : BK * PA, B_EL = B_KC ? BN * PB : BK * PB;
  static constexpr int STAGE = A_EL + B_EL;
  static constexpr int AC = BM * BK / 8 / NT, BC = BN * BK / 8 / NT;  // 16-byte chunks per thread
  static constexpr int RM = BM / 64, RN = BN / 64, WM = BM / 2, WN = BN / 2;
  static constexpr size_t LDS = 2 * (size_t)STAGE * 2;
};

// chunk q of a staged operand image: K-contiguous -> (row, 8-wide k group), K-major -> (k row,
// 8-wide column group)
template <bool KC, int ROWS>
__device__ __forceinline__ void chunk_pos(int q, int& a, int& b) {
  if (KC) {
    a = q >> 2;  // BK / 8 = 4 groups per row
    b = q & 3;
  } else {
    constexpr int G = ROWS / 8;
    a = q / G;
    b = q % G;
  }
}

template <int BM, int BN, int MODE, bool C4>
struct Stager {
  using G = Geo<BM, BN, MODE>;
  rsrc_t ra, rb;
  // per chunk: fixed parts of the gather (unpacked once; the K-step adds its tap / channel base)
  int a0[G::AC], a1[G::AC], a2[G::AC];  // FWD/DGRAD A: b*H(o), spatial bases; WGRAD A: column
  int b0[G::BC];                        // B: row (n) or column group offset
  int alds[G::AC], blds[G::BC];         // LDS element offsets
  uint4 va[G::AC], vb[G::BC];

  __device__ void init(const CsConvNhwcArgs& p, int m0, int n0) {
#pragma unroll
    for (int i = 0; i < G::AC; ++i) {
      const int q = threadIdx.x + G::NT * i;
      int r, c;
      chunk_pos<G::A_G, G::BM>(q, r, c);
      if constexpr (MODE == CS_CONV_FWD) {  // output pixel m -> (b, oh*st - pad, ow*st - pad)
        const int m = m0 + r;
        const int ow = m % p.Wo, t = m / p.Wo, oh = t % p.Ho, b = t / p.Ho;
        a0[i] = m < p.M ? b * p.H : -(1 << 28);
        a1[i] = oh * p.st - p.pad;
        a2[i] = ow * p.st - p.pad;
        alds[i] = r * G::PA + 8 * c;
      } else if constexpr (MODE == CS_CONV_DGRAD) {  // input pixel m -> (b, ih + pad, iw + pad)
        const int m = m0 + r;
        const int iw = m % p.W, t = m / p.W, ih = t % p.H, b = t / p.H;
        a0[i] = m < p.M ? b * p.Ho : -(1 << 28);
        a1[i] = ih + p.pad;
        a2[i] = iw + p.pad;
        alds[i] = r * G::PA + 8 * c;
      } else {  // WGRAD A = dy^T: k row = pixel (added per K-step), columns = output channels;
                // stored transposed: element j of the chunk -> image row 8c + j, column r
        a0[i] = r;
        a1[i] = m0 + 8 * c;
        a2[i] = 0;
        alds[i] = 8 * c * G::PA + r;
      }
    }
#pragma unroll
    for (int i = 0; i < G::BC; ++i) {
      const int q = threadIdx.x + G::NT * i;
      int r, c;
      chunk_pos<G::B_KC, BN>(q, r, c);
      if constexpr (MODE != CS_CONV_WGRAD) {  // weights [N][K], K-contiguous
        const int n = n0 + r;
        b0[i] = n < p.N ? n * p.K + 8 * c : -1;
        blds[i] = r * G::PB + 8 * c;
      } else {  // WGRAD B = im2col(x): k row = pixel, columns n = (r, s, c) in groups of 8
        b0[i] = (r << 16) | (n0 + 8 * c);
        blds[i] = r * G::PB + 8 * c;
      }
    }
    const int64_t xb = (int64_t)p.B * p.H * p.W * p.C * 2, yb = (int64_t)p.B * p.Ho * p.Wo * p.Co * 2;
    if constexpr (MODE == CS_CONV_FWD) {
      ra = rsrc(p.x, xb);
      rb = rsrc(p.w, (int64_t)p.N * p.K * 2);
    } else if constexpr (MODE == CS_CONV_DGRAD) {
      ra = rsrc(p.dy, yb);
      rb = rsrc(p.w, (int64_t)p.N * p.K * 2);
    } else {
      ra = rsrc(p.dy, yb);
      rb = rsrc(p.x, xb);
    }
  }

  // global -> registers for the K-step starting at k0 (GEMM K index)
  __device__ __forceinline__ void load(const CsConvNhwcArgs& p, int k0) {
    if constexpr (MODE == CS_CONV_FWD && C4) {
      const int r = k0 >> 5;  // one kernel row per K-step; chunk cq = taps 2cq, 2cq + 1
#pragma unroll
      for (int i = 0; i < G::AC; ++i) {
        const int ih = a1[i] + r, cq = (threadIdx.x + G::NT * i) & 3;
        const bool okr = a0[i] >= 0 && (unsigned)ih < (unsigned)p.H;
        va[i] = pix_pair(ra, okr, a0[i] + ih, a2[i] + 2 * cq, p.W);
      }
    } else if constexpr (MODE == CS_CONV_FWD) {
      const int tap = k0 / p.C, c0 = k0 - tap * p.C;
      const int r = tap / p.S, s = tap - r * p.S;
#pragma unroll
      for (int i = 0; i < G::AC; ++i) {
        const int ih = a1[i] + r, iw = a2[i] + s;
        const int cq = (threadIdx.x + G::NT * i) & 3;
        const bool ok = a0[i] >= 0 && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        va[i] = bload16(ra, ok ? (((a0[i] + ih) * p.W + iw) * p.C + c0 + 8 * cq) * 2 : kOOB);
      }
    } else if constexpr (MODE == CS_CONV_DGRAD) {
      const int tap = k0 / p.Co, c0 = k0 - tap * p.Co;
      const int r = tap / p.S, s = tap - r * p.S;
#pragma unroll
      for (int i = 0; i < G::AC; ++i) {
        const int th = a1[i] - r, tw = a2[i] - s;
        const int oh = th / p.st, ow = tw / p.st;
        const int cq = (threadIdx.x + G::NT * i) & 3;
        const bool ok = a0[i] >= 0 && th >= 0 && tw >= 0 && oh * p.st == th && ow * p.st == tw && oh < p.Ho &&
                        ow < p.Wo;
        va[i] = bload16(ra, ok ? (((a0[i] + oh) * p.Wo + ow) * p.Co + c0 + 8 * cq) * 2 : kOOB);
      }
    } else {
#pragma unroll
      for (int i = 0; i < G::AC; ++i) {
        const int pix = k0 + a0[i];
        const bool ok = pix < p.K && a1[i] < p.M;
        va[i] = bload16(ra, ok ? (pix * p.Co + a1[i]) * 2 : kOOB);
      }
    }
    if constexpr (MODE != CS_CONV_WGRAD) {
#pragma unroll
      for (int i = 0; i < G::BC; ++i) vb[i] = bload16(rb, b0[i] >= 0 ? (b0[i] + k0) * 2 : kOOB);
    } else if constexpr (C4) {
#pragma unroll
      for (int i = 0; i < G::BC; ++i) {
        const int pix = k0 + (b0[i] >> 16), n = b0[i] & 0xffff;
        const int ow = pix % p.Wo, t = pix / p.Wo, oh = t % p.Ho, b = t / p.Ho;
        const int r = n >> 5, s = (n >> 2) & 7;  // n = (r, s, c): a chunk is taps s, s + 1 of row r
        const int ih = oh * p.st - p.pad + r;
        const bool okr = pix < p.K && n < p.N && (unsigned)ih < (unsigned)p.H;
        vb[i] = pix_pair(rb, okr, b * p.H + ih, ow * p.st - p.pad + s, p.W);
      }
    } else {
#pragma unroll
      for (int i = 0; i < G::BC; ++i) {
        const int pix = k0 + (b0[i] >> 16), n = b0[i] & 0xffff;
        const int ow = pix % p.Wo, t = pix / p.Wo, oh = t % p.Ho, b = t / p.Ho;
        const int tap = n / p.C, c = n - tap * p.C;
        const int r = tap / p.S, s = tap - r * p.S;
        const int ih = oh * p.st - p.pad + r, iw = ow * p.st - p.pad + s;
        const bool ok = pix < p.K && n < p.N && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        vb[i] = bload16(rb, ok ? (((b * p.H + ih) * p.W + iw) * p.C + c) * 2 : kOOB);
      }
    }
  }

  __device__ __forceinline__ void store(__bf16* As, __bf16* Bs) const {
#pragma unroll
    for (int i = 0; i < G::AC; ++i) {
      if constexpr (G::A_G) {
        *reinterpret_cast<uint4*>(As + alds[i]) = va[i];
      } else {
        const unsigned w[4] = {va[i].x, va[i].y, va[i].z, va[i].w};
        unsigned short* a = reinterpret_cast<unsigned short*>(As + alds[i]);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j * G::PA] = (unsigned short)(w[j >> 1] >> (16 * (j & 1)));
      }
    }
#pragma unroll
    for (int i = 0; i < G::BC; ++i) *reinterpret_cast<uint4*>(Bs + blds[i]) = vb[i];
  }
};

// MFMA fragments (32x32x16: lane row / column = lane & 31, element j <-> k = 16*(lane >> 5) +
// 8*h + j for the h-th 16-wide half of the K-step — A and B read with the same map, so the
// permutation of K cancels) of R 32-row groups from a staged image
template <int R, bool KC, int P>
__device__ __forceinline__ void frag(const __bf16* img, int base, int h, int lane, bf16x8 (&f)[R]) {
#pragma unroll
  for (int i = 0; i < R; ++i) {
    if constexpr (KC) {
      const int row = base + i * 32 + (lane & 31);
      f[i] = *reinterpret_cast<const bf16x8*>(img + row * P + 16 * (lane >> 5) + 8 * h);
    } else {
      // transpose read: in each 16-lane group, 4 lanes x 4 k rows of a 4 x 4 block
      const int grp = lane >> 4, l16 = lane & 15;
      const int col = base + i * 32 + 16 * (grp & 1) + 4 * (l16 & 3);
      const int kr = 16 * (grp >> 1) + 8 * h + (l16 >> 2);
      const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(img + kr * P + col));
      const i16x4 hi =
          __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(img + (kr + 4) * P + col));
      f[i] = __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo), __builtin_bit_cast(bf16x4, hi), 0, 1, 2, 3, 4, 5, 6,
                                     7);
    }
  }
}

template <int BM, int BN, int MODE, bool C4>
__global__ __launch_bounds__(256) void conv_nhwc_kernel(CsConvNhwcArgs p) {
  using G = Geo<BM, BN, MODE>;
  extern __shared__ __attribute__((aligned(16))) __bf16 lds[];
  const int ntn = (p.N + BN - 1) / BN, ntiles = ((p.M + G::BM - 1) / G::BM) * ntn;
  const int nsplit = (p.ksteps + p.ksteps_per_split - 1) / p.ksteps_per_split;
  const int lin = blockIdx.x;
  const int split = lin / ntiles;
  const int tile = cs::xcd_remap(lin % ntiles, ntiles);
  const int mt = tile / ntn, nt = tile - mt * ntn;
  const int m0 = mt * G::BM, n0 = nt * BN;
  const int kb = split * p.ksteps_per_split, ke = min(p.ksteps, kb + p.ksteps_per_split);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wm = wv >> 1, wn = wv & 1;

  f32x16 acc[G::RM][G::RN];
#pragma unroll
  for (int i = 0; i < G::RM; ++i)
#pragma unroll
    for (int j = 0; j < G::RN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  Stager<BM, BN, MODE, C4> st;
  st.init(p, m0, n0);
  if (kb < ke) {
    st.load(p, kb * BK);
    st.store(lds, lds + G::A_EL);
  }
  __syncthreads();
  for (int t = kb; t < ke; ++t) {
    const int cur = (t - kb) & 1;
    if (t + 1 < ke) st.load(p, (t + 1) * BK);  // next K-step's gathers in flight under the MFMAs
    const __bf16* As = lds + cur * G::STAGE;
    const __bf16* Bs = As + G::A_EL;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 af[G::RM], bfr[G::RN];
      frag<G::RM, G::A_KC, G::PA>(As, wm * G::WM, h, lane, af);
      frag<G::RN, G::B_KC, G::PB>(Bs, wn * G::WN, h, lane, bfr);
#pragma unroll
      for (int i = 0; i < G::RM; ++i)
#pragma unroll
        for (int j = 0; j < G::RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < ke) st.store(lds + (cur ^ 1) * G::STAGE, lds + (cur ^ 1) * G::STAGE + G::A_EL);
    __syncthreads();
  }

  // epilogue (C/D map: col = lane & 31, row = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5))
  if constexpr (MODE == CS_CONV_WGRAD) {
    float* dst = p.dw + (size_t)split * p.M * p.N;
    const rsrc_t ro = rsrc(dst, (int64_t)p.M * p.N * 4);
#pragma unroll
    for (int i = 0; i < G::RM; ++i)
#pragma unroll
      for (int j = 0; j < G::RN; ++j) {
        const int n = n0 + wn * G::WN + j * 32 + (lane & 31);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * G::WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          // (copy the element first: hipcc 7.2 lowered bit_cast of an indexed f32x16 element
          // to element 0 for every e — all 16 stores wrote a0)
          const float v = acc[i][j][e];
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), ro,
                                                (m < p.M && n < p.N) ? (m * p.N + n) * 4 : kOOB, 0, 0);
        }
      }
  } else {
    const rsrc_t ro = rsrc(p.y, (int64_t)p.M * p.N * 2);
#pragma unroll
    for (int i = 0; i < G::RM; ++i)
#pragma unroll
      for (int j = 0; j < G::RN; ++j) {
        const int n = n0 + wn * G::WN + j * 32 + (lane & 31);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * G::WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          const __bf16 v = (__bf16)acc[i][j][e];
          __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, v), ro,
                                                (m < p.M && n < p.N) ? (m * p.N + n) * 2 : kOOB, 0, 0);
        }
      }
  }
}

// dW = sum of the split slabs, fp32 [M][N]: a block is CB float4 columns x SL split lanes (CB*SL =
// 256); lane l sums slabs l, l + SL, ... in order, then the SL lane sums are added in lane order
// through LDS — a fixed order for a given split count (SL is a function of it): deterministic. The
// stem's weight gradient has hundreds of slabs over a small [64][224] output, so the slabs are
// spread over lanes as well as columns.
__global__ __launch_bounds__(256) void conv_nhwc_reduce_kernel(const float* __restrict__ part, int splits, int SL,
                                                               int64_t n4, float* __restrict__ out) {
  __shared__ float4 sh[256];
  const int CB = 256 / SL, cl = threadIdx.x % CB, sl = threadIdx.x / CB;
  const int64_t i = (int64_t)blockIdx.x * CB + cl;
  const float4* p4 = reinterpret_cast<const float4*>(part);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4)
    for (int z = sl; z < splits; z += SL) {
      const float4 t = p4[(int64_t)z * n4 + i];
      a.x += t.x; a.y += t.y; a.z += t.z; a.w += t.w;
    }
  sh[threadIdx.x] = a;
  __syncthreads();
  if (sl != 0 || i >= n4) return;
  for (int l = 1; l < SL; ++l) {
    const float4 t = sh[l * CB + cl];
    a.x += t.x; a.y += t.y; a.z += t.z; a.w += t.w;
  }
  reinterpret_cast<float4*>(out)[i] = a;
}

template <int BM, int BN, int MODE, bool C4 = false>
hipError_t launch(const CsConvNhwcArgs& p, int splits, hipStream_t stream) {
  using G = Geo<BM, BN, MODE>;
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  hipLaunchKernelGGL((conv_nhwc_kernel<BM, BN, MODE, C4>), dim3(tiles * splits), dim3(256), G::LDS, stream, p);
  return hipGetLastError();
}

}  // namespace

// out[n] = sum over z of part[z][n] (z in order within each split lane, lanes in order): the
// deterministic slab sum of the weight-gradient GEMMs, also used by ops/cnn_nhwc._wgrad for its
// row-chunk partials (n % 4 == 0, 16-byte aligned buffers)
hipError_t cs_slab_sum(const float* part, int splits, int64_t n, float* out, hipStream_t stream) {
  if (n % 4 || splits < 1) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  int SL = 1;
  while (SL < 16 && SL * 32 < splits) SL *= 2;
  const int64_t blocks = (n4 + 256 / SL - 1) / (256 / SL);
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(conv_nhwc_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, part, splits, SL, n4, out);
  return hipGetLastError();
}

int cs_conv_nhwc_splits(int mode, int B, int H, int W, int C, int Co, int R, int S, int st, int pad) {
  if (mode != CS_CONV_WGRAD) return 1;
  const int Ho = (H + 2 * pad - R) / st + 1, Wo = (W + 2 * pad - S) / st + 1;
  const int64_t pix = (int64_t)B * Ho * Wo, ksteps = (pix + BK - 1) / BK;
  const int64_t kc = C == 4 ? (int64_t)R * 32 : (int64_t)R * S * C;
  const int64_t tiles = (int64_t)((Co + 127) / 128) * ((kc + 127) / 128);
  int64_t s = 1;  // ~2 waves of 256 CUs, >= 8 K-steps per split, slabs within 1 GiB
  while (tiles * s * 2 <= 1024 && ksteps / (2 * s) >= 8 && 2 * s * Co * kc * 4 <= (1ll << 30)) s *= 2;
  return (int)s;
}

hipError_t cs_conv_nhwc(int mode, const CsConvNhwcArgs& in, int splits, hipStream_t stream) {
  CsConvNhwcArgs p = in;
  // C4: the 4-channel stem, forward and weight gradient, kernel rows of at most 8 taps
  const bool c4 = p.C == 4 && p.S <= 8 && mode != CS_CONV_DGRAD;
  if ((p.C % 32 && !c4) || p.Co % 32 || p.R < 1 || p.S < 1 || p.st < 1 || p.pad < 0) return hipErrorInvalidValue;
  p.Ho = (p.H + 2 * p.pad - p.R) / p.st + 1;
  p.Wo = (p.W + 2 * p.pad - p.S) / p.st + 1;
  if (p.Ho < 1 || p.Wo < 1) return hipErrorInvalidValue;
  const int64_t xe = (int64_t)p.B * p.H * p.W * p.C, ye = (int64_t)p.B * p.Ho * p.Wo * p.Co;
  const int64_t kc = c4 ? (int64_t)p.R * 32 : (int64_t)p.R * p.S * p.C;
  if (mode == CS_CONV_FWD) {
    p.M = (int)((int64_t)p.B * p.Ho * p.Wo);
    p.N = p.Co;
    p.K = (int)kc;
  } else if (mode == CS_CONV_DGRAD) {
    p.M = (int)((int64_t)p.B * p.H * p.W);
    p.N = p.C;
    p.K = p.R * p.S * p.Co;
  } else {
    p.M = p.Co;
    p.N = (int)kc;
    p.K = (int)((int64_t)p.B * p.Ho * p.Wo);
    if (kc > 0xffff) return hipErrorInvalidValue;  // packed column index in the WGRAD gather
  }
  // 32-bit byte offsets in every buffer descriptor
  if (2 * std::max(xe, ye) >= 0x7ffffff0ll || 2 * (int64_t)p.Co * kc >= 0x7ffffff0ll) return hipErrorInvalidValue;
  p.ksteps = (p.K + BK - 1) / BK;
  if (mode != CS_CONV_WGRAD) splits = 1;
  if (splits < 1) splits = 1;
  if (splits > p.ksteps) splits = p.ksteps;
  p.ksteps_per_split = (p.ksteps + splits - 1) / splits;
  splits = (p.ksteps + p.ksteps_per_split - 1) / p.ksteps_per_split;
  if (mode == CS_CONV_WGRAD && (p.dw == nullptr || (int64_t)splits * p.M * p.N * 4 >= 0x7ffffff0ll))
    return hipErrorInvalidValue;
  if (mode != CS_CONV_WGRAD && p.y == nullptr) return hipErrorInvalidValue;
  const bool wide = p.N >= 128 && p.N % 128 == 0;
  hipError_t e;
  if (c4 && mode == CS_CONV_FWD)
    e = wide ? launch<128, 128, CS_CONV_FWD, true>(p, 1, stream) : launch<128, 64, CS_CONV_FWD, true>(p, 1, stream);
  else if (c4)
    e = p.M <= 64 ? launch<64, 64, CS_CONV_WGRAD, true>(p, splits, stream)
                  : launch<128, 64, CS_CONV_WGRAD, true>(p, splits, stream);
  else if (mode == CS_CONV_FWD)
    e = wide ? launch<128, 128, CS_CONV_FWD>(p, 1, stream) : launch<128, 64, CS_CONV_FWD>(p, 1, stream);
  else if (mode == CS_CONV_DGRAD)
    e = wide ? launch<128, 128, CS_CONV_DGRAD>(p, 1, stream) : launch<128, 64, CS_CONV_DGRAD>(p, 1, stream);
  else if (p.M <= 64)  // 64 output channels: a 64-row tile (no half-empty MFMA rows)
    e = wide ? launch<64, 128, CS_CONV_WGRAD>(p, splits, stream) : launch<64, 64, CS_CONV_WGRAD>(p, splits, stream);
  else
    e = wide ? launch<128, 128, CS_CONV_WGRAD>(p, splits, stream) : launch<128, 64, CS_CONV_WGRAD>(p, splits, stream);
  if (e != hipSuccess || mode != CS_CONV_WGRAD) return e;
  // the caller's dw_out receives the split-ordered sum (slabs in p.dw)
  return cs_slab_sum(p.dw, splits, (int64_t)p.M * p.N, p.dw_out, stream);
}
