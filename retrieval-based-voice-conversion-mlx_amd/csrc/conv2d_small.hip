// 3x3 / pad 1 2-D convolution for few channels (C_in, N in {16, 32}) on v_mfma_f32_16x16x4_f32 (exact f32), and in
// the two-plane fp16 split on v_mfma_f32_16x16x32_f16 (k_conv2d_h16 below, the default arithmetic).
//
// The RMVPE U-Net's outer levels (RMVPE.py:13-57 ConvBlockRes at 16 and 32 channels over 1568 x 128 and
// 784 x 64 NHWC images) are 4x under-filled on the general kernel's 32x32x2 tiles (N = 16 fills half a
// 32-wide tile, C_in = 16 half a 32-channel chunk: 9.6 TF measured). Here the contraction index is
// (tap, channel) with a 16x16 output fragment per MFMA:
//   * a block stages a PIX-pixel tile of the image (RH full rows of W pixels) with its 1-pixel halo in
//     LDS once, channels contiguous (+4 floats per pixel so a quarter-wave's 16-B reads hit distinct
//     banks), and all 9 x N x C_in weights;
//   * wave w owns PIX/4 pixels as 16-pixel fragments; lane l supplies A = X[pixel l&15][4(l>>4) + j] and
//     B = W[tap][n l&15][4(l>>4) + j] for MFMA j: one ds_read_b128 per operand feeds 4 MFMAs;
//   * the epilogue (bias, act, residual) is the general kernel's, applied per output element.
// Exact f32 (MFMA f32 = fmaf chain), so results equal the general path up to summation order.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "rvcx_kernels.h"
#include "split_bf16.h"

namespace rvcx {

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));

}  // namespace

constexpr int SIT = 17;  // staging rounds of 256 float4 per block: (RH + 2) x (W + 2) x CIN / 4 <= 17 x 256 (all U-Net levels)

template <int CIN, int NOUT, int PIX>
__global__ __launch_bounds__(256) void k_conv2d_small(const ConvArgs a, const int RH) {
  constexpr int CP = CIN + 4;   // LDS floats per pixel
  constexpr int NT = NOUT / 16;  // 16-wide output fragments
  constexpr int CG = CIN / 16;   // 16-channel groups
  constexpr int TPW = PIX / 64;  // 16-pixel fragments per wave
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int W = a.W_out, H = a.T_out;
  const int AW = W + 2;
  float* As = sm;                                   // [RH + 2][W + 2][CP]
  float* Bs = sm + (size_t)(RH + 2) * AW * CP;      // [9][NOUT][CP]
  const int b = blockIdx.z;
  const int h0 = blockIdx.x * RH;
  const float* X = a.x + (long long)b * a.x_bs;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // ---- stage the halo tile and the weights: every thread's loads are issued before its first LDS store (the
  // tile is <= SIT rounds of 256 float4), so a block waits for one load latency instead of one per round
  const int rows = RH + 2;
  const int na = rows * AW * (CIN / 4);
  constexpr int NW = 9 * NOUT * (CIN / 4);
  constexpr int WIT = (NW + 255) / 256;
  {
    f32x4 v[SIT];
    f32x4 wv[WIT];
#pragma unroll
    for (int it = 0; it < SIT; ++it) {
      const int idx = it * 256 + tid;
      const int q = idx % (CIN / 4);
      const int pix = idx / (CIN / 4);
      const int r = pix / AW, cc = pix - r * AW;
      const int gh = h0 - 1 + r, gw = cc - 1;
      v[it] = (idx < na && gh >= 0 && gh < H && gw >= 0 && gw < W)
                  ? *reinterpret_cast<const f32x4*>(X + ((long long)gh * W + gw) * a.ldx + 4 * q)
                  : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int idx = it * 256 + tid;
      const int q = idx % (CIN / 4);
      const int tn = idx / (CIN / 4);  // tap * NOUT + n
      const int tap = tn / NOUT, n = tn % NOUT;
      // N < NOUT (RMVPE's 16 -> 3 output conv on the 16-wide tile): the missing weight rows read row 0, zeroed below
      if (NW % 256 == 0 || idx < NW) {
        wv[it] = *reinterpret_cast<const f32x4*>(a.w + (long long)tap * a.w_ts + (long long)(n < a.N ? n : 0) * a.ldw +
                                                 4 * q);
        if (n >= a.N) wv[it] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int it = 0; it < SIT; ++it) {
      const int idx = it * 256 + tid;
      if (idx < na) *reinterpret_cast<f32x4*>(As + (size_t)(idx / (CIN / 4)) * CP + 4 * (idx % (CIN / 4))) = v[it];
    }
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int idx = it * 256 + tid;
      if (NW % 256 == 0 || idx < NW)
        *reinterpret_cast<f32x4*>(Bs + (size_t)(idx / (CIN / 4)) * CP + 4 * (idx % (CIN / 4))) = wv[it];
    }
  }
  __syncthreads();
  // ---- MFMA main loop: 9 taps x CG channel groups x TPW pixel fragments x NT output fragments x 4
  f32x4 acc[TPW][NT];
#pragma unroll
  for (int p = 0; p < TPW; ++p)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[p][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int li = lane & 15, kq = lane >> 4;
  int pr[TPW], pc[TPW];
#pragma unroll
  for (int p = 0; p < TPW; ++p) {
    const int pix = wave * (PIX / 4) + p * 16 + li;  // pixel of this lane's A row within the tile
    pr[p] = pix / W;
    pc[p] = pix % W;
  }
  // per (tap, channel group): every A and B fragment read first (one exposed LDS latency), then the MFMAs k-slice
  // major so consecutive ones feed TPW x NT independent accumulators (v_mfma_f32_16x16x4_f32 issues every 32 cycles
  // but a dependent one waits 40; the pixel-major order chained 4 dependent MFMAs per fragment and read A one
  // fragment at a time: 2x the MFMA time)
  int abase[TPW];
#pragma unroll
  for (int p = 0; p < TPW; ++p) abase[p] = (pr[p] * AW + pc[p]) * CP + 4 * kq;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int dh = tap / 3, dw = tap % 3;
#pragma unroll
    for (int g = 0; g < CG; ++g) {
      f32x4 bf[NT], af[TPW];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        bf[t] = *reinterpret_cast<const f32x4*>(Bs + (size_t)(tap * NOUT + t * 16 + li) * CP + g * 16 + 4 * kq);
#pragma unroll
      for (int p = 0; p < TPW; ++p)
        af[p] = *reinterpret_cast<const f32x4*>(As + abase[p] + (dh * AW + dw) * CP + g * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int p = 0; p < TPW; ++p)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[p][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[p][j], bf[t][j], acc[p][t], 0, 0, 0);
    }
  }
  // ---- epilogue: lane holds rows (pixels) 4*kq + i of fragment p, column (channel) li of fragment t. The uniform
  // switches (alpha, act, residual) are tested once per 4-pixel group around the group-wide operation (per element
  // they were ~10 scalar branches per output, as in store_tile16)
  float* Y = a.y + (long long)b * a.y_bs;
  const float* R = a.res ? a.res + (long long)b * a.res_bs : nullptr;
  const bool res = a.res_mode == RES_ADD_POST;
  const int act = a.act;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = t * 16 + li;
    const bool n_ok = n < a.N;
    const float bn = (a.bias && n_ok) ? a.bias[n] : 0.f;
#pragma unroll
    for (int p = 0; p < TPW; ++p) {
      long long m[4];
      bool ok[4];
      f32x4 v = acc[p][t], rv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pix = wave * (PIX / 4) + p * 16 + 4 * kq + i;
        const int gh = h0 + pix / W, gw = pix % W;
        ok[i] = gh < H && n_ok;
        m[i] = (long long)(gh < H ? gh : 0) * W + gw;
      }
      if (res) {
#pragma unroll
        for (int i = 0; i < 4; ++i) rv[i] = R[m[i] * a.ldr + (n_ok ? n : 0)];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] += bn;
      if (a.alpha != 1.f) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] *= a.alpha;
      }
      if (act == ACT_RELU) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] > 0.f ? v[i] : 0.f;
      } else if (act == ACT_LRELU) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] > 0.f ? v[i] : v[i] * a.slope;
      }
      if (res) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] + rv[i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (ok[i]) Y[m[i] * a.ldy + n] = v[i];
    }
  }
}

// ---- The same convs in the two-plane fp16 split (split_bf16.h put_h16x4; rvcx_set_conv_math mode 3, the default):
// v_mfma_f32_16x16x32_f16, K = 32 = two taps of 16 channels (C_in 16; the 10th tap slot reads a zero pixel) or one
// tap of 32 channels, three products per K step (h h' into acc, l h' + h l' into acc2). The f32 kernel above spends
// 32 cycles per 16x16x4 MFMA: 9216 MFMA cycles per wave at level 0; here 1920. The weights come pre-split (k_s2d_wsplit,
// once per tensor, cached by the runtime as WSPLIT_S2D): [K step][16-column group][plane][64 lanes][16 B], lane l holding
// K rows 8 (l / 16) .. + 7 of column l % 16 (one ds_read_b128 per fragment), then the per-column 1 / (scale 2^-4) tail; a
// block copies it into LDS beside its tile (a block building it from the fp32 weights itself ran 10-45 % slower than
// the exact-f32 kernel, r04l). A pixel's LDS row is [hi plane | lo plane | 16 B pad] (80 or 144 B: a quarter-wave's
// 16-B reads of 16 consecutive pixels hit distinct bank groups).
namespace {
using namespace splitbf16;
constexpr int SIT_H = 13;  // staging rounds of 256 float4 per block (the 32 -> 16 decoder conv at W = 128: 12.2)
}  // namespace

template <int CIN, int NOUT, int PIX>
__global__ __launch_bounds__(256) void k_conv2d_h16(const ConvArgs a, const int RH) {
  constexpr int KS = CIN == 16 ? 5 : 9;  // K steps of 32
  constexpr int NT = NOUT / 16;
  constexpr int TPW = PIX / 64;  // 16-pixel fragments per wave
  constexpr int PS = CIN * 4 + 16;  // LDS bytes per pixel
  extern __shared__ __attribute__((aligned(16))) char smh[];
  const int W = a.W_out, H = a.T_out;
  const int AW = W + 2;
  const int npix = (RH + 2) * AW;  // + one zero pixel at index npix
  char* As = smh;
  char* Bs = smh + (((size_t)(npix + 1) * PS + 15) & ~(size_t)15);  // [KS][NT][plane][64 lanes][16 B]
  const int b = blockIdx.z;
  const int h0 = blockIdx.x * RH;
  const float* X = a.x + (long long)b * a.x_bs;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // ---- the epilogue's residual operands, loaded first (their latency then overlaps the staging and the MFMAs
  // instead of following them): lane holds rows 4 (lane / 16) + i of fragment p, column t * 16 + lane % 16
  const float* R = a.res ? a.res + (long long)b * a.res_bs : nullptr;
  const bool res = R && a.res_mode == RES_ADD_POST;
  f32x4 rv[TPW][NT];
#pragma unroll
  for (int p = 0; p < TPW; ++p)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      rv[p][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (res) {
        const int n = t * 16 + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int pix = wave * (PIX / 4) + p * 16 + 4 * (lane >> 4) + i;
          const int gh = h0 + pix / W, gw = pix % W;
          rv[p][t][i] = R[((long long)(gh < H ? gh : 0) * W + gw) * a.ldr + (n < a.N ? n : 0)];
        }
      }
    }
  // ---- halo tile: issue every load first, then split into LDS
  const int na = npix * (CIN / 4);
  {
    f32x4 v[SIT_H];
#pragma unroll
    for (int it = 0; it < SIT_H; ++it) {
      const int idx = it * 256 + tid;
      const int q = idx % (CIN / 4);
      const int pix = idx / (CIN / 4);
      const int r = pix / AW, cc = pix - r * AW;
      const int gh = h0 - 1 + r, gw = cc - 1;
      const bool ok = idx < na && gh >= 0 && gh < H && gw >= 0 && gw < W;
      v[it] = *reinterpret_cast<const f32x4*>(X + ((long long)(ok ? gh : 0) * W + (ok ? gw : 0)) * a.ldx + 4 * q);
      if (!ok) v[it] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // the pre-split weight image (k_s2d_wsplit: built once per weight tensor), issued beside the tile's loads
    constexpr int NBV = KS * NT * 2 * 64;  // 16-B vectors
    constexpr int BIT = (NBV + 255) / 256;
    uint4 bv[BIT];
    const uint4* wimg = static_cast<const uint4*>(a.wsplit);
#pragma unroll
    for (int it = 0; it < BIT; ++it) {
      const int idx = it * 256 + tid;
      bv[it] = wimg[idx < NBV ? idx : 0];
    }
#pragma unroll
    for (int it = 0; it < BIT; ++it) {
      const int idx = it * 256 + tid;
      if (idx < NBV) reinterpret_cast<uint4*>(Bs)[idx] = bv[it];
    }
#pragma unroll
    for (int it = 0; it < SIT_H; ++it) {
      const int idx = it * 256 + tid;
      if (idx < na) {
        f32x4 val = v[it];
#pragma unroll
        for (int j = 0; j < 4; ++j) val[j] *= H16_XS;
        // put_h16x4's layout with the plane stride of this kernel's rows: hi at 2c, lo at 2 CIN + 2c
        char* row = As + (size_t)(idx / (CIN / 4)) * PS;
        const int c4 = 4 * (idx % (CIN / 4));
        uint2 hh, ll;
        hh.x = pk_f16(val[0], val[1]);
        hh.y = pk_f16(val[2], val[3]);
        ll.x = pk_f16((val[0] - f16lo_f(hh.x)) * H16_LO, (val[1] - f16hi_f(hh.x)) * H16_LO);
        ll.y = pk_f16((val[2] - f16lo_f(hh.y)) * H16_LO, (val[3] - f16hi_f(hh.y)) * H16_LO);
        *reinterpret_cast<uint2*>(row + c4 * 2) = hh;
        *reinterpret_cast<uint2*>(row + CIN * 2 + c4 * 2) = ll;
      }
    }
    if (tid < PS / 16) reinterpret_cast<uint4*>(As + (size_t)npix * PS)[tid] = make_uint4(0u, 0u, 0u, 0u);
  }
  __syncthreads();

  // ---- MFMA loop
  f32x4 acc[TPW][NT], acc2[TPW][NT];
#pragma unroll
  for (int p = 0; p < TPW; ++p)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[p][t] = acc2[p][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int li = lane & 15, g = lane >> 4;
  int pbase[TPW];  // LDS byte offset of the fragment row's pixel (tap (0, 0)) + this lane's channel slot
#pragma unroll
  for (int p = 0; p < TPW; ++p) {
    const int pix = wave * (PIX / 4) + p * 16 + li;
    pbase[p] = ((pix / W) * AW + pix % W) * PS + (CIN == 16 ? 16 * (g & 1) : 16 * g);
  }
  const int zoff = npix * PS;  // the zero pixel (CIN 16: the 10th tap slot)
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int tap = CIN == 16 ? 2 * ks + (g >> 1) : ks;
    const int toff = ((tap / 3) * AW + tap % 3) * PS;
    f16x8 bh[NT], bl[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const char* src = Bs + ((size_t)((ks * NT + t) * 2) * 64 + lane) * 16;
      bh[t] = *reinterpret_cast<const f16x8*>(src);
      bl[t] = *reinterpret_cast<const f16x8*>(src + 64 * 16);
    }
#pragma unroll
    for (int p = 0; p < TPW; ++p) {
      const int ao = (CIN == 16 && tap >= 9) ? zoff : pbase[p] + toff;
      const f16x8 ah = *reinterpret_cast<const f16x8*>(As + ao);
      const f16x8 al = *reinterpret_cast<const f16x8*>(As + ao + CIN * 2);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[p][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[t], acc[p][t], 0, 0, 0);
        f32x4 c = acc2[p][t];
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[t], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[t], c, 0, 0, 0);
        acc2[p][t] = c;
      }
    }
  }
  // ---- epilogue (k_conv2d_small's): acc + 2^-11 acc2, times 1 / (column weight scale x activation scale) from the
  // image tail
  const float* invt = static_cast<const float*>(a.wsplit) + KS * NT * 2 * 64 * 4;
  float* Y = a.y + (long long)b * a.y_bs;
  const int act = a.act;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = t * 16 + li;
    const bool n_ok = n < a.N;
    const float bn = (a.bias && n_ok) ? a.bias[n] : 0.f;
    const float inv = invt[n];
#pragma unroll
    for (int p = 0; p < TPW; ++p) {
      long long m[4];
      bool ok[4];
      f32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = (acc[p][t][i] + acc2[p][t][i] * H16_LO_INV) * inv;
        const int pix = wave * (PIX / 4) + p * 16 + 4 * g + i;
        const int gh = h0 + pix / W, gw = pix % W;
        ok[i] = gh < H && n_ok;
        m[i] = (long long)(gh < H ? gh : 0) * W + gw;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] += bn;
      if (a.alpha != 1.f) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] *= a.alpha;
      }
      if (act == ACT_RELU) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] > 0.f ? v[i] : 0.f;
      } else if (act == ACT_LRELU) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] > 0.f ? v[i] : v[i] * a.slope;
      }
      if (res) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] + rv[p][t][i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (ok[i]) Y[m[i] * a.ldy + n] = v[i];
    }
  }
}

namespace {
template <int CIN, int NOUT, int PIX>
hipError_t launch_small(const ConvArgs& a, hipStream_t s) {
  const int W = a.W_out;
  const int RH = PIX / W;
  const size_t lds = ((size_t)(RH + 2) * (W + 2) * (CIN + 4) + (size_t)9 * NOUT * (CIN + 4)) * sizeof(float);
  if (lds > 160 * 1024 || (long long)(RH + 2) * (W + 2) * (CIN / 4) > (long long)SIT * 256) return hipErrorInvalidValue;
  auto kern = k_conv2d_small<CIN, NOUT, PIX>;
  static size_t lds_set = 64 * 1024;  // per instantiation: raise the dynamic-LDS limit once, not per launch
  if (lds > lds_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    lds_set = lds;
  }
  dim3 grid((a.T_out + RH - 1) / RH, 1, a.batch);
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a, RH);
  return hipGetLastError();
}
// the image: one block; max |w| per output column (LDS atomics on the bits), each column's power-of-two scale (conv_wsb.hip
// k_wsplit_h16's rule), then the lane-major fragments and the tail inv[32] = 1 / (scale_n 2^-4)
__global__ __launch_bounds__(256) void k_s2d_wsplit(const float* __restrict__ w, long long w_ts, int ldw, int N, int CIN,
                                                    int NT, unsigned short* __restrict__ out) {
  __shared__ unsigned cmax[32];
  const int tid = threadIdx.x;
  if (tid < 32) cmax[tid] = 0u;
  __syncthreads();
  for (int i = tid; i < 9 * N * CIN; i += 256) {
    const int c = i % CIN, tn = i / CIN;
    atomicMax(&cmax[tn % N], __float_as_uint(fabsf(w[(long long)(tn / N) * w_ts + (long long)(tn % N) * ldw + c])));
  }
  __syncthreads();
  const int KS = CIN == 16 ? 5 : 9;
  for (int e = tid; e < KS * NT * 64; e += 256) {
    const int l = e & 63, knt = e >> 6;
    const int nt = knt % NT, ks = knt / NT;
    const int n = nt * 16 + (l & 15), g = l >> 4;
    const int tap = CIN == 16 ? 2 * ks + (g >> 1) : ks;
    const int c0 = CIN == 16 ? 8 * (g & 1) : 8 * g;
    const bool ok = tap < 9 && n < N;
    const float sc = h16_weight_scale(cmax[n]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = ok ? w[(long long)tap * w_ts + (long long)n * ldw + c0 + j] * sc : 0.f;
      const unsigned h = pk_f16(v, 0.f);
      out[((size_t)(knt * 2) * 64 + l) * 8 + j] = (unsigned short)h;
      out[((size_t)(knt * 2 + 1) * 64 + l) * 8 + j] = (unsigned short)pk_f16((v - f16lo_f(h)) * H16_LO, 0.f);
    }
  }
  if (tid < 32) {
    float* tail = reinterpret_cast<float*>(out + (size_t)KS * NT * 2 * 64 * 8);
    tail[tid] = 1.f / (h16_weight_scale(cmax[tid]) * H16_XS);
  }
}

// the fp16-split form: PIX 512 (C_in 16) / 128 (C_in 32) pixels per block: one round of blocks at the U-Net sizes
template <int CIN, int NOUT>
hipError_t launch_h16(const ConvArgs& a, hipStream_t s) {
  constexpr int PIX = CIN == 16 ? 512 : 128;  // C_in 16 at 256: 784 blocks for 768 slots (two rounds), 19 us at level 0
  const int W = a.W_out;
  if (PIX % W) return hipErrorInvalidValue;
  const int RH = PIX / W;
  const size_t ps = CIN * 4 + 16;
  const size_t abytes = (((size_t)((RH + 2) * (W + 2) + 1) * ps) + 15) & ~(size_t)15;
  const size_t lds = abytes + (size_t)(CIN == 16 ? 5 : 9) * (NOUT / 16) * 2 * 1024;
  if (lds > 160 * 1024 || (long long)(RH + 2) * (W + 2) * (CIN / 4) > (long long)SIT_H * 256) return hipErrorInvalidValue;
  auto kern = k_conv2d_h16<CIN, NOUT, PIX>;
  static size_t lds_set = 64 * 1024;
  if (lds > lds_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    lds_set = lds;
  }
  dim3 grid((a.T_out + RH - 1) / RH, 1, a.batch);
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a, RH);
  return hipGetLastError();
}
}  // namespace

bool conv2d_small_fits(const ConvArgs& a) {
  const bool shape = a.KH == 3 && a.KW == 3 && a.taps == 9 && a.padh == 1 && a.padw == 1 && a.T_in == a.T_out &&
                     a.W_in == a.W_out && (a.C_in == 16 || a.C_in == 32) && (a.N == 32 || (a.N >= 1 && a.N <= 16));
  if (!shape) return false;
  const int pix = a.C_in == 16 ? 512 : 256;
  if (a.W_out < 16 || pix % a.W_out) return false;
  if ((long long)(pix / a.W_out + 2) * (a.W_out + 2) * (a.C_in / 4) > (long long)SIT * 256) return false;
  const bool epi = a.out_map == OUT_ROWS && a.acc_mode == ACC_STORE && !a.mask && a.pre_act == ACT_NONE &&
                   !a.pre_mask && a.batch_inner == 1 && !a.b_kn && a.stride == 1 &&
                   (a.res_mode == RES_NONE || a.res_mode == RES_ADD_POST) &&
                   (a.act == ACT_NONE || a.act == ACT_RELU || a.act == ACT_LRELU) && a.w_bs == 0 && a.bias_bs == 0;
  const bool align = (a.ldx % 4 == 0) && (a.x_bs % 4 == 0) && (a.ldw % 4 == 0) && (a.w_ts % 4 == 0) &&
                     ((reinterpret_cast<uintptr_t>(a.x) & 15) == 0) && ((reinterpret_cast<uintptr_t>(a.w) & 15) == 0) &&
                     a.ldx >= a.C_in && a.ldw >= a.C_in;
  return epi && align;
}

static int s2d_nt(const ConvArgs& a) { return a.N <= 16 ? 1 : 2; }
long long small2d_wsplit_bytes(const ConvArgs& a) {
  return (long long)(a.C_in == 16 ? 5 : 9) * s2d_nt(a) * 2 * 1024 + 256;
}
hipError_t small2d_wsplit_build(const ConvArgs& a, void* out, hipStream_t s) {
  if (!conv2d_small_fits(a)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_s2d_wsplit, dim3(1), dim3(256), 0, s, a.w, a.w_ts, a.ldw, a.N, a.C_in, s2d_nt(a),
                     static_cast<unsigned short*>(out));
  return hipGetLastError();
}

hipError_t conv2d_small(const ConvArgs& a, hipStream_t s) {
  // the fp16 split (conv math 3) reads the pre-split image; the exact-f32 form serves conv math 1-2
  if (conv_math_of(a) == 3 && a.wsplit && a.wsplit_fmt == WSPLIT_S2D) {
    hipError_t e = hipErrorInvalidValue;
    if (a.C_in == 16) e = a.N <= 16 ? launch_h16<16, 16>(a, s) : launch_h16<16, 32>(a, s);
    else e = a.N <= 16 ? launch_h16<32, 16>(a, s) : launch_h16<32, 32>(a, s);
    if (e != hipErrorInvalidValue) return e;
  }
  if (a.C_in == 16 && a.N <= 16) return launch_small<16, 16, 512>(a, s);
  if (a.C_in == 16 && a.N == 32) return launch_small<16, 32, 512>(a, s);
  if (a.C_in == 32 && a.N <= 16) return launch_small<32, 16, 256>(a, s);
  if (a.C_in == 32 && a.N == 32) return launch_small<32, 32, 256>(a, s);
  return hipErrorInvalidValue;
}

}  // namespace rvcx
