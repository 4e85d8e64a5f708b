// 3x3 / pad 1 2-D convolution for few channels (C_in, N in {16, 32}) on v_mfma_f32_16x16x4_f32.
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

#include "rvcx_kernels.h"

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

hipError_t conv2d_small(const ConvArgs& a, hipStream_t s) {
  if (a.C_in == 16 && a.N <= 16) return launch_small<16, 16, 512>(a, s);
  if (a.C_in == 16 && a.N == 32) return launch_small<16, 32, 512>(a, s);
  if (a.C_in == 32 && a.N <= 16) return launch_small<32, 16, 256>(a, s);
  if (a.C_in == 32 && a.N == 32) return launch_small<32, 32, 256>(a, s);
  return hipErrorInvalidValue;
}

}  // namespace rvcx
