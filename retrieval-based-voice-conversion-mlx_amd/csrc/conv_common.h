// Shared pieces of the implicit-GEMM conv kernels (conv_gemm.hip: exact fp32 MFMA; conv_emu.hip: fp32 through
// three bf16 planes): activations, the fused epilogue, and the accumulator -> HBM store of one block tile.
#pragma once
#include "rvcx_kernels.h"

namespace rvcx {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int CONV_THREADS = 256;  // 4 waves per block in every conv kernel

static __device__ __noinline__ float act_fn_slow(float v, int act, float slope) {
  switch (act) {
    case ACT_GELU: return 0.5f * v * (1.f + erff(v * 0.70710678118654752440f));
    case ACT_TANH: return tanhf(v);
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    case ACT_LOGCLAMP: return logf(fmaxf(v, slope));
    default: return v;
  }
}

// cheap activations inline, transcendental ones out of line (keeps the unrolled epilogue small
// enough that the accumulators stay in registers)
static __device__ __forceinline__ float act_fn(float v, int act, float slope) {
  if (act == ACT_NONE) return v;
  if (act == ACT_LRELU) return v > 0.f ? v : v * slope;
  if (act == ACT_RELU) return v > 0.f ? v : 0.f;
  return act_fn_slow(v, act, slope);
}

// Pre-activation chosen at compile time (kernel MODE bits 0-1: 0 none, 1 leaky ReLU, 2 any other via act_fn): a
// runtime act switch per element put ~30-120 scalar branches into every A staging pass of the streamed kernels
enum { PA_NONE = 0, PA_LRELU = 1, PA_ANY = 2 };
template <int PA>
static __device__ __forceinline__ float pre_fn(float v, int act, float slope) {
  if constexpr (PA == PA_NONE) return v;
  else if constexpr (PA == PA_LRELU) return v > 0.f ? v : v * slope;
  else return act_fn(v, act, slope);
}
static inline int pre_mode(int act) { return act == ACT_NONE ? PA_NONE : (act == ACT_LRELU ? PA_LRELU : PA_ANY); }

static __device__ __forceinline__ void epilogue_store(const ConvArgs& a, float v, float bn, long long m, int n, int oh,
                                                      int ow, const float* R, const float* MK, float* Y) {
  if (a.bias) v += bn;
  if (a.res_mode == RES_ADD_PRE) v = v + R[m * a.ldr + n];
  if (a.alpha != 1.f) v *= a.alpha;
  v = act_fn(v, a.act, a.slope);
  if (a.res_mode == RES_ADD_POST) v = v + R[m * a.ldr + n];
  else if (a.res_mode == RES_RSUB_POST) v = R[m * a.ldr + n] - v;
  float* dst;
  if (a.out_map == OUT_UPSAMPLE2D) {
    const int cv = a.out_cv;
    const int ph = n / (2 * cv), pw = (n / cv) & 1, co = n % cv;
    dst = Y + ((long long)(2 * oh + ph) * (2 * a.W_out) + (2 * ow + pw)) * a.ldy + co;
  } else {
    dst = Y + m * a.ldy + n;
  }
  if (a.acc_mode == ACC_ADD) v = *dst + v;
  else if (a.acc_mode == ACC_ADD_DIV) v = (*dst + v) / a.acc_div;
  if (MK) v *= MK[m];
  *dst = v;
}

// The 16x16 accumulator tiles of a wave (v_mfma_f32_16x16x32 C layout: lane l holds column l % 16, rows 4 (l / 16) + r)
// -> HBM or the split-K slab, with the shared epilogue (epilogue_store's order of operations, bit-identical). The
// epilogue switches are uniform and tested once per 4-element group, each around its group-wide operation: tested
// per element (as epilogue_store does) they cost ~25 scalar branches per output, as much as a short tile's MMA loop.
// + the NSF noise conv (ConvArgs::nz_*) of output column n, rows mb .. mb + 3 (those with ok[r]): KK = nz_kk at
// compile time. k_noise_add's order: an fma chain over q from 0, + bias, + v
template <int KK>
__device__ __forceinline__ void noise_rows(const ConvArgs& a, int b, long long mb, int n, const bool (&ok)[4],
                                           f32x4& v) {
  const int stride = a.nz_stride, C = a.nz_C;
  const int p = n / C, c = n - p * C;
  const float* hb = a.nz_har + (long long)b * a.nz_bs;
  float wq[KK];
  {
    int tap = 0, j = 0;
#pragma unroll
    for (int q = 0; q < KK; ++q) {
      wq[q] = a.nz_w[((long long)tap * C + c) * stride + j];
      if (++j == stride) {
        j = 0;
        ++tap;
      }
    }
  }
  const float nb = a.nz_b[c];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float* x = hb + ((ok[r] ? mb + r : 0) * a.nz_u + p) * stride;
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < KK; ++q) acc = fmaf(wq[q], x[q], acc);
    v[r] = v[r] + (acc + nb);
  }
}

// UP2D: the instantiation may see the ConvTranspose2d phase layout (OUT_UPSAMPLE2D: the 2-D gather-streamed kernel
// only; compiled out elsewhere)
template <int TM16, int TN16, int WM, int WN, bool UP2D = false>
__device__ __forceinline__ void store_tile16(const ConvArgs& a, int m0, int n0, int b, int zsplit, int ksplit,
                                             long long Mtot, f32x4 (&acc)[TM16][TN16]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lc = lane & 15, lg = lane >> 4;
  if (ksplit > 1) {
#pragma unroll
    for (int tn = 0; tn < TN16; ++tn) {
      const int n = n0 + wn * TN16 * 16 + tn * 16 + lc;
#pragma unroll
      for (int tm = 0; tm < TM16; ++tm) {
        const long long mb = (long long)m0 + wm * TM16 * 16 + tm * 16 + 4 * lg;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n < a.N && mb + r < Mtot) a.ws[(((long long)b * ksplit + zsplit) * a.ws_rows + mb + r) * a.N + n] = acc[tm][tn][r];
      }
    }
    return;
  }
  const float* bias = a.bias ? a.bias + (long long)b * a.bias_bs : nullptr;
  const float* R = a.res ? a.res + (long long)b * a.res_bs : nullptr;
  const float* MK = a.mask ? a.mask + (long long)b * a.mask_bs : nullptr;
  float* Y = a.y + (long long)b * a.y_bs;
  const bool need_r = R && a.res_mode != RES_NONE;
  const bool need_d = a.acc_mode != ACC_STORE;
  const int act = a.act;
#pragma unroll
  for (int tn = 0; tn < TN16; ++tn) {
    const int n = n0 + wn * TN16 * 16 + tn * 16 + lc;
    const bool n_ok = n < a.N;
    const float bn = (bias && n_ok) ? bias[n] : 0.f;
#pragma unroll
    for (int tm = 0; tm < TM16; ++tm) {
      const long long mb = (long long)m0 + wm * TM16 * 16 + tm * 16 + 4 * lg;
      bool ok[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) ok[r] = n_ok && mb + r < Mtot;
      f32x4 v = acc[tm][tn];
      f32x4 rv = {0.f, 0.f, 0.f, 0.f}, dv = {0.f, 0.f, 0.f, 0.f}, mv = {1.f, 1.f, 1.f, 1.f};
      // gather first (residual / accumulate / mask operands), then the arithmetic, then the stores
      if (need_r) {
#pragma unroll
        for (int r = 0; r < 4; ++r) rv[r] = ok[r] ? R[(mb + r) * a.ldr + n] : 0.f;
      }
      if (need_d) {
#pragma unroll
        for (int r = 0; r < 4; ++r) dv[r] = ok[r] ? Y[(mb + r) * a.ldy + n] : 0.f;
      }
      if (MK) {
#pragma unroll
        for (int r = 0; r < 4; ++r) mv[r] = ok[r] ? MK[mb + r] : 1.f;
      }
      if (bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bn;
      }
      if (a.res_mode == RES_ADD_PRE) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] + rv[r];
      }
      if (a.alpha != 1.f) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] *= a.alpha;
      }
      if (act == ACT_LRELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
      } else if (act == ACT_RELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
      } else if (act != ACT_NONE) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_fn_slow(v[r], act, a.slope);
      }
      if (a.res_mode == RES_ADD_POST) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] + rv[r];
      } else if (a.res_mode == RES_RSUB_POST) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = rv[r] - v[r];
      }
      if (a.acc_mode == ACC_ADD) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = dv[r] + v[r];
      } else if (a.acc_mode == ACC_ADD_DIV) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (dv[r] + v[r]) / a.acc_div;
      }
      if (a.nz_har && n_ok) {
        // the NSF noise conv of these 4 outputs (ConvArgs::nz_*): k_noise_add's arithmetic, y + (sum + b); one
        // tap (the last stage's stride-1 noise conv: the dispatcher admits nz_kk = 1 only)
        noise_rows<1>(a, b, mb, n, ok, v);
      }
      if (MK) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] *= mv[r];
      }
      if (UP2D && a.out_map == OUT_UPSAMPLE2D) {
        // the 2x2-phase ConvTranspose2d (epilogue_store's mapping): virtual column n = (ph, pw, co) of input pixel m
        const int cv = a.out_cv;
        const int ph = n / (2 * cv), pw = (n / cv) & 1, co = n - (n / cv) * cv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (!ok[r]) continue;
          const long long m = mb + r;
          const long long oh = m / a.W_out, ow = m - oh * a.W_out;
          Y[((2 * oh + ph) * (2 * a.W_out) + (2 * ow + pw)) * a.ldy + co] = v[r];
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (ok[r]) Y[(mb + r) * a.ldy + n] = v[r];
    }
  }
}

// store_tile16 for the transposed accumulator layout D = W X^T (conv_wsb.hip): lane (lc, lg) of a 16x16 tile holds
// row lc, columns 4 lg + r, so the residual / accumulate operands and the outputs move as one 16-byte vector per lane
// and tile where the rows are 16-byte aligned (vec: N, the row strides and the bases multiples of 4 floats) -- a
// quarter of store_tile16's memory instructions, whose issue rate, not HBM, bounded the epilogue. Same per-element
// order of operations (bit-identical results); 1-D OUT_ROWS only.
template <int TM16, int TN16, int WM, int WN>
__device__ __forceinline__ void store_tile16t(const ConvArgs& a, int m0, int n0, int b, int zsplit, int ksplit,
                                              long long Mtot, f32x4 (&acc)[TM16][TN16]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lc = lane & 15, lg = lane >> 4;
  const bool nvec = (a.N & 3) == 0;
  if (ksplit > 1) {
    float* W = a.ws + ((long long)b * ksplit + zsplit) * a.ws_rows * a.N;
#pragma unroll
    for (int tm = 0; tm < TM16; ++tm) {
      const long long m = (long long)m0 + wm * TM16 * 16 + tm * 16 + lc;
      if (m >= Mtot) continue;
#pragma unroll
      for (int tn = 0; tn < TN16; ++tn) {
        const int n = n0 + wn * TN16 * 16 + tn * 16 + 4 * lg;
        float* dst = W + m * a.N + n;
        if (nvec && n + 3 < a.N) {
          *reinterpret_cast<f32x4*>(dst) = acc[tm][tn];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < a.N) dst[r] = acc[tm][tn][r];
        }
      }
    }
    return;
  }
  const float* bias = a.bias ? a.bias + (long long)b * a.bias_bs : nullptr;
  const float* R = a.res ? a.res + (long long)b * a.res_bs : nullptr;
  const float* MK = a.mask ? a.mask + (long long)b * a.mask_bs : nullptr;
  float* Y = a.y + (long long)b * a.y_bs;
  const bool need_r = R && a.res_mode != RES_NONE;
  const bool need_d = a.acc_mode != ACC_STORE;
  const int act = a.act;
  const bool vec = nvec && ((reinterpret_cast<uintptr_t>(Y) & 15) == 0) && (a.ldy & 3) == 0 &&
                   (!need_r || (((reinterpret_cast<uintptr_t>(R) & 15) == 0) && (a.ldr & 3) == 0));
#pragma unroll
  for (int tn = 0; tn < TN16; ++tn) {
    const int n = n0 + wn * TN16 * 16 + tn * 16 + 4 * lg;
    f32x4 bn = {0.f, 0.f, 0.f, 0.f};
    if (bias) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bn[r] = n + r < a.N ? bias[n + r] : 0.f;
    }
#pragma unroll
    for (int tm = 0; tm < TM16; ++tm) {
      const long long m = (long long)m0 + wm * TM16 * 16 + tm * 16 + lc;
      const bool m_ok = m < Mtot;
      const bool full = m_ok && n + 3 < a.N;
      bool ok[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) ok[r] = m_ok && n + r < a.N;
      f32x4 v = acc[tm][tn];
      f32x4 rv = {0.f, 0.f, 0.f, 0.f}, dv = {0.f, 0.f, 0.f, 0.f};
      float mv = 1.f;
      // gather first (residual / accumulate / mask operands), then the arithmetic, then the stores
      if (need_r) {
        const float* src = R + m * a.ldr + n;
        if (vec && full) {
          rv = *reinterpret_cast<const f32x4*>(src);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) rv[r] = ok[r] ? src[r] : 0.f;
        }
      }
      if (need_d) {
        const float* src = Y + m * a.ldy + n;
        if (vec && full) {
          dv = *reinterpret_cast<const f32x4*>(src);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) dv[r] = ok[r] ? src[r] : 0.f;
        }
      }
      if (MK) mv = m_ok ? MK[m] : 1.f;
      if (bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bn[r];
      }
      if (a.res_mode == RES_ADD_PRE) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] + rv[r];
      }
      if (a.alpha != 1.f) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] *= a.alpha;
      }
      if (act == ACT_LRELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
      } else if (act == ACT_RELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
      } else if (act != ACT_NONE) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_fn_slow(v[r], act, a.slope);
      }
      if (a.res_mode == RES_ADD_POST) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] + rv[r];
      } else if (a.res_mode == RES_RSUB_POST) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = rv[r] - v[r];
      }
      if (a.acc_mode == ACC_ADD) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = dv[r] + v[r];
      } else if (a.acc_mode == ACC_ADD_DIV) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (dv[r] + v[r]) / a.acc_div;
      }
      if (a.nz_har) {
        // the NSF noise conv of these 4 outputs, one tap (the dispatcher admits nz_kk = 1 only): k_noise_add's
        // arithmetic, y + (w x + b)
        const float* hb = a.nz_har + (long long)b * a.nz_bs;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (!ok[r]) continue;
          const int p = (n + r) / a.nz_C, c = n + r - p * a.nz_C;
          const float x = hb[(m * a.nz_u + p) * a.nz_stride];
          v[r] = v[r] + (fmaf(a.nz_w[(long long)c * a.nz_stride], x, 0.f) + a.nz_b[c]);
        }
      }
      if (MK) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] *= mv;
      }
      float* dst = Y + m * a.ldy + n;
      if (vec && full) {
        *reinterpret_cast<f32x4*>(dst) = v;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (ok[r]) dst[r] = v[r];
      }
    }
  }
}

// Where a block tile sits: output rows m0.. (1-D) or the rh x rw pixel window at (h0, w0) (2-D), output channels
// n0.., outer/inner batch (b, bi), split-K slice zsplit of ksplit for batch entry zb.
struct TilePos {
  int m0, h0, w0, rw, rh, n0, b, bi, zb, zsplit, ksplit;
};

// The block's accumulators -> HBM. Wave (wm, wn) holds TM x TN 32x32 tiles in the MFMA C layout: lane (li, hk),
// register r is row (r&3) + 8(r>>2) + 4hk, column li. Split-K slices write their partial tile to the slab
// (splitk_reduce_kernel applies the epilogue); otherwise the fused epilogue runs here.
template <int TM, int TN, int WM, int WN, bool TWO_D>
__device__ __forceinline__ void conv_store_tile(const ConvArgs& a, const TilePos& p, f32x16 (&acc)[TM][TN],
                                                float* smem) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 31, hk = lane >> 5;
  const float* bias = a.bias ? a.bias + (long long)p.b * a.bias_bs + (long long)p.bi * a.bias_bs2 : nullptr;
  const float* R = a.res ? a.res + (long long)p.b * a.res_bs + (long long)p.bi * a.res_bs2 : nullptr;
  const float* MK = a.mask ? a.mask + (long long)p.b * a.mask_bs : nullptr;
  float* Y = a.y + (long long)p.b * a.y_bs + (long long)p.bi * a.y_bs2;
  auto emit = [&](float v, int ml, int n, bool n_ok, float bn) {
    long long m;
    int oh = 0, ow = 0;
    bool ok;
    if (!TWO_D) {
      m = p.m0 + ml;
      ok = n_ok && (m < a.T_out);
    } else {
      oh = p.h0 + ml / p.rw;
      ow = p.w0 + ml % p.rw;
      ok = n_ok && (ml < p.rh * p.rw) && (oh < a.T_out) && (ow < a.W_out);
      m = (long long)oh * a.W_out + ow;
    }
    if (ok) {
      if (p.ksplit > 1) {
        a.ws[(((long long)p.zb * p.ksplit + p.zsplit) * a.ws_rows + m) * a.N + n] = v;
      } else {
        epilogue_store(a, v, bn, m, n, oh, ow, R, MK, Y);
      }
    }
  };
  if (!TWO_D && p.ksplit == 1 && a.out_map == OUT_ROWS) {
    // 1-D rows: every accumulator of the wave straight from registers, one 32x32 tile after another, gather
    // first: the residual, accumulate and mask operands of the lane's 16 outputs of a tile are all loaded before
    // the first store. The stores may alias them (an in-place residual reads the very element it writes), so
    // the compiler cannot hoist the loads across the stores itself and would expose one load latency per output
    // (16 per lane): the short-contraction convs (ResBlock k=3 at 32/64 channels) were latency-bound on exactly
    // that. Each element is read and written by this lane only, so the reorder is exact.
    const bool need_r = R && a.res_mode != RES_NONE;
    const bool need_d = a.acc_mode != ACC_STORE;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int n = p.n0 + wn * TN * 32 + tn * 32 + li;
        const bool n_ok = n < a.N;
        const float bn = (bias && n_ok) ? bias[n] : 0.f;
        // element r sits at row mb + (r&3) + 8(r>>2) of column n: per-lane base pointers, constant row offsets
        const int mb = p.m0 + wm * TM * 32 + tm * 32 + 4 * hk;
        const bool full = p.m0 + wm * TM * 32 + tm * 32 + 32 <= a.T_out;
        const float* Rl = need_r ? R + (long long)mb * a.ldr + n : nullptr;
        float* Yl = Y + (long long)mb * a.ldy + n;
        const float* Ml = MK ? MK + mb : nullptr;
        auto row_ok = [&](int r) { return n_ok && (full || mb + (r & 3) + 8 * (r >> 2) < a.T_out); };
        // two halves of 8 elements: one exposed load latency each, 24 staging registers instead of 48 (the
        // VGPR count sets the workgroups per CU of this latency-bound kernel)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float rv[8], dv[8], mv[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int r = 8 * h + i;
            const int ro = (r & 3) + 8 * (r >> 2);
            const bool ok = row_ok(r);
            rv[i] = (ok && need_r) ? Rl[ro * a.ldr] : 0.f;
            dv[i] = (ok && need_d) ? Yl[ro * a.ldy] : 0.f;
            mv[i] = (ok && MK) ? Ml[ro] : 1.f;
          }
          // the uniform switches once per 8-element half, each around its half-wide operation (store_tile16)
          float v[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] = acc[tm][tn][8 * h + i];
          if (a.bias) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] += bn;
          }
          if (a.res_mode == RES_ADD_PRE) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = v[i] + rv[i];
          }
          if (a.alpha != 1.f) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] *= a.alpha;
          }
          if (a.act == ACT_LRELU) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = v[i] > 0.f ? v[i] : v[i] * a.slope;
          } else if (a.act == ACT_RELU) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = v[i] > 0.f ? v[i] : 0.f;
          } else if (a.act != ACT_NONE) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = act_fn_slow(v[i], a.act, a.slope);
          }
          if (a.res_mode == RES_ADD_POST) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = v[i] + rv[i];
          } else if (a.res_mode == RES_RSUB_POST) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = rv[i] - v[i];
          }
          if (a.acc_mode == ACC_ADD) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = dv[i] + v[i];
          } else if (a.acc_mode == ACC_ADD_DIV) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = (dv[i] + v[i]) / a.acc_div;
          }
          if (MK) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] *= mv[i];
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int r = 8 * h + i;
            if (row_ok(r)) Yl[((r & 3) + 8 * (r >> 2)) * a.ldy] = v[i];
          }
        }
      }
    }
    return;
  }
  if constexpr (TM * TN == 1) {
    // one accumulator per wave: straight from registers (fully unrolled, 16 values per lane)
    const int n = p.n0 + wn * 32 + li;
    const bool n_ok = n < a.N;
    const float bn = (bias && n_ok) ? bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) emit(acc[0][0][r], wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hk, n, n_ok, bn);
  } else {
    // several accumulators per wave: stage one 32x32 tile at a time through the wave's own LDS slot
    // (32 x 33 floats) and emit rows 2i + hk, column li; accumulator registers are only indexed with
    // compile-time constants, so the large wave tiles keep them out of scratch
    __syncthreads();  // every wave is done with the A/B tiles: their LDS becomes the staging area
    float* Cs = smem + wave * (32 * 33);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
        for (int r = 0; r < 16; ++r) Cs[((r & 3) + 8 * (r >> 2) + 4 * hk) * 33 + li] = acc[tm][tn][r];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int n = p.n0 + wn * TN * 32 + tn * 32 + li;
        const bool n_ok = n < a.N;
        const float bn = (bias && n_ok) ? bias[n] : 0.f;
        for (int i = 0; i < 16; ++i) {
          const int rr = 2 * i + hk;
          emit(Cs[rr * 33 + li], wm * TM * 32 + tm * 32 + rr, n, n_ok, bn);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
  }
}

// Block -> tile: the grid is 1-D over (M tile, N tile) with N fastest when ntn > 0, and the linear workgroup id
// is remapped so each XCD (workgroups are dealt to the 8 XCDs round-robin) owns one contiguous run of tiles: the
// N tiles of an M tile then share its A halo through one L2 instead of re-reading it from HBM/L3 (bijective
// remap, cdna_hip_programming.md T1). ntn = 0: the plain (x = M, y = N) grid.
__device__ __forceinline__ void conv_block_coords(int ntn, int& bx, int& by, int& bz) {
  bx = blockIdx.x;
  by = blockIdx.y;
  bz = blockIdx.z;
  if (ntn > 0) {
    const int X = gridDim.x, total = X * gridDim.z;
    const int orig = blockIdx.z * X + blockIdx.x;
    const int xcd = orig & 7, q = total >> 3, r = total & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
    bz = wg / X;
    const int t = wg - bz * X;
    bx = t / ntn;
    by = t - bx * ntn;
  }
}

// conv_emu.hip: fp32 convolution on bf16 MFMA through a 3-way operand split (defined there)
// cfg: 10.. (cfg_tile_emu); returns hipErrorInvalidValue when the tile's LDS does not fit
hipError_t conv_emu_launch(const ConvArgs& a, int cfg, bool two_d, bool pipe, int ksplit, int ntn_enable,
                           hipStream_t s);
bool conv_emu_tile(int cfg, int& BM, int& BN);

}  // namespace rvcx
