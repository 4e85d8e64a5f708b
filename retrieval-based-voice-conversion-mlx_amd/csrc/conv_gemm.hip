// Implicit-GEMM convolution on CDNA4 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// One kernel family covers every contraction of the RVC path:
//   * 1-D conv (time-major [T][C]): NSF ResBlock dilated convs, conv_pre, flow WaveNet,
//     TextEncoder FFN, HuBERT strided feature convs, the grouped positional conv (batch=group),
//     ConvTranspose1d as a polyphase conv (u*C_out virtual outputs), STFT-as-GEMM framing;
//   * GEMM (taps=1): all Linear / 1x1 convs, attention QK^T and PV (batch = head);
//   * 2-D 3x3 conv on NHWC images (RMVPE U-Net), ConvTranspose2d as a 2x2-tap phase conv.
//
// Tiling: a 256-thread block (4 waves) owns BM output rows x BN output channels. The A tile is
// staged once per 32-channel chunk with its full tap halo ((BM-1)*stride + (taps-1)*dil + 1 rows,
// or the (RH+KH-1) x (RW+KW-1) pixel window in 2-D), the pre-activation applied on the way into
// LDS; each tap then re-reads shifted rows of that tile (no im2col in HBM). B (weights packed
// [tap][N][C]) is staged per tap. Each wave holds TM x TN 32x32 fp32 accumulators; one
// ds_read_b128 per operand feeds 4 MFMAs (the k-pair of MFMA j is channels {8kk+j, 8kk+4+j}).
// fp32 in / fp32 accumulate MFMA is a bit-exact fp32 fma chain at the FP32 vector peak rate.
#include <algorithm>
#include <cstdlib>
#include <string>

#include "conv_common.h"

namespace rvcx {

constexpr int CK = 32;   // contraction channels per LDS chunk
constexpr int NTHREADS = CONV_THREADS;

template <int BM, int BN, int WM, int WN, bool TWO_D, bool PIPE, int ASB, int CKT = CK>
__global__ __launch_bounds__(NTHREADS, 2) void conv_gemm_kernel(const ConvArgs a, const int nrows_a, const int rw,
                                                             const int rh, const int tiles_w, const int vec_a,
                                                             const int vec_b, const int ksplit, const int ntn) {
  constexpr int CKP = CKT + 4;  // padded LDS row: rows i..i+15 land on distinct 16-B bank slots
  constexpr int C4 = CKT / 4;   // float4 per LDS row
  constexpr int TM = BM / (WM * 32);
  constexpr int TN = BN / (WN * 32);
  static_assert(WM * WN == 4, "4 waves per block");
  static_assert(TM >= 1 && TN >= 1, "tile too small");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;
  float* Bs0 = smem + nrows_a * CKP;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 31, hk = lane >> 5;
  // Tile order (ntn > 0): the grid is 1-D over (M tile, N tile) with N fastest, and the linear workgroup
  // id is remapped so each XCD (workgroups are dealt to the 8 XCDs round-robin) owns one contiguous run of
  // tiles: the N tiles of an M tile then share its A halo through one L2 instead of re-reading it from
  // HBM/L3 (bijective remap, cdna_hip_programming.md T1). ntn = 0: the plain (x = M, y = N) grid.
  int bx, by, bz;
  conv_block_coords(ntn, bx, by, bz);
  const int zsplit = bz % ksplit;     // split-K slice
  const int zb = bz / ksplit;
  const int b = zb / a.batch_inner;   // outer batch
  const int bi = zb % a.batch_inner;  // inner batch (heads / groups)
  const int n0 = by * BN;
  int m0 = 0, h0 = 0, w0 = 0;
  if (!TWO_D) {
    m0 = bx * BM;
  } else {
    h0 = (bx / tiles_w) * rh;
    w0 = (bx % tiles_w) * rw;
  }
  const float* X = a.x + (long long)b * a.x_bs + (long long)bi * a.x_bs2;
  const float* Wb = a.w + (long long)b * a.w_bs + (long long)bi * a.w_bs2;
  const float* PM = a.pre_mask ? a.pre_mask + (long long)b * a.pre_mask_bs : nullptr;
  const int aw = TWO_D ? rw + a.KW - 1 : 0;
  const int row0 = TWO_D ? 0 : m0 * a.stride - a.pad;

  int base[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int ml = wm * TM * 32 + tm * 32 + li;
    if (!TWO_D) {
      base[tm] = ml * a.stride;
    } else {
      base[tm] = (ml < rh * rw) ? (ml / rw) * aw + (ml % rw) : 0;
    }
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tm][tn][r] = 0.f;

  // B tile loader: global -> registers (BN x 32 floats of (tap, chunk)); NK or KN weight layout
  constexpr int BV = (BN * C4 + NTHREADS - 1) / NTHREADS;  // float4 per thread
  // NK layout: thread v-slot reads row n0 + idx / C4, channels c0 + 4 (idx % C4): the row offset is fixed for
  // the whole kernel, so it is computed once (32-bit: one layer's weights are < 2^31 floats)
  int b_row_off[BV];
  bool b_row_ok[BV];
#pragma unroll
  for (int v = 0; v < BV; ++v) {
    const int idx = tid + v * NTHREADS;
    const int gn = n0 + idx / C4;
    b_row_ok[v] = idx < BN * C4 && gn < a.N;
    b_row_off[v] = gn * a.ldw + ((idx % C4) << 2);
  }
  auto load_b = [&](int tap, int c0, f32x4 (&reg)[BV]) {
    const float* Wt = Wb + (long long)tap * a.w_ts;
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int idx = tid + v * NTHREADS;
      f32x4 val = {0.f, 0.f, 0.f, 0.f};
      if (idx < BN * C4) {
        if (!a.b_kn) {
          const int c = c0 + ((idx % C4) << 2);
          if (b_row_ok[v] && c < a.C_in) {
            const float* src = Wt + c0 + b_row_off[v];
            if (vec_b && c + 4 <= a.C_in) {
              val = *reinterpret_cast<const f32x4*>(src);
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) val[j] = (c + j < a.C_in) ? src[j] : 0.f;
            }
          }
        } else {
          const int cc = idx / (BN / 4);
          const int n4 = (idx - cc * (BN / 4)) << 2;
          const int gc = c0 + cc, gn = n0 + n4;
          if (gc < a.C_in && gn < a.N) {
            const float* src = Wt + (long long)gc * a.ldw + gn;
            if (vec_b && gn + 4 <= a.N) {
              val = *reinterpret_cast<const f32x4*>(src);
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) val[j] = (gn + j < a.N) ? src[j] : 0.f;
            }
          }
        }
      }
      reg[v] = val;
    }
  };
  auto store_b = [&](float* Bs, const f32x4 (&reg)[BV]) {
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int idx = tid + v * NTHREADS;
      if (idx < BN * C4) {
        if (!a.b_kn) {
          *reinterpret_cast<f32x4*>(&Bs[(idx / C4) * CKP + ((idx % C4) << 2)]) = reg[v];
        } else {
          const int cc = idx / (BN / 4);
          const int n4 = (idx - cc * (BN / 4)) << 2;
#pragma unroll
          for (int j = 0; j < 4; ++j) Bs[(n4 + j) * CKP + cc] = reg[v][j];
        }
      }
    }
  };
  // A tile: nrows_a x 32 channels of chunk c0 -> LDS, pre-activation applied, zero outside the input
  auto stage_a_serial = [&](int c0) {
    if constexpr (!TWO_D) {
      // 1-D: a thread keeps one 4-channel column and walks rows NTHREADS / C4 apart, so the source and LDS
      // addresses advance by constants (no per-element 64-bit index math)
      constexpr int RSTEP = NTHREADS / C4;
      const int c4 = (tid % C4) << 2;
      const int c = c0 + c4;
      const bool c_ok = c < a.C_in;
      const bool c_vec = vec_a && c + 4 <= a.C_in;
      int r = tid / C4;
      int g = row0 + r;
      const float* src = X + (long long)g * a.ldx + c;
      const long long src_step = (long long)RSTEP * a.ldx;
      for (; r < nrows_a; r += RSTEP, g += RSTEP, src += src_step) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (c_ok && g >= 0 && g < a.T_in) {
          if (c_vec) {
            v = *reinterpret_cast<const f32x4*>(src);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (c + j < a.C_in) ? src[j] : 0.f;
          }
          if (a.pre_act != ACT_NONE) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = act_fn(v[j], a.pre_act, a.pre_slope);
          }
          if (PM) {
            const float mk = PM[g];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] *= mk;
          }
        }
        *reinterpret_cast<f32x4*>(&As[r * CKP + c4]) = v;
      }
      return;
    }
    for (int idx = tid; idx < nrows_a * C4; idx += NTHREADS) {
      const int r = idx / C4;
      const int c4 = (idx % C4) << 2;
      const int c = c0 + c4;
      long long grow;
      bool valid;
      if (!TWO_D) {
        const int g = row0 + r;
        valid = (g >= 0) && (g < a.T_in);
        grow = g;
      } else {
        const int ah = r / aw, awi = r - ah * aw;
        const int gh = h0 - a.padh + ah, gw = w0 - a.padw + awi;
        valid = (gh >= 0) && (gh < a.T_in) && (gw >= 0) && (gw < a.W_in);
        grow = (long long)gh * a.W_in + gw;
      }
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (valid && c < a.C_in) {
        const float* src = X + grow * a.ldx + c;
        if (vec_a && c + 4 <= a.C_in) {
          v = *reinterpret_cast<const f32x4*>(src);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (c + j < a.C_in) ? src[j] : 0.f;
        }
        if (a.pre_act != ACT_NONE) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = act_fn(v[j], a.pre_act, a.pre_slope);
        }
        if (PM) {
          const float mk = PM[grow];
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] *= mk;
        }
      }
      *reinterpret_cast<f32x4*>(&As[r * CKP + c4]) = v;
    }
  };
  // batched staging: ASB float4 loads per thread in flight before the first wait, then the transform
  auto stage_a = [&](int c0) {
    if constexpr (ASB <= 1) {
      stage_a_serial(c0);
    } else {
      const int total = nrows_a * C4;
      for (int base = 0; base < total; base += ASB * NTHREADS) {
        f32x4 rv[ASB];
        float mk[ASB];
#pragma unroll
        for (int q = 0; q < ASB; ++q) {
          const int idx = base + tid + q * NTHREADS;
          rv[q] = f32x4{0.f, 0.f, 0.f, 0.f};
          mk[q] = 0.f;
          if (idx < total) {
            const int r = idx / C4;
            const int c = c0 + ((idx % C4) << 2);
            long long grow;
            bool valid;
            if (!TWO_D) {
              const int g = row0 + r;
              valid = (g >= 0) && (g < a.T_in);
              grow = g;
            } else {
              const int ah = r / aw, awi = r - ah * aw;
              const int gh = h0 - a.padh + ah, gw = w0 - a.padw + awi;
              valid = (gh >= 0) && (gh < a.T_in) && (gw >= 0) && (gw < a.W_in);
              grow = (long long)gh * a.W_in + gw;
            }
            if (valid && c < a.C_in) {
              mk[q] = PM ? PM[grow] : 1.f;
              const float* src = X + grow * a.ldx + c;
              if (vec_a && c + 4 <= a.C_in) {
                rv[q] = *reinterpret_cast<const f32x4*>(src);
              } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) rv[q][j] = (c + j < a.C_in) ? src[j] : 0.f;
              }
            }
          }
        }
#pragma unroll
        for (int q = 0; q < ASB; ++q) {
          const int idx = base + tid + q * NTHREADS;
          if (idx < total) {
            f32x4 v = rv[q];
            if (mk[q] != 0.f) {
              if (a.pre_act != ACT_NONE) {
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = act_fn(v[j], a.pre_act, a.pre_slope);
              }
              if (PM) {
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] *= mk[q];
              }
            } else {
              v = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            *reinterpret_cast<f32x4*>(&As[(idx / C4) * CKP + ((idx % C4) << 2)]) = v;
          }
        }
      }
    }
  };
  auto compute = [&](const float* Bs, int tap) {
    const int toff = TWO_D ? (tap / a.KW) * aw + (tap % a.KW) : tap * a.dil;
#pragma unroll
    for (int kk = 0; kk < CKT; kk += 8) {
      float av[TM][4], bv[TN][4];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(&As[(base[tm] + toff) * CKP + kk + hk * 4]);
        av[tm][0] = t[0]; av[tm][1] = t[1]; av[tm][2] = t[2]; av[tm][3] = t[3];
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(&Bs[(wn * TN * 32 + tn * 32 + li) * CKP + kk + hk * 4]);
        bv[tn][0] = t[0]; bv[tn][1] = t[1]; bv[tn][2] = t[2]; bv[tn][3] = t[3];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[tm][j], bv[tn][j], acc[tm][tn], 0, 0, 0);
    }
  };

  const int nchunks = (a.C_in + CKT - 1) / CKT;
  if (!PIPE) {
    f32x4 breg[BV];
    const int total = nchunks * a.taps;
    const int per = (total + ksplit - 1) / ksplit;
    const int it0 = zsplit * per, it1 = min(total, it0 + per);
    int it = it0;
    while (it < it1) {
      const int ch = it / a.taps;
      __syncthreads();
      stage_a(ch * CKT);
      for (int tap = it - ch * a.taps; tap < a.taps && it < it1; ++tap, ++it) {
        if (it > it0 && tap != it0 - ch * a.taps) __syncthreads();
        load_b(tap, ch * CKT, breg);
        store_b(Bs0, breg);
        __syncthreads();
        compute(Bs0, tap);
      }
    }
  } else {
    // PIPE (1-D, taps == 1, stride 1: a plain GEMM over C_in): A and B both double-buffered in LDS; the next
    // chunk's tiles are fetched into registers while the MFMAs consume the current ones, then written to
    // the other buffers; one barrier per chunk. Small-M GEMMs (HuBERT at 775 rows, TextEncoder/flow at
    // 1550) otherwise expose two dependent global-load latencies per 32-channel chunk.
    constexpr int AV = (BM * C4 + NTHREADS - 1) / NTHREADS;
    float* const A0 = smem;
    float* const A1 = smem + BM * CKP;
    float* const B0 = smem + 2 * BM * CKP;
    float* const B1 = B0 + BN * CKP;
    f32x4 areg[AV];
    float amk[AV];
    f32x4 breg[BV];
    auto load_a = [&](int c0) {
#pragma unroll
      for (int v = 0; v < AV; ++v) {
        const int idx = tid + v * NTHREADS;
        areg[v] = f32x4{0.f, 0.f, 0.f, 0.f};
        amk[v] = 0.f;
        if (idx < BM * C4) {
          const int r = idx / C4;
          const int c = c0 + ((idx % C4) << 2);
          const int g = row0 + r;
          if (g >= 0 && g < a.T_in && c < a.C_in) {
            amk[v] = PM ? PM[g] : 1.f;
            const float* src = X + (long long)g * a.ldx + c;
            if (vec_a && c + 4 <= a.C_in) {
              areg[v] = *reinterpret_cast<const f32x4*>(src);
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) areg[v][j] = (c + j < a.C_in) ? src[j] : 0.f;
            }
          }
        }
      }
    };
    auto store_a = [&](float* dst) {
#pragma unroll
      for (int v = 0; v < AV; ++v) {
        const int idx = tid + v * NTHREADS;
        if (idx < BM * C4) {
          f32x4 val = areg[v];
          if (amk[v] != 0.f) {
            if (a.pre_act != ACT_NONE) {
#pragma unroll
              for (int j = 0; j < 4; ++j) val[j] = act_fn(val[j], a.pre_act, a.pre_slope);
            }
            if (PM) {
#pragma unroll
              for (int j = 0; j < 4; ++j) val[j] *= amk[v];
            }
          } else {
            val = f32x4{0.f, 0.f, 0.f, 0.f};
          }
          *reinterpret_cast<f32x4*>(&dst[(idx / C4) * CKP + ((idx % C4) << 2)]) = val;
        }
      }
    };
    const int per = (nchunks + ksplit - 1) / ksplit;
    const int it0 = zsplit * per, it1 = min(nchunks, it0 + per);
    if (it0 < it1) {
      load_a(it0 * CKT);
      load_b(0, it0 * CKT, breg);
      store_a(A0);
      store_b(B0, breg);
      __syncthreads();
      for (int it = it0; it < it1; ++it) {
        const bool odd = (it - it0) & 1;
        const bool more = it + 1 < it1;
        if (more) {
          load_a((it + 1) * CKT);
          load_b(0, (it + 1) * CKT, breg);
        }
        As = odd ? A1 : A0;
        compute(odd ? B1 : B0, 0);
        if (more) {
          store_a(odd ? A0 : A1);
          store_b(odd ? B0 : B1, breg);
        }
        __syncthreads();
      }
    }
  }

  // ---- epilogue
  conv_store_tile<TM, TN, WM, WN, TWO_D>(a, TilePos{m0, h0, w0, rw, rh, n0, b, bi, zb, zsplit, ksplit}, acc, smem);
}

// split-K combine: sums the ksplit partial tiles in slice order (deterministic) and applies the epilogue. Grid
// (x: elements of one batch entry, y: batch entry); 32-bit element index within an entry (launch checks), all
// ksplit slab loads of an element issued before the ordered sum
__global__ void splitk_reduce_kernel(const ConvArgs a, const int ksplit, const int two_d) {
  const unsigned per_b = (unsigned)(a.ws_rows * a.N);
  const int zb = blockIdx.y;
  const int b = zb / a.batch_inner, bi = zb - (zb / a.batch_inner) * a.batch_inner;
  const float* bias = a.bias ? a.bias + (long long)b * a.bias_bs + (long long)bi * a.bias_bs2 : nullptr;
  const float* R = a.res ? a.res + (long long)b * a.res_bs + (long long)bi * a.res_bs2 : nullptr;
  const float* MK = a.mask ? a.mask + (long long)b * a.mask_bs : nullptr;
  float* Y = a.y + (long long)b * a.y_bs + (long long)bi * a.y_bs2;
  const float* base = a.ws + (long long)zb * ksplit * per_b;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < per_b; i += gridDim.x * blockDim.x) {
    const unsigned m = i / (unsigned)a.N;
    const int n = (int)(i - m * (unsigned)a.N);
    const float* p = base + i;
    float v = 0.f;
    int s = 0;
    for (; s + 4 <= ksplit; s += 4) {
      const float p0 = p[(long long)s * per_b], p1 = p[(long long)(s + 1) * per_b];
      const float p2 = p[(long long)(s + 2) * per_b], p3 = p[(long long)(s + 3) * per_b];
      v += p0;
      v += p1;
      v += p2;
      v += p3;
    }
    for (; s < ksplit; ++s) v += p[(long long)s * per_b];
    int oh = 0, ow = 0;
    if (two_d) {
      oh = (int)(m / (unsigned)a.W_out);
      ow = (int)(m - (unsigned)oh * (unsigned)a.W_out);
    }
    epilogue_store(a, v, bias ? bias[n] : 0.f, m, n, oh, ow, R, MK, Y);
  }
}

// split-K combine + the post-norm LayerNorm (ConvArgs::ln_g): one 256-thread block per output row, thread t holding
// columns t + 256 j (N <= 1024); every slab load of a column issued before its ordered sum, as in splitk_reduce_kernel
// (a wave per row with the loads in a column loop measured 16 us against 5.6 + 7 for the two passes). The arithmetic
// is splitk_reduce_kernel's epilogue followed by k_layernorm's on (res + v); the mean and variance sum the columns in
// another order (block-wide), so the result equals the two passes to fp32 rounding of those sums.
__device__ __forceinline__ float wave_sum64(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__global__ __launch_bounds__(256) void splitk_reduce_ln_kernel(const ConvArgs a, const int ksplit) {
  __shared__ float red[2][4];
  const long long row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = (int)(row / a.ws_rows);
  const long long m = row - (long long)b * a.ws_rows;
  const long long per_b = a.ws_rows * a.N;
  const float* bias = a.bias ? a.bias + (long long)b * a.bias_bs : nullptr;
  const float* R = a.res + (long long)b * a.res_bs + m * a.ldr;
  const float mk = a.mask ? a.mask[(long long)b * a.mask_bs + m] : 1.f;
  float* Y = a.y + (long long)b * a.y_bs + m * a.ldy;
  const float* base = a.ws + (long long)b * ksplit * per_b + m * a.N;
  float v[4];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = tid + j * 256;
    float t = 0.f;
    if (n < a.N) {
      const float* p = base + n;
      float acc = 0.f;
      int k = 0;
      for (; k + 4 <= ksplit; k += 4) {  // splitk_reduce_kernel's order
        const float p0 = p[(long long)k * per_b], p1 = p[(long long)(k + 1) * per_b];
        const float p2 = p[(long long)(k + 2) * per_b], p3 = p[(long long)(k + 3) * per_b];
        acc += p0;
        acc += p1;
        acc += p2;
        acc += p3;
      }
      for (; k < ksplit; ++k) acc += p[(long long)k * per_b];
      if (bias) acc += bias[n];  // epilogue_store's order: bias, alpha, act, (mask)
      if (a.alpha != 1.f) acc *= a.alpha;
      acc = act_fn(acc, a.act, a.slope);
      if (a.mask) acc *= mk;
      t = R[n];
      t = t + acc;
    }
    v[j] = t;
    s += t;
  }
  s = wave_sum64(s);
  if (lane == 0) red[0][wave] = s;
  __syncthreads();
  const float mean = ((red[0][0] + red[0][1]) + (red[0][2] + red[0][3])) / (float)a.N;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = tid + j * 256;
    if (n < a.N) {
      const float d = v[j] - mean;
      q += d * d;
    }
  }
  q = wave_sum64(q);
  if (lane == 0) red[1][wave] = q;
  __syncthreads();
  const float var = ((red[1][0] + red[1][1]) + (red[1][2] + red[1][3])) / (float)a.N;
  const float rstd = 1.f / sqrtf(var + a.ln_eps);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = tid + j * 256;
    if (n < a.N) Y[n] = (v[j] - mean) * rstd * a.ln_g[n] + a.ln_b[n];
  }
}

// Contractions far shorter than one 32-channel MFMA chunk (C_in <= 4 and at most 16 MACs per output: RMVPE's 3x3
// and 1x1 convs on the 1-channel mel image, the generator's last 1-tap noise conv) would run the MFMA tile on
// >= 87 % zero padding: one thread per output element instead, an fp32 fma chain over (tap, channel), then the
// shared epilogue. (The long-tap C_in = 1 noise convs stay on the MFMA kernel: 80 dependent loads per output
// measured 351 vs 110 us.) Outputs are n-fastest,
// so stores and weight reads coalesce and a thread group shares its input rows through L1.
template <bool TWO_D>
__global__ void conv_tiny_kernel(const ConvArgs a) {
  // 32-bit index math (launch_tiny checks the sizes): one output element per thread, n fastest
  const int rows = TWO_D ? a.T_out * a.W_out : a.T_out;
  const int per_b = rows * a.N;
  const int total = per_b * a.batch * a.batch_inner;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int zb = i / per_b;
    const int rem = i - zb * per_b;
    const int m = rem / a.N;
    const int n = rem - m * a.N;
    const int b = zb / a.batch_inner, bi = zb - (zb / a.batch_inner) * a.batch_inner;
    const float* X = a.x + (long long)b * a.x_bs + (long long)bi * a.x_bs2;
    const float* Wb = a.w + (long long)b * a.w_bs + (long long)bi * a.w_bs2;
    const float* PM = a.pre_mask ? a.pre_mask + (long long)b * a.pre_mask_bs : nullptr;
    int oh = 0, ow = 0;
    if (TWO_D) {
      oh = m / a.W_out;
      ow = m - oh * a.W_out;
    }
    float acc = 0.f;
    for (int tap = 0; tap < a.taps; ++tap) {
      int g;
      if (!TWO_D) {
        g = m * a.stride - a.pad + tap * a.dil;
        if (g < 0 || g >= a.T_in) continue;
      } else {
        const int kh = tap / a.KW;
        const int gh = oh - a.padh + kh, gw = ow - a.padw + (tap - kh * a.KW);
        if (gh < 0 || gh >= a.T_in || gw < 0 || gw >= a.W_in) continue;
        g = gh * a.W_in + gw;
      }
      const float pm = (PM && !TWO_D) ? PM[g] : 1.f;
      const float* Wt = Wb + (long long)tap * a.w_ts;
      for (int c = 0; c < a.C_in; ++c) {
        const float v = act_fn(X[(long long)g * a.ldx + c], a.pre_act, a.pre_slope) * pm;
        const float wv = a.b_kn ? Wt[(long long)c * a.ldw + n] : Wt[(long long)n * a.ldw + c];
        acc = fmaf(v, wv, acc);
      }
    }
    const float* bias = a.bias ? a.bias + (long long)b * a.bias_bs + (long long)bi * a.bias_bs2 : nullptr;
    const float* R = a.res ? a.res + (long long)b * a.res_bs + (long long)bi * a.res_bs2 : nullptr;
    const float* MK = a.mask ? a.mask + (long long)b * a.mask_bs : nullptr;
    float* Y = a.y + (long long)b * a.y_bs + (long long)bi * a.y_bs2;
    epilogue_store(a, acc, bias ? bias[n] : 0.f, m, n, oh, ow, R, MK, Y);
  }
}

// The tiny contractions whose epilogue is only bias + activation + store (the RMVPE U-Net's first ConvBlockRes on the
// 1-channel mel image: the 3x3 1 -> 16 conv and the 1x1 shortcut), one thread per output ROW computing all N <= 32
// outputs: the weights and bias in LDS, the <= 16 inputs read once instead of once per output, the activation a
// compile-time choice, float4 stores. (conv_tiny_kernel's per-element index math, activation switch and shared epilogue
// took 100-135 us for these two 3.2 M-output convs.)
template <bool TWO_D, int N, int ACT>
__global__ __launch_bounds__(256) void conv_tiny_rows_kernel(const ConvArgs a) {
  __shared__ float ws[16 * 32], bs[32];
  const int ck = a.C_in * a.taps;  // <= 16
  for (int i = threadIdx.x; i < ck * N; i += blockDim.x) {
    const int tap = i / (a.C_in * N), r = i - tap * (a.C_in * N);
    const int n = r / a.C_in, c = r - n * a.C_in;
    ws[(tap * a.C_in + c) * N + n] = a.w[(long long)tap * a.w_ts + (long long)n * a.ldw + c];
  }
  if (threadIdx.x < N) bs[threadIdx.x] = a.bias ? a.bias[threadIdx.x] : 0.f;
  __syncthreads();
  const int rows = TWO_D ? a.T_out * a.W_out : a.T_out;
  const int total = rows * a.batch;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int b = i / rows, m = i - b * rows;
    const float* X = a.x + (long long)b * a.x_bs;
    float acc[N];
#pragma unroll
    for (int n = 0; n < N; ++n) acc[n] = 0.f;
    int oh = 0, ow = m;
    if (TWO_D) {
      oh = m / a.W_out;
      ow = m - oh * a.W_out;
    }
    for (int tap = 0; tap < a.taps; ++tap) {
      int g;
      if (!TWO_D) {
        g = m * a.stride - a.pad + tap * a.dil;
        if (g < 0 || g >= a.T_in) continue;
      } else {
        const int kh = tap / a.KW;
        const int gh = oh - a.padh + kh, gw = ow - a.padw + (tap - kh * a.KW);
        if (gh < 0 || gh >= a.T_in || gw < 0 || gw >= a.W_in) continue;
        g = gh * a.W_in + gw;
      }
      for (int c = 0; c < a.C_in; ++c) {
        const float v = X[(long long)g * a.ldx + c];
        const float* wr = ws + (tap * a.C_in + c) * N;
#pragma unroll
        for (int n = 0; n < N; ++n) acc[n] = fmaf(v, wr[n], acc[n]);
      }
    }
    float* Y = a.y + (long long)b * a.y_bs + (long long)m * a.ldy;
#pragma unroll
    for (int n = 0; n < N; n += 4) {
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[n + e] + bs[n + e];  // conv_tiny_kernel's order: the fma chain, then the bias
        if (ACT == ACT_RELU) v = v > 0.f ? v : 0.f;
        else if (ACT == ACT_LRELU) v = v > 0.f ? v : v * a.slope;
        o[e] = v;
      }
      *reinterpret_cast<f32x4*>(Y + n) = o;
    }
  }
}

// 1x1 convs with few inputs and outputs (the U-Net's ConvBlockRes shortcuts: 16 -> 32, 64 -> 32, 32 -> 16 channels on
// 50 k - 200 k pixels; round 5): one thread per pixel, its C_in inputs as float4 loads, the weights [C_in][N] and bias in
// LDS (broadcast reads), N fp32 fma chains, bias + activation, float4 stores. Exact fp32 (the native-f32 MFMA GEMM it
// replaces took 13-23 us for these byte-bound shapes).
template <int N, int ACT>
__global__ __launch_bounds__(256) void conv_rows1x1_kernel(const ConvArgs a) {
  // (staging the block's input rows through LDS for coalesced loads measured slower: 16 / 20 us vs 12 / 18, r05aq)
  __shared__ __attribute__((aligned(16))) float ws[64 * 32];
  __shared__ float bs[32];
  const int C = a.C_in;
  for (int i = threadIdx.x; i < C * N; i += blockDim.x) {
    const int n = i / C, c = i - n * C;
    ws[c * N + n] = a.w[(long long)n * a.ldw + c];
  }
  if (threadIdx.x < N) bs[threadIdx.x] = a.bias ? a.bias[threadIdx.x] : 0.f;
  __syncthreads();
  const int rows = a.W_out > 0 ? a.T_out * a.W_out : a.T_out;
  const int total = rows * a.batch;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int b = i / rows, m = i - b * rows;
    const f32x4* X = reinterpret_cast<const f32x4*>(a.x + (long long)b * a.x_bs + (long long)m * a.ldx);
    float acc[N];
#pragma unroll
    for (int n = 0; n < N; ++n) acc[n] = 0.f;
    for (int c4 = 0; c4 < C / 4; ++c4) {
      const f32x4 v = X[c4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const f32x4* wr = reinterpret_cast<const f32x4*>(ws + (4 * c4 + e) * N);
#pragma unroll
        for (int n4 = 0; n4 < N / 4; ++n4) {
          const f32x4 w = wr[n4];
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[4 * n4 + k] = fmaf(v[e], w[k], acc[4 * n4 + k]);
        }
      }
    }
    float* Y = a.y + (long long)b * a.y_bs + (long long)m * a.ldy;
#pragma unroll
    for (int n = 0; n < N; n += 4) {
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[n + e] + bs[n + e];
        if (ACT == ACT_RELU) v = v > 0.f ? v : 0.f;
        else if (ACT == ACT_LRELU) v = v > 0.f ? v : v * a.slope;
        o[e] = v;
      }
      *reinterpret_cast<f32x4*>(Y + n) = o;
    }
  }
}

namespace {

// conv_tiny_rows_kernel's shapes: only bias + activation in the epilogue, N in {16, 32}, 16-B aligned output rows
inline bool tiny_rows_fits(const ConvArgs& a) {
  return (a.N == 16 || a.N == 32) && a.pre_act == ACT_NONE && !a.pre_mask && !a.b_kn && a.batch_inner == 1 &&
         a.out_map == OUT_ROWS && a.res_mode == RES_NONE && !a.mask && a.acc_mode == ACC_STORE && a.alpha == 1.f &&
         (a.act == ACT_NONE || a.act == ACT_RELU || a.act == ACT_LRELU) && (a.ldy & 3) == 0 && (a.y_bs & 3) == 0 &&
         (reinterpret_cast<uintptr_t>(a.y) & 15) == 0 && a.gate_h == 0;
}

constexpr int TINY_MAX_CIN = 4;
inline bool tiny_fits(const ConvArgs& a) {
  const long long rows = a.W_out > 0 ? (long long)a.T_out * a.W_out : a.T_out;
  return a.C_in <= TINY_MAX_CIN && a.C_in * a.taps <= 16 && a.force_cfg < 0 &&
         rows * a.N * a.batch * a.batch_inner < (1LL << 30);
}

// conv_rows1x1_kernel's shapes: a 1x1 / stride-1 conv (1-D or 2-D) with C_in a multiple of 4 up to 64, 16-B aligned
// input rows, and conv_tiny_rows_kernel's epilogue conditions
inline bool rows1x1_fits(const ConvArgs& a, bool two_d) {
  if (a.taps != 1 || a.stride != 1 || a.dil != 1 || a.pad != 0 || a.force_cfg >= 0) return false;
  if (two_d && (a.KH != 1 || a.KW != 1 || a.padh != 0 || a.padw != 0 || a.T_in != a.T_out || a.W_in != a.W_out))
    return false;
  const long long rows = two_d ? (long long)a.T_out * a.W_out : a.T_out;
  return tiny_rows_fits(a) && a.C_in % 4 == 0 && a.C_in >= 4 && a.C_in <= 64 && (a.ldx & 3) == 0 &&
         (a.x_bs & 3) == 0 && (reinterpret_cast<uintptr_t>(a.x) & 15) == 0 && rows * a.batch < (1LL << 31) - 65536LL * 256;
}

hipError_t launch_rows1x1(const ConvArgs& a, bool two_d, hipStream_t s) {
  const long long rows = two_d ? (long long)a.T_out * a.W_out : a.T_out;
  const unsigned nb = (unsigned)std::min<long long>((rows * a.batch + 255) / 256, 65536);
  ConvArgs b = a;
  if (!two_d) b.W_out = 0;
#define ROWS1(NN, AC) hipLaunchKernelGGL((conv_rows1x1_kernel<NN, AC>), dim3(nb), dim3(256), 0, s, b)
  const int act = a.act;
  if (a.N == 16) { if (act == ACT_RELU) ROWS1(16, ACT_RELU); else if (act == ACT_LRELU) ROWS1(16, ACT_LRELU); else ROWS1(16, ACT_NONE); }
  else { if (act == ACT_RELU) ROWS1(32, ACT_RELU); else if (act == ACT_LRELU) ROWS1(32, ACT_LRELU); else ROWS1(32, ACT_NONE); }
#undef ROWS1
  return hipGetLastError();
}

hipError_t launch_tiny(const ConvArgs& a, bool two_d, hipStream_t s) {
  const long long rows = two_d ? (long long)a.T_out * a.W_out : a.T_out;
  const long long total = rows * a.N * a.batch * a.batch_inner;
  if (total >= (1LL << 31) - 65536LL * 256) return hipErrorInvalidValue;  // 32-bit indexing in the kernel
  if (tiny_rows_fits(a)) {
    const long long nr = total / a.N;
    const unsigned nbr = (unsigned)std::min<long long>((nr + 255) / 256, 65536);
#define TINY_ROWS(TD, NN, AC) hipLaunchKernelGGL((conv_tiny_rows_kernel<TD, NN, AC>), dim3(nbr), dim3(256), 0, s, a)
    const int act = a.act;
    if (two_d) {
      if (a.N == 16) { if (act == ACT_RELU) TINY_ROWS(true, 16, ACT_RELU); else if (act == ACT_LRELU) TINY_ROWS(true, 16, ACT_LRELU); else TINY_ROWS(true, 16, ACT_NONE); }
      else { if (act == ACT_RELU) TINY_ROWS(true, 32, ACT_RELU); else if (act == ACT_LRELU) TINY_ROWS(true, 32, ACT_LRELU); else TINY_ROWS(true, 32, ACT_NONE); }
    } else {
      if (a.N == 16) { if (act == ACT_RELU) TINY_ROWS(false, 16, ACT_RELU); else if (act == ACT_LRELU) TINY_ROWS(false, 16, ACT_LRELU); else TINY_ROWS(false, 16, ACT_NONE); }
      else { if (act == ACT_RELU) TINY_ROWS(false, 32, ACT_RELU); else if (act == ACT_LRELU) TINY_ROWS(false, 32, ACT_LRELU); else TINY_ROWS(false, 32, ACT_NONE); }
    }
#undef TINY_ROWS
    return hipGetLastError();
  }
  long long nb = (total + 255) / 256;
  if (nb > 65536) nb = 65536;
  if (two_d) hipLaunchKernelGGL(conv_tiny_kernel<true>, dim3((unsigned)nb), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(conv_tiny_kernel<false>, dim3((unsigned)nb), dim3(256), 0, s, a);
  return hipGetLastError();
}

// the split-K combine of a gated WaveNet in_layer (ConvArgs::gate_h): the pair (c, c + H) of one output row per thread
// (k_gate's arithmetic, aux_kernels.hip), acts [rows][ldy]
__global__ void splitk_reduce_gate_kernel(const ConvArgs a, const int ksplit) {
  const unsigned H = (unsigned)a.gate_h;
  const unsigned per_b = (unsigned)(a.ws_rows * a.N), per_o = (unsigned)a.ws_rows * H;
  const int b = blockIdx.y;
  const float* g = a.gate_g + (long long)b * a.gate_g_bs;
  float* Y = a.y + (long long)b * a.y_bs;
  const float* base = a.ws + (long long)b * ksplit * per_b;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < per_o; i += gridDim.x * blockDim.x) {
    const unsigned m = i / H, c = i - m * H;
    const float* p = base + (size_t)m * a.N + c;
    float u = 0.f, v = 0.f;
    for (int s = 0; s < ksplit; ++s) {
      u += p[(long long)s * per_b];
      v += p[(long long)s * per_b + H];
    }
    if (a.bias) {
      u += a.bias[c];
      v += a.bias[c + H];
    }
    const float ta = u + g[c], sb = v + g[c + H];
    Y[(long long)m * a.ldy + c] = tanhf(ta) * (1.f / (1.f + expf(-sb)));
  }
}

hipError_t launch_splitk_reduce(const ConvArgs& a, int ksplit, bool two_d, hipStream_t s) {
  if (a.ln_g) {
    if (two_d || a.batch_inner != 1 || a.N > 1024 || !a.ln_b || !a.res || a.res_mode != RES_NONE ||
        a.acc_mode != ACC_STORE || a.out_map != OUT_ROWS || a.gate_h > 0)
      return hipErrorInvalidValue;
    const long long rows = (long long)a.batch * a.ws_rows;
    if (rows >= (1LL << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(splitk_reduce_ln_kernel, dim3((unsigned)rows), dim3(256), 0, s, a, ksplit);
    return hipGetLastError();
  }
  if (a.gate_h > 0) {
    if (two_d || a.batch_inner != 1 || a.N != 2 * a.gate_h || !a.gate_g) return hipErrorInvalidValue;
    const long long per_o = a.ws_rows * a.gate_h;
    hipLaunchKernelGGL(splitk_reduce_gate_kernel, dim3((unsigned)std::min<long long>((per_o + 255) / 256, 4096),
                                                       (unsigned)a.batch), dim3(256), 0, s, a, ksplit);
    return hipGetLastError();
  }
  const long long per_b = (long long)a.ws_rows * a.N;
  const int nz = a.batch * a.batch_inner;
  if (per_b >= (1LL << 31) || nz > 65535) return hipErrorInvalidValue;  // 32-bit element index, grid y
  long long nb = (per_b + 255) / 256;
  if (nb > 8192) nb = 8192;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)nb, (unsigned)nz), dim3(256), 0, s, a, ksplit,
                     two_d ? 1 : 0);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, bool TWO_D, bool PIPE = false, int ASB = 1, int CKT = CK>
hipError_t launch_cfg(const ConvArgs& a, hipStream_t s) {
  constexpr int CKP = CKT + 4;
  int nrows_a, rw = 0, rh = 0, tiles_w = 1, mtiles;
  if (!TWO_D) {
    nrows_a = (BM - 1) * a.stride + (a.taps - 1) * a.dil + 1;
    mtiles = (a.T_out + BM - 1) / BM;
  } else {
    rw = a.W_out < BM ? a.W_out : BM;
    rh = BM / rw;
    tiles_w = (a.W_out + rw - 1) / rw;
    mtiles = ((a.T_out + rh - 1) / rh) * tiles_w;
    nrows_a = (rh + a.KH - 1) * (rw + a.KW - 1);
  }
  if (PIPE && (TWO_D || a.taps != 1 || a.stride != 1)) return hipErrorInvalidValue;
  size_t smem = (size_t)(PIPE ? 2 : 1) * (nrows_a + BN) * CKP * sizeof(float);
  smem = std::max(smem, (size_t)4 * 32 * 33 * sizeof(float));  // epilogue staging slots (2x2-per-wave tiles)
  if (smem > 160 * 1024) return hipErrorInvalidValue;
  const int vec_a = ((a.ldx & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.x) & 15) == 0) &&
                    ((a.x_bs & 3) == 0) && ((a.x_bs2 & 3) == 0);
  const int vec_b = ((a.ldw & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.w) & 15) == 0) &&
                    ((a.w_bs & 3) == 0) && ((a.w_bs2 & 3) == 0) && ((a.w_ts & 3) == 0);
  if (a.batch_inner < 1) return hipErrorInvalidValue;
  int ksplit = 1;
  if (a.ws && a.ksplit > 1) ksplit = a.ksplit;
  const int ntiles = (a.N + BN - 1) / BN;
  const int ntn = ntiles;  // XCD-contiguous tile runs (conv_block_coords)
  dim3 grid(ntn ? mtiles * ntiles : mtiles, ntn ? 1 : ntiles, a.batch * a.batch_inner * ksplit);
  auto kern = conv_gemm_kernel<BM, BN, WM, WN, TWO_D, PIPE, ASB, CKT>;
  static size_t smem_set = 64 * 1024;  // per instantiation: raise the dynamic-LDS limit once, not per launch
  if (smem > smem_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    smem_set = smem;
  }
  hipLaunchKernelGGL(kern, grid, dim3(NTHREADS), smem, s, a, nrows_a, rw, rh, tiles_w, vec_a, vec_b, ksplit, ntn);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || ksplit == 1) return e;
  return launch_splitk_reduce(a, ksplit, TWO_D, s);
}

template <bool TWO_D, bool PIPE, int ASB>
hipError_t launch_forced_asb(const ConvArgs& a, hipStream_t s) {
  switch (a.force_cfg) {
    case 0: return launch_cfg<256, 32, 4, 1, TWO_D, PIPE, ASB>(a, s);
    case 1: return launch_cfg<128, 32, 4, 1, TWO_D, PIPE, ASB>(a, s);
    case 2: return launch_cfg<128, 64, 2, 2, TWO_D, PIPE, ASB>(a, s);
    case 3: return launch_cfg<64, 64, 2, 2, TWO_D, PIPE, ASB>(a, s);
    case 4: return launch_cfg<128, 128, 2, 2, TWO_D, PIPE, ASB>(a, s);
    case 5: return launch_cfg<64, 128, 2, 2, TWO_D, PIPE, ASB>(a, s);
    case 6: return launch_cfg<256, 64, 4, 1, TWO_D, PIPE, ASB>(a, s);
    case 7: return launch_cfg<64, 64, 2, 2, TWO_D, PIPE, ASB, 64>(a, s);
    case 8: return launch_cfg<128, 32, 4, 1, TWO_D, PIPE, ASB, 64>(a, s);
    case 9: return launch_cfg<128, 128, 2, 2, TWO_D, PIPE, ASB, 64>(a, s);
    default: return hipErrorInvalidValue;
  }
}

// A-tile staging: serial (1, the default) or 4 loads in flight per thread (ConvArgs::astage = 4)
template <bool TWO_D, bool PIPE>
hipError_t launch_forced(const ConvArgs& a, hipStream_t s) {
  const int asb = a.astage > 0 ? a.astage : 1;
  if (!PIPE && asb >= 4) return launch_forced_asb<TWO_D, false, 4>(a, s);
  return launch_forced_asb<TWO_D, PIPE, 1>(a, s);
}

// Tile per shape class, measured on MI355X (same-box A/B of the whole pipeline, tools/ab_policy.sh):
// one 32x32 accumulator per wave with 4 waves per block beats the larger per-wave tiles in the pipeline:
// 128x32 for N <= 32 and for the long-tap 1-D convs (the generator's dilated ResBlock convs), 64x64
// otherwise; split-K when the output grid cannot fill 256 CUs.
inline int env_cfg(const char* name, int dflt) {
  const char* e = rvcx_knob(name);
  return e ? std::atoi(e) : dflt;
}
// contraction arithmetic: 1 = native fp32 MFMA (conv_gemm_kernel), 2 = fp32 through the 3-way bf16 split everywhere
// (conv_emu.hip), 3 (the default) = as 2 except the weight-streamed kernel and the fused ResBlock pairs (the generator),
// which take the two-plane fp16 split (the WSPLIT_H16 / RB_WF16 images: three MFMA products per step instead of six,
// measured as accurate as native fp32, bench_conv / tests/test_gpu_conv_math.py); ConvArgs::math overrides
// RVCX_CONV_MATH (f32 | split | h16)
inline int conv_math(const ConvArgs& a) {
  static const int env = [] {
    const char* e = rvcx_knob("RVCX_CONV_MATH");
    if (e && (std::string(e) == "f32" || std::string(e) == "1")) return 1;
    if (e && (std::string(e) == "split" || std::string(e) == "2")) return 2;
    return 3;
  }();
  return a.math > 0 ? a.math : env;
}

// Tile per shape class in split mode, from build/bench_conv on MI355X (TF/s, split vs the native fp32 kernel):
// long-tap convs 128x32 (C128 k11 155 vs 114, C256 k11 138 vs 106), short taps and GEMMs 64x64 (C128 k3 + residual
// 101 vs 78, HuBERT qkv 52 vs 38), narrow short convs (N <= 32, taps < 5: the 32-channel ResBlock k=3, latency
// bound) stay on the native kernel (53 vs 47): both arithmetics are fp32 accurate, so the choice is per shape. The
// U-Net's 3x3 convs: 64x64 (C2 26.7 -> 25.9 ms vs 128x64)
template <bool TWO_D>
int pick_emu(const ConvArgs& a) {
  if (TWO_D) return a.N <= 32 ? 12 : 13;
  if (a.N <= 32) return a.taps >= 5 ? 12 : 1;
  if (a.taps >= 5) return 12;
  return 13;
}

template <bool TWO_D>
int pick_cfg(const ConvArgs& a) {
  if (a.force_cfg >= 0) return a.force_cfg;
  if (conv_math(a) >= 2) return pick_emu<TWO_D>(a);
  // N <= 32 and the 1-D convs with taps >= 5 (A/B: 32.8 vs 33.6 ms): 128 x 32; everything else 64 x 64
  if (a.N <= 32) return 1;
  if (!TWO_D && a.taps >= 5) return 1;
  return 3;
}

inline void cfg_tile(int cfg, int& BM, int& BN) {
  if (conv_emu_tile(cfg, BM, BN)) return;
  static const int t[10][2] = {{256, 32}, {128, 32}, {128, 64}, {64, 64}, {128, 128}, {64, 128}, {256, 64},
                               {64, 64}, {128, 32}, {128, 128}};
  BM = t[cfg][0];
  BN = t[cfg][1];
}

// weight-streamed split kernel (conv_wsb.hip) tiles: 256x32 for N <= 32, else 128x64 (2 x 2 waves of 64 x 32;
// RVCX_WCFG_* override). bench_conv on MI355X with the register epilogue (TF/s, vs the LDS-staged split kernel's
// best tile): C256 k11 174 vs 142, C128 k11 204 vs 160, C128 k7 185 vs 144, C128 k3 124 vs 118, ConvTranspose
// phases 105 / 124 / 94 vs 95 / 117 / 96; the 32-channel convs lose (C32 k11 95 vs 115).
// Round 3: the same tiles on v_mfma_f32_16x16x32_bf16 (cfg 24 / 23) hold a higher clock under the power-limited load
// (bench_conv r03h, same box, 32x32x16 -> 16x16x32 TF/s: C128 k11 198 -> 214, k7 181 -> 194, k3 124 -> 131, C256 k11
// 171 -> 182, C64 k11 177 -> 190, ConvTranspose phases 108 / 125 / 94 -> 114 / 129 / 99).
// Round 3, wave layout per shape (cfg 23 = 2 x 2 waves of 64 x 32, 27 = 1 x 4 waves of 128 x 16, 28 = 256 x 64 as
// 2 x 2 waves of 128 x 32). bench_conv r03bc (warm, TF/s): short taps (k = 3 ResBlock convs, ConvTranspose phases)
// gain on 27 (C128 k3+res 141 -> 159, C64 k3+res 90 -> 109, up3 152 -> 159: a wave's 3 B loads per step feed 8 row
// blocks), k = 7 / 11 at C_in <= 128 a little on 28 (C128 k11 244 -> 252), C256 k11 loses on 28 (208 -> 171). In the
// C2 step (rocprof r03ab, weight-streamed time per step): 27 for k <= 3 7969 -> 7919 us, 28 for k = 7 / 11 +147 us
// (cold activations, 2 workgroups per CU), so the long convs stay on 23 (RVCX_WCFG_LONG=28 to compare)
// Round 6: the 128-channel k = 7 / 11 convs on 128 x 128 tiles (cfg 25, 2 x 2 waves of 64 x 64: C128 k11 402 vs 380
// TF, k7 346 vs 340 in bench_conv r06a; same-box C2 12.91 / 12.99 vs 13.04 / 13.01 ms, r06b); at 256 input channels
// (C256 k11 288 vs 330) and 64 output channels (half of each tile idle) cfg 23 stays. RVCX_WCFG_LONG forces one tile
// for every long conv (A/B aid)
inline int pick_wsb(const ConvArgs& a) {
  static const int c_long = env_cfg("RVCX_WCFG_LONG", 0);
  if (a.wsb == 2) return 30;  // gather-streamed (conv_gs.hip): the short contractions
  if (a.N <= 32) return 24;
  // the wide ConvTranspose phase group of the second upsample (18600 rows x 1280 columns, 2 taps) on 128 x 128 tiles:
  // bench_conv r06a h25 254.6 vs h27 232.2 TF (the first one, 1550 rows x 3072, loses there: 189 vs 206)
  if (a.taps <= 3 && a.N >= 1024 && a.T_out >= 8192 && a.C_in < 512 && c_long == 0) return 25;
  if (a.taps <= 3) return 27;
  if (c_long > 0) return c_long;
  return (a.C_in < 256 && a.N >= 128) ? 25 : 23;
}
}  // namespace
int conv_wsb_pick(const ConvArgs& a) {
  ConvArgs b = a;
  b.wsb = 1;
  return pick_wsb(b);
}
thread_local int g_conv_kind = CK_OTHER;
int conv_last_kind() { return g_conv_kind; }
const char* conv_kind_name(int k) {
  static const char* const names[CK_COUNT] = {"conv_wsb16_kernel", "conv_wsb_kernel", "conv_gs16_kernel",
                                              "conv_gsw16_kernel", "k_rb_pair", "k_conv2d_h16/k_conv2d_small",
                                              "conv_emu_kernel", "conv_gemm_kernel", "conv_tiny_kernel",
                                              "conv_wst16_kernel", "other"};
  return (k >= 0 && k < CK_COUNT) ? names[k] : "other";
}

namespace {

template <bool TWO_D>
hipError_t dispatch(const ConvArgs& a_in, hipStream_t s) {
  const ConvArgs& a = a_in;
  if (a.N <= 0 || a.T_out <= 0 || a.batch <= 0) return hipSuccess;
  if (a.C_in <= 0 || a.taps <= 0) return hipErrorInvalidValue;
  // the fused noise conv lives in store_tile16's unsplit epilogue only (the caller routes it to such a kernel)
  const bool nz = a.nz_har != nullptr;
  if (nz && (TWO_D || (a.ws && a.ksplit > 1) || a.nz_C <= 0 || a.nz_stride <= 0 ||
             a.nz_kk != 1 ||
             a.N != a.nz_u * a.nz_C || a.out_map != OUT_ROWS))
    return hipErrorInvalidValue;
  // the gate and the LayerNorm are applied by the combine
  if ((a.gate_h > 0 || a.ln_g) && !(a.ws && a.ksplit > 1)) return hipErrorInvalidValue;
  if (tiny_fits(a)) {
    if (nz) return hipErrorInvalidValue;
    g_conv_kind = CK_TINY;
    return launch_tiny(a, TWO_D, s);
  }
  if (!nz && !(a.ws && a.ksplit > 1) && rows1x1_fits(a, TWO_D)) {
    g_conv_kind = CK_TINY;
    return launch_rows1x1(a, TWO_D, s);
  }
  if (a.wsb == 2 && a.wsplit && conv_math(a) >= 2 && conv_gs_eligible(a, TWO_D)) {
    const int ks = (a.ws && a.ksplit > 1) ? a.ksplit : 1;
    const int cfg = a.force_cfg >= 30 ? a.force_cfg : pick_wsb(a);
    g_conv_kind = (TWO_D && cfg == 30 && conv_gsw_eligible(a)) ? CK_GSW : CK_GS;
    hipError_t e = conv_gs_launch(a, cfg, 1, s, TWO_D, ks);
    if (e == hipSuccess && ks > 1) e = launch_splitk_reduce(a, ks, TWO_D, s);
    if (e != hipErrorInvalidValue) return e;
  }
  if (a.wsb == 1 && a.wsplit && conv_math(a) >= 2 && conv_wsb_eligible(a, TWO_D)) {
    const int ks = (a.ws && a.ksplit > 1) ? a.ksplit : 1;
    // the short 64 / 128-channel convs on the weight-stationary kernel (conv_wst.hip; force_cfg 20..39 keeps a
    // weight-streamed tile for comparisons)
    if (ks == 1 && (a.force_cfg < 20 || a.force_cfg == 40) && conv_wst_fits(a, TWO_D)) {
      g_conv_kind = CK_WST;
      hipError_t e = conv_wst_launch(a, s);
      if (e != hipErrorInvalidValue) return e;
    }
    const int cfg = a.force_cfg >= 20 && a.force_cfg < 40 ? a.force_cfg : pick_wsb(a);
    g_conv_kind = CK_WSB16;
    hipError_t e = conv_wsb_launch(a, cfg, 1, s, TWO_D, ks);
    if (e == hipSuccess && ks > 1) e = launch_splitk_reduce(a, ks, TWO_D, s);
    if (e != hipErrorInvalidValue) return e;
  }
  if (nz) return hipErrorInvalidValue;  // no store_tile16 kernel took it
  // 3x3 convs with 16/32 channels: 16x16x4 MFMA fragments (conv2d_small.hip)
  if (TWO_D && a.force_cfg < 0 && conv2d_small_fits(a)) {
    g_conv_kind = CK_SMALL2D;
    return conv2d_small(a, s);
  }
  const int cfg = pick_cfg<TWO_D>(a);
  g_conv_kind = cfg >= 10 ? CK_EMU : CK_GEMM;
  ConvArgs b = a;
  b.force_cfg = cfg;
  // plain GEMMs (1-D, one tap, stride 1) take the double-buffered pipeline unless a.pipe < 0; a.pipe > 0 forces it
  // (benchmarks)
  const bool gemm = !TWO_D && a.taps == 1 && a.stride == 1;
  const bool pipe = gemm && a.pipe >= 0;
  if (cfg >= 10) {
    auto run = [&](int c, bool p) -> hipError_t {
      const int ksplit = (b.ws && b.ksplit > 1) ? b.ksplit : 1;
      hipError_t e = conv_emu_launch(b, c, TWO_D, p, ksplit, 1, s);
      if (e != hipSuccess || ksplit == 1) return e;
      return launch_splitk_reduce(b, ksplit, TWO_D, s);
    };
    hipError_t e = run(cfg, pipe);
    if (e == hipErrorInvalidValue && pipe) e = run(cfg, false);  // tile without a GEMM-pipeline instantiation
    if (e == hipErrorInvalidValue && a.force_cfg < 0) {
      // the tile's halo does not fit in LDS (long strided taps) or the shape class has no such instantiation
      for (int alt : {13, 12}) {
        if (alt == cfg) continue;
        e = run(alt, false);
        if (e != hipErrorInvalidValue) break;
      }
    }
    return e;
  }
  hipError_t e = pipe ? launch_forced<TWO_D, true>(b, s) : launch_forced<TWO_D, false>(b, s);
  if (e == hipErrorInvalidValue && a.force_cfg < 0) {
    // the chosen tile's halo does not fit in LDS (long strided taps): fall back to smaller tiles
    for (int alt : {3, 1}) {
      if (alt == cfg) continue;
      b.force_cfg = alt;
      e = launch_forced<TWO_D, false>(b, s);
      if (e != hipErrorInvalidValue) break;
    }
  }
  return e;
}

}  // namespace

long long conv_plan_splitk(ConvArgs& a, bool two_d) {
  a.ksplit = 1;
  if (a.N <= 0 || a.T_out <= 0 || a.no_splitk) return 0;
  if (tiny_fits(a)) return 0;
  if (two_d && a.force_cfg < 0 && conv2d_small_fits(a)) return 0;
  int BM, BN;
  if (a.wsb == 2) {  // the gather-streamed tile
    conv_gs_tile(a.force_cfg >= 30 ? a.force_cfg : pick_wsb(a), BM, BN);
  } else if (a.wsb) {  // the weight-streamed tile (pick_wsb)
    if (!conv_wsb_tile(a.force_cfg >= 20 ? a.force_cfg : pick_wsb(a), BM, BN)) return 0;
  } else {
    cfg_tile(two_d ? pick_cfg<true>(a) : pick_cfg<false>(a), BM, BN);
  }
  long long mtiles;
  if (!two_d) {
    mtiles = (a.T_out + BM - 1) / BM;
  } else {
    const int rw = a.W_out < BM ? a.W_out : BM;
    const int rh = BM / rw;
    mtiles = (long long)((a.T_out + rh - 1) / rh) * ((a.W_out + rw - 1) / rw);
  }
  const long long tiles = mtiles * ((a.N + BN - 1) / BN) * a.batch * a.batch_inner;
  const int iters = ((a.C_in + CK - 1) / CK) * a.taps;
  const double M = two_d ? (double)a.T_out * a.W_out : (double)a.T_out;
  const double flops = 2.0 * M * a.N * (double)a.C_in * a.taps * a.batch * a.batch_inner;
  // split only where the output grid leaves CUs idle AND the contraction is long enough to pay
  // for the extra combine launch (~5-10 us): a tile's (chunk, tap) steps are a serial chain of
  // ~1.5-2 us each (global B load -> LDS -> barrier -> MFMA), so a handful of tiles walking >= 16 steps
  // is latency-bound whatever the FLOP count (RMVPE's deepest levels at streaming sizes: 8 tiles x 144
  // steps = 264 us unsplit)
  // same-box A/B of C2 (round 2, with the 32-bit combine): (target, tiles, min_iters) = (512, 192, 4) 22.59 ms,
  // (768, 384, 8) 22.82, (512, 256, 4) 22.70, (384, 256, 4) 22.64, (1024, 384, 8) 23.33
  static const int target = env_cfg("RVCX_SPLITK_TARGET", 512);  // workgroups a split launch aims for
  constexpr int min_tiles = 192;  // grids with at least this many tiles stay unsplit
  constexpr int min_iters = 4;    // shortest contraction worth a split
  // a gated WaveNet in_layer always splits: its gate lives in the combine (ConvArgs::gate_h)
  const bool combine_epi = a.gate_h > 0 || a.ln_g;  // an epilogue only the combine applies: always split
  if (!combine_epi && (tiles >= min_tiles || iters < min_iters || (flops < 1.0e8 && iters < 16))) return 0;
  int ks = (int)((target + tiles - 1) / tiles);
  // the gather-streamed kernels keep >= 8 (chunk, tap) steps per slice: below that a slice is all prologue and
  // epilogue and the extra slab + combine launch cost more than the parallelism gains (bench_gs r03s, cold: HuBERT
  // 768 -> 768 ks 1 22.1 us vs ks 4 27.6, TextEncoder 1x1 ks 1 11.6 vs ks 3 14.4, U-Net 196 px ks 8 19.8 vs ks 16
  // 21.8, 3136 px ks 2 20.2 vs ks 6 27.3; the 3072 -> 768 linear keeps ks 4: 48.6 vs 62.8 unsplit)
  constexpr int gs_min_steps = 8;  // same-box C2: 2 17.73, 8 17.72, 16 17.86, 24 17.97 ms
  ks = std::min(ks, a.wsb == 2 ? iters / gs_min_steps : iters / 2);
  ks = std::min(ks, 32);
  // the windowed 2-D gather-streamed kernel splits by whole 32-channel chunks (bench_gs: U-Net 784 px ks 8 and 3136 px
  // ks 4 beat the 10 and 6 the step count would give)
  if (a.wsb == 2 && two_d && (a.force_cfg < 0 || a.force_cfg == 30) && conv_gsw_eligible(a))
    ks = std::min(ks, (a.C_in + CK - 1) / CK);
  if (combine_epi && iters >= 2) ks = std::max(ks, 2);
  if (ks < 2) return 0;
  a.ksplit = ks;
  a.ws_rows = two_d ? (long long)a.T_out * a.W_out : a.T_out;
  return std::max((long long)ks * a.ws_rows * a.N * a.batch * a.batch_inner, tiles * ks * BM * BN);
}

bool conv_wsb_wants(const ConvArgs& a) {
  if (conv_math(a) < 2 || !conv_wsb_eligible(a)) return false;
  // where it measured faster (bench_conv, profiles/r02i_bench_conv.txt: 128 x 64 tiles of 2 x 2 waves of 64 x 32
  // with the register epilogue; C2 A/B): N >= 64 with >= 2 taps (ResBlock convs at 64-256 channels incl. k = 3, the
  // polyphase ConvTranspose phases; the 64-channel stage on 128x64 tiles beat the fused pair), on a grid that fills
  // the chip
  constexpr int min_taps = 2, min_tiles = 512, min_n = 64;
  if (a.N < min_n || a.taps < min_taps) return false;
  const long long tiles = (long long)((a.T_out + 127) / 128) * ((a.N + 63) / 64) * a.batch;
  return tiles >= min_tiles;
}

int conv_wsb_route(const ConvArgs& a, bool two_d) {
  if (conv_math(a) < 2 || tiny_fits(a)) return 0;
  if (two_d && conv2d_small_fits(a)) return 0;
  // the weight-streamed kernel on small grids (split-K) and on the U-Net's 3x3 convs measured slower than the
  // gather-streamed one (HuBERT / TextEncoder GEMMs +0.7 ms, U-Net +0.8 ms: with few M tiles every wave re-streams its
  // B fragments from L2)
  if (!two_d && conv_wsb_wants(a)) return 1;
  // everything else with a static weight, 32-channel chunks and >= 64 outputs: the short contractions
  if (a.N >= 64 && conv_gs_eligible(a, two_d)) return 2;
  return 0;
}

int conv_math_of(const ConvArgs& a) { return conv_math(a); }
hipError_t conv1d(const ConvArgs& a, hipStream_t s) { return dispatch<false>(a, s); }
hipError_t conv2d(const ConvArgs& a, hipStream_t s) { return dispatch<true>(a, s); }

}  // namespace rvcx
