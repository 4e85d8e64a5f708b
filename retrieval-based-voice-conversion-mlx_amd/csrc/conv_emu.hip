// fp32 implicit-GEMM convolution on CDNA4 bf16 MFMA (v_mfma_f32_32x32x16_bf16) through a 3-way operand split.
//
// gfx950 has no xf32: its fp32-input MFMA (conv_gemm.hip) runs at the FP32 vector rate, 1/16 of bf16. Every
// fp32 operand x is split exactly into three bf16 planes, x = x0 + x1 + x2 (x0 = bf16(x), x1 = bf16(x - x0),
// x2 = bf16(x - x0 - x1); each difference is exact in fp32 and the three planes carry all 24 significand bits),
// and a product is summed as the six plane products with i + j <= 2:
//     x*y ~= x2*y0 + x1*y1 + x0*y2 + x1*y0 + x0*y1 + x0*y0        (smallest first, one fp32 accumulator)
// Each bf16 x bf16 product is exact in fp32; the dropped terms x1*y2 + x2*y1 + x2*y2 are below 2^-25 |x*y|, under
// the fp32 rounding every fma of the native path incurs. So the contraction is fp32 accurate (no reduced
// precision anywhere: tests/test_gpu_conv_math.py measures the error against fp64 next to the native fp32 MFMA
// path) at 6 x 32 cycles per 32x32x16 step instead of 8 x 64 for the f32 form: 2.67x the MFMA throughput.
//
// The split happens once, on the way into LDS (A: the halo tile of one 32-channel chunk, reused by every tap;
// B: the per-tap weight tile), so the MFMA loop reads ready bf16 fragments. LDS row = [hi | mid | lo] x 32
// channels + 16 B pad (208 B = 52 dwords: 16 consecutive rows hit 16 distinct 4-bank groups). B is double
// buffered with a one-tap register prefetch (one barrier per tap); A is staged synchronously per chunk for the
// halo convs, double buffered with register prefetch for plain GEMMs (taps 1, stride 1).
#include <algorithm>
#include <cstdlib>

#include "conv_common.h"
#include "split_bf16.h"

namespace rvcx {

namespace {

using namespace splitbf16;

template <int BM, int BN, int WM, int WN, bool TWO_D, bool PIPE>
__global__ __launch_bounds__(CONV_THREADS, 2) void conv_emu_kernel(const ConvArgs a, const int nrows_a, const int rw,
                                                                   const int rh, const int tiles_w, const int vec_a,
                                                                   const int vec_b, const int ksplit, const int ntn) {
  constexpr int NT = CONV_THREADS;
  constexpr int TM = BM / (WM * 32);
  constexpr int TN = BN / (WN * 32);
  static_assert(WM * WN == 4, "4 waves per block");
  static_assert(TM >= 1 && TN >= 1, "tile too small");
  static_assert(!(PIPE && TWO_D), "the GEMM pipeline is 1-D");
  extern __shared__ __attribute__((aligned(16))) char smem_e[];
  // non-PIPE: A [nrows_a] | B0 [BN] | B1 [BN] ; PIPE: A0 [BM] | A1 [BM] | B0 | B1   (rows of ERS bytes)
  char* const A0 = smem_e;
  char* const A1 = PIPE ? smem_e + BM * ERS : smem_e;
  char* const B0 = smem_e + (PIPE ? 2 * BM : nrows_a) * ERS;
  char* const B1 = B0 + BN * ERS;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 31, hk = lane >> 5;
  int bx, by, bz;
  conv_block_coords(ntn, bx, by, bz);
  const int zsplit = bz % ksplit;
  const int zb = bz / ksplit;
  const int b = zb / a.batch_inner;
  const int bi = zb % a.batch_inner;
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

  // byte offsets of this lane's fragment rows (tap 0, K16 step 0)
  int aoff[TM], boff[TN];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int ml = wm * TM * 32 + tm * 32 + li;
    int r;
    if (!TWO_D) {
      r = ml * a.stride;
    } else {
      r = (ml < rh * rw) ? (ml / rw) * aw + (ml % rw) : 0;
    }
    aoff[tm] = r * ERS + hk * 16;
  }
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) boff[tn] = (wn * TN * 32 + tn * 32 + li) * ERS + hk * 16;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tm][tn][r] = 0.f;

  // ---- B: global fp32 -> registers -> split into LDS
  constexpr int BV = (BN * EC4 + NT - 1) / NT;
  const int brow = store_row(tid / EC4);  // row of this thread's float4 within each 32-row slab
  int b_row_off[BV];
  bool b_row_ok[BV];
#pragma unroll
  for (int v = 0; v < BV; ++v) {
    const int idx = tid + v * NT;
    const int gn = n0 + v * (NT / EC4) + brow;
    b_row_ok[v] = idx < BN * EC4 && gn < a.N;
    b_row_off[v] = gn * a.ldw + ((idx % EC4) << 2);
  }
  // whole tile in range, 16-B aligned rows, full chunks: one unconditional dwordx4 per slot
  const bool b_fast = vec_b && !a.b_kn && (a.C_in % EK) == 0 && n0 + BN <= a.N;
  auto load_b = [&](int tap, int c0, f32x4 (&reg)[BV]) {
    const float* Wt = Wb + (long long)tap * a.w_ts;
    if (b_fast) {
#pragma unroll
      for (int v = 0; v < BV; ++v)
        if (BN * EC4 % NT == 0 || tid + v * NT < BN * EC4)
          reg[v] = *reinterpret_cast<const f32x4*>(Wt + c0 + b_row_off[v]);
      return;
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int idx = tid + v * NT;
      f32x4 val = {0.f, 0.f, 0.f, 0.f};
      if (idx < BN * EC4) {
        if (!a.b_kn) {
          const int c = c0 + ((idx % EC4) << 2);
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
  auto store_b = [&](char* Bs, const f32x4 (&reg)[BV]) {
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int idx = tid + v * NT;
      if (idx < BN * EC4) {
        if (!a.b_kn) {
          put_split4(Bs + (v * (NT / EC4) + brow) * ERS, (idx % EC4) << 2, reg[v]);
        } else {
          const int cc = idx / (BN / 4);
          const int n4 = (idx - cc * (BN / 4)) << 2;
#pragma unroll
          for (int j = 0; j < 4; ++j) put_split1(Bs + (n4 + j) * ERS, cc, reg[v][j]);
        }
      }
    }
  };

  // ---- A (halo convs): one chunk's nrows_a x 32 tile, pre-activation and row mask applied, split into LDS
  auto stage_a = [&](char* As, int c0) {
    if constexpr (!TWO_D) {
      // a thread keeps one 4-channel column and walks rows NT / EC4 apart: constant address steps
      constexpr int RSTEP = NT / EC4;
      const int c4 = (tid % EC4) << 2;
      const int c = c0 + c4;
      const bool c_ok = c < a.C_in;
      const bool c_vec = vec_a && c + 4 <= a.C_in;
      int r = tid / EC4;
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
        put_split4(As + r * ERS, c4, v);
      }
    } else {
      for (int idx = tid; idx < nrows_a * EC4; idx += NT) {
        const int r = idx / EC4;
        const int c4 = (idx % EC4) << 2;
        const int c = c0 + c4;
        const int ah = r / aw, awi = r - ah * aw;
        const int gh = h0 - a.padh + ah, gw = w0 - a.padw + awi;
        const bool valid = (gh >= 0) && (gh < a.T_in) && (gw >= 0) && (gw < a.W_in);
        const long long grow = (long long)gh * a.W_in + gw;
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
        }
        put_split4(As + r * ERS, c4, v);
      }
    }
  };

  // ---- A (1-D): register prefetch of a whole chunk tile, issued one chunk ahead and written (split) at the chunk
  // change; tiles up to BM + 64 rows (every halo conv of the path but HuBERT's strided feature convs)
  // 2-D (the (rh + KH - 1) x (rw + KW - 1) pixel window) measured slower with the prefetch (U-Net 64x64 convs
  // 2.58 vs 2.47 ms per C2 step: 134 vs 105 VGPRs), so 2-D tiles stage synchronously (AP = 1 never fits)
  constexpr int AP = TWO_D ? 1 : ((BM + 64) * EC4 + NT - 1) / NT;
  f32x4 apre[AP];
  float apm[TWO_D ? 1 : AP];  // 1-D: 0 outside the input, else the row mask; 2-D: folded into apre
  const bool a_pre = !PIPE && nrows_a * EC4 <= AP * NT &&
                     (!TWO_D || a.pre_act == ACT_NONE || a.pre_act == ACT_LRELU || a.pre_act == ACT_RELU);
  const bool a_fast = vec_a && (a.C_in % EK) == 0;
  const int arow = store_row(tid / EC4), ac4 = (tid % EC4) << 2;
  auto load_a_regs = [&](int c0) {
    const float* src0 = X + c0 + ac4;
#pragma unroll
    for (int v = 0; v < AP; ++v) {
      const int r = v * (NT / EC4) + arow;
      long long g;
      bool ok;
      if constexpr (!TWO_D) {
        g = row0 + r;
        ok = r < nrows_a && g >= 0 && g < a.T_in;
      } else {
        const int ah = r / aw, awi = r - ah * aw;
        const int gh = h0 - a.padh + ah, gw = w0 - a.padw + awi;
        ok = r < nrows_a && gh >= 0 && gh < a.T_in && gw >= 0 && gw < a.W_in;
        g = (long long)gh * a.W_in + gw;
      }
      f32x4 val = {0.f, 0.f, 0.f, 0.f};
      if constexpr (!TWO_D) apm[v] = 0.f;
      if (ok) {
        const float* src = src0 + g * a.ldx;
        if (a_fast) {
          val = *reinterpret_cast<const f32x4*>(src);
        } else {
          const int c = c0 + ac4;
#pragma unroll
          for (int j = 0; j < 4; ++j) val[j] = (c + j < a.C_in) ? src[j] : 0.f;
        }
        if constexpr (!TWO_D) apm[v] = PM ? PM[g] : 1.f;
      }
      apre[v] = val;
    }
  };
  auto write_a_regs = [&](char* As) {
#pragma unroll
    for (int v = 0; v < AP; ++v) {
      const int r = v * (NT / EC4) + arow;
      if (r < nrows_a) {
        f32x4 val = apre[v];
        if (a.pre_act != ACT_NONE) {
#pragma unroll
          for (int j = 0; j < 4; ++j) val[j] = act_fn(val[j], a.pre_act, a.pre_slope);  // act(0) = 0
        }
        if constexpr (!TWO_D) {
#pragma unroll
          for (int j = 0; j < 4; ++j) val[j] *= apm[v];  // 0 outside the input, the row mask inside
        }
        put_split4(As + r * ERS, ac4, val);
      }
    }
  };

  // ---- MFMA: 2 K16 steps x (TM x TN tiles) x 6 plane products, smallest terms first
  auto compute = [&](const char* As, const char* Bs, int tap) {
    const int toff = (TWO_D ? (tap / a.KW) * aw + (tap % a.KW) : tap * a.dil) * ERS;
    // every fragment of both K16 steps is requested before the first MFMA: one exposed LDS latency per tap
    bf16x8 af2[2][TM][3], bf2[2][TN][3];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int q = 0; q < 3; ++q)
          af2[s][tm][q] = *reinterpret_cast<const bf16x8*>(As + aoff[tm] + toff + q * PLANE + s * 32);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int q = 0; q < 3; ++q)
          bf2[s][tn][q] = *reinterpret_cast<const bf16x8*>(Bs + boff[tn] + q * PLANE + s * 32);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      auto& af = af2[s];
      auto& bfr = bf2[s];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          f32x16 c = acc[tm][tn];
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm][2], bfr[tn][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm][1], bfr[tn][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm][0], bfr[tn][2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm][1], bfr[tn][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm][0], bfr[tn][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm][0], bfr[tn][0], c, 0, 0, 0);
          acc[tm][tn] = c;
        }
    }
  };

  const int nchunks = (a.C_in + EK - 1) / EK;
  f32x4 breg[BV];
  if constexpr (!PIPE) {
    // (chunk, tap) iterations of this split-K slice; B of the next iteration is in flight during the MFMAs
    const int total = nchunks * a.taps;
    const int per = (total + ksplit - 1) / ksplit;
    const int it0 = zsplit * per, it1 = min(total, it0 + per);
    if (it0 < it1) {
      int ch = it0 / a.taps, tap = it0 - ch * a.taps;
      load_b(tap, ch * EK, breg);
      if (a_pre) {
        load_a_regs(ch * EK);
        write_a_regs(A0);
        if ((ch + 1) * a.taps < it1) load_a_regs((ch + 1) * EK);  // in flight across this chunk's taps
      } else {
        stage_a(A0, ch * EK);
      }
      store_b(B0, breg);
      __syncthreads();
      bool odd = false;
      for (int it = it0; it < it1; ++it) {
        const bool more = it + 1 < it1;
        int nch = ch, ntap = tap + 1;
        if (ntap == a.taps) {
          ntap = 0;
          ++nch;
        }
        if (more) load_b(ntap, nch * EK, breg);
        compute(A0, odd ? B1 : B0, tap);
        if (more) {
          if (nch != ch) {
            __syncthreads();  // every wave is done with this chunk's A tile
            if (a_pre) {
              write_a_regs(A0);
              if ((nch + 1) * a.taps < it1) load_a_regs((nch + 1) * EK);
            } else {
              stage_a(A0, nch * EK);
            }
          }
          store_b(odd ? B0 : B1, breg);
          __syncthreads();
          odd = !odd;
        }
        ch = nch;
        tap = ntap;
      }
    }
  } else {
    // plain GEMM: A and B both double buffered, the next chunk's tiles in registers during the MFMAs
    constexpr int AV = (BM * EC4 + NT - 1) / NT;
    f32x4 areg[AV];
    float amk[AV];
    auto load_a = [&](int c0) {
#pragma unroll
      for (int v = 0; v < AV; ++v) {
        const int idx = tid + v * NT;
        areg[v] = f32x4{0.f, 0.f, 0.f, 0.f};
        amk[v] = 0.f;
        if (idx < BM * EC4) {
          const int r = idx / EC4;
          const int c = c0 + ((idx % EC4) << 2);
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
    auto store_a = [&](char* dst) {
#pragma unroll
      for (int v = 0; v < AV; ++v) {
        const int idx = tid + v * NT;
        if (idx < BM * EC4) {
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
          put_split4(dst + (idx / EC4) * ERS, (idx % EC4) << 2, val);
        }
      }
    };
    const int per = (nchunks + ksplit - 1) / ksplit;
    const int it0 = zsplit * per, it1 = min(nchunks, it0 + per);
    if (it0 < it1) {
      load_a(it0 * EK);
      load_b(0, it0 * EK, breg);
      store_a(A0);
      store_b(B0, breg);
      __syncthreads();
      for (int it = it0; it < it1; ++it) {
        const bool odd = (it - it0) & 1;
        const bool more = it + 1 < it1;
        if (more) {
          load_a((it + 1) * EK);
          load_b(0, (it + 1) * EK, breg);
        }
        compute(odd ? A1 : A0, odd ? B1 : B0, 0);
        if (more) {
          store_a(odd ? A0 : A1);
          store_b(odd ? B0 : B1, breg);
        }
        __syncthreads();
      }
    }
  }

  conv_store_tile<TM, TN, WM, WN, TWO_D>(a, TilePos{m0, h0, w0, rw, rh, n0, b, bi, zb, zsplit, ksplit}, acc,
                                         reinterpret_cast<float*>(smem_e));
}

template <int BM, int BN, int WM, int WN, bool TWO_D, bool PIPE>
hipError_t launch_emu(const ConvArgs& a, int ksplit, int ntn_enable, hipStream_t s) {
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
  if (PIPE && (a.taps != 1 || a.stride != 1)) return hipErrorInvalidValue;
  size_t smem = (size_t)(PIPE ? 2 * (BM + BN) : nrows_a + 2 * BN) * ERS;
  smem = std::max(smem, (size_t)4 * 32 * 33 * sizeof(float));  // epilogue staging slots
  if (smem > 160 * 1024) return hipErrorInvalidValue;
  smem = std::min(smem + (size_t)std::max(0, a.lds_pad), (size_t)160 * 1024);  // occupancy throttle, clamped
  const int vec_a = ((a.ldx & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.x) & 15) == 0) && ((a.x_bs & 3) == 0) &&
                    ((a.x_bs2 & 3) == 0);
  const int vec_b = ((a.ldw & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.w) & 15) == 0) && ((a.w_bs & 3) == 0) &&
                    ((a.w_bs2 & 3) == 0) && ((a.w_ts & 3) == 0);
  if (a.batch_inner < 1) return hipErrorInvalidValue;
  const int ntiles = (a.N + BN - 1) / BN;
  const int ntn = ntn_enable ? ntiles : 0;
  dim3 grid(ntn ? mtiles * ntiles : mtiles, ntn ? 1 : ntiles, a.batch * a.batch_inner * ksplit);
  auto kern = conv_emu_kernel<BM, BN, WM, WN, TWO_D, PIPE>;
  static size_t smem_set = 64 * 1024;  // per instantiation: raise the dynamic-LDS limit once
  if (smem > smem_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    smem_set = smem;
  }
  hipLaunchKernelGGL(kern, grid, dim3(CONV_THREADS), smem, s, a, nrows_a, rw, rh, tiles_w, vec_a, vec_b, ksplit,
                     ntn);
  return hipGetLastError();
}

}  // namespace

// cfg ids of the split kernel (10..16): BM x BN, waves WM x WN, per-wave tile (BM/WM) x (BN/WN)
bool conv_emu_tile(int cfg, int& BM, int& BN) {
  static const int t[7][2] = {{128, 64}, {256, 32}, {128, 32}, {64, 64}, {128, 128}, {64, 128}, {256, 64}};
  if (cfg < 10 || cfg > 16) return false;
  BM = t[cfg - 10][0];
  BN = t[cfg - 10][1];
  return true;
}

hipError_t conv_emu_launch(const ConvArgs& a, int cfg, bool two_d, bool pipe, int ksplit, int ntn_enable,
                           hipStream_t s) {
  if (two_d) {
    switch (cfg) {
      case 10: return launch_emu<128, 64, 2, 2, true, false>(a, ksplit, ntn_enable, s);
      case 12: return launch_emu<128, 32, 4, 1, true, false>(a, ksplit, ntn_enable, s);
      case 13: return launch_emu<64, 64, 2, 2, true, false>(a, ksplit, ntn_enable, s);
      case 14: return launch_emu<128, 128, 2, 2, true, false>(a, ksplit, ntn_enable, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (pipe) {
    switch (cfg) {
      case 10: return launch_emu<128, 64, 2, 2, false, true>(a, ksplit, ntn_enable, s);
      case 12: return launch_emu<128, 32, 4, 1, false, true>(a, ksplit, ntn_enable, s);
      case 13: return launch_emu<64, 64, 2, 2, false, true>(a, ksplit, ntn_enable, s);
      case 14: return launch_emu<128, 128, 2, 2, false, true>(a, ksplit, ntn_enable, s);
      case 15: return launch_emu<64, 128, 2, 2, false, true>(a, ksplit, ntn_enable, s);
      default: return hipErrorInvalidValue;
    }
  }
  switch (cfg) {
    case 10: return launch_emu<128, 64, 2, 2, false, false>(a, ksplit, ntn_enable, s);
    case 11: return launch_emu<256, 32, 4, 1, false, false>(a, ksplit, ntn_enable, s);
    case 12: return launch_emu<128, 32, 4, 1, false, false>(a, ksplit, ntn_enable, s);
    case 13: return launch_emu<64, 64, 2, 2, false, false>(a, ksplit, ntn_enable, s);
    case 14: return launch_emu<128, 128, 2, 2, false, false>(a, ksplit, ntn_enable, s);
    case 15: return launch_emu<64, 128, 2, 2, false, false>(a, ksplit, ntn_enable, s);
    case 16: return launch_emu<256, 64, 4, 1, false, false>(a, ksplit, ntn_enable, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace rvcx
