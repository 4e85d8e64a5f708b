// Weight-stationary form of the two-plane fp16 conv (conv_wst16_kernel) for the generator's short, long-running 1-D
// convs: the k = 3 ResBlock convs at 64 / 128 channels (residuals.py:71-80, ResBlock.forward; convs1 dilated, convs2
// not) and the ConvTranspose phases of the last two upsample stages (hifigan_nsf.py:184-199, two taps per phase).
//
// Why a separate kernel: at C_in <= 128 and k <= 3 the weight-streamed kernel (conv_wsb.hip, cfg 27) re-reads a
// tile's whole weight image from L2 for every 128 output rows -- as many bytes per tile as the activations it
// convolves -- and pays a cold prologue (halo load, split, barrier) per workgroup, so it ran these HBM-bound shapes at
// ~3 TB/s with 14-24 % MFMA busy. Here the whole weight image of a wave's 16 output columns
// (NCH x TAPS steps x 2 planes x 16 B per lane: 96 VGPRs at 128 channels, k = 3) is loaded into registers ONCE, and
// a persistent workgroup streams a contiguous run of 64-row time tiles through a double-buffered LDS image:
//   iteration t:  MFMAs of tile t (LDS buffer t % 2, weights in registers; no memory operation in the loop)
//                 split tile t + 1's prefetched rows into the other buffer, issue tile t + 2's row loads
//                 epilogue of tile t (its residual / accumulate rows were loaded one tile ahead), issue tile t + 1's
//                 one barrier
// Every global load is unconditional (indices clamped to the run's last tile) and issued a whole tile before it is
// consumed, in the order it is consumed, so each vmcnt wait finds its load done and never waits for a younger one.
//
// Arithmetic: exactly conv_wsb16_kernel's (split_bf16.h put_h16x4 activations at 2^-4, the per-column-scaled
// k_wsplit_h16 image, three v_mfma_f32_16x16x32_f16 products per (chunk, tap) step in the same order, acc + 2^-11 acc2
// times the column's inverse scale, then store_tile16's epilogue order), with the MFMA operands swapped (D = W X^T, so
// a lane's accumulators are four channels of one time row): the two kernels are bit-identical
// (tests/test_gpu_conv_wst.py compares them element for element). Measured against the weight-streamed tile it
// replaces (profiles/r06t_ab_wst.txt): bench_conv C128 k3 198 -> 262 TF, the up3 phase group 151 -> 224, C2 -0.2 ms.
// What bounds it (r06v/w variants): the MFMA loop alone runs 43 us of the 70 us C128 k3 launch and the loads, split
// and stores alone 34 us (5.6 TB/s); a ping-pong schedule meant to overlap them measured slower (r06r/s).
#include <algorithm>

#include "conv_common.h"
#include "split_bf16.h"

namespace rvcx {

namespace {

using namespace splitbf16;

constexpr int WST_BM = 64;                      // output rows per tile
constexpr int WST_HMAX = 16;                    // max (taps - 1) * dil
constexpr int WST_NR = WST_BM + WST_HMAX;       // LDS rows per chunk image
// LDS row stride of the two-plane image: 160 B (40 dwords). The A-fragment read (ds_read_b128, lane l: row l % 16,
// 16 B at (l / 16) * 16) is serviced in four 16-lane groups of a fixed odd membership (MI355X_MICROARCH.md, LDS
// table: {0-3, 12-15, 20-27}, ...); at the weight-streamed kernel's 144 B every group has 2-way bank conflicts, at
// 160 B none (a brute-force check over row strides 128-304 B: 160, 224 and 288 are the conflict-free ones)
constexpr int WST_RS = 2 * PLANE + 32;
// one 32-channel chunk image, + 64 B so consecutive chunks start 16 banks apart: the split's 8-byte stores (16-lane
// groups spanning two chunks of one row) are conflict-free
constexpr int WST_CHB = WST_NR * WST_RS + 64;
constexpr int WST_WBLK = 1024;                  // conv_wsb.hip's (step, 16-column group, plane) block

// NCH 32-channel input chunks, TAPS taps, NW waves (= N / 16 output columns, one 16-column group per wave), EPI bit 0:
// a residual (RES_ADD_POST), bit 1: an accumulate target (ACC_ADD / ACC_ADD_DIV) -- compile-time, so their loads are
// never behind a branch whose join would make the waitcnt pass drain the row prefetch; bit 2: the leaky-ReLU
// pre-activation (convs1 and the ConvTranspose phases; convs2 reads an already activated input)
template <int NCH, int TAPS, int NW, int EPI>
__global__ __launch_bounds__(NW * 64, 2) void conv_wst16_kernel(const ConvArgs a,
                                                                              const char* __restrict__ wsp,
                                                                              const int Npad, const int mtiles,
                                                                              const int total) {
  constexpr int NT = NW * 64;
  constexpr int NSTEP = NCH * TAPS;
  constexpr int TM16 = WST_BM / 16;
  constexpr int C4 = NCH * EC4;  // float4 groups per input row
  constexpr int XI = (WST_NR * C4 + NT - 1) / NT;
  static_assert(NT % C4 == 0 && (WST_NR * C4) % NT == 0, "whole rows per prefetch instruction");
  constexpr bool NEED_R = (EPI & 1) != 0, NEED_D = (EPI & 2) != 0, PRE = (EPI & 4) != 0;
  extern __shared__ __attribute__((aligned(16))) char smem_wst[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lc = lane & 15, lg = lane >> 4;
  // MFMA orientation D[out channel][time] (A = the weight fragment, B = the activation fragment): accumulator element r
  // of lane (lc, lg) is output channel n0 + r of time row lc of its 16-row block, so the epilogue moves 16 B per lane
  // (four channels) where the [time][channel] orientation stored one float per lane and instruction (the epilogue's
  // store issue, not HBM, was its cost)
  const int n0 = wave * 16 + 4 * lg;  // the lane's four output channels
  const int per = (total + (int)gridDim.x - 1) / (int)gridDim.x;
  const int t_begin = blockIdx.x * per, t_end = min(total, t_begin + per);
  if (t_begin >= t_end) return;
  const int t_last = t_end - 1;

  // ---- the wave's weight image -> registers, once
  const size_t bstep = (size_t)Npad * 2 * PLANE;
  f16x8 wr[NSTEP][2];
#pragma unroll
  for (int it = 0; it < NSTEP; ++it)
#pragma unroll
    for (int q = 0; q < 2; ++q)
      wr[it][q] = *reinterpret_cast<const f16x8*>(wsp + it * bstep + (size_t)wave * 2 * WST_WBLK + q * WST_WBLK +
                                                  lane * 16);
  const f32x4 iv = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(wsp + NSTEP * bstep) + n0);
  const bool has_bias = a.bias != nullptr;
  f32x4 bn = f32x4{0.f, 0.f, 0.f, 0.f};
  if (has_bias) {
#pragma unroll
    for (int r = 0; r < 4; ++r) bn[r] = a.bias[n0 + r];
  }

  // ---- tile cursors: a run's tiles are consecutive (batch-major), so each consumer (the row prefetch, the residual
  // prefetch, the epilogue) steps its own (batch, row tile) pair instead of dividing; element offsets inside one batch
  // entry are 32-bit (conv_wst_fits: rows < 2^24, row strides < 2^24, rows x stride < 2^31) on full-rate 24-bit
  // multiplies (the 64-bit index products were a third of the loop's VALU work)
  struct Cur {
    int t, b, mi;
  };
  auto cur_at = [&](int t) { Cur c; c.t = t; c.b = t / mtiles; c.mi = t - c.b * mtiles; return c; };
  auto cur_next = [&](Cur& c) {  // clamped to the run's last tile (its loads repeat, harmlessly)
    if (c.t < t_last) {
      ++c.t;
      if (++c.mi == mtiles) {
        c.mi = 0;
        ++c.b;
      }
    }
  };
  // ---- rows of a tile: input rows m0 - pad + r, r < nr (zero outside [0, T_in): the conv's padding)
  const int nr = WST_BM + (TAPS - 1) * a.dil;
  constexpr int RPV = NT / C4;  // rows per prefetch instruction
  const int xr0 = tid / C4, xc4 = (tid % C4) * 4;
  f32x4 xr[XI];
  unsigned xok = 0u;
  auto load_x = [&](const Cur& c) __attribute__((always_inline)) {
    const float* X = a.x + (long long)c.b * a.x_bs + xc4;
    const int g0 = c.mi * WST_BM - a.pad + xr0;
    xok = 0u;
#pragma unroll
    for (int v = 0; v < XI; ++v) {
      const int g = g0 + v * RPV;
      const bool ok = xr0 + v * RPV < nr && g >= 0 && g < a.T_in;
      xr[v] = *reinterpret_cast<const f32x4*>(X + (ok ? __umul24((unsigned)g, (unsigned)a.ldx) : 0u));
      xok |= ok ? (1u << v) : 0u;
    }
  };
  auto write_x = [&](char* buf) __attribute__((always_inline)) {
    char* const dst0 = buf + (xc4 / EK) * WST_CHB + xr0 * WST_RS + (xc4 % EK) * 2;
#pragma unroll
    for (int v = 0; v < XI; ++v) {
      if (xr0 + v * RPV < nr) {
        f32x4 val = xr[v];
        const bool ok = (xok >> v) & 1u;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          val[j] = ok ? pre_fn<PRE ? PA_LRELU : PA_NONE>(val[j], ACT_LRELU, a.pre_slope) * H16_XS : 0.f;
        put_h16x4<2>(dst0 + v * RPV * WST_RS, 0, val);
      }
    }
  };
  // ---- the residual / accumulate rows of the lane's outputs (rows past T_out read the last row; not stored)
  f32x4 rv[TM16], dv[TM16];
  const int tlast_row = a.T_out - 1;
  auto load_rd = [&](const Cur& c) __attribute__((always_inline)) {
    const float* R = NEED_R ? a.res + (long long)c.b * a.res_bs + n0 : nullptr;
    const float* Y = a.y + (long long)c.b * a.y_bs + n0;
    const int m0 = c.mi * WST_BM + lc;
#pragma unroll
    for (int tm = 0; tm < TM16; ++tm) {
      const unsigned m = (unsigned)min(m0 + tm * 16, tlast_row);
      if constexpr (NEED_R) rv[tm] = *reinterpret_cast<const f32x4*>(R + __umul24(m, (unsigned)a.ldr));
      if constexpr (NEED_D) dv[tm] = *reinterpret_cast<const f32x4*>(Y + __umul24(m, (unsigned)a.ldy));
    }
  };

  f32x4 acc[TM16], acc2[TM16];
  // A fragments run a ring of RING register slots AHEAD (step, row block) units ahead of the MFMAs that use
  // them: every slot index is compile-time in the unrolled unit loop and the reads are pinned above each unit's MFMAs
  // (left to itself the scheduler reused one register pair and waited out every read's latency, lgkmcnt(0) per 3
  // MFMAs; a whole step's fragments one step ahead needed 64 registers and spilled at 128 channels). Pairs of row
  // blocks per unit with their MFMAs interleaved (no MFMA waiting on the one before) measured no faster (r06t)
  constexpr int NU = NSTEP * TM16, RING = 4, AHEAD = 3;
  f16x8 af[RING][2];
  auto compute = [&](const char* buf) __attribute__((always_inline)) {
#pragma unroll
    for (int tm = 0; tm < TM16; ++tm) acc[tm] = acc2[tm] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* base = buf + lc * WST_RS + lg * 16;
    auto read_a = [&](int u, f16x8(&f)[2]) __attribute__((always_inline)) {
      const int it = u / TM16, tm = u - it * TM16;
      const int ch = it / TAPS, tap = it - ch * TAPS;
      const char* p = base + ch * WST_CHB + (tap * a.dil + tm * 16) * WST_RS;
      f[0] = *reinterpret_cast<const f16x8*>(p);
      f[1] = *reinterpret_cast<const f16x8*>(p + PLANE);
    };
#pragma unroll
    for (int u = 0; u < AHEAD; ++u) read_a(u, af[u % RING]);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      if (u + AHEAD < NU) read_a(u + AHEAD, af[(u + AHEAD) % RING]);
      __builtin_amdgcn_sched_barrier(0);
      const int it = u / TM16, tm = u - it * TM16;
      const f16x8 ah = af[u % RING][0], al = af[u % RING][1];
      acc[tm] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[it][0], ah, acc[tm], 0, 0, 0);
      f32x4 c = acc2[tm];
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[it][0], al, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[it][1], ah, c, 0, 0, 0);
      acc2[tm] = c;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // store_tile16's order of operations, per element: (acc + 2^-11 acc2) * inv, + bias, act, + residual, accumulate,
  // + the fused noise conv (one tap: k_noise_add's y + (w x + b))
  auto epilogue = [&](const Cur& c) __attribute__((always_inline)) {
    const int b = c.b;
    float* Yn = a.y + (long long)b * a.y_bs + n0;
    // the noise conv of these four columns (one phase p of nz_u: C % 4 == 0) -- conv_wst_fits admits nz_kk = 1 only
    const float* hb = a.nz_har ? a.nz_har + (long long)b * a.nz_bs : nullptr;
    const int nzp = a.nz_har ? n0 / a.nz_C : 0, nzc = a.nz_har ? n0 - nzp * a.nz_C : 0;
#pragma unroll
    for (int tm = 0; tm < TM16; ++tm) {
      const int m = c.mi * WST_BM + tm * 16 + lc;
      const bool ok = m < a.T_out;
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = acc[tm][r];
        x += acc2[tm][r] * H16_LO_INV;
        v[r] = x * iv[r];
      }
      if (has_bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bn[r];
      }
      if (a.act == ACT_LRELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
      }
      if constexpr (NEED_R) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] + rv[tm][r];
      }
      if constexpr (NEED_D) {
        if (a.acc_mode == ACC_ADD) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = dv[tm][r] + v[r];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (dv[tm][r] + v[r]) / a.acc_div;
        }
      }
      if (hb) {
        const float hx = hb[((long long)(ok ? m : 0) * a.nz_u + nzp) * a.nz_stride];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float w = a.nz_w[(long long)(nzc + r) * a.nz_stride];
          v[r] = v[r] + (fmaf(w, hx, 0.f) + a.nz_b[nzc + r]);
        }
      }
      if (ok) *reinterpret_cast<f32x4*>(Yn + __umul24((unsigned)m, (unsigned)a.ldy)) = v;
    }
  };

  char* const buf0 = smem_wst;
  char* const buf1 = smem_wst + NCH * WST_CHB;
  Cur ce = cur_at(t_begin);  // the tile computed / stored
  Cur cx = ce;               // the row prefetch (one to two tiles ahead)
  Cur cr = ce;               // the residual / accumulate prefetch (one tile ahead)
  load_x(cx);
  write_x(buf0);
  cur_next(cx);
  load_x(cx);
  load_rd(cr);
  __syncthreads();
  bool cur1 = false;
#pragma unroll 1
  for (int tile = t_begin; tile < t_end; ++tile) {
    char* const bc = cur1 ? buf1 : buf0;
    char* const bnx = cur1 ? buf0 : buf1;
    compute(bc);
    write_x(bnx);  // tile + 1 (at the run's end: the last tile again, never read)
    cur_next(cx);
    load_x(cx);
    epilogue(ce);
    cur_next(ce);
    cur_next(cr);
    load_rd(cr);
    __syncthreads();  // the next buffer complete; this one free
    cur1 = !cur1;
  }
}

template <int NCH, int TAPS, int NW>
hipError_t launch_wst_epi(const ConvArgs& a, hipStream_t s) {
  const int epi = (a.res_mode == RES_ADD_POST ? 1 : 0) | (a.acc_mode != ACC_STORE ? 2 : 0) |
                  (a.pre_act == ACT_LRELU ? 4 : 0);
  void (*kern)(const ConvArgs, const char*, int, int, int);
  switch (epi) {
#define WST_CASE(E) \
  case E: kern = conv_wst16_kernel<NCH, TAPS, NW, E>; break;
    WST_CASE(0) WST_CASE(1) WST_CASE(2) WST_CASE(3) WST_CASE(4) WST_CASE(5) WST_CASE(6) WST_CASE(7)
#undef WST_CASE
    default: return hipErrorInvalidValue;
  }
  const size_t smem = (size_t)2 * NCH * WST_CHB;
  // per instantiation: the dynamic-LDS limit raised once, the resident workgroups per CU measured once
  static bool attr_set[8] = {};
  static int occ[8] = {};
  if (!attr_set[epi]) {
    if (smem > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
      if (e != hipSuccess) return e;
    }
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kern, NW * 64, smem) != hipSuccess || o < 1) o = 1;
    occ[epi] = o;
    attr_set[epi] = true;
  }
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  const int mtiles = (a.T_out + WST_BM - 1) / WST_BM;
  const long long total = (long long)mtiles * a.batch;
  if (total >= (1LL << 31)) return hipErrorInvalidValue;
  const int grid = (int)std::min<long long>(total, (long long)ncu * occ[epi]);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), smem, s, a, static_cast<const char*>(a.wsplit), a.wsplit_npad,
                     mtiles, (int)total);
  return hipGetLastError();
}

}  // namespace

bool conv_wst_fits(const ConvArgs& a, bool two_d) {
  const bool vec_a = ((a.ldx & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.x) & 15) == 0) && ((a.x_bs & 3) == 0);
  // 16-byte epilogue operands: y / res rows (and their batch strides) 16-B aligned
  const bool vec_y = ((reinterpret_cast<uintptr_t>(a.y) & 15) == 0) && (a.ldy & 3) == 0 && (a.y_bs & 3) == 0 &&
                     (a.res_mode == RES_NONE ||
                      (((reinterpret_cast<uintptr_t>(a.res) & 15) == 0) && (a.ldr & 3) == 0 && (a.res_bs & 3) == 0)) &&
                     (!a.nz_har || (a.nz_C % 4 == 0 && a.nz_kk == 1));
  const bool shape = (a.C_in == 128 && a.N == 128 && (a.taps == 3 || a.taps == 2)) ||
                     (a.C_in == 64 && a.N == 64 && (a.taps == 3 || a.taps == 2));
  return !two_d && shape && vec_a && vec_y && a.wsb == 1 && a.wsplit && a.wsplit_fmt == WSPLIT_H16 && !a.lowp &&
         a.wsplit_npad >= a.N && a.batch_inner == 1 && !a.b_kn && a.out_map == OUT_ROWS && a.stride == 1 &&
         a.dil >= 1 && (a.taps - 1) * a.dil <= WST_HMAX && (a.pre_act == ACT_LRELU || a.pre_act == ACT_NONE) &&
         !a.pre_mask && a.alpha == 1.f &&
         !a.mask && (a.act == ACT_NONE || a.act == ACT_LRELU) &&
         (a.res_mode == RES_NONE || (a.res_mode == RES_ADD_POST && a.res)) && a.bias_bs == 0 && a.gate_h == 0 &&
         !a.ln_g && !(a.ws && a.ksplit > 1) && a.T_out > 0 && a.T_in > 0 && a.batch > 0 &&
         // 32-bit element offsets on 24-bit multiplies inside a batch entry (the kernel's cursors)
         a.T_in < (1 << 24) && a.T_out + WST_BM < (1 << 24) && a.ldx < (1 << 24) && a.ldy < (1 << 24) &&
         a.ldr < (1 << 24) && (long long)a.T_in * a.ldx < (1LL << 31) && (long long)a.T_out * a.ldy < (1LL << 31) &&
         (long long)a.T_out * a.ldr < (1LL << 31);
}

hipError_t conv_wst_launch(const ConvArgs& a, hipStream_t s) {
  if (!conv_wst_fits(a, false)) return hipErrorInvalidValue;
  if (a.C_in == 128) return a.taps == 3 ? launch_wst_epi<4, 3, 8>(a, s) : launch_wst_epi<4, 2, 8>(a, s);
  return a.taps == 3 ? launch_wst_epi<2, 3, 4>(a, s) : launch_wst_epi<2, 2, 4>(a, s);
}

}  // namespace rvcx
