// fp32 implicit-GEMM convolution for the SHORT contractions of the path (HuBERT's linears and feature convs, the
// TextEncoder / flow convs, the RMVPE U-Net's 3x3 convs, split-K partial tiles): "gather-streamed" on
// v_mfma_f32_16x16x32_bf16, same exact 3-plane bf16 arithmetic as conv_emu.hip / conv_wsb.hip.
//
// These contractions have few output tiles (M = 196..3200 rows) and short per-tile K walks (after split-K, 4..24
// (chunk, tap) steps), so the LDS-staged kernel's one-step register prefetch leaves every step waiting out a full
// global-load latency (~1-2 us per step against ~0.2 us of MFMA work). Here both operands run a 3-deep register
// prefetch ring and nothing waits on a load issued less than two steps earlier:
//   * B: the weights pre-split once into bf16 planes in HBM (conv_wsb.hip's lane-major image, k_wsplit), per lane
//     one 16-byte fragment per (plane, 16-column tile) straight from L2 into registers -- no LDS, no conversion;
//   * A: every (chunk, tap) step GATHERS its BM rows x 32 channels from global memory (no halo reuse: the taps of
//     these convs are 1..9, so re-reading the shifted rows from L2 costs less than a serial halo stage), a
//     1-D row at m * stride - pad + tap * dil, a 2-D output pixel's input pixel at (oh - padh + kh, ow - padw + kw);
//     the pre-activation and row mask are applied and the tile split into an LDS double buffer (one barrier/step).
// Split-K slices write partial tiles to the slab (splitk_reduce_kernel applies the epilogue), as elsewhere.
#include <algorithm>
#include <cstdlib>

#include "conv_common.h"
#include "split_bf16.h"

namespace rvcx {

namespace {

using namespace splitbf16;

constexpr int GS_BLK = 1024;       // bytes of one (step, 16-column group, plane) block of that image
#ifndef GS_DEPTH
#define GS_DEPTH 3
#endif
constexpr int GS_D = GS_DEPTH;      // prefetch ring depth (steps in flight per operand)

// one (tm) row block of 16x16x32 fp16 MFMAs of the two-plane arithmetic: acc += h*h', acc2 += l*h' + h*l'
template <int TN16>
__device__ __forceinline__ void mma_h16(const bf16x8 (&af)[2], const bf16x8 (&bf)[TN16][2], f32x4 (&acc)[TN16],
                                        f32x4 (&acc2)[TN16]) {
  const f16x8 ah = __builtin_bit_cast(f16x8, af[0]), al = __builtin_bit_cast(f16x8, af[1]);
#pragma unroll
  for (int tn = 0; tn < TN16; ++tn) {
    const f16x8 bh = __builtin_bit_cast(f16x8, bf[tn][0]);
    acc[tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[tn], 0, 0, 0);
    f32x4 c = acc2[tn];
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, __builtin_bit_cast(f16x8, bf[tn][1]), c, 0, 0, 0);
    acc2[tn] = c;
  }
}
// acc + 2^-11 acc2, times 1 / (column weight scale x activation scale) from the fp16 image's tail (at tail_off bytes:
// one inverse scale per output column, conv_wsb.hip k_wsplit_h16); lane column n0 + wn * TN16 * 16 + tn * 16 + lane % 16
template <int TM16, int TN16, int WN>
__device__ __forceinline__ void h16_finish(const char* wsp, size_t tail_off, int n0, f32x4 (&acc)[TM16][TN16],
                                           const f32x4 (&acc2)[TM16][TN16]) {
  const int wn = (threadIdx.x >> 6) % WN;
  const float* inv = reinterpret_cast<const float*>(wsp + tail_off) + n0 + wn * TN16 * 16 + (threadIdx.x & 15);
#pragma unroll
  for (int tn = 0; tn < TN16; ++tn) {
    const float iv = inv[tn * 16];
#pragma unroll
    for (int tm = 0; tm < TM16; ++tm)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[tm][tn][r] = (acc[tm][tn][r] + acc2[tm][tn][r] * H16_LO_INV) * iv;
  }
}

// MODE bits 0-1: the pre-activation (pre_fn: none, leaky ReLU, other), bit 2: a 1-D pre-mask row multiplier --
// compile-time, so the step loop carries no per-element activation switch and no conditional mask load (both put ~30
// scalar branches and a load-history merge into every step); bit 4: the two-plane fp16 arithmetic (split_bf16.h
// put_h16x4, the WSPLIT_H16 image: three MFMA products into two accumulators instead of six)
template <int BM, int BN, int WM, int WN, bool TWO_D, int MODE>
__global__ __launch_bounds__(CONV_THREADS, 2) void conv_gs16_kernel(const ConvArgs a, const char* __restrict__ wsp,
                                                                    const int Npad, const int ntn, const int ksplit,
                                                                    const int mfast) {
  constexpr int NT = CONV_THREADS;
  constexpr int TM16 = BM / (WM * 16);
  constexpr int TN16 = BN / (WN * 16);
  constexpr int AV = BM * EC4 / NT;  // float4 groups of the A tile per thread
  constexpr int PA = MODE & 3;
  constexpr bool PMASK = !TWO_D && (MODE & 4) != 0;
  constexpr bool H16 = (MODE & 16) != 0;
  constexpr int NQ = H16 ? 2 : 3;            // planes per operand
  constexpr int RS = H16 ? ERS_H : ERS;      // LDS row stride
  static_assert(WM * WN == 4 && TM16 >= 1 && TN16 >= 1 && BM * EC4 % NT == 0, "tile shape");
  extern __shared__ __attribute__((aligned(16))) char smem_gs[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lc = lane & 15, lg = lane >> 4;
  int bx, by, bz;
  conv_block_coords(ntn, bx, by, bz);
  if (mfast && ntn > 0) {
    // each XCD's contiguous run of tiles walks M fastest: it streams only its share of the weight columns (the big
    // operand of these GEMMs) through its L2 while every XCD re-reads the small activation tile set
    const int t = bx * ntn + by;
    const int mt = (int)gridDim.x / ntn;
    bx = t % mt;
    by = t / mt;
  }
  const int zsplit = bz % ksplit;
  const int b = bz / ksplit;
  const int n0 = by * BN;
  const int m0 = bx * BM;
  const long long Mtot = TWO_D ? (long long)a.T_out * a.W_out : a.T_out;
  const float* X = a.x + (long long)b * a.x_bs;
  const float* PM = PMASK ? a.pre_mask + (long long)b * a.pre_mask_bs : nullptr;

  // (chunk, tap) steps [it0, it1) of this split-K slice
  const int taps = a.taps;
  const int total = (a.C_in / EK) * taps;
  const int per = (total + ksplit - 1) / ksplit;
  const int it0 = zsplit * per, it1 = min(total, it0 + per);
  const int last = it1 - 1;

  // ---- A gather: thread rows r_v = v * 32 + arow, channels ac4..ac4+3 of the step's chunk
  const int arow = store_row(tid / EC4), ac4 = (tid % EC4) << 2;
  int g0[AV];   // 1-D: input row of tap 0 (m * stride - pad); 2-D: oh - padh
  int w0v[AV];  // 2-D: ow - padw
  bool rok[AV];
#pragma unroll
  for (int v = 0; v < AV; ++v) {
    const long long m = (long long)m0 + v * (NT / EC4) + arow;
    rok[v] = m < Mtot;
    if constexpr (!TWO_D) {
      g0[v] = (int)m * a.stride - a.pad;
      w0v[v] = 0;
    } else {
      const int mm = rok[v] ? (int)m : 0;
      const int oh = mm / a.W_out;
      g0[v] = oh - a.padh;
      w0v[v] = mm - oh * a.W_out - a.padw;
    }
  }
  // The next step to gather, kept incrementally (no division per load): a_st with its chunk, tap and (2-D) kernel
  // row / column; loads past the slice's last step reload it (clamped), harmlessly.
  int a_st = it0, a_ch = it0 / taps, a_tap = it0 - (it0 / taps) * taps, a_kh = 0, a_kw = 0;
  if constexpr (TWO_D) {
    a_kh = a_tap / a.KW;
    a_kw = a_tap - a_kh * a.KW;
  }
  // Loads are branch-free: a row outside the input is read at row 0 (always valid) and zeroed when the slot is split
  // into LDS (its bit in aok clear). A conditional load (`ok ? load : 0`) merges the loaded and the zero value at the
  // branch join, and the waitcnt pass then waits for the load right there or at the register's next reuse: with it
  // the ring ran one step ahead instead of GS_D - 1 (every step waited out a load latency).
  f32x4 ar[GS_D][AV];
  float am[GS_D][AV];  // pre-mask value of the row (PMASK only)
  unsigned aok[GS_D];  // bit v: row v of the slot lies inside the input
  auto load_a = [&](f32x4 (&dst)[AV], float (&dm)[AV], unsigned& okb) __attribute__((always_inline)) {
    const float* src = X + a_ch * EK + ac4;
    okb = 0u;
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      int g;
      bool ok;
      if constexpr (!TWO_D) {
        g = g0[v] + a_tap * a.dil;
        ok = rok[v] && (unsigned)g < (unsigned)a.T_in;
      } else {
        const int ih = g0[v] + a_kh, iw = w0v[v] + a_kw;
        ok = rok[v] && (unsigned)ih < (unsigned)a.T_in && (unsigned)iw < (unsigned)a.W_in;
        g = ih * a.W_in + iw;
      }
      const unsigned gc = ok ? (unsigned)g : 0u;
      dst[v] = *reinterpret_cast<const f32x4*>(src + gc * (unsigned)a.ldx);  // conv_gs_eligible: 32-bit offsets
      if constexpr (PMASK) dm[v] = PM[gc];
      okb |= ok ? (1u << v) : 0u;
    }
    if (a_st < last) {
      ++a_st;
      if (++a_tap == taps) {
        a_tap = 0;
        ++a_ch;
        a_kh = 0;
        a_kw = 0;
      } else if constexpr (TWO_D) {
        if (++a_kw == a.KW) {
          a_kw = 0;
          ++a_kh;
        }
      }
    }
  };
  auto store_a = [&](char* As, const f32x4 (&src)[AV], const float (&sm)[AV], unsigned okb) __attribute__((always_inline)) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      f32x4 val = src[v];
      const bool ok = (okb >> v) & 1u;
#pragma unroll
      for (int j = 0; j < 4; ++j) val[j] = pre_fn<PA>(val[j], a.pre_act, a.pre_slope);
      if constexpr (PMASK) {
#pragma unroll
        for (int j = 0; j < 4; ++j) val[j] = ok ? val[j] * sm[v] : 0.f;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) val[j] = ok ? val[j] : 0.f;
      }
      if constexpr (H16) {
#pragma unroll
        for (int j = 0; j < 4; ++j) val[j] *= H16_XS;
        put_h16x4<2>(As + (v * (NT / EC4) + arow) * RS, ac4, val);
      } else {
        put_split4(As + (v * (NT / EC4) + arow) * RS, ac4, val);
      }
    }
  };

  // ---- B: pre-split fragments from L2
  typedef bf16x8 BFrag[TN16][NQ];
  BFrag br[GS_D];
  // the image's lane-major blocks (conv_wsb.hip k_wsplit): lane l reads 16-B slot l, one contiguous 1 KB per load
  const char* bp = wsp + (size_t)((n0 + wn * TN16 * 16) >> 4) * (NQ * GS_BLK) + lane * 16;
  const size_t bstep = (size_t)Npad * NQ * PLANE;
  auto load_b = [&](int st, BFrag& dst) __attribute__((always_inline)) {
    const char* p = bp + (size_t)st * bstep;
#pragma unroll
    for (int tn = 0; tn < TN16; ++tn)
#pragma unroll
      for (int q = 0; q < NQ; ++q) dst[tn][q] = *reinterpret_cast<const bf16x8*>(p + tn * (NQ * GS_BLK) + q * GS_BLK);
  };

  f32x4 acc[TM16][TN16], acc2[H16 ? TM16 : 1][H16 ? TN16 : 1];
#pragma unroll
  for (int tm = 0; tm < TM16; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN16; ++tn) {
      acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (H16) acc2[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  int aoff[TM16];
#pragma unroll
  for (int tm = 0; tm < TM16; ++tm) aoff[tm] = (wm * TM16 * 16 + tm * 16 + lc) * RS + lg * 16;
  auto compute = [&](const char* As, const BFrag& bf) __attribute__((always_inline)) {
#pragma unroll
    for (int tm = 0; tm < TM16; ++tm) {
      bf16x8 af[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) af[q] = *reinterpret_cast<const bf16x8*>(As + aoff[tm] + q * PLANE);
      if constexpr (H16) {
        mma_h16(af, bf, acc[tm], acc2[tm]);
        continue;
      }
#pragma unroll
      for (int tn = 0; tn < TN16; ++tn) {
        f32x4 c = acc[tm][tn];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2], bf[tn][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], bf[tn][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[tn][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], bf[tn][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[tn][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[tn][0], c, 0, 0, 0);
        acc[tm][tn] = c;
      }
    }
  };

  // Step i: issue B(i + D - 1), MFMAs on A(i) (LDS buffer i % 2) and B(i), then A(i + 1) -> LDS buffer (i + 1) % 2,
  // issue A(i + D), one barrier (load indices clamped to the slice: the tail reloads its last step, harmlessly). Ring
  // slots are (step - it0) % D, compile-time after the D-fold unroll. The whole groups of D steps run without a
  // branch inside (a skipped step would merge two load histories at its join and shorten every wait after it to the
  // skipped path's), the < D remaining steps after them; the prologue issues its loads in the order the steady state
  // leaves them (B(i), A(i + 1), B(i + 1), ...), so the loop header merges two identical pending-load histories.
  if (it0 < it1) {
    auto clampst = [&](int st) { return st < last ? st : last; };
    load_a(ar[0], am[0], aok[0]);
#pragma unroll
    for (int p = 1; p < GS_D; ++p) {
      load_b(clampst(it0 + p - 1), br[p - 1]);
      load_a(ar[p], am[p], aok[p]);
    }
    store_a(smem_gs, ar[0], am[0], aok[0]);
    __syncthreads();
    auto step = [&](int i, int p) __attribute__((always_inline)) {
      load_b(clampst(i + GS_D - 1), br[(p + GS_D - 1) % GS_D]);
      __builtin_amdgcn_sched_barrier(0);
      compute(smem_gs + (size_t)((i - it0) & 1) * BM * RS, br[p]);
      // A(i + 1) -> the other LDS buffer (on the last step a harmless copy of A(last) nobody reads), then A(i + D)
      // into the slot A(i) left
      store_a(smem_gs + (size_t)((i + 1 - it0) & 1) * BM * RS, ar[(p + 1) % GS_D], am[(p + 1) % GS_D],
              aok[(p + 1) % GS_D]);
      load_a(ar[p], am[p], aok[p]);
      __syncthreads();
    };
    int base = it0;
    for (; base + GS_D <= it1; base += GS_D) {
#pragma unroll
      for (int p = 0; p < GS_D; ++p) step(base + p, p);
    }
#pragma unroll
    for (int p = 0; p < GS_D - 1; ++p)
      if (base + p < it1) step(base + p, p);
  }
  if constexpr (H16) h16_finish<TM16, TN16, WN>(wsp, (size_t)total * bstep, n0, acc, acc2);
  store_tile16<TM16, TN16, WM, WN, TWO_D>(a, m0, n0, b, zsplit, ksplit, Mtot, acc);
}

template <int BM, int BN, int WM, int WN, bool TWO_D, int MODE>
void launch_gs_mode(const ConvArgs& a, dim3 grid, size_t smem, int ntn, int ksplit, int mfast, hipStream_t s) {
  static size_t smem_set = 64 * 1024;  // per instantiation: raise the dynamic-LDS limit once (ConvArgs::lds_pad)
  if (smem > smem_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv_gs16_kernel<BM, BN, WM, WN, TWO_D, MODE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    smem_set = smem;
  }
  hipLaunchKernelGGL((conv_gs16_kernel<BM, BN, WM, WN, TWO_D, MODE>), grid, dim3(CONV_THREADS), smem, s, a,
                     static_cast<const char*>(a.wsplit), a.wsplit_npad, ntn, ksplit, mfast);
}

template <int BM, int BN, int WM, int WN, bool TWO_D>
hipError_t launch_gs(const ConvArgs& a, int ntn_enable, int ksplit, hipStream_t s) {
  const long long Mtot = TWO_D ? (long long)a.T_out * a.W_out : a.T_out;
  const long long mtiles = (Mtot + BM - 1) / BM;
  if (mtiles > INT32_MAX / 64 || a.wsplit_npad % BN != 0 || ksplit < 1 || (ksplit > 1 && !a.ws)) return hipErrorInvalidValue;
  const int ntiles = (a.N + BN - 1) / BN;
  const int ntn = ntn_enable ? ntiles : 0;
  dim3 grid((unsigned)(ntn ? mtiles * ntiles : mtiles), ntn ? 1 : ntiles, a.batch * ksplit);
  const bool h16 = a.wsplit_fmt == WSPLIT_H16;
  // the throttle pad (ConvArgs::lds_pad) is clamped to the CU's 160 KB: above 80 KB it means one workgroup per CU
  const size_t smem = std::min((size_t)2 * BM * (h16 ? ERS_H : ERS) + (size_t)std::max(0, a.lds_pad),
                               std::max((size_t)2 * BM * (h16 ? ERS_H : ERS), (size_t)160 * 1024));
  // M-fastest tile runs when the pre-split weight (6 B per element) outweighs the activation operand (4 B)
  const double wbytes = 6.0 * a.N * a.C_in * a.taps, abytes = 4.0 * (double)Mtot * a.C_in * a.batch;
  const int mfast = wbytes > abytes ? 1 : 0;
  const int mode = pre_mode(a.pre_act) | (!TWO_D && a.pre_mask ? 4 : 0) | (h16 ? 16 : 0);
  constexpr bool HI = true;
  switch (mode) {
    case 0: launch_gs_mode<BM, BN, WM, WN, TWO_D, 0>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 1: launch_gs_mode<BM, BN, WM, WN, TWO_D, 1>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 2: launch_gs_mode<BM, BN, WM, WN, TWO_D, 2>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 4: launch_gs_mode<BM, BN, WM, WN, TWO_D, 4>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 5: launch_gs_mode<BM, BN, WM, WN, TWO_D, 5>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 6: launch_gs_mode<BM, BN, WM, WN, TWO_D, 6>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 16: launch_gs_mode<BM, BN, WM, WN, TWO_D, HI ? 16 : 0>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 17: launch_gs_mode<BM, BN, WM, WN, TWO_D, HI ? 17 : 0>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 18: launch_gs_mode<BM, BN, WM, WN, TWO_D, HI ? 18 : 0>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 20: launch_gs_mode<BM, BN, WM, WN, TWO_D, HI && !TWO_D ? 20 : 0>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 21: launch_gs_mode<BM, BN, WM, WN, TWO_D, HI && !TWO_D ? 21 : 0>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 22: launch_gs_mode<BM, BN, WM, WN, TWO_D, HI && !TWO_D ? 22 : 0>(a, grid, smem, ntn, ksplit, mfast, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---- 3x3 / pad-1 2-D convs on images at most 32 pixels wide (the RMVPE U-Net's deep levels, 4..32 wide):
// "windowed" gather-streamed kernel. A 64-pixel tile is rh = 64 / W whole image rows, so its outputs are 64
// consecutive flattened pixels (the 1-D store_tile16 and split-K slab apply unchanged). Per 32-channel chunk the
// tile's (rh + 2) x (W + 2) input window is split into LDS ONCE and all 9 taps read their shifted A fragments from
// it (the per-tap gather of conv_gs16_kernel re-loaded and re-split every input pixel 9 times: ~90 VALU of its ~200
// instructions per step); the next chunk's window is prefetched into registers during the current chunk's taps.
// B streams from the lane-major image through the same 3-deep register ring. Split-K slices are whole chunks, so
// chunk switches fall on 3-step group boundaries and the 9 unrolled taps per chunk carry no branch.
constexpr int GSW_MAXW = 32;
constexpr int GSW_WROWS = (64 / GSW_MAXW + 2) * (GSW_MAXW + 2);  // largest window: rh = 2 (4 x 34 = 136 pixels)
// B ring depth of the windowed kernel (3 or 9: the ring slot of a tap is tap % depth). 9 deep issues a whole chunk's
// weights in one burst (236 VGPRs, no spill) and was no faster in the C2 step (same-box A/B r05k: 3 deep 13.36 /
// 13.53 / 13.38 ms against 9 deep 13.66 / 13.60 / 13.39): these launches are not waiting on the B loads
#ifndef GSW_DEPTH
#define GSW_DEPTH 3
#endif
constexpr int GSW_D = GSW_DEPTH;
static_assert(9 % GSW_D == 0, "the ring slot of a tap is tap % GSW_D: whole chunks of 9 taps");

// MODE bits 0-1 the pre-activation, bit 4 the two-plane fp16 arithmetic (as conv_gs16_kernel)
template <int MODE>
__global__ __launch_bounds__(CONV_THREADS, 2) void conv_gsw16_kernel(const ConvArgs a, const char* __restrict__ wsp,
                                                                     const int Npad, const int ntn, const int ksplit,
                                                                     const int mfast) {
  constexpr int BM = 64, BN = 64, WM = 2, WN = 2;
  constexpr int NT = CONV_THREADS;
  constexpr int TM16 = BM / (WM * 16), TN16 = BN / (WN * 16);
  constexpr int PA = MODE & 3;
  constexpr bool H16 = (MODE & 16) != 0;
  constexpr int NQ = H16 ? 2 : 3;
  constexpr int RS = H16 ? ERS_H : ERS;
  constexpr int D = H16 ? GSW_D : GS_D;  // the three-plane form (NQ = 3) keeps the 3-deep ring: 9 deep spills
  constexpr int WV = (GSW_WROWS * EC4 + NT - 1) / NT;  // float4 groups of the window per thread
  extern __shared__ __attribute__((aligned(16))) char smem_gsw[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lc = lane & 15, lg = lane >> 4;
  int bx, by, bz;
  conv_block_coords(ntn, bx, by, bz);
  if (mfast && ntn > 0) {
    const int t = bx * ntn + by;
    const int mt = (int)gridDim.x / ntn;
    bx = t % mt;
    by = t / mt;
  }
  const int zsplit = bz % ksplit;
  const int b = bz / ksplit;
  const int n0 = by * BN;
  const int W = a.W_out, H = a.T_out;
  const int rh = BM / W, aw = W + 2;
  const int h0 = bx * rh;
  const int nwin = (rh + 2) * aw;
  const float* X = a.x + (long long)b * a.x_bs;
  const int nch = a.C_in / EK;
  const int pc = (nch + ksplit - 1) / ksplit;  // whole chunks per split-K slice
  const int c0 = zsplit * pc, c1 = min(nch, c0 + pc);

  // ---- window staging: thread rows v * 32 + arow (window pixel (wr / aw, wr % aw)), channels ac4..ac4+3
  const int arow = store_row(tid / EC4), ac4 = (tid % EC4) << 2;
  f32x4 wr_[WV];
  unsigned wok = 0u;
  auto load_win = [&](int ch) __attribute__((always_inline)) {
    const float* src = X + ch * EK + ac4;
    wok = 0u;
#pragma unroll
    for (int v = 0; v < WV; ++v) {
      const int r = v * (NT / EC4) + arow;
      const int wh = r / aw, wc = r - wh * aw;
      const int ih = h0 - 1 + wh, iw = wc - 1;
      const bool ok = r < nwin && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      const unsigned g = ok ? (unsigned)(ih * W + iw) : 0u;
      wr_[v] = *reinterpret_cast<const f32x4*>(src + g * (unsigned)a.ldx);  // branch-free (conv_gs16_kernel)
      wok |= ok ? (1u << v) : 0u;
    }
  };
  auto store_win = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int v = 0; v < WV; ++v) {
      const int r = v * (NT / EC4) + arow;
      if (r < nwin) {
        f32x4 val = wr_[v];
        const bool ok = (wok >> v) & 1u;
#pragma unroll
        for (int j = 0; j < 4; ++j) val[j] = ok ? pre_fn<PA>(val[j], a.pre_act, a.pre_slope) : 0.f;
        if constexpr (H16) {
#pragma unroll
          for (int j = 0; j < 4; ++j) val[j] *= H16_XS;
          put_h16x4<2>(smem_gsw + r * RS, ac4, val);
        } else {
          put_split4(smem_gsw + r * RS, ac4, val);
        }
      }
    }
  };

  // ---- B ring (conv_gs16_kernel's)
  typedef bf16x8 BFrag[TN16][NQ];
  BFrag br[D];
  const char* bp = wsp + (size_t)((n0 + wn * TN16 * 16) >> 4) * (NQ * GS_BLK) + lane * 16;
  const size_t bstep = (size_t)Npad * NQ * PLANE;
  auto load_b = [&](int st, BFrag& dst) __attribute__((always_inline)) {
    const char* p = bp + (size_t)st * bstep;
#pragma unroll
    for (int tn = 0; tn < TN16; ++tn)
#pragma unroll
      for (int q = 0; q < NQ; ++q) dst[tn][q] = *reinterpret_cast<const bf16x8*>(p + tn * (NQ * GS_BLK) + q * GS_BLK);
  };

  f32x4 acc[TM16][TN16], acc2[H16 ? TM16 : 1][H16 ? TN16 : 1];
#pragma unroll
  for (int tm = 0; tm < TM16; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN16; ++tn) {
      acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (H16) acc2[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  // A fragment rows: tile pixel ml = (r, c) -> window pixel (r + kh, c + kw)
  int aoff[TM16];
#pragma unroll
  for (int tm = 0; tm < TM16; ++tm) {
    const int ml = wm * TM16 * 16 + tm * 16 + lc;
    const int r = ml / W, c = ml - r * W;
    aoff[tm] = (r * aw + c) * RS + lg * 16;
  }
  auto compute = [&](int tap, const BFrag& bf) __attribute__((always_inline)) {
    const int toff = ((tap / 3) * aw + (tap % 3)) * RS;
#pragma unroll
    for (int tm = 0; tm < TM16; ++tm) {
      bf16x8 af[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) af[q] = *reinterpret_cast<const bf16x8*>(smem_gsw + aoff[tm] + toff + q * PLANE);
      if constexpr (H16) {
        mma_h16(af, bf, acc[tm], acc2[tm]);
        continue;
      }
#pragma unroll
      for (int tn = 0; tn < TN16; ++tn) {
        f32x4 cc = acc[tm][tn];
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2], bf[tn][0], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], bf[tn][1], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[tn][2], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], bf[tn][0], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[tn][1], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[tn][0], cc, 0, 0, 0);
        acc[tm][tn] = cc;
      }
    }
  };

  if (c0 < c1) {
    const int it0 = c0 * 9, last = c1 * 9 - 1;
    auto clampst = [&](int st) { return st < last ? st : last; };
    load_win(c0);
#pragma unroll
    for (int p = 0; p < D - 1; ++p) load_b(clampst(it0 + p), br[p]);
    store_win();
    if (c0 + 1 < c1) load_win(c0 + 1);
    __syncthreads();
    for (int ch = c0; ch < c1; ++ch) {
      const int base = ch * 9;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int p = tap % D;  // ring slot: (step - it0) % D = tap % D (whole chunks of 9 steps)
        load_b(clampst(base + tap + D - 1), br[(p + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);
        compute(tap, br[p]);
      }
      if (ch + 1 < c1) {
        __syncthreads();  // every wave is done with this chunk's window
        store_win();
        if (ch + 2 < c1) load_win(ch + 2);
        __syncthreads();
      }
    }
  }
  if constexpr (H16) h16_finish<TM16, TN16, WN>(wsp, (size_t)nch * 9 * bstep, n0, acc, acc2);
  store_tile16<TM16, TN16, WM, WN>(a, h0 * W, n0, b, zsplit, ksplit, (long long)H * W, acc);
}

template <int MODE>
void launch_gsw_mode(const ConvArgs& a, dim3 grid, size_t smem, int ntn, int ksplit, int mfast, hipStream_t s) {
  hipLaunchKernelGGL((conv_gsw16_kernel<MODE>), grid, dim3(CONV_THREADS), smem, s, a,
                     static_cast<const char*>(a.wsplit), a.wsplit_npad, ntn, ksplit, mfast);
}

hipError_t launch_gsw(const ConvArgs& a, int ntn_enable, int ksplit, hipStream_t s) {
  const int W = a.W_out, rh = 64 / W;
  const long long mtiles = (a.T_out + rh - 1) / rh;
  if (a.wsplit_npad % 64 != 0 || ksplit < 1 || (ksplit > 1 && !a.ws) || mtiles > INT32_MAX / 64) return hipErrorInvalidValue;
  const int ntiles = (a.N + 63) / 64;
  const int ntn = ntn_enable ? ntiles : 0;
  dim3 grid((unsigned)(ntn ? mtiles * ntiles : mtiles), ntn ? 1 : ntiles, a.batch * ksplit);
  const bool h16 = a.wsplit_fmt == WSPLIT_H16;
  const size_t smem = (size_t)(rh + 2) * (W + 2) * (h16 ? ERS_H : ERS);
  const double wbytes = 6.0 * a.N * a.C_in * 9, abytes = 4.0 * (double)a.T_out * W * a.C_in * a.batch;
  const int mfast = wbytes > abytes ? 1 : 0;
  switch (pre_mode(a.pre_act) | (h16 ? 16 : 0)) {
    case 0: launch_gsw_mode<0>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 1: launch_gsw_mode<1>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 2: launch_gsw_mode<2>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 16: launch_gsw_mode<16>(a, grid, smem, ntn, ksplit, mfast, s); break;
    case 17: launch_gsw_mode<17>(a, grid, smem, ntn, ksplit, mfast, s); break;
    default: launch_gsw_mode<18>(a, grid, smem, ntn, ksplit, mfast, s); break;
  }
  return hipGetLastError();
}

}  // namespace

bool conv_gs_eligible(const ConvArgs& a, bool two_d) {
  const bool vec_a = ((a.ldx & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.x) & 15) == 0) && ((a.x_bs & 3) == 0);
  // the 2x2-phase ConvTranspose2d output (OUT_UPSAMPLE2D, the U-Net decoder's up-convs, round 5) with the plain epilogue
  // (store_tile16 maps it; a split launch's combine does, as for the LDS-staged kernel)
  const bool up2d = two_d && a.out_map == OUT_UPSAMPLE2D && a.out_cv > 0 && a.N == 4 * a.out_cv && !a.res &&
                    a.acc_mode == ACC_STORE && !a.mask && !a.nz_har;
  const bool common = a.batch_inner == 1 && !a.b_kn && a.C_in % EK == 0 && a.C_in > 0 && a.taps >= 1 && vec_a &&
                      (a.out_map == OUT_ROWS || up2d) && a.stride >= 1 && a.dil >= 1;
  if (!common) return false;
  // 32-bit element offsets within one batch entry (the A gather)
  const long long rows_in = two_d ? (long long)a.T_in * a.W_in : a.T_in;
  if (rows_in * a.ldx + a.C_in >= INT32_MAX) return false;
  if (!two_d) return (long long)a.T_out * a.stride < INT32_MAX / 2 && a.T_in < INT32_MAX / 2;
  return a.taps == a.KH * a.KW && !a.pre_mask && a.stride == 1 && a.W_out >= 1 && a.W_in >= 1;
}

// cfg 30: 64 x 64 (2 x 2 waves of 32 x 32). Round 5's 64 x 32 tiles with the K walk split over the 4 waves of a
// workgroup (the windowed form, cfg 33) and the 128 x 64 / 64 x 128 tiles (31, 32) measured no faster and are gone
bool conv_gs_tile(int cfg, int& BM, int& BN) {
  if (cfg != 30) return false;
  BM = 64;
  BN = 64;
  return true;
}

// the windowed 2-D kernel: 3x3 / pad 1 / stride 1, same-size images at most 32 pixels wide with 32 % W == 0
bool conv_gsw_eligible(const ConvArgs& a) {
  return conv_gs_eligible(a, true) && a.KH == 3 && a.KW == 3 && a.padh == 1 && a.padw == 1 &&
         a.T_in == a.T_out && a.W_in == a.W_out && a.W_out <= GSW_MAXW && GSW_MAXW % a.W_out == 0 && a.W_out >= 4;
}

hipError_t conv_gs_launch(const ConvArgs& a, int cfg, int ntn_enable, hipStream_t s, bool two_d, int ksplit) {
  if (!a.wsplit || !conv_gs_eligible(a, two_d) || a.lowp) return hipErrorInvalidValue;
  if (cfg != 30) return hipErrorInvalidValue;
  if (two_d && conv_gsw_eligible(a)) return launch_gsw(a, ntn_enable, ksplit, s);
  return two_d ? launch_gs<64, 64, 2, 2, true>(a, ntn_enable, ksplit, s)
               : launch_gs<64, 64, 2, 2, false>(a, ntn_enable, ksplit, s);
}

}  // namespace rvcx
