// The weight-streamed fp16-split convolution (conv_wsb.hip conv_wsb16_kernel, MODE bit 4) with a UNIFORM load schedule,
// for the generator's long ResBlock convs (taps >= 5, one split-K slice).
//
// Why a second form: vmcnt retires in issue order, and the waitcnt pass merges the load histories of a loop's paths
// pessimistically. conv_wsb16_kernel loads the next chunk's whole A halo at the chunk switch (a branch taken once per
// `taps` steps); on the steps after a switch the B-fragment waits then also waited for those HBM loads. bench_conv with
// the halo loads removed ran +24 % (C128 k11) to +26 % (C64 k11) faster (r04h, build/exp).
//
// Here every step issues the same loads in the same order, so the compiler's waits are exact on every path:
//   step s (tap t of chunk c):  B fragments of step s + 1  |  MFMAs of step s (wait for B(s) only)  |
//                               LDS write of the halo part(s) loaded at step s - 2 (into the idle halo buffer)  |
//                               load of halo part(s) t * PPS .. of chunk c + 1 (clamped: past the window, the last
//                               part again)  |  at the chunk's last tap: one barrier, the halo buffers swap
// A part loaded at step s is first waited for at step s + 2 (by the B(s + 2) wait that follows it in issue order), which
// is also where it is written. PPS parts per step, PPS = ceil(parts / (taps - 2)), so every part of chunk c + 1 is
// written by the last tap of chunk c. The duplicates (clamped parts) land in the buffer of chunk c + 2 before its own
// part is written there, so they are overwritten. Two halo buffers in LDS, one barrier per chunk.
// Arithmetic, image layout, tile shape and epilogue are conv_wsb16_kernel's (bit-identical results).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "conv_common.h"
#include "split_bf16.h"

namespace rvcx {

namespace {

using namespace splitbf16;

constexpr int WBLK_C = 1024;  // conv_wsb.hip WBLK: bytes of one (step, 16-column group, plane) image block
constexpr int WSC_HALO = 64;  // max (taps - 1) * dil
constexpr int WSC_BM = 128, WSC_BN = 64;
constexpr int WSC_AP = ((WSC_BM + WSC_HALO) * EC4 + CONV_THREADS - 1) / CONV_THREADS;  // halo parts (6)

// MODE: bits 0-1 the pre-activation (pre_fn), bit 3 the reduced-precision hi-plane product alone
template <int PPS, int WM, int WN, int MODE>
__global__ __launch_bounds__(CONV_THREADS, 3) void conv_wsc16_kernel(const ConvArgs a, const char* __restrict__ wsp,
                                                                     const int Npad, const int nrows_a, const int ntn) {
  constexpr int NT = CONV_THREADS;
  constexpr int PA = MODE & 3;
  constexpr bool LOWP = (MODE & 8) != 0;
  constexpr int NQ = LOWP ? 1 : 2;  // planes an MFMA step reads
  constexpr int NQI = 2;            // planes of the image
  constexpr int RS = ERS_H;
  constexpr int BM = WSC_BM, BN = WSC_BN, AP = WSC_AP;
  constexpr int TM16 = BM / (WM * 16);
  constexpr int TN16 = BN / (WN * 16);
  static_assert(WM * WN == 4 && TM16 >= 1 && TN16 >= 1, "4 waves, whole 16x16 sub-tiles");
  extern __shared__ __attribute__((aligned(16))) char smem_wc[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lc = lane & 15, lg = lane >> 4;
  int bx, by, bz;
  conv_block_coords(ntn, bx, by, bz);
  const int b = bz;
  const int n0 = by * BN;
  const int m0 = bx * BM;
  const float* X = a.x + (long long)b * a.x_bs;
  const int row0 = m0 - a.pad;
  const int hbuf = (nrows_a + 1) * RS;  // one halo image + a dummy row (the writes of rows past the halo land there)
  const int aoff0 = (wm * TM16 * 16 + lc) * RS + lg * 16;  // A fragments: tm / plane offsets are immediates
  unsigned boff[TN16];  // lane l reads 16-B slot l of each block: one contiguous 1 KB per wave load
#pragma unroll
  for (int tn = 0; tn < TN16; ++tn)
    boff[tn] = (unsigned)(((n0 + wn * TN16 * 16 + tn * 16) >> 4) * (NQI * WBLK_C) + lane * 16);
  const size_t bstep = (size_t)Npad * NQI * PLANE;

  f32x4 acc[TM16][TN16], acc2[LOWP ? 1 : TM16][LOWP ? 1 : TN16];
#pragma unroll
  for (int tm = 0; tm < TM16; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN16; ++tn) {
      acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (!LOWP) acc2[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

  // ---- halo part p: rows p * (NT / EC4) + arow (store_row order), channels ac4 .. ac4 + 3 of a chunk
  const int arow = store_row(tid / EC4), ac4 = (tid % EC4) << 2;
  // ASM = true: an inline-asm load, absent from hipcc's waitcnt bookkeeping (the loop counts it itself, see `step`)
  auto load_part = [&](int p, int c0, f32x4& v, bool& ok, auto asmc) __attribute__((always_inline)) {
    const int r = p * (NT / EC4) + arow;
    const int g = row0 + r;
    ok = r < nrows_a && g >= 0 && g < a.T_in;
    const int gc = ok ? g : 0;
    const float* src = X + c0 + (unsigned)(gc * a.ldx + ac4);  // < 2^30 (launch check)
    if constexpr (decltype(asmc)::value) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(src));
    else v = *reinterpret_cast<const f32x4*>(src);
  };
  auto write_part = [&](int p, f32x4 v, bool ok, char* buf) __attribute__((always_inline)) {
    const int r = p * (NT / EC4) + arow;
    const int rr = r < nrows_a ? r : nrows_a;  // rows past the halo: the dummy row (branch-free)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = ok ? pre_fn<PA>(v[j], a.pre_act, a.pre_slope) * H16_XS : 0.f;
    put_h16x4<NQ>(buf + rr * RS, ac4, v);
  };
  typedef bf16x8 BFrag[TN16][NQ];
  auto load_b = [&](const char* base, BFrag& dst) __attribute__((always_inline)) {  // inline asm (counted by `step`)
#pragma unroll
    for (int tn = 0; tn < TN16; ++tn) {
      const char* src = base + boff[tn];
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst[tn][0]) : "v"(src));
      if constexpr (NQ > 1) asm volatile("global_load_dwordx4 %0, %1, off offset:1024" : "=v"(dst[tn][1]) : "v"(src));
    }
  };
  static_assert(WBLK_C == 1024, "the asm B loads address plane 1 at offset:1024");
  auto compute = [&](const char* ap, const BFrag& bf) __attribute__((always_inline)) {
#pragma unroll
    for (int tm = 0; tm < TM16; ++tm) {
      bf16x8 af[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) af[q] = *reinterpret_cast<const bf16x8*>(ap + tm * 16 * RS + q * PLANE);
      const f16x8 ah = __builtin_bit_cast(f16x8, af[0]);
#pragma unroll
      for (int tn = 0; tn < TN16; ++tn) {
        const f16x8 bh = __builtin_bit_cast(f16x8, bf[tn][0]);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[tm][tn], 0, 0, 0);
        if constexpr (!LOWP) {
          f32x4 c = acc2[tm][tn];
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, af[NQ - 1]), bh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, __builtin_bit_cast(f16x8, bf[tn][NQ - 1]), c, 0, 0, 0);
          acc2[tm][tn] = c;
        }
      }
    }
  };

  const int taps = a.taps, nch = a.C_in / EK;
  const int total = nch * taps;
  const char* const blast = wsp + (size_t)(total - 1) * bstep;  // B prefetches past the last step re-read it
  const int dstride = a.dil * RS;
  char* cur = smem_wc;         // halo of the chunk being computed
  char* nxt = smem_wc + hbuf;  // halo of the next chunk, being written

  // prologue: chunk 0's halo into `cur`; then the loads in flight at the loop head in the steady state's order (ring
  // slot 0, B of step 0, ring slot 1), so the waitcnt state entering the loop equals the one on its back edge. The
  // ring slots start with the last part of chunk 1, a duplicate that its own write overwrites later.
  {
    f32x4 v[AP];
    bool ok[AP];
#pragma unroll
    for (int p = 0; p < AP; ++p) load_part(p, 0, v[p], ok[p], std::false_type{});
#pragma unroll
    for (int p = 0; p < AP; ++p) write_part(p, v[p], ok[p], cur);
  }
  __syncthreads();
  int tap = 0, ch = 0;
  int cnext = (nch > 1 ? 1 : 0) * EK;
  BFrag bq0, bq1;
  f32x4 r0[PPS], r1[PPS];
  int p0[PPS], p1[PPS];
  bool k0[PPS], k1[PPS];
#pragma unroll
  for (int u = 0; u < PPS; ++u) {
    p0[u] = p1[u] = AP - 1;
    load_part(AP - 1, cnext, r0[u], k0[u], std::true_type{});
  }
  load_b(wsp, bq0);
#pragma unroll
  for (int u = 0; u < PPS; ++u) load_part(AP - 1, cnext, r1[u], k1[u], std::true_type{});
  const char* bnext = wsp + bstep < blast ? wsp + bstep : blast;
  // In issue order every step is: B(s + 1) | wait | MFMAs of step s | write A(s - 2) | load A(s) | (barrier). At the
  // wait the loads younger than B(s) are A(s - 1) and B(s + 1): vmcnt(PPS + NB) retires B(s) and, older, A(s - 2). The
  // empty asm statements after it make those registers opaque there, so no consumer is scheduled above the wait.
  constexpr int NB = TN16 * NQ;
  auto step = [&](BFrag& bcur, BFrag& bnxt, f32x4 (&rs)[PPS], int (&ps)[PPS], bool (&ks)[PPS])
      __attribute__((always_inline)) {
    load_b(bnext, bnxt);
    bnext = bnext + bstep < blast ? bnext + bstep : blast;
    asm volatile("s_waitcnt vmcnt(%c0)" ::"i"(PPS + NB));
#pragma unroll
    for (int tn = 0; tn < TN16; ++tn)
#pragma unroll
      for (int q = 0; q < NQ; ++q) asm volatile("" : "+v"(bcur[tn][q]));
#pragma unroll
    for (int u = 0; u < PPS; ++u) asm volatile("" : "+v"(rs[u]));
    compute(cur + tap * dstride + aoff0, bcur);
#pragma unroll
    for (int u = 0; u < PPS; ++u) write_part(ps[u], rs[u], ks[u], nxt);
#pragma unroll
    for (int u = 0; u < PPS; ++u) {
      ps[u] = min(tap * PPS + u, AP - 1);
      load_part(ps[u], cnext, rs[u], ks[u], std::true_type{});
    }
    if (++tap == taps) {
      tap = 0;
      ++ch;
      cnext = min(ch + 1, nch - 1) * EK;
      // the halo writes of every wave land before any wave reads the buffer; a bare barrier, so the loads in flight
      // stay in flight (__syncthreads' fence may drain them)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      char* const t = cur;
      cur = nxt;
      nxt = t;
    }
  };
  for (int s = 0; s < total; s += 2) {
    step(bq0, bq1, r0, p0, k0);
    if (s + 1 < total) step(bq1, bq0, r1, p1, k1);
  }
  // the ring's last loads (duplicates) must land before their registers are reused
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // acc + 2^-11 acc2, times 1 / (weight scale x activation scale) from the image tail: exact powers of two
  const float inv = *reinterpret_cast<const float*>(wsp + (size_t)total * bstep + sizeof(float));
#pragma unroll
  for (int tm = 0; tm < TM16; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN16; ++tn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[tm][tn][r];
        if constexpr (!LOWP) v += acc2[tm][tn][r] * H16_LO_INV;
        acc[tm][tn][r] = v * inv;
      }
  store_tile16<TM16, TN16, WM, WN>(a, m0, n0, b, 0, 1, (long long)a.T_out, acc);
}

template <int PPS, int WM, int WN>
hipError_t launch_wsc(const ConvArgs& a, int ntn_enable, hipStream_t s) {
  const int nrows_a = WSC_BM + (a.taps - 1) * a.dil;
  const size_t smem = 2 * (size_t)(nrows_a + 1) * ERS_H;
  const int mtiles = (a.T_out + WSC_BM - 1) / WSC_BM;
  const int ntiles = (a.N + WSC_BN - 1) / WSC_BN;
  const int ntn = ntn_enable ? ntiles : 0;
  dim3 grid(ntn ? mtiles * ntiles : mtiles, ntn ? 1 : ntiles, a.batch);
  const int mode = pre_mode(a.pre_act) | (a.lowp ? 8 : 0);
  void (*kern)(const ConvArgs, const char*, int, int, int);
  switch (mode) {
    case 0: kern = conv_wsc16_kernel<PPS, WM, WN, 0>; break;
    case 1: kern = conv_wsc16_kernel<PPS, WM, WN, 1>; break;
    case 8: kern = conv_wsc16_kernel<PPS, WM, WN, 8>; break;
    case 9: kern = conv_wsc16_kernel<PPS, WM, WN, 9>; break;
    default: return hipErrorInvalidValue;
  }
  static size_t smem_set[16] = {};
  if (smem > 64 * 1024 && smem > smem_set[mode]) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    smem_set[mode] = smem;
  }
  hipLaunchKernelGGL(kern, grid, dim3(CONV_THREADS), smem, s, a, static_cast<const char*>(a.wsplit), a.wsplit_npad,
                     nrows_a, ntn);
  return hipGetLastError();
}

}  // namespace

bool conv_wsc_enabled() {
  static const bool v = [] {  // RVCX_WSC=1: the k >= 5 generator convs on this kernel (validation pending: off)
    const char* e = std::getenv("RVCX_WSC");
    return e && std::atoi(e) == 1;
  }();
  return v;
}

// the fp16 image, 1-D, one split-K slice, the tile shape of cfg 23 (2 x 2 waves of 64 x 32), taps >= 5, 32-bit
// in-tensor offsets; hipErrorInvalidValue otherwise (the caller falls back to conv_wsb16_kernel)
hipError_t conv_wsc_launch(const ConvArgs& a, int cfg, int ntn_enable, int ksplit, hipStream_t s) {
  if (!conv_wsc_enabled() || cfg != 23 || a.wsplit_fmt != WSPLIT_H16 || ksplit != 1 || a.pre_mask || a.stride != 1 ||
      a.C_in % EK != 0 || a.C_in < EK || a.wsplit_npad % WSC_BN != 0 || a.taps < 5 ||
      (a.taps - 1) * a.dil > WSC_HALO || pre_mode(a.pre_act) == PA_ANY || (long long)a.T_in * a.ldx >= (1ll << 30))
    return hipErrorInvalidValue;
  // every part of the next chunk is written by the chunk's last tap: PPS * (taps - 2) >= parts
  if (a.taps - 2 >= WSC_AP) return launch_wsc<1, 2, 2>(a, ntn_enable, s);
  if (2 * (a.taps - 2) >= WSC_AP) return launch_wsc<2, 2, 2>(a, ntn_enable, s);
  return hipErrorInvalidValue;
}

}  // namespace rvcx
