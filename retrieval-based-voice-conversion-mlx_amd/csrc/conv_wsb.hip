// fp32 implicit-GEMM convolution with the weights pre-split in HBM ("weight-streamed B"), for the long 1-D convs of
// the generator (ResBlocks, ConvTranspose phases, conv_pre). Two arithmetics in one kernel (conv_wsb16_kernel): the
// default two-plane fp16 split (split_bf16.h put_h16x4: x = h + 2^-11 l, three v_mfma_f32_16x16x32_f16 products per
// step, the weights from the per-column-scaled k_wsplit_h16 image), and the exact 3-plane bf16 split of conv_emu.hip
// (x = x0 + x1 + x2, six plane products smallest first; rvcx_set_conv_math mode 2). The kernel is restructured so the
// (chunk, tap) loop has no barrier and no conversion work:
//   * the weights are split ONCE (k_wsplit / k_wsplit_h16, cached per weight tensor by the runtime) into lane-major
//     1 KB plane blocks per (chunk, tap, 16-column group), so every lane loads its MFMA B fragments straight from
//     L2/L1 as 16-byte vectors, one iteration ahead, into registers (two register sets);
//   * only the activation halo goes through LDS (split once per 32-channel chunk and reused by every tap); the
//     next chunk's halo is prefetched into registers during the current chunk's taps;
//   * barriers only at chunk changes (two per 32 input channels).
#include <algorithm>
#include <cstdlib>

#include "conv_common.h"
#include "split_bf16.h"

namespace rvcx {

namespace {

using namespace splitbf16;

constexpr int WROW = 3 * PLANE;  // bytes of one (chunk, tap, column) row of split weights in HBM
constexpr int WSB_HALO = 64;     // max (taps - 1) * dil: the A prefetch registers cover BM + 64 rows

// w [tap][n][c] (ldw, w_ts) -> the pre-split image: per (chunk, tap) step, per 16-column group and plane a 1 KB
// block laid out lane-major for the 16x16x32 MFMA B operand: 16-B slot g * 16 + j holds channels 8g..8g+7 of column
// 16 * group + j, so one wave's fragment load of a plane is one contiguous 1 KB (8 whole 128-B lines) -- the earlier
// [column][hi | mid | lo] rows made every such load touch 16-24 lines for 64-B pieces of each. Zero beyond N and
// C_in. The plane arithmetic is put_split1's.
constexpr int WBLK = 1024;  // bytes of one (step, 16-column group, plane) block
__global__ void k_wsplit(const float* __restrict__ w, int ldw, long long w_ts, int N, int C_in, int taps, int nchunks,
                         int Npad, unsigned short* __restrict__ out) {
  const long long total = (long long)nchunks * taps * Npad * EK;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % EK);
    const long long r = i / EK;
    const int n = (int)(r % Npad);
    const long long ct = r / Npad;
    const int tap = (int)(ct % taps), ch = (int)(ct / taps);
    const int cc = ch * EK + c;
    const float v = (n < N && cc < C_in) ? w[tap * w_ts + (long long)n * ldw + cc] : 0.f;
    const unsigned h = pk_bf16(v, 0.f);
    const float rr = v - lo_f(h);
    const unsigned m = pk_bf16(rr, 0.f);
    const unsigned l = pk_bf16(rr - lo_f(m), 0.f);
    const long long blk = (ct * (Npad / 16) + n / 16) * 3;
    unsigned short* o = out + blk * (WBLK / 2) + ((c >> 3) * 16 + (n & 15)) * 8 + (c & 7);
    o[0] = (unsigned short)h;
    o[WBLK / 2] = (unsigned short)m;
    o[WBLK] = (unsigned short)l;
  }
}

// The two-plane fp16 image (split_bf16.h put_h16x4 arithmetic) of the same weights: per (chunk, tap) step and 16-column
// group two 1 KB blocks [h | l], lane-major as k_wsplit's. Each output column n is scaled by its own power of two s_n
// (max over the column's taps and channels of |w| s_n in [128, 256): a column far below the tensor's largest -- a dead
// or near-dead weight-norm channel -- keeps its full 22 significand bits instead of sinking into fp16's subnormals), the
// activations by 2^-4 (inputs up to 2^20 stay finite). The image's tail holds inv[Npad] = 1 / (s_n 2^-4), which the
// kernels' epilogues multiply back in per column (exact powers of two), then the columns' max |w| bits (build scratch).
constexpr int WROW_H = 2 * PLANE;  // bytes of one (chunk, tap, column) row of the fp16 image
// max |w| of each column (one wave per column; columns >= N get 0) into colmax[Npad]
__global__ void k_wmax_col(const float* __restrict__ w, int ldw, long long w_ts, int N, int C_in, int taps, int Npad,
                           unsigned* __restrict__ colmax) {
  const int n = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= Npad) return;
  float m = 0.f;
  if (n < N)
    for (int tap = 0; tap < taps; ++tap)
      for (int c = lane; c < C_in; c += 64) m = fmaxf(m, fabsf(w[tap * w_ts + (long long)n * ldw + c]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if (lane == 0) colmax[n] = __float_as_uint(m);
}
__global__ void k_wsplit_h16(const float* __restrict__ w, int ldw, long long w_ts, int N, int C_in, int taps,
                             int nchunks, int Npad, unsigned short* __restrict__ out, float* __restrict__ tail) {
  const unsigned* colmax = reinterpret_cast<const unsigned*>(tail) + Npad;
  const long long total = (long long)nchunks * taps * Npad * EK;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % EK);
    const long long r = i / EK;
    const int n = (int)(r % Npad);
    const long long ct = r / Npad;
    const int tap = (int)(ct % taps), ch = (int)(ct / taps);
    const int cc = ch * EK + c;
    const float sc = h16_weight_scale(colmax[n]);
    if (ct == 0 && c == 0) tail[n] = 1.f / (sc * H16_XS);
    const float v = (n < N && cc < C_in) ? w[tap * w_ts + (long long)n * ldw + cc] * sc : 0.f;
    const unsigned h = pk_f16(v, 0.f);
    const unsigned l = pk_f16((v - f16lo_f(h)) * H16_LO, 0.f);
    const long long blk = (ct * (Npad / 16) + n / 16) * 2;
    unsigned short* o = out + blk * (WBLK / 2) + ((c >> 3) * 16 + (n & 15)) * 8 + (c & 7);
    o[0] = (unsigned short)h;
    o[WBLK / 2] = (unsigned short)l;
  }
}

// ---- the contraction on v_mfma_f32_16x16x32 (1-D). One MFMA covers a whole 32-channel chunk (lane group g = lane / 16
// holds channels 8g..8g+7 of its row / column), so a (chunk, tap) step is, per wave of TM16 x TN16 16x16 tiles,
// NQ*TM16 LDS reads, NQ*TN16 global B loads and 3 (fp16) or 6 (bf16) x TM16*TN16 MFMAs of 16 cycles. The chip holds a
// higher clock on this shape than on 32x32x16 under power-limited load (MI355X_MICROARCH.md "DVFS give-back" item 7):
// a 32x32x16 form of the fp16 kernel (round 6, same tile and image) measured slower on every generator shape (C128 k11
// 352 vs 380 TF, k7 317 vs 340, C2 +0.2 ms; profiles/r06a_bench_conv_wsb32h.txt) although an MFMA of it blocks vector
// issue for 8 of 32 cycles instead of 8 of 16.
// The MFMA runs D = W X^T (weight fragment as the A operand): lane l of a 16x16 tile holds row (time) l % 16, columns
// (output channels) 4 (l / 16) + r, r = 0..3, so the epilogue (store_tile16t) moves 16 B per lane (a [time][channel]
// D held one float per lane and store: C128 k7 / k11 and C64 k11 ... r06 A/B in profiles/r06t_ab_wst.txt).
// MODE: bits 0-1 the pre-activation (pre_fn), bit 2 a pre-mask row multiplier (conv_gs.hip's MODE), bit 4 the
// two-plane fp16 arithmetic (split_bf16.h put_h16x4; weights from the k_wsplit_h16 image), bit 3 (with bit 4) the
// opt-in reduced precision: the fp16 hi planes' product alone. The weight image comes from k_wsplit (bf16) or
// k_wsplit_h16 (fp16); only the activation halo goes through LDS (split once per 32-channel chunk, reused by every tap)
template <int BM, int BN, int WM, int WN, int MODE>
__global__ __launch_bounds__(CONV_THREADS, (BM / WM) * (BN / WN) > 64 * 32 ? 2 : 3) void conv_wsb16_kernel(const ConvArgs a, const char* __restrict__ wsp,
                                                                     const int Npad, const int nrows_a, const int ntn,
                                                                     const int ksplit) {
  constexpr int NT = CONV_THREADS;
  constexpr int PA = MODE & 3;
  constexpr bool PMASK = (MODE & 4) != 0;
  constexpr bool H16 = (MODE & 16) != 0;
  constexpr bool LOWP = H16 && (MODE & 8) != 0;
  constexpr int NQ = LOWP ? 1 : (H16 ? 2 : 3);  // planes an MFMA step reads
  constexpr int NQI = H16 ? 2 : 3;               // planes of the weight image
  constexpr int RS = H16 ? ERS_H : ERS;          // LDS row stride
  constexpr int TM16 = BM / (WM * 16);
  constexpr int TN16 = BN / (WN * 16);
  static_assert(WM * WN == 4 && TM16 >= 1 && TN16 >= 1, "4 waves, whole 16x16 sub-tiles");
  extern __shared__ __attribute__((aligned(16))) char smem_w16[];
  char* const As = smem_w16;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lc = lane & 15, lg = lane >> 4;
  int bx, by, bz;
  conv_block_coords(ntn, bx, by, bz);
  const int zsplit = bz % ksplit;
  const int b = bz / ksplit;
  const int n0 = by * BN;
  const int m0 = bx * BM;
  const float* X = a.x + (long long)b * a.x_bs;
  const float* PM = PMASK ? a.pre_mask + (long long)b * a.pre_mask_bs : nullptr;
  const int row0 = m0 - a.pad;

  int aoff[TM16];
#pragma unroll
  for (int tm = 0; tm < TM16; ++tm) aoff[tm] = (wm * TM16 * 16 + tm * 16 + lc) * RS + lg * 16;
  const char* bp[TN16];  // lane l reads 16-B slot l of each block: one contiguous 1 KB per wave load
#pragma unroll
  for (int tn = 0; tn < TN16; ++tn)
    bp[tn] = wsp + (size_t)((n0 + wn * TN16 * 16 + tn * 16) >> 4) * (NQI * WBLK) + lane * 16;
  const size_t bstep = (size_t)Npad * NQI * PLANE;

  f32x4 acc[TM16][TN16], acc2[H16 && !LOWP ? TM16 : 1][H16 && !LOWP ? TN16 : 1];
#pragma unroll
  for (int tm = 0; tm < TM16; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN16; ++tn) {
      acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (H16 && !LOWP) acc2[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

  constexpr int AP = ((BM + WSB_HALO) * EC4 + NT - 1) / NT;
  f32x4 apre[AP];
  float apm[AP];
  unsigned aok = 0u;  // branch-free prefetch: rows outside the input read row 0 and are zeroed when split into LDS
  const int arow = store_row(tid / EC4), ac4 = (tid % EC4) << 2;
  auto load_a_regs = [&](int c0) __attribute__((always_inline)) {
    const float* src0 = X + c0 + ac4;
    aok = 0u;
#pragma unroll
    for (int v = 0; v < AP; ++v) {
      const int r = v * (NT / EC4) + arow;
      const long long g = row0 + r;
      const bool ok = r < nrows_a && g >= 0 && g < a.T_in;
      const long long gc = ok ? g : 0;
      apre[v] = *reinterpret_cast<const f32x4*>(src0 + gc * a.ldx);
      if constexpr (PMASK) apm[v] = PM[gc];
      aok |= ok ? (1u << v) : 0u;
    }
  };
  auto write_a_regs = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int v = 0; v < AP; ++v) {
      const int r = v * (NT / EC4) + arow;
      if (r < nrows_a) {
        f32x4 val = apre[v];
        const bool ok = (aok >> v) & 1u;
#pragma unroll
        for (int j = 0; j < 4; ++j) val[j] = pre_fn<PA>(val[j], a.pre_act, a.pre_slope);
        if constexpr (PMASK) {
#pragma unroll
          for (int j = 0; j < 4; ++j) val[j] = ok ? val[j] * apm[v] : 0.f;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) val[j] = ok ? val[j] : 0.f;
        }
        if constexpr (H16) {
#pragma unroll
          for (int j = 0; j < 4; ++j) val[j] *= H16_XS;
          put_h16x4<NQ>(As + r * RS, ac4, val);
        } else {
          put_split4(As + r * RS, ac4, val);
        }
      }
    }
  };
  typedef bf16x8 BFrag[TN16][NQ];
  auto load_b = [&](int it, BFrag& dst) __attribute__((always_inline)) {
    const size_t o = (size_t)it * bstep;
#pragma unroll
    for (int tn = 0; tn < TN16; ++tn)
#pragma unroll
      for (int q = 0; q < NQ; ++q) dst[tn][q] = *reinterpret_cast<const bf16x8*>(bp[tn] + o + q * WBLK);
  };
  auto compute = [&](int tap, const BFrag& bf) __attribute__((always_inline)) {
    const int toff = tap * a.dil * RS;
#pragma unroll
    for (int tm = 0; tm < TM16; ++tm) {
      bf16x8 af[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) af[q] = *reinterpret_cast<const bf16x8*>(As + aoff[tm] + toff + q * PLANE);
      if constexpr (H16) {
        const f16x8 ah = __builtin_bit_cast(f16x8, af[0]);
#pragma unroll
        for (int tn = 0; tn < TN16; ++tn) {
          const f16x8 bh = __builtin_bit_cast(f16x8, bf[tn][0]);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh, ah, acc[tm][tn], 0, 0, 0);
          if constexpr (!LOWP) {
            f32x4 c = acc2[tm][tn];
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh, __builtin_bit_cast(f16x8, af[NQ - 1]), c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, bf[tn][NQ - 1]), ah, c, 0, 0, 0);
            acc2[tm][tn] = c;
          }
        }
        continue;
      }
#pragma unroll
      for (int tn = 0; tn < TN16; ++tn) {
        f32x4 c = acc[tm][tn];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[tn][0], af[NQ - 1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[tn][NQ / 2], af[NQ / 2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[tn][NQ - 1], af[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[tn][0], af[NQ / 2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[tn][NQ / 2], af[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[tn][0], af[0], c, 0, 0, 0);
        acc[tm][tn] = c;
      }
    }
  };

  const int taps = a.taps, total = (a.C_in / EK) * taps;
  const int per = (total + ksplit - 1) / ksplit;
  const int it0 = zsplit * per, it1 = min(total, it0 + per);
  if (it0 < it1) {
    BFrag b0, b1;
    int ch = it0 / taps, tap = it0 - ch * taps;
    load_a_regs(ch * EK);
    write_a_regs();
    if ((ch + 1) * taps < it1) load_a_regs((ch + 1) * EK);
    load_b(it0, b0);
    __syncthreads();
    auto step = [&](int it, const BFrag& cur, BFrag& nxt) __attribute__((always_inline)) {
      // unconditional (the last step reloads its own fragments): with a conditional load the waitcnt pass merges the
      // load-issued and load-skipped paths and waits for the prefetch itself inside this step; the scheduling barrier
      // keeps the loads at the top of the step (the machine scheduler otherwise sinks them below the MFMAs, so the
      // next step waits out their whole latency)
      load_b(it + 1 < it1 ? it + 1 : it, nxt);
      __builtin_amdgcn_sched_barrier(0);
      compute(tap, cur);
      if (++tap == taps) {
        tap = 0;
        if (++ch * taps < it1) {
          __syncthreads();
          write_a_regs();
          if ((ch + 1) * taps < it1) load_a_regs((ch + 1) * EK);
          __syncthreads();
        }
      }
    };
    for (int it = it0; it < it1; it += 2) {
      step(it, b0, b1);
      if (it + 1 < it1) step(it + 1, b1, b0);
    }
  }
  if constexpr (H16) {
    // acc + 2^-11 acc2, times 1 / (column weight scale x activation scale) from the image tail: exact powers of two
    // (the image's padded columns carry scales too, so the 4-column vector is always in bounds)
    const float* inv = reinterpret_cast<const float*>(wsp + (size_t)total * bstep) + n0 + wn * TN16 * 16 + 4 * lg;
#pragma unroll
    for (int tn = 0; tn < TN16; ++tn) {
      const f32x4 iv = *reinterpret_cast<const f32x4*>(inv + tn * 16);
#pragma unroll
      for (int tm = 0; tm < TM16; ++tm)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[tm][tn][r];
          if constexpr (!LOWP) v += acc2[tm][tn][r] * H16_LO_INV;
          acc[tm][tn][r] = v * iv[r];
        }
    }
  }
  store_tile16t<TM16, TN16, WM, WN>(a, m0, n0, b, zsplit, ksplit, (long long)a.T_out, acc);
}

template <int BM, int BN, int WM, int WN>
hipError_t launch_wsb16(const ConvArgs& a, int ntn_enable, int ksplit, hipStream_t s) {
  const int nrows_a = BM + (a.taps - 1) * a.dil;
  const int mtiles = (a.T_out + BM - 1) / BM;
  const bool h16 = a.wsplit_fmt == WSPLIT_H16;
  const size_t smem = (size_t)nrows_a * (h16 ? ERS_H : ERS);
  if (a.wsplit_npad % BN != 0 || ksplit < 1 || (ksplit > 1 && !a.ws)) return hipErrorInvalidValue;
  if (a.lowp && !h16) return hipErrorInvalidValue;  // the reduced-precision mode reads the fp16 image's hi plane
  const int ntiles = (a.N + BN - 1) / BN;
  const int ntn = ntn_enable ? ntiles : 0;
  dim3 grid(ntn ? mtiles * ntiles : mtiles, ntn ? 1 : ntiles, a.batch * ksplit);
  // the reduced-precision opt-in only without a pre-mask (the generator's convs)
  const int mode = pre_mode(a.pre_act) | (a.pre_mask ? 4 : 0) | (h16 ? 16 : 0) | (h16 && a.lowp && !a.pre_mask ? 8 : 0);
  void (*kern)(const ConvArgs, const char*, int, int, int, int);
  switch (mode) {
#define WSB16_CASE(M) \
  case M: kern = conv_wsb16_kernel<BM, BN, WM, WN, M>; break;
    WSB16_CASE(0) WSB16_CASE(1) WSB16_CASE(2) WSB16_CASE(4) WSB16_CASE(5) WSB16_CASE(6)
    WSB16_CASE(16) WSB16_CASE(17) WSB16_CASE(18) WSB16_CASE(20) WSB16_CASE(21) WSB16_CASE(22)
    WSB16_CASE(24) WSB16_CASE(25) WSB16_CASE(26)
#undef WSB16_CASE
    default: return hipErrorInvalidValue;
  }
  // per instantiation: raise the dynamic-LDS limit once, not per launch
  static size_t smem_set[32] = {};
  if (smem > 64 * 1024 && smem > smem_set[mode & 31]) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    smem_set[mode & 31] = smem;
  }
  hipLaunchKernelGGL(kern, grid, dim3(CONV_THREADS), smem, s, a, static_cast<const char*>(a.wsplit), a.wsplit_npad,
                     nrows_a, ntn, ksplit);
  return hipGetLastError();
}

}  // namespace

bool conv_wsb_eligible(const ConvArgs& a, bool two_d) {
  const bool vec_a = ((a.ldx & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.x) & 15) == 0) && ((a.x_bs & 3) == 0);
  return !two_d && a.batch_inner == 1 && !a.b_kn && a.C_in % EK == 0 && a.C_in > 0 && a.taps >= 1 && vec_a &&
         a.out_map == OUT_ROWS && a.stride == 1 && (a.taps - 1) * a.dil <= WSB_HALO && a.dil >= 1;
}

int conv_wsplit_npad(int N) { return (N + 127) / 128 * 128; }

// chunks of 32 input channels, the last one zero-padded; the fp16 image carries a tail of 2 x Npad words (the columns'
// inverse scales, then their max |w| bits)
long long conv_wsplit_bytes(const ConvArgs& a) {
  if (a.wsplit_fmt == WSPLIT_S2D) return small2d_wsplit_bytes(a);
  const long long steps = (long long)((a.C_in + EK - 1) / EK) * a.taps * conv_wsplit_npad(a.N);
  return a.wsplit_fmt == WSPLIT_H16 ? steps * WROW_H + 8LL * conv_wsplit_npad(a.N) : steps * WROW;
}

hipError_t conv_wsplit_build(const ConvArgs& a, void* out, hipStream_t s) {
  if (a.wsplit_fmt == WSPLIT_S2D) return small2d_wsplit_build(a, out, s);
  const int nch = (a.C_in + EK - 1) / EK, Npad = conv_wsplit_npad(a.N);
  if (nch < 1 || a.taps < 1 || a.N < 1) return hipErrorInvalidValue;
  const long long total = (long long)nch * a.taps * Npad * EK;
  const long long nb = std::min<long long>((total + 255) / 256, 1 << 20);
  if (a.wsplit_fmt == WSPLIT_H16) {
    float* tail = reinterpret_cast<float*>(static_cast<char*>(out) + (long long)nch * a.taps * Npad * WROW_H);
    hipLaunchKernelGGL(k_wmax_col, dim3((unsigned)(Npad / 4)), dim3(256), 0, s, a.w, a.ldw, a.w_ts, a.N, a.C_in, a.taps,
                       Npad, reinterpret_cast<unsigned*>(tail) + Npad);
    hipLaunchKernelGGL(k_wsplit_h16, dim3((unsigned)nb), dim3(256), 0, s, a.w, a.ldw, a.w_ts, a.N, a.C_in, a.taps, nch,
                       Npad, static_cast<unsigned short*>(out), tail);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_wsplit, dim3((unsigned)nb), dim3(256), 0, s, a.w, a.ldw, a.w_ts, a.N, a.C_in, a.taps, nch, Npad,
                     static_cast<unsigned short*>(out));
  return hipGetLastError();
}

// cfg 23: 128 x 64 as 2 x 2 waves of 64 x 32, 24: 256 x 32 as 4 x 1 waves of 64 x 32 (N <= 32), 25: 128 x 128 as
// 2 x 2 waves of 64 x 64 (round 6: the 128-channel k = 7 / 11 convs, C128 k11 402 vs 380 TF, k7 346 vs 340 in
// bench_conv r06a; C2 -0.05 to -0.1 ms same box), 27: 128 x 64 as 1 x 4 waves of 128 x 16 (k <= 3). The 32x32x16
// bf16 kernel of rounds 2-3 (cfg 20-22), 256 x 64 tiles (26, 28) and a 32x32x16 fp16 form (r06a) measured slower and
// are gone. A persistent form of the kernel (contiguous tile runs per workgroup, A halos and B prefetched across tile
// boundaries) measured slower on every shape (bench_conv r03k: C128 k3 118 vs 129 TF, k11 198 vs 219, up-phases 88-111
// vs 97-128): three independent one-tile workgroups per CU already overlap each other's prologue and epilogue
bool conv_wsb_tile(int cfg, int& BM, int& BN) {
  switch (cfg) {
    case 23: BM = 128; BN = 64; return true;
    case 24: BM = 256; BN = 32; return true;
    case 25: BM = 128; BN = 128; return true;
    case 27: BM = 128; BN = 64; return true;
    default: return false;
  }
}

hipError_t conv_wsb_launch(const ConvArgs& a, int cfg, int ntn_enable, hipStream_t s, bool two_d, int ksplit) {
  if (!a.wsplit || !conv_wsb_eligible(a, two_d)) return hipErrorInvalidValue;
  switch (cfg) {
    case 23: return launch_wsb16<128, 64, 2, 2>(a, ntn_enable, ksplit, s);
    case 24: return launch_wsb16<256, 32, 4, 1>(a, ntn_enable, ksplit, s);
    case 25: return launch_wsb16<128, 128, 2, 2>(a, ntn_enable, ksplit, s);
    case 27: return launch_wsb16<128, 64, 1, 4>(a, ntn_enable, ksplit, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace rvcx
