// One ResBlock dilation pair of the HiFi-GAN generators as ONE kernel (residuals.py:71-80, ResBlock.forward;
// hifigan_mrf.py:45-50, MRFLayer.forward):
//     t   = lrelu(conv1_d(lrelu(x)) + b1)          (k taps, dilation d, zero padding)
//     out = conv2(t) + b2 + x                      (k taps, dilation 1, zero padding)
//     y   = out | y + out | (y + out) / div        (the ResBlock mean of hifigan_nsf.py:190-207 on the last pair)
// The intermediate t never leaves the CU: a workgroup loads its x tile (+ both convs' halo) once, splits lrelu(x)
// into bf16 planes in LDS, runs conv1 into a second LDS image of t and conv2 out of it, and writes only the pair's
// output. Per pair that is one read and one write of the [T][C] activation instead of five passes (x, t written,
// t read, x re-read as the residual, out), and one launch instead of two latency-bound ones at 32/64 channels.
//
// Arithmetic (FMT): the exact 3-plane bf16 split of conv_emu.hip (x = x0 + x1 + x2, six plane products with i + j <= 2
// summed smallest first into one fp32 accumulator per output); or the two-plane fp16 split of split_bf16.h
// (put_h16x4: three products into two accumulators, weights and activations scaled by powers of two); or its hi plane
// alone (the realtime hop's reduced-precision generator, rvcx_rt_opts::gen_precision).
//
// Orientation: D[out channel][time] = W[out ch][in ch] * X^T[in ch][time] on v_mfma_f32_32x32x16_bf16, so a lane
// of the accumulator holds 16 output channels of ONE time step. Inside each 16-channel chunk the contraction slots
// are permuted (slot j <-> channel rb_pi(j), bits 2 and 3 swapped) so those 16 registers are exactly two chunks'
// worth of 8 consecutive slots: conv1's epilogue writes its t image with 16-byte LDS stores (6 per 32x32 tile),
// already in conv2's B-fragment layout. Weights are pre-split once into the same slot order, per lane one 16-byte
// A fragment per (tap, chunk, plane), loaded from L1/L2 one step ahead.
#include <algorithm>

#include "conv_common.h"
#include "split_bf16.h"

namespace rvcx {

namespace {

using namespace splitbf16;

constexpr int RB_THREADS = 256;
constexpr int RB_MAXH1 = 30;  // conv1 halo rows per side supported: (k - 1) / 2 * d

__host__ __device__ constexpr int rb_pi(int j) { return (j & 3) | (((j >> 3) & 1) << 2) | (((j >> 2) & 1) << 3); }

// activation / weight formats: planes per value and element type
enum RbFmt : int { RB_BF16X3 = 0, RB_F16X2 = 1, RB_F16X1 = 2 };
__host__ __device__ constexpr int rb_planes(int fmt) { return fmt == RB_BF16X3 ? 3 : (fmt == RB_F16X2 ? 2 : 1); }

template <int C, int FMT = RB_BF16X3>
struct RbGeo {
  static constexpr int NCH = C / 16;                           // 16-channel contraction chunks
  static constexpr int NP = rb_planes(FMT);
  static constexpr int ROW = NCH * NP * 32 + 16;  // LDS bytes per time row: [chunk][plane][16 slots] + pad
};

// w [tap][C_out][C_in] fp32 -> ((tap * NCH + s) * 3 + q) planes of [C_out][16 slots] bf16, slot j = channel
// 16 s + rb_pi(j) (put_split1's arithmetic)
__global__ void k_rb_wsplit(const float* __restrict__ w, int C, int k, unsigned short* __restrict__ out) {
  const int NCH = C / 16;
  const long long total = (long long)k * NCH * C * 16;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(i & 15);
    long long r = i >> 4;
    const int och = (int)(r % C);
    r /= C;
    const int s = (int)(r % NCH), tap = (int)(r / NCH);
    const float v = w[((long long)tap * C + och) * C + 16 * s + rb_pi(j)];
    const unsigned h = pk_bf16(v, 0.f);
    const float rr = v - lo_f(h);
    const unsigned m = pk_bf16(rr, 0.f);
    const unsigned l = pk_bf16(rr - lo_f(m), 0.f);
    const long long base = (((long long)(tap * NCH + s) * 3) * C + och) * 16 + j;
    out[base] = (unsigned short)h;
    out[base + (long long)C * 16] = (unsigned short)m;
    out[base + 2LL * C * 16] = (unsigned short)l;
  }
}

// the fp16 images: ((tap * NCH + s) * NP + q) planes of [C_out][16 slots] fp16 (q = 0 hi, 1 the 2^11-scaled residual:
// put_h16x4's arithmetic) of w * sc_o, sc_o a power of two per OUTPUT CHANNEL with max |w[., o, .]| sc_o in [128, 256)
// (conv_wsb.hip k_wsplit_h16's rule); the image's tail (after the planes) holds inv[C] = 1 / (sc_o * RB_XS), then the
// channels' max |w| bits (build scratch). Activations are split at RB_XS = 2^-4.
constexpr float RB_XS = 1.f / 16.f;
// one wave per output channel o: max over taps and input channels of |w[tap][o][c]|
__global__ void k_rb_wmax(const float* __restrict__ w, int C, int k, unsigned* __restrict__ chmax) {
  const int o = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (o >= C) return;
  float m = 0.f;
  for (int tap = 0; tap < k; ++tap)
    for (int c = lane; c < C; c += 64) m = fmaxf(m, fabsf(w[((long long)tap * C + o) * C + c]));
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if (lane == 0) chmax[o] = __float_as_uint(m);
}
__global__ void k_rb_wsplit_h16(const float* __restrict__ w, int C, int k, int NP, unsigned short* __restrict__ out,
                                float* __restrict__ tail) {
  const unsigned* chmax = reinterpret_cast<const unsigned*>(tail) + C;
  const int NCH = C / 16;
  const long long total = (long long)k * NCH * C * 16;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(i & 15);
    long long r = i >> 4;
    const int och = (int)(r % C);
    r /= C;
    const int s = (int)(r % NCH), tap = (int)(r / NCH);
    const float sc = h16_weight_scale(chmax[och]);
    if (r == 0 && j == 0) tail[och] = 1.f / (sc * RB_XS);
    const float v = w[((long long)tap * C + och) * C + 16 * s + rb_pi(j)] * sc;
    const unsigned h = pk_f16(v, 0.f);
    const long long base = (((long long)(tap * NCH + s) * NP) * C + och) * 16 + j;
    out[base] = (unsigned short)h;
    if (NP > 1) out[base + (long long)C * 16] = (unsigned short)pk_f16((v - f16lo_f(h)) * H16_LO, 0.f);
  }
}

// 8 fp32 values -> three 16-byte planes (hi, mid, lo)
__device__ __forceinline__ void split8(const float (&v)[8], uint4& h, uint4& m, uint4& l) {
  unsigned hh[4], mm[4], ll[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    hh[p] = pk_bf16(v[2 * p], v[2 * p + 1]);
    float r0 = v[2 * p] - lo_f(hh[p]), r1 = v[2 * p + 1] - hi_f(hh[p]);
    mm[p] = pk_bf16(r0, r1);
    r0 -= lo_f(mm[p]);
    r1 -= hi_f(mm[p]);
    ll[p] = pk_bf16(r0, r1);
  }
  h = make_uint4(hh[0], hh[1], hh[2], hh[3]);
  m = make_uint4(mm[0], mm[1], mm[2], mm[3]);
  l = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}

// 8 fp32 values (already scaled by RB_XS) -> the fp16 hi plane and the 2^11-scaled residual plane
__device__ __forceinline__ void split8_h16(const float (&v)[8], uint4& h, uint4& l) {
  unsigned hh[4], ll[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    hh[p] = pk_f16(v[2 * p], v[2 * p + 1]);
    ll[p] = pk_f16((v[2 * p] - f16lo_f(hh[p])) * H16_LO, (v[2 * p + 1] - f16hi_f(hh[p])) * H16_LO);
  }
  h = make_uint4(hh[0], hh[1], hh[2], hh[3]);
  l = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}

__device__ __forceinline__ float lrelu01(float v) { return v > 0.f ? v : v * 0.1f; }

// C channels, NBT 32-row time blocks per workgroup tile, TN time blocks per wave unit, ACCM the output's accumulate
// mode (ACC_STORE / ACC_ADD / ACC_ADD_DIV: compile-time, so the accumulate target's loads are not a uniform branch
// whose join would cost the weight ring its depth)
// MODE: bits 0-1 the accumulate mode ACCM; bits 2-3 the arithmetic FMT (RbFmt: the exact bf16 split, the two-plane
// fp16 split, or the realtime hop's reduced-precision fp16 hi planes)
template <int C, int NBT, int TN, int MODE>
__global__ __launch_bounds__(RB_THREADS, 3) void k_rb_pair(const RbPairArgs a, const int ntiles) {
  constexpr int ACCM = MODE & 3;
  constexpr int FMT = (MODE >> 2) & 3;
  constexpr bool H16 = FMT != RB_BF16X3;
  constexpr int NQ = rb_planes(FMT);              // planes of the activations in LDS and of an MFMA step
  constexpr int NQI = H16 ? 2 : 3;               // planes of the weight image (the fp16 image always holds two)
  constexpr int CB = NQ * 32;  // LDS bytes of one 16-channel chunk of a row
  constexpr int NCH = RbGeo<C, FMT>::NCH, ROW = RbGeo<C, FMT>::ROW, OB = C / 32;
  constexpr int UNITS = OB * NBT / TN;  // wave work units per conv: (out-channel block, TN time blocks)
  static_assert(UNITS % 4 == 0, "whole units per wave");
  constexpr int UPW = UNITS / 4;
  constexpr int C4 = C / 4;
  constexpr int XROWS_MAX = NBT * 32 + 2 * RB_MAXH1;
  constexpr int XITER = (XROWS_MAX * C4 + RB_THREADS - 1) / RB_THREADS;
  extern __shared__ __attribute__((aligned(16))) char rb_smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, hk = lane >> 5;
  const int k = a.k, h2 = (k - 1) / 2, h1 = h2 * a.d;
  const int nx = NBT * 32 + 2 * h1;  // XS rows: conv1 inputs
  const int TT = NBT * 32 - 2 * h2;  // valid outputs per tile
  char* const XS = rb_smem;
  char* const TS = rb_smem + (size_t)nx * ROW;
  // persistent: workgroup g takes a contiguous run of the B * ntiles (batch-major) tiles; the next tile's x is
  // loaded into registers while the current one computes
  const int total = ntiles * a.B;

  // ---- the wave's jobs: UPW conv1 units, then UPW conv2 units. A unit is one 32-channel output block x TN time
  // blocks; one (tap, chunk) step of it is 3 A fragments (weights, global/L2, two steps ahead), 3 * TN B fragments
  // (LDS, one step ahead) and 6 * TN MFMAs.
  constexpr size_t QS = (size_t)C * 32;  // bytes of one plane of one (tap, chunk) step of the weight image
  typedef bf16x8 AFrag[NQ];
  typedef bf16x8 BFrag[TN][NQ];
  const int nsteps = k * NCH;
  auto unit_ob = [&](int job) { return (wave + 4 * (job % UPW)) % OB; };
  auto unit_tg = [&](int job) { return (wave + 4 * (job % UPW)) / OB; };
  auto wl_of = [&](int job) {
    const char* w = static_cast<const char*>(job < UPW ? a.w1s : a.w2s);
    return w + (size_t)(unit_ob(job) * 32 + li) * 32 + hk * 16;
  };
  auto load_a = [&](const char* wl, int st, AFrag& f) __attribute__((always_inline)) {
    const char* p = wl + (size_t)st * NQI * QS;
#pragma unroll
    for (int q = 0; q < NQ; ++q) f[q] = *reinterpret_cast<const bf16x8*>(p + q * QS);
  };
  auto load_b = [&](const char* bl, int dil, int st, BFrag& f) __attribute__((always_inline)) {
    const int tap = st / NCH, s = st - tap * NCH;
    const char* bp = bl + (size_t)tap * dil * ROW + s * CB;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int q = 0; q < NQ; ++q) f[tn][q] = *reinterpret_cast<const bf16x8*>(bp + (size_t)tn * 32 * ROW + q * 32);
  };
  typedef _Float16 f16x8_ __attribute__((ext_vector_type(8)));
  auto mma = [&](const AFrag& af, const BFrag& bf, f32x16(&acc)[TN], f32x16(&acc2)[TN]) __attribute__((always_inline)) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      if constexpr (H16) {
        const f16x8_ ah = __builtin_bit_cast(f16x8_, af[0]), bh = __builtin_bit_cast(f16x8_, bf[tn][0]);
        acc[tn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[tn], 0, 0, 0);
        if constexpr (NQ > 1) {
          f32x16 c2 = acc2[tn];
          c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_, af[1]), bh, c2, 0, 0, 0);
          c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, __builtin_bit_cast(f16x8_, bf[tn][1]), c2, 0, 0, 0);
          acc2[tn] = c2;
        }
        continue;
      }
      f32x16 c = acc[tn];
      {
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[NQ - 1], bf[tn][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[NQ / 2], bf[tn][NQ / 2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bf[tn][NQ - 1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[NQ / 2], bf[tn][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bf[tn][NQ / 2], c, 0, 0, 0);
      }
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bf[tn][0], c, 0, 0, 0);
      acc[tn] = c;
    }
  };
  // Weight fragments run a 3-slot register ring two steps ahead, LDS fragments one step ahead (their own 3 slots, so
  // every slot index is compile-time in the 3-fold unrolled loop). Every load is unconditional (indices clamped to
  // the last step: the tail reloads it, harmlessly) and issued at the top of its step, pinned there: a conditional
  // load's join made the waitcnt pass wait for the ring at every step (vmcnt(0) before each MFMA group), and the
  // scheduler sank the loads below the MFMAs.
  AFrag ring[3];
  BFrag bring[3];
  auto run_conv = [&](const char* wl, const char* bl, int dil, f32x16(&acc)[TN], f32x16(&acc2)[TN])
                      __attribute__((always_inline)) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tn][r] = acc2[tn][r] = 0.f;
    const int last = nsteps - 1;
    load_a(wl, 0, ring[0]);
    load_a(wl, 1 < last ? 1 : last, ring[1]);
    load_b(bl, dil, 0, bring[0]);
    auto step = [&](int i, int p) __attribute__((always_inline)) {
      load_a(wl, i + 2 < last ? i + 2 : last, ring[(p + 2) % 3]);
      load_b(bl, dil, i + 1 < last ? i + 1 : last, bring[(p + 1) % 3]);
      __builtin_amdgcn_sched_barrier(0);
      mma(ring[p], bring[p], acc, acc2);
    };
    int cur = 0;
    for (; cur + 3 <= nsteps; cur += 3) {
#pragma unroll
      for (int p = 0; p < 3; ++p) step(cur + p, p);
    }
#pragma unroll
    for (int p = 0; p < 2; ++p)
      if (cur + p < nsteps) step(cur + p, p);
  };

  // ---- x tile -> XS = split(lrelu(x)); row r <-> time t0 - h2 - h1 + r, zero outside [0, T) (conv1's padding)
  f32x4 xv[XITER];
  auto load_x = [&](int tile) __attribute__((always_inline)) {
    const int bb = tile / ntiles, tb = (tile - bb * ntiles) * TT - h2 - h1;
    const float* Xb = a.x + (long long)bb * a.x_bs;
#pragma unroll
    for (int it = 0; it < XITER; ++it) {
      const int i = it * RB_THREADS + tid;
      const int r = i / C4, c4 = (i % C4) * 4;
      const int t = tb + r;
      const bool ok = r < nx && t >= 0 && t < a.T;
      xv[it] = ok ? *reinterpret_cast<const f32x4*>(Xb + (long long)t * C + c4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto write_x = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XITER; ++it) {
      const int i = it * RB_THREADS + tid;
      const int r = i / C4, c4 = (i % C4) * 4;
      if (r < nx) {
        // channels 16 s + 8 p + 4 q + e sit at slots 8 q + 4 p + e
        const int s = c4 >> 4, o = c4 & 15;
        const int slot = ((o >> 2) & 1) * 8 + (o >> 3) * 4;
        char* row = XS + (size_t)r * ROW + s * CB + slot * 2;
        const float x0 = lrelu01(xv[it][0]), x1 = lrelu01(xv[it][1]), x2 = lrelu01(xv[it][2]),
                    x3 = lrelu01(xv[it][3]);
        if constexpr (H16) {
          uint2 hh, ll;
          const float y0 = x0 * RB_XS, y1 = x1 * RB_XS, y2 = x2 * RB_XS, y3 = x3 * RB_XS;
          hh.x = pk_f16(y0, y1);
          hh.y = pk_f16(y2, y3);
          *reinterpret_cast<uint2*>(row) = hh;
          if constexpr (NQ > 1) {
            ll.x = pk_f16((y0 - f16lo_f(hh.x)) * H16_LO, (y1 - f16hi_f(hh.x)) * H16_LO);
            ll.y = pk_f16((y2 - f16lo_f(hh.y)) * H16_LO, (y3 - f16hi_f(hh.y)) * H16_LO);
            *reinterpret_cast<uint2*>(row + 32) = ll;
          }
          continue;
        }
        uint2 hh, mm, ll;
        hh.x = pk_bf16(x0, x1);
        hh.y = pk_bf16(x2, x3);
        float r0 = x0 - lo_f(hh.x), r1 = x1 - hi_f(hh.x), r2 = x2 - lo_f(hh.y), r3 = x3 - hi_f(hh.y);
        mm.x = pk_bf16(r0, r1);
        mm.y = pk_bf16(r2, r3);
        r0 -= lo_f(mm.x);
        r1 -= hi_f(mm.x);
        r2 -= lo_f(mm.y);
        r3 -= hi_f(mm.y);
        ll.x = pk_bf16(r0, r1);
        ll.y = pk_bf16(r2, r3);
        *reinterpret_cast<uint2*>(row) = hh;
        *reinterpret_cast<uint2*>(row + 32) = mm;
        *reinterpret_cast<uint2*>(row + 64) = ll;
      }
    }
  };

  // contiguous runs of tiles per workgroup: the next tile's halo rows were just read by this workgroup (same XCD
  // L2), instead of by a neighbour on another XCD
  const int per = (total + (int)gridDim.x - 1) / (int)gridDim.x;
  int tile = blockIdx.x * per;
  const int tile_end = min(total, tile + per);
  if (tile >= tile_end) return;
  // (a next-tile x prefetch into registers measured slower: contiguous runs find the next tile in L2 already, and the
  // first weight wait after it stalls on the HBM load, A/B 22.30 vs 22.19 ms)
#pragma unroll 1
  for (; tile < tile_end; ++tile) {
  load_x(tile);
  const int b = tile / ntiles;
  const int t0 = (tile - b * ntiles) * TT;
  const float* X = a.x + (long long)b * a.x_bs;
  // XS is dead once every wave passed the previous tile's mid barrier; the barrier below also orders this tile's
  // conv1 (writing TS) after every wave's conv2 of the previous tile (reading TS)
  write_x();
  __syncthreads();
  float* Y = a.y + (long long)b * a.y_bs;
#pragma unroll 1
  for (int job = 0; job < 2 * UPW; ++job) {
    const bool second = job >= UPW;
    if (job == UPW) __syncthreads();  // TS complete (XS dead)
    const int ob = unit_ob(job), tg = unit_tg(job);
    const float* bias = second ? a.b2 : a.b1;
    float bv[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[m][e] = bias[ob * 32 + 8 * m + 4 * hk + e];
    // conv2: the residual (and the accumulate target) of the lane's outputs, loaded before the MFMAs
    f32x4 rv[TN][4], dv[TN][4];
    if (second) {
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int o = (tg * TN + tn) * 32 + li;
        const int t = t0 + o;
        const bool ok = o < TT && t < a.T;
        const long long off = (long long)(ok ? t : 0) * C + ob * 32 + 4 * hk;
#pragma unroll
        for (int m = 0; m < 4; ++m) {  // branch-free: rows past the tile read row 0 (their results are not stored)
          rv[tn][m] = *reinterpret_cast<const f32x4*>(X + off + 8 * m);
          if constexpr (ACCM != ACC_STORE) dv[tn][m] = *reinterpret_cast<const f32x4*>(Y + off + 8 * m);
        }
      }
    }
    f32x16 acc[TN], acc2[TN];
    run_conv(wl_of(job), (second ? TS : XS) + (size_t)(tg * TN * 32 + li) * ROW + hk * 16, second ? 1 : a.d, acc, acc2);
    if constexpr (H16) {
      // acc + 2^-11 acc2, times 1 / (output-channel weight scale x activation scale) from the weight image's tail:
      // accumulator element r is output channel ob * 32 + 8 (r / 4) + 4 hk + r % 4 (the bias layout above)
      const float* invp = reinterpret_cast<const float*>(static_cast<const char*>(second ? a.w2s : a.w1s) +
                                                         (size_t)nsteps * NQI * QS) + ob * 32 + 4 * hk;
      f32x4 inv[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) inv[m] = *reinterpret_cast<const f32x4*>(invp + 8 * m);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          acc[tn][r] = (NQ > 1 ? acc[tn][r] + acc2[tn][r] * H16_LO_INV : acc[tn][r]) * inv[r >> 2][r & 3];
    }
    if (!second) {
      // conv1 -> TS = split(lrelu(conv1 + b1)); TS row p <-> time t0 - h2 + p, zero outside [0, T)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int p = (tg * TN + tn) * 32 + li;
        const int t = t0 - h2 + p;
        const bool ok = t >= 0 && t < a.T;
        char* row = TS + (size_t)p * ROW + hk * 16;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          float v[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int r = 8 * hh + i;
            const float x = lrelu01(acc[tn][r] + bv[r >> 2][r & 3]);
            v[i] = ok ? (H16 ? x * RB_XS : x) : 0.f;
          }
          char* dst = row + (2 * ob + hh) * CB;
          if constexpr (H16) {
            uint4 Hh, Ll;
            split8_h16(v, Hh, Ll);
            *reinterpret_cast<uint4*>(dst) = Hh;
            if constexpr (NQ > 1) *reinterpret_cast<uint4*>(dst + 32) = Ll;
          } else {
            uint4 H, M, L;
            split8(v, H, M, L);
            *reinterpret_cast<uint4*>(dst) = H;
            *reinterpret_cast<uint4*>(dst + 32) = M;
            *reinterpret_cast<uint4*>(dst + 64) = L;
          }
        }
      }
    } else {
      // conv2 + b2 + x -> y (acc mode); output row o <-> time t0 + o, valid for o < TT, t < T
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int o = (tg * TN + tn) * 32 + li;
        const int t = t0 + o;
        if (o < TT && t < a.T) {
          const long long off = (long long)t * C + ob * 32 + 4 * hk;
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            f32x4 o4;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float v = acc[tn][4 * m + e] + bv[m][e];
              v = v + rv[tn][m][e];
              if constexpr (ACCM == ACC_ADD) v = dv[tn][m][e] + v;
              else if constexpr (ACCM == ACC_ADD_DIV) v = (dv[tn][m][e] + v) / a.acc_div;
              o4[e] = v;
            }
            *reinterpret_cast<f32x4*>(Y + off + 8 * m) = o4;
          }
        }
      }
    }
  }
  }  // tiles
}

// The k = 3 pairs at 32 channels in the two-plane fp16 split (the 32-channel stage's first ResBlock, residuals.py:71-80
// with d = 1, 3, 5): both convs' images -- 3 taps x 2 chunks x 2 planes, one 16-byte A fragment each per lane, 96
// VGPRs -- are loaded into registers once per persistent workgroup, so the conv loops issue no global loads and the
// next tile's x rows are prefetched into registers across both convs (in the streamed-weight form such a prefetch
// stalled the first weight wait behind its HBM latency: vmcnt retires in issue order). Biases and inverse weight
// scales sit in LDS. Same tile (128 rows, 126 outputs), the same MFMA sequence and epilogue order as k_rb_pair: the
// results are bit-identical to it (tests/test_gpu_resblock_fused.py::test_k3_pair_matches_streamed_form).
template <int ACCM>
__global__ __launch_bounds__(RB_THREADS, 2) void k_rb_pair3(const RbPairArgs a, const int ntiles) {
  constexpr int C = 32, NBT = 4, NCH = 2, NQ = 2, CB = NQ * 32, ROW = RbGeo<C, RB_F16X2>::ROW, NST = 3 * NCH;
  constexpr int C4 = C / 4;
  constexpr int XITER = ((NBT * 32 + 2 * RB_MAXH1) * C4 + RB_THREADS - 1) / RB_THREADS;
  constexpr size_t QS = (size_t)C * 32;
  typedef _Float16 f16x8_ __attribute__((ext_vector_type(8)));
  extern __shared__ __attribute__((aligned(16))) char rb_smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, hk = lane >> 5;
  const int h1 = a.d;  // conv1 halo (k = 3); conv2's is 1
  const int nx = NBT * 32 + 2 * h1;
  constexpr int TT = NBT * 32 - 2;
  char* const XS = rb_smem;
  char* const TS = rb_smem + (size_t)nx * ROW;
  float* const prm = reinterpret_cast<float*>(TS + (size_t)(NBT * 32 + 2) * ROW);  // b1, inv1, b2, inv2
  const int total = ntiles * a.B;
  const int per = (total + (int)gridDim.x - 1) / (int)gridDim.x;
  int tile = blockIdx.x * per;
  const int tile_end = min(total, tile + per);
  if (tile >= tile_end) return;

  // ---- once: the weight fragments (A operand: out channel li, slots hk * 8 ..) and the per-channel constants
  f16x8_ w1r[NST][NQ], w2r[NST][NQ];
  {
    const char* p1 = static_cast<const char*>(a.w1s) + (size_t)li * 32 + hk * 16;
    const char* p2 = static_cast<const char*>(a.w2s) + (size_t)li * 32 + hk * 16;
#pragma unroll
    for (int st = 0; st < NST; ++st)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        w1r[st][q] = *reinterpret_cast<const f16x8_*>(p1 + (size_t)st * 2 * QS + q * QS);
        w2r[st][q] = *reinterpret_cast<const f16x8_*>(p2 + (size_t)st * 2 * QS + q * QS);
      }
  }
  if (tid < 4 * C) {
    const int which = tid / C, c = tid % C;
    const float* inv1 = reinterpret_cast<const float*>(static_cast<const char*>(a.w1s) + NST * 2 * QS);
    const float* inv2 = reinterpret_cast<const float*>(static_cast<const char*>(a.w2s) + NST * 2 * QS);
    prm[tid] = which == 0 ? a.b1[c] : which == 1 ? inv1[c] : which == 2 ? a.b2[c] : inv2[c];
  }

  // ---- x tile -> XS = split(lrelu(x)); row r <-> time t0 - 1 - h1 + r, zero outside [0, T) (conv1's padding)
  f32x4 xv[XITER];
  unsigned xok = 0u;  // rows outside [0, T) are loaded from row 0 and zeroed when split (no select on the loads)
  auto load_x = [&](int tl) __attribute__((always_inline)) {
    const int bb = tl / ntiles, tb = (tl - bb * ntiles) * TT - 1 - h1;
    const float* Xb = a.x + (long long)bb * a.x_bs;
    xok = 0u;
#pragma unroll
    for (int it = 0; it < XITER; ++it) {
      const int i = it * RB_THREADS + tid;
      const int r = i / C4, c4 = (i % C4) * 4;
      const int t = tb + r;
      const bool ok = r < nx && t >= 0 && t < a.T;
      xv[it] = *reinterpret_cast<const f32x4*>(Xb + (long long)(ok ? t : 0) * C + c4);
      xok |= ok ? (1u << it) : 0u;
    }
  };
  auto write_x = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < XITER; ++it) {
      const int i = it * RB_THREADS + tid;
      const int r = i / C4, c4 = (i % C4) * 4;
      if (r < nx) {
        const int s = c4 >> 4, o = c4 & 15;
        const int slot = ((o >> 2) & 1) * 8 + (o >> 3) * 4;
        char* row = XS + (size_t)r * ROW + s * CB + slot * 2;
        const bool ok = (xok >> it) & 1u;
        const float y0 = ok ? lrelu01(xv[it][0]) * RB_XS : 0.f, y1 = ok ? lrelu01(xv[it][1]) * RB_XS : 0.f,
                    y2 = ok ? lrelu01(xv[it][2]) * RB_XS : 0.f, y3 = ok ? lrelu01(xv[it][3]) * RB_XS : 0.f;
        uint2 hh, ll;
        hh.x = pk_f16(y0, y1);
        hh.y = pk_f16(y2, y3);
        ll.x = pk_f16((y0 - f16lo_f(hh.x)) * H16_LO, (y1 - f16hi_f(hh.x)) * H16_LO);
        ll.y = pk_f16((y2 - f16lo_f(hh.y)) * H16_LO, (y3 - f16hi_f(hh.y)) * H16_LO);
        *reinterpret_cast<uint2*>(row) = hh;
        *reinterpret_cast<uint2*>(row + 32) = ll;
      }
    }
  };
  // one conv over the wave's 32-row block: B fragments from LDS one step ahead (two register slots)
  auto conv = [&](const char* bl, int dil, const f16x8_(&w)[NST][NQ], f32x16& acc, f32x16& acc2)
                  __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = acc2[r] = 0.f;
    f16x8_ bf[2][NQ];
    auto load_b = [&](int st, f16x8_(&f)[NQ]) __attribute__((always_inline)) {
      const int tap = st / NCH, s = st - tap * NCH;
      const char* bp = bl + (size_t)tap * dil * ROW + s * CB;
#pragma unroll
      for (int q = 0; q < NQ; ++q) f[q] = *reinterpret_cast<const f16x8_*>(bp + q * 32);
    };
    load_b(0, bf[0]);
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      if (st + 1 < NST) load_b(st + 1, bf[(st + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      const f16x8_ bh = bf[st & 1][0];
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(w[st][0], bh, acc, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(w[st][1], bh, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(w[st][0], bf[st & 1][1], acc2, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // acc + 2^-11 acc2 times 1 / (channel weight scale x activation scale): element r is channel 8 (r / 4) + 4 hk + r % 4
  auto finish = [&](f32x16& acc, const f32x16& acc2, const float* inv) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const f32x4 iv = *reinterpret_cast<const f32x4*>(inv + 8 * m + 4 * hk);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[4 * m + e] = (acc[4 * m + e] + acc2[4 * m + e] * H16_LO_INV) * iv[e];
    }
  };

  load_x(tile);
#pragma unroll 1
  for (; tile < tile_end; ++tile) {
    const int b = tile / ntiles;
    const int t0 = (tile - b * ntiles) * TT;
    write_x();
    __syncthreads();  // XS complete; TS free (every wave's conv2 of the previous tile is done)
    // this tile's residual (and accumulate) operands, then the next tile's rows: issued in the order they are used
    const float* X = a.x + (long long)b * a.x_bs;
    float* Y = a.y + (long long)b * a.y_bs;
    const int o = wave * 32 + li;
    const int t = t0 + o;
    const bool out_ok = o < TT && t < a.T;
    const long long off = (long long)(out_ok ? t : 0) * C + 4 * hk;
    f32x4 rv[4], dv[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      rv[m] = *reinterpret_cast<const f32x4*>(X + off + 8 * m);
      if constexpr (ACCM != ACC_STORE) dv[m] = *reinterpret_cast<const f32x4*>(Y + off + 8 * m);
    }
    load_x(min(tile + 1, tile_end - 1));
    // conv1 -> TS = split(lrelu(conv1 + b1)); TS row p <-> time t0 - 1 + p, zero outside [0, T)
    {
      f32x16 acc, acc2;
      conv(XS + (size_t)(wave * 32 + li) * ROW + hk * 16, a.d, w1r, acc, acc2);
      finish(acc, acc2, prm + C);
      const int p = wave * 32 + li;
      const int tp = t0 - 1 + p;
      const bool ok = tp >= 0 && tp < a.T;
      char* row = TS + (size_t)p * ROW + hk * 16;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int r = 8 * hh + i;
          const float bv = prm[8 * (r >> 2) + 4 * hk + (r & 3)];
          const float x = lrelu01(acc[r] + bv);
          v[i] = ok ? x * RB_XS : 0.f;
        }
        uint4 Hh, Ll;
        split8_h16(v, Hh, Ll);
        char* dst = row + hh * CB;
        *reinterpret_cast<uint4*>(dst) = Hh;
        *reinterpret_cast<uint4*>(dst + 32) = Ll;
      }
    }
    __syncthreads();  // TS complete; XS free
    // conv2 + b2 + x -> y (acc mode); output row o <-> time t0 + o
    {
      f32x16 acc, acc2;
      conv(TS + (size_t)(wave * 32 + li) * ROW + hk * 16, 1, w2r, acc, acc2);
      finish(acc, acc2, prm + 3 * C);
      if (out_ok) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const f32x4 bv = *reinterpret_cast<const f32x4*>(prm + 2 * C + 8 * m + 4 * hk);
          f32x4 o4;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = acc[4 * m + e] + bv[e];
            v = v + rv[m][e];
            if constexpr (ACCM == ACC_ADD) v = dv[m][e] + v;
            else if constexpr (ACCM == ACC_ADD_DIV) v = (dv[m][e] + v) / a.acc_div;
            o4[e] = v;
          }
          *reinterpret_cast<f32x4*>(Y + off + 8 * m) = o4;
        }
      }
    }
  }
}

template <int ACCM>
hipError_t launch_rb3(const RbPairArgs& a, hipStream_t s) {
  constexpr int ROW = RbGeo<32, RB_F16X2>::ROW;
  const int TT = 4 * 32 - 2;
  const size_t smem = (size_t)(4 * 32 + 2 * a.d) * ROW + (size_t)(4 * 32 + 2) * ROW + 4 * 32 * sizeof(float);
  auto kern = k_rb_pair3<ACCM>;
  static size_t smem_set = 64 * 1024;
  if (smem > smem_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)smem);
    if (e != hipSuccess) return e;
    smem_set = smem;
  }
  const int ntiles = (a.T + TT - 1) / TT;
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || ncu <= 0)
      ncu = 256;
  }
  const long long tiles = (long long)ntiles * a.B;
  const int grid = (int)std::min<long long>(tiles, (long long)ncu * 2);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(RB_THREADS), smem, s, a, ntiles);
  return hipGetLastError();
}

template <int C, int NBT, int TN, int MODE>
hipError_t launch_rb_acc(const RbPairArgs& a, hipStream_t s) {
  constexpr int ROW = RbGeo<C, (MODE >> 2) & 3>::ROW;
  const int h2 = (a.k - 1) / 2, h1 = h2 * a.d;
  const int TT = NBT * 32 - 2 * h2;
  const size_t smem = (size_t)(NBT * 32 + 2 * h1) * ROW + (size_t)(NBT * 32 + 2 * h2) * ROW;
  auto kern = k_rb_pair<C, NBT, TN, MODE>;
  static size_t smem_set = 64 * 1024;
  if (smem > smem_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)smem);
    if (e != hipSuccess) return e;
    smem_set = smem;
  }
  const int ntiles = (a.T + TT - 1) / TT;
  // persistent grid: as many workgroups as fit on the chip at once (LDS-limited), at most one per tile
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || ncu <= 0)
      ncu = 256;
  }
  const int per_cu = std::max(1, std::min(3, (int)((160 * 1024) / smem)));
  const long long tiles = (long long)ntiles * a.B;
  const int grid = (int)std::min<long long>(tiles, (long long)ncu * per_cu);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(RB_THREADS), smem, s, a, ntiles);
  return hipGetLastError();
}

template <int C, int NBT, int TN>
hipError_t launch_rb(const RbPairArgs& a, hipStream_t s) {
  // the weight images' format decides the arithmetic; the reduced-precision mode reads the fp16 image's hi plane
  const int fmt = a.wfmt == RB_WF16 ? (a.lowp ? RB_F16X1 : RB_F16X2) : RB_BF16X3;
  if (a.lowp && a.wfmt != RB_WF16) return hipErrorInvalidValue;
  switch (a.acc_mode | (fmt << 2)) {
#define RB_CASE(M) \
  case M: return launch_rb_acc<C, NBT, TN, M>(a, s);
    RB_CASE(0) RB_CASE(1) RB_CASE(2) RB_CASE(4) RB_CASE(5) RB_CASE(6) RB_CASE(8) RB_CASE(9) RB_CASE(10)
#undef RB_CASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool rb_pair_fits(int C, int k, int d) {
  if (!(C == 32 || C == 64)) return false;
  if (k < 1 || (k & 1) == 0 || d < 1) return false;
  const int h2 = (k - 1) / 2;
  return h2 * d <= RB_MAXH1 && 2 * h2 < 32;
}

// the fp16 image: two planes + a tail of 2 x C words (the output channels' inverse scales, their max |w| bits)
long long rb_wsplit_bytes(int C, int k, int wfmt) {
  return wfmt == RB_WF16 ? (long long)k * (C / 16) * 2 * C * 32 + 8LL * C : (long long)k * (C / 16) * 3 * C * 32;
}

hipError_t rb_wsplit_build(const float* w, int C, int k, void* out, hipStream_t s, int wfmt) {
  if (C % 16 != 0 || k < 1) return hipErrorInvalidValue;
  const long long total = (long long)k * (C / 16) * C * 16;
  const long long nb = std::min<long long>((total + 255) / 256, 1 << 20);
  if (wfmt == RB_WF16) {
    float* tail = reinterpret_cast<float*>(static_cast<char*>(out) + (long long)k * (C / 16) * 2 * C * 32);
    hipLaunchKernelGGL(k_rb_wmax, dim3((unsigned)((C + 3) / 4)), dim3(256), 0, s, w, C, k,
                       reinterpret_cast<unsigned*>(tail) + C);
    hipLaunchKernelGGL(k_rb_wsplit_h16, dim3((unsigned)nb), dim3(256), 0, s, w, C, k, 2,
                       static_cast<unsigned short*>(out), tail);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_rb_wsplit, dim3((unsigned)nb), dim3(256), 0, s, w, C, k, static_cast<unsigned short*>(out));
  return hipGetLastError();
}

// (C, NBT, TN) = 32: (4, 1), 64: (2, 1). The (8, 2) / (4, 2) tiles (two time blocks per wave) measured slower (+0.35 ms
// in the C2 step) and are gone. cfg 0: the k = 3, 32-channel fp16 pairs on the weight-resident kernel (k_rb_pair3),
// the rest on k_rb_pair; cfg 1: k_rb_pair for every shape (comparisons)
hipError_t rb_pair(const RbPairArgs& a, int cfg, hipStream_t s) {
  if (cfg != 0 && cfg != 1) return hipErrorInvalidValue;
  if (!rb_pair_fits(a.C, a.k, a.d) || a.T < 1 || a.B < 1 || !a.x || !a.y || !a.w1s || !a.w2s || !a.b1 || !a.b2 ||
      a.x == a.y)
    return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(a.x) & 15) || (reinterpret_cast<uintptr_t>(a.y) & 15) || (a.x_bs & 3) ||
      (a.y_bs & 3))
    return hipErrorInvalidValue;
  if (cfg == 0 && a.C == 32 && a.k == 3 && a.wfmt == RB_WF16 && !a.lowp) {
    switch (a.acc_mode) {
      case ACC_STORE: return launch_rb3<ACC_STORE>(a, s);
      case ACC_ADD: return launch_rb3<ACC_ADD>(a, s);
      case ACC_ADD_DIV: return launch_rb3<ACC_ADD_DIV>(a, s);
      default: return hipErrorInvalidValue;
    }
  }
  switch (a.C) {
    case 32: return launch_rb<32, 4, 1>(a, s);
    case 64: return launch_rb<64, 2, 1>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace rvcx
