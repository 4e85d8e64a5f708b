// Fused multi-head attention without a [B][heads][T][T] score buffer (flash-style online softmax), for the
// TextEncoder's windowed relative-position attention (rvc/lib/algorithm/attentions.py:79-185: scores =
// (q/sqrt(d)) k^T + band of (q/sqrt(d)) rel_k^T, masked_fill(mask == 0, -1e4), softmax, p v + band(p) rel_v) and
// HuBERT's plain attention (modeling_hubert.py HubertAttention: softmax((q * d^-0.5) k^T) v).
//
// One wave per (32-query block, key split, batch x head). The wave works in the transposed frame so that no
// fragment needs an LDS transpose: S^T = K Q^T (A = K rows, B = Q^T; MFMA C layout puts one query per lane
// column), the softmax statistics of a query are a lane's own 16 registers plus its partner lane (lane ^ 32),
// and O^T = V^T P^T takes P^T straight from the S^T registers as the B fragment (the K16 slots of a lane are its
// C rows, the same key permutation on the A side). Every product uses the two-plane fp16 split (below; fp32
// accurate). Key splits write unnormalised partials (O, running max, running sum) that k_flash_combine merges; the
// relative-value band is folded into each split's O before it is written.
#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <string>

#include "split_bf16.h"

namespace rvcx {

namespace {

using namespace splitbf16;

constexpr int FA_Q = 32;    // queries per wave
constexpr int FA_K = 32;    // keys per block
constexpr int FA_NW = 32;   // max relative window 2w+1 (LDS table width)

// key row of C register r for the half-wave hk (MFMA 32x32 C layout)
__device__ __forceinline__ int crow(int r, int hk) { return (r & 3) + 8 * (r >> 2) + 4 * hk; }

// ---- The arithmetic: the two-plane fp16 split (split_bf16.h put_h16x4; since round 4): three v_mfma_f32_32x32x16_f16
// products per step into two accumulators (h h' and l h' + h l', combined as acc + 2^-11 acc2) instead of the six bf16
// products of rounds 2-3's three-plane kernel (removed in round 6), and K / V from fragment-major images built once
// per call by k_kv_split16 (every query-block wave of the bf16 kernel re-split the same K and V blocks). q, k, v and
// the relative tables are scaled by 2^-4 before the split (inputs up to 2^20 stay finite fp16; the softmax
// probabilities need none) and the scales are multiplied back exactly: S by 2^8, O by 2^4.
// Image of one (batch x head, 32-key block): K: [NS][plane][64 lanes][8 fp16] (lane (li, hk): key li, dims
// 16 s + 8 hk ..), then V: [NT][2][plane][64 lanes][8 fp16] (lane (li, hk): dim 32 t + li, keys crow(8 s2 + e, hk)).
constexpr float FA_XS = 1.f / 16.f;

__device__ __forceinline__ void split8h(const float (&v)[8], f16x8 (&out)[2]) {
  unsigned h[4], l[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    h[p] = pk_f16(v[2 * p], v[2 * p + 1]);
    l[p] = pk_f16((v[2 * p] - f16lo_f(h[p])) * H16_LO, (v[2 * p + 1] - f16hi_f(h[p])) * H16_LO);
  }
  out[0] = __builtin_bit_cast(f16x8, make_uint4(h[0], h[1], h[2], h[3]));
  out[1] = __builtin_bit_cast(f16x8, make_uint4(l[0], l[1], l[2], l[3]));
}

__device__ __forceinline__ void mfma3(const f16x8 (&a)[2], const f16x8 (&b)[2], f32x16& c, f32x16& c2) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], c, 0, 0, 0);
  c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], c2, 0, 0, 0);
  c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], c2, 0, 0, 0);
}

// one wave per (key block, batch x head, fragment): blockIdx.z < NS a K step, else a V^T (t, s2) pair
template <int DK>
__global__ __launch_bounds__(64) void k_kv_split16(const float* __restrict__ qkv, int ldq, int T, int nh, int H,
                                                   uint4* __restrict__ img) {
  constexpr int NS = DK / 16, NT = DK / 32;
  constexpr int FR = NS * 2 + NT * 2 * 2;  // 1 KB fragment planes per (bh, key block)
  const int lane = threadIdx.x, li = lane & 31, hk = lane >> 5;
  const int kb = blockIdx.x, bh = blockIdx.y, f = blockIdx.z, nkb = gridDim.x;
  const int b = bh / nh, h = bh % nh;
  const float* base = qkv + (long long)b * T * ldq;
  uint4* out = img + ((long long)bh * nkb + kb) * FR * 64 + lane;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int fr;
  if (f < NS) {  // K: key li, dims 16 f + 8 hk ..
    const int j = kb * FA_K + li;
    if (j < T) {
      const float4* src = reinterpret_cast<const float4*>(base + (long long)j * ldq + H + h * DK + 16 * f + 8 * hk);
      const float4 x0 = src[0], x1 = src[1];
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    }
    fr = 2 * f;
  } else {  // V^T: dim 32 t + li, keys crow(8 s2 + e, hk)
    const int t = (f - NS) >> 1, s2 = (f - NS) & 1;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int jj = kb * FA_K + crow(8 * s2 + e, hk);
      if (jj < T) v[e] = base[(long long)jj * ldq + 2 * H + h * DK + 32 * t + li];
    }
    fr = 2 * NS + (t * 2 + s2) * 2;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] *= FA_XS;
  f16x8 q[2];
  split8h(v, q);
  out[fr * 64] = __builtin_bit_cast(uint4, q[0]);
  out[(fr + 1) * 64] = __builtin_bit_cast(uint4, q[1]);
}

// NW waves per block: the same query block, key splits blockIdx.y * NW + wave, merged in LDS at the end into one
// partial per block (the split partials written to HBM and re-read by k_flash_combine drop NW-fold; NW = 1: one
// wave, one partial each)
template <int DK, int NW>
__global__ __launch_bounds__(64 * NW, 2) void k_flash_attn_h16(
    const float* __restrict__ qkv, int ldq, int T, int nh, int H, float qscale, int kb_per_split,
    const float* __restrict__ rel_k, const float* __restrict__ rel_v, int window, const float* __restrict__ mask,
    const uint4* __restrict__ img, float* __restrict__ part_o, float* __restrict__ part_ml) {
  constexpr int NS = DK / 16;
  constexpr int NT = DK / 32;
  constexpr int FR = NS * 2 + NT * 2 * 2;
  __shared__ float relq_s[NW][FA_Q][FA_NW + 1];
  __shared__ float pband_s[NW][FA_Q][FA_NW + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 31, hk = lane >> 5;
  float (*relq)[FA_NW + 1] = relq_s[wave];
  float (*pband)[FA_NW + 1] = pband_s[wave];
  const int q0 = blockIdx.x * FA_Q, split = blockIdx.y * NW + wave, bh = blockIdx.z;
  const int b = bh / nh, h = bh % nh;
  const int BH = gridDim.z;
  const float* base = qkv + (long long)b * T * ldq;
  const int i = q0 + li;
  const bool qok = i < T;
  const int nw = rel_k ? 2 * window + 1 : 0;
  const float* mk = mask ? mask + (long long)b * T : nullptr;
  const float mi = (mk && qok) ? mk[i] : 1.f;
  const int nkb = (T + FA_K - 1) / FA_K;
  const uint4* kvimg = img + (long long)bh * nkb * FR * 64 + lane;

  // Q^T fragments (scaled by qscale 2^-4), kept for the whole key range. Queries past T read row T - 1 and are
  // zeroed: no load sits under a lane condition, so all NS steps' loads are in flight together (one round trip, not NS)
  f16x8 qf[NS][2];
  {
    const float4* src = reinterpret_cast<const float4*>(base + (long long)min(i, T - 1) * ldq + h * DK + 8 * hk);
    float4 xq[NS][2];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      xq[s][0] = src[4 * s];
      xq[s][1] = src[4 * s + 1];
    }
    const float qs = qscale * FA_XS;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const float4 x0 = xq[s][0], x1 = xq[s][1];
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (qok) {
        v[0] = x0.x * qs; v[1] = x0.y * qs; v[2] = x0.z * qs; v[3] = x0.w * qs;
        v[4] = x1.x * qs; v[5] = x1.y * qs; v[6] = x1.z * qs; v[7] = x1.w * qs;
      }
      split8h(v, qf[s]);
    }
  }
  const int kb0 = split * kb_per_split, kb1 = min(nkb, kb0 + kb_per_split);
  const bool band_split = nw && kb0 < kb1 && (kb1 * FA_K - 1 >= q0 - window) && (kb0 * FA_K <= q0 + FA_Q - 1 + window);
  if (band_split) {
    f32x16 rq, rq2;
#pragma unroll
    for (int r = 0; r < 16; ++r) rq[r] = rq2[r] = 0.f;
    // rows past the window read row nw - 1 and are zeroed: no load sits under a lane condition, so the NS steps'
    // loads issue back to back instead of one round trip per step
    const float* rk = rel_k + min(li, nw - 1) * DK + 8 * hk;
    f32x4 rkv[NS][2];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      rkv[s][0] = *reinterpret_cast<const f32x4*>(rk + 16 * s);
      rkv[s][1] = *reinterpret_cast<const f32x4*>(rk + 16 * s + 4);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = li < nw ? rkv[s][e >> 2][e & 3] * FA_XS : 0.f;
      f16x8 rf[2];
      split8h(v, rf);
      mfma3(rf, qf[s], rq, rq2);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int od = crow(r, hk);
      relq[li][od] = (rq[r] + rq2[r] * H16_LO_INV) * 256.f;
      pband[li][od] = 0.f;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  f32x16 o[NT], o2[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[t][r] = o2[t][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  for (int kb = kb0; kb < kb1; ++kb) {
    const int j0 = kb * FA_K;
    const uint4* fr = kvimg + (long long)kb * FR * 64;
    // S^T = K Q^T for keys j0.. (rows) x this wave's queries (columns)
    // the key block's K fragments issued in batches of KB steps ahead of their products (one round trip per batch
    // instead of one per K step: the scheduler otherwise interleaves load -> wait -> MFMA per step); DK = 96 takes
    // two batches, all six in flight would not fit beside the accumulators in 256 VGPRs
    constexpr int KB = DK == 64 ? NS : NS / 2;
    f32x16 sc, sc2;
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[r] = sc2[r] = 0.f;
#pragma unroll
    for (int s0 = 0; s0 < NS; s0 += KB) {
      uint4 kraw[KB][2];
#pragma unroll
      for (int s = 0; s < KB; ++s) {
        kraw[s][0] = fr[(2 * (s0 + s)) * 64];
        kraw[s][1] = fr[(2 * (s0 + s) + 1) * 64];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < KB; ++s) {
        f16x8 kf[2];
        kf[0] = __builtin_bit_cast(f16x8, kraw[s][0]);
        kf[1] = __builtin_bit_cast(f16x8, kraw[s][1]);
        mfma3(kf, qf[s0 + s], sc, sc2);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // the V^T fragments: for DK = 64 all issued now, in flight under the softmax; for DK = 96 per half of the key
    // block (s2) just before its products (all of them here would not fit in 256 VGPRs)
    uint4 vraw[NT][2][2];
    auto load_v = [&](int s2) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int f = 2 * NS + (t * 2 + s2) * 2;
        vraw[t][s2][0] = fr[f * 64];
        vraw[t][s2][1] = fr[(f + 1) * 64];
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    if constexpr (DK == 64) {
      load_v(0);
      load_v(1);
    }
    // band blocks only (wave-uniform): the 16 relative-key terms gathered in one batch of LDS reads (clamped
    // column, out-of-window values discarded)
    const bool band = band_split && (j0 + FA_K - 1 >= q0 - window) && (j0 <= q0 + FA_Q - 1 + window);
    float rqv[16];
    if (band) {
#pragma unroll
      for (int r = 0; r < 16; ++r) rqv[r] = relq[li][min(max(j0 + crow(r, hk) - i + window, 0), FA_NW)];
    }
    float mloc = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = j0 + crow(r, hk);
      float v = (sc[r] + sc2[r] * H16_LO_INV) * 256.f;
      if (band) {
        const int od = j - i + window;
        if (od >= 0 && od < nw) v = v + rqv[r];
      }
      if (mk && j < T && mi * mk[j] == 0.f) v = -1e4f;
      if (j >= T) v = -INFINITY;
      sc[r] = v;
      mloc = fmaxf(mloc, v);
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32));
    const float m_new = fmaxf(m_run, mloc);
    const float alpha = expf(m_run - m_new);
    float lsum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sc[r] = expf(sc[r] - m_new);
      lsum += sc[r];
    }
    lsum += __shfl_xor(lsum, 32);
    l_run = l_run * alpha + lsum;
    m_run = m_new;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        o[t][r] *= alpha;
        o2[t][r] *= alpha;
      }
    if (band_split) {
      // rescale the band sums when a running max moved (alpha == 1 exactly otherwise): the two lanes of a query
      // take 16 of its 32 columns each, unrolled so the reads issue back to back
      if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
        for (int e = 0; e < 16; ++e) pband[li][16 * hk + e] *= alpha;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (band) {
        // a lane's 16 keys sit on 16 distinct diagonals (the other lane of its query on 16 others): all reads can
        // precede all writes
        float pb[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) pb[r] = pband[li][min(max(j0 + crow(r, hk) - i + window, 0), FA_NW)];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int od = j0 + crow(r, hk) - i + window;
          if (od >= 0 && od < nw) pband[li][od] = pb[r] + sc[r];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // O^T += V^T P^T
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      if constexpr (DK != 64) load_v(s2);
      float pv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) pv[e] = sc[8 * s2 + e];
      f16x8 pf[2];
      split8h(pv, pf);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f16x8 vf[2];
        vf[0] = __builtin_bit_cast(f16x8, vraw[t][s2][0]);
        vf[1] = __builtin_bit_cast(f16x8, vraw[t][s2][1]);
        mfma3(vf, pf, o[t], o2[t]);
      }
    }
  }
  if (band_split) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      float pv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) pv[e] = pband[li][16 * s2 + 8 * hk + e];
      f16x8 pf[2];
      split8h(pv, pf);
      // every rel_v load unconditional (rows past the window read row nw - 1, zeroed below): all 8 x NT in flight
      float rv[NT][8];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) rv[t][e] = rel_v[min(16 * s2 + 8 * hk + e, nw - 1) * DK + 32 * t + li];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int od = 16 * s2 + 8 * hk + e;
          v[e] = od < nw ? rv[t][e] * FA_XS : 0.f;
        }
        f16x8 vf[2];
        split8h(v, vf);
        mfma3(vf, pf, o[t], o2[t]);
      }
    }
  }
  if constexpr (NW == 1) {
    float* ot = &relq[0][0];
    const long long slab = ((long long)split * BH + bh) * T;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int r = 0; r < 16; ++r) ot[li * (FA_NW + 1) + crow(r, hk)] = (o[t][r] + o2[t][r] * H16_LO_INV) * 16.f;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int idx = k * 64 + lane, rr = idx >> 3, c4 = (idx & 7) * 4;
        if (q0 + rr < T) {
          const float* src = ot + rr * (FA_NW + 1) + c4;
          const f32x4 v = {src[0], src[1], src[2], src[3]};
          *reinterpret_cast<f32x4*>(part_o + (slab + q0 + rr) * DK + 32 * t + c4) = v;
        }
      }
    }
    if (qok && hk == 0) {
      const long long row = slab + i;
      part_ml[2 * row] = m_run;
      part_ml[2 * row + 1] = l_run;
    }
  } else {
    // block merge: M = max of the waves' running maxima per query, each wave's tile scaled by e^(m_w - M) and
    // summed into LDS in wave order (deterministic), L likewise; one partial (M, L, sum) per block
    __shared__ float mrow[NW][FA_Q];
    __shared__ float lsum[FA_Q];
    __shared__ float acc[FA_Q][DK + 4];
    if (hk == 0) mrow[wave][li] = m_run;
    __syncthreads();
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, mrow[w][li]);
    const float e = m_run == -INFINITY ? 0.f : expf(m_run - M);
    for (int w = 0; w < NW; ++w) {
      if (wave == w) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float v = (o[t][r] + o2[t][r] * H16_LO_INV) * 16.f * e;
            float& a = acc[li][32 * t + crow(r, hk)];
            a = w == 0 ? v : a + v;
          }
        if (hk == 0) lsum[li] = w == 0 ? l_run * e : lsum[li] + l_run * e;
      }
      __syncthreads();
    }
    const long long slab = ((long long)blockIdx.y * BH + bh) * T;
    for (int idx = threadIdx.x; idx < FA_Q * DK / 4; idx += 64 * NW) {
      const int rr = idx / (DK / 4), c4 = (idx - rr * (DK / 4)) * 4;
      if (q0 + rr < T) {
        const f32x4 v = {acc[rr][c4], acc[rr][c4 + 1], acc[rr][c4 + 2], acc[rr][c4 + 3]};
        *reinterpret_cast<f32x4*>(part_o + (slab + q0 + rr) * DK + c4) = v;
      }
    }
    if (wave == 0 && qok && hk == 0) {
      const long long row = slab + i;
      part_ml[2 * row] = M;
      part_ml[2 * row + 1] = lsum[li];
    }
  }
}

// out[b][i][h*DK + d] = sum_s O_s[d] e^(m_s - M) / sum_s l_s e^(m_s - M)
// Merges the key splits: one row (bh, query i) per DK/4 lanes, each lane a float4 of the head dimension. The split
// weights exp(m_s - M) are computed per lane group (was: per output element, with 64-bit index divisions per element),
// every load is a 16-B vector or a broadcast, and the sum runs over the splits in order (same arithmetic as before).
template <int DK>
__global__ __launch_bounds__(256) void k_flash_combine(const float* __restrict__ part_o,
                                                       const float* __restrict__ part_ml, int nsplit, int BH, int T,
                                                       int nh, float* __restrict__ out, int ldo) {
  constexpr int LPR = DK / 4;          // lanes per row
  constexpr int RPW = 64 / LPR;        // rows per wave
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / LPR, d4 = (lane - sub * LPR) * 4;
  if (sub >= RPW) return;  // DK = 96: lanes 48..63 idle
  const int rows = BH * T;
  const int row = (blockIdx.x * 4 + wave) * RPW + sub;
  if (row >= rows) return;
  const unsigned split_rows = (unsigned)rows;  // rows per split slab
  float M = -INFINITY;
  for (int sp = 0; sp < nsplit; ++sp) M = fmaxf(M, part_ml[2u * (sp * split_rows + (unsigned)row)]);
  float L = 0.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int sp = 0; sp < nsplit; ++sp) {
    const unsigned r = sp * split_rows + (unsigned)row;
    const float ms = part_ml[2u * r];
    if (ms == -INFINITY) continue;  // an empty split
    const float e = expf(ms - M);
    L += part_ml[2u * r + 1] * e;
    const f32x4 o = *reinterpret_cast<const f32x4*>(part_o + r * (unsigned)DK + d4);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] += o[j] * e;
  }
  const int bh = row / T, i = row - bh * T;
  const int b = bh / nh, h = bh - b * nh;
  f32x4 res;
#pragma unroll
  for (int j = 0; j < 4; ++j) res[j] = acc[j] / L;
  *reinterpret_cast<f32x4*>(out + ((long long)b * T + i) * ldo + h * DK + d4) = res;
}

}  // namespace

// key splits: ~4096 query-block x split waves (the kernel is latency-bound per key block), at least 2 key blocks
// per split
int flash_attn_splits(int B, int nh, int T) {
  static const int waves = [] {  // RVCX_FA_WAVES: target query-block x split waves (A/B aid)
    const char* e = rvcx_knob("RVCX_FA_WAVES");
    return e ? std::max(1, std::atoi(e)) : 4096;  // same-box C2: 512 18.12, 1024 17.91, 2048 17.98, 4096 17.84 ms
  }();
  const int qb = (T + FA_Q - 1) / FA_Q, kb = (T + FA_K - 1) / FA_K;
  int ns = (waves + qb * B * nh - 1) / (qb * B * nh);
  ns = std::max(1, std::min(ns, std::max(1, kb / 2)));
  return ns;
}

// part_o's floats: the split partials, then the K / V fragment images
long long flash_attn_ws_floats(int B, int nh, int T, int dk, int nsplit) {
  const long long parts = (long long)nsplit * B * nh * T * dk;
  const long long nkb = (T + FA_K - 1) / FA_K;
  const long long img = (long long)B * nh * nkb * (dk / 16 * 2 + dk / 32 * 4) * 64 * 4;  // uint4 = 4 floats
  return parts + img;
}

hipError_t flash_attn(const float* qkv, int ldq, int B, int T, int nh, int dk, float qscale, const float* rel_k,
                      const float* rel_v, int window, const float* mask, float* part_o, float* part_ml, int nsplit,
                      float* out, int ldo, hipStream_t s) {
  if (T <= 0) return hipSuccess;
  if ((ldq & 3) != 0 || (reinterpret_cast<uintptr_t>(qkv) & 15) != 0) return hipErrorInvalidValue;  // float4 rows
  if ((rel_k != nullptr) != (rel_v != nullptr) || (rel_k && 2 * window + 1 > FA_NW) || nsplit < 1)
    return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(rel_k) & 15) != 0) return hipErrorInvalidValue;  // float4 rel_k rows (h16 kernel)
  const int H = nh * dk;
  const int qb = (T + FA_Q - 1) / FA_Q, kb = (T + FA_K - 1) / FA_K;
  if (dk != 64 && dk != 96) return hipErrorInvalidValue;
  int nparts = nsplit;  // partials the combine merges
  {
    // the K / V images after the partials (the caller sized part_o with flash_attn_ws_floats)
    uint4* img = reinterpret_cast<uint4*>(part_o + (long long)nsplit * B * nh * T * dk);
    if ((reinterpret_cast<uintptr_t>(img) & 15) != 0) return hipErrorInvalidValue;
    dim3 g2(kb, B * nh, dk / 16 + dk / 16);  // NS K steps + 2 NT V^T pairs (NS = 2 NT)
    // four key splits per block merged in LDS (one wave per split, every split a partial, below four splits; four
    // waves per block cut the HBM partials and the combine's reads 4-fold: TE combine 17.0 -> 6.7 us, r04zg)
    const int NWB = nsplit >= 4 ? 4 : 1;
    nparts = (nsplit + NWB - 1) / NWB;
    const int per_w = (kb + nparts * NWB - 1) / (nparts * NWB);
    dim3 gw(qb, nparts, B * nh);
    if (dk == 64) {
      hipLaunchKernelGGL(k_kv_split16<64>, g2, dim3(64), 0, s, qkv, ldq, T, nh, H, img);
      if (NWB == 4)
        hipLaunchKernelGGL((k_flash_attn_h16<64, 4>), gw, dim3(256), 0, s, qkv, ldq, T, nh, H, qscale, per_w, rel_k,
                           rel_v, window, mask, img, part_o, part_ml);
      else
        hipLaunchKernelGGL((k_flash_attn_h16<64, 1>), gw, dim3(64), 0, s, qkv, ldq, T, nh, H, qscale, per_w, rel_k,
                           rel_v, window, mask, img, part_o, part_ml);
    } else {
      hipLaunchKernelGGL(k_kv_split16<96>, g2, dim3(64), 0, s, qkv, ldq, T, nh, H, img);
      if (NWB == 4)
        hipLaunchKernelGGL((k_flash_attn_h16<96, 4>), gw, dim3(256), 0, s, qkv, ldq, T, nh, H, qscale, per_w, rel_k,
                           rel_v, window, mask, img, part_o, part_ml);
      else
        hipLaunchKernelGGL((k_flash_attn_h16<96, 1>), gw, dim3(64), 0, s, qkv, ldq, T, nh, H, qscale, per_w, rel_k,
                           rel_v, window, mask, img, part_o, part_ml);
    }
  }
  const long long rows = (long long)B * nh * T;
  if (rows * nsplit * dk >= (1LL << 31) || (ldo & 3) != 0 || (reinterpret_cast<uintptr_t>(out) & 15) != 0)
    return hipErrorInvalidValue;  // 32-bit slab offsets, float4 output rows
  const int rpb = 4 * (64 / (dk / 4));  // rows per 256-thread block
  const unsigned nb = (unsigned)((rows + rpb - 1) / rpb);
  if (dk == 64)
    hipLaunchKernelGGL(k_flash_combine<64>, dim3(nb), dim3(256), 0, s, part_o, part_ml, nparts, B * nh, T, nh, out, ldo);
  else
    hipLaunchKernelGGL(k_flash_combine<96>, dim3(nb), dim3(256), 0, s, part_o, part_ml, nparts, B * nh, T, nh, out, ldo);
  return hipGetLastError();
}

}  // namespace rvcx
