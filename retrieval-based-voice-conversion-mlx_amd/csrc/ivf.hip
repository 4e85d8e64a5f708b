// FAISS IndexIVFFlat search and the pipeline's speaker-embedding retrieval on device.
//
// Reference call site: rvc/infer/pipeline.py:378-388 (_retrieve_speaker_embeddings; identical in
// rvc_mlx/infer/pipeline_mlx.py:183-201):  score, ix = index.search(feats, k=8);
// w = (1/score)^2 / sum;  npy = sum_j big_npy[ix_j] * w_j;  feats = npy * rate + (1 - rate) * feats.
// Search semantics restate faiss 1.7.4 IndexIVF::search (L2): coarse top-nprobe centroids, exact L2
// scan of the probed lists, k best kept by strict-less admission in scan order, output ordered by
// (distance, id), missing results (+inf, -1).
//
// Layout in HBM (built by index_ivf.cpp): centroids [nlist][d]; the inverted lists' vectors back to
// back in list order [ntotal][d] with offsets off[nlist+1]; ids [ntotal] (int64, list order);
// slot_of_id [ntotal] (int32: big_npy row id -> storage slot, so big_npy[ix] is a gather of the
// stored vectors and no second copy exists).
//
// The work is tiny next to the synthesizer (775 queries x ~40 vectors x 768 at C2), so the kernels
// are plain VALU: one wave per vector row, coalesced 64-lane row reads, butterfly reductions.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>

#include "rvcx_kernels.h"

namespace rvcx {

namespace {

constexpr int WAVE = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}

// (dist, tie) lexicographic "a strictly before b"
__device__ __forceinline__ bool key_lt(float da, long long ta, float db, long long tb) {
  return da < db || (da == db && ta < tb);
}

}  // namespace

// ------------------------------------------------------------------ coarse distances
// cd[q][l] = sum_i (x[q][i] - cent[l][i])^2. Block: 4 waves x QB queries staged in LDS; blockIdx.x
// covers 64 centroids (16 per wave), blockIdx.y covers QB queries.
constexpr int IVF_QB = 8;
__global__ void __launch_bounds__(256) k_ivf_coarse(const float* __restrict__ x, int n, int d,
                                                    const float* __restrict__ cent, int nlist,
                                                    float* __restrict__ cd) {
  extern __shared__ float xs[];  // [IVF_QB][d]
  const int q0 = blockIdx.y * IVF_QB;
  const int nq = min(IVF_QB, n - q0);
  for (int i = threadIdx.x; i < IVF_QB * d; i += blockDim.x) {
    const int q = i / d;
    xs[i] = q < nq ? x[(long long)(q0 + q) * d + (i % d)] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l_end = min(nlist, (int)(blockIdx.x + 1) * 64);
  for (int l = blockIdx.x * 64 + w; l < l_end; l += 4) {
    const float* c = cent + (long long)l * d;
    float acc[IVF_QB];
#pragma unroll
    for (int q = 0; q < IVF_QB; ++q) acc[q] = 0.f;
    for (int i = lane; i < d; i += WAVE) {
      const float cv = c[i];
#pragma unroll
      for (int q = 0; q < IVF_QB; ++q) {
        const float t = xs[q * d + i] - cv;
        acc[q] = fmaf(t, t, acc[q]);
      }
    }
#pragma unroll
    for (int q = 0; q < IVF_QB; ++q) acc[q] = wave_sum(acc[q]);
    if (lane < nq) {
      float v = acc[0];
#pragma unroll
      for (int q = 1; q < IVF_QB; ++q)
        if (lane == q) v = acc[q];
      cd[(long long)(q0 + lane) * nlist + l] = v;
    }
  }
}

// ------------------------------------------------------------------ probe selection
// probe[q][p] = p-th smallest (cd, list id); one wave per query, nprobe passes of a wave argmin over
// the keys strictly after the previous pick.
__global__ void __launch_bounds__(64) k_ivf_probe(const float* __restrict__ cd, int n, int nlist, int nprobe,
                                                  int* __restrict__ probe) {
  const int q = blockIdx.x;
  if (q >= n) return;
  const int lane = threadIdx.x;
  const float* row = cd + (long long)q * nlist;
  float pd = -FLT_MAX;
  long long pl = -1;
  for (int p = 0; p < nprobe; ++p) {
    float bd = FLT_MAX;
    long long bl = LLONG_MAX;
    for (int l = lane; l < nlist; l += WAVE) {
      const float v = row[l];
      if (key_lt(pd, pl, v, l) && key_lt(v, l, bd, bl)) {
        bd = v;
        bl = l;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float od = __shfl_xor(bd, o, WAVE);
      const long long ol = __shfl_xor(bl, o, WAVE);
      if (key_lt(od, ol, bd, bl)) {
        bd = od;
        bl = ol;
      }
    }
    if (lane == 0) probe[(long long)q * nprobe + p] = bl == LLONG_MAX ? -1 : (int)bl;
    pd = bd;
    pl = bl;
  }
}

// ------------------------------------------------------------------ list scan (+ retrieval blend)
// One block (4 waves) per query. Each wave scans every 4th vector of the probed lists (scan position
// pos) and keeps its K best (dist, pos) in lanes 0..K-1 (lane j = j-th best), inserting with one
// shuffle. The 4 wave lists are merged by rank; the k results are ordered by (dist, id).
// When `out` is set, the retrieval blend of pipeline.py:380-387 follows with numpy/torch float32
// rounding: w_j = (1/d_j)^2, w_j /= pairwise_sum(w) (numpy pairwise order), npy = ((p_0 + p_1) + ...)
// with p_j = big[ix_j] * w_j rounded, out = npy * f32(rate) + f32(1 - rate) * feats.
#pragma clang fp contract(off)
__global__ void __launch_bounds__(256) k_ivf_scan(const float* __restrict__ x, int n, int d,
                                                  const float* __restrict__ vecs, const long long* __restrict__ off,
                                                  const long long* __restrict__ ids, const int* __restrict__ probe,
                                                  int nprobe, int k, float* __restrict__ dist_out,
                                                  long long* __restrict__ ids_out, const int* __restrict__ slot_of_id,
                                                  long long ntotal, float rate, float one_minus_rate,
                                                  float* __restrict__ out) {
  extern __shared__ float sm[];
  float* xs = sm;                                   // [d]
  float* cd = xs + d;                               // [4*16] candidate dists
  long long* cp = reinterpret_cast<long long*>(cd + 64);  // [64] candidate pos
  long long* cs = cp + 64;                          // [64] candidate slot
  float* rd = reinterpret_cast<float*>(cs + 64);    // [16] result dists
  long long* ri = reinterpret_cast<long long*>(rd + 16);  // [16] result ids
  float* rw = reinterpret_cast<float*>(ri + 16);    // [16] weights
  long long* rs = reinterpret_cast<long long*>(rw + 16);  // [16] storage slots of the results
  __shared__ long long sid_sh[64];
  __shared__ int sel_sh[64];
  const int q = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* xq = x + (long long)q * d;
  for (int i = threadIdx.x; i < d; i += blockDim.x) xs[i] = xq[i];
  __syncthreads();

  float kd = INFINITY;
  long long kp = LLONG_MAX, ks = -1;
  long long pos0 = 0;
  for (int p = 0; p < nprobe; ++p) {
    const int l = probe[(long long)q * nprobe + p];
    if (l < 0) break;
    const long long base = off[l], cnt = off[l + 1] - base;
    for (long long j = w; j < cnt; j += 4) {
      const float* v = vecs + (base + j) * d;
      float acc = 0.f;
      for (int i = lane; i < d; i += WAVE) {
        const float t = xs[i] - v[i];
        acc = __fadd_rn(acc, __fmul_rn(t, t));
      }
      const float dist = wave_sum(acc);
      const long long pos = pos0 + j;
      const float worst = __shfl(kd, k - 1, WAVE);
      if (dist < worst) {  // strict admission (faiss CMax::cmp); NaN never admitted
        const bool gt = lane < k && key_lt(dist, pos, kd, kp);
        const bool pgt = __shfl_up(gt ? 1 : 0, 1, WAVE) != 0 && lane > 0;
        const float ud = __shfl_up(kd, 1, WAVE);
        const long long up = __shfl_up(kp, 1, WAVE), us = __shfl_up(ks, 1, WAVE);
        if (gt) {
          kd = pgt ? ud : dist;
          kp = pgt ? up : pos;
          ks = pgt ? us : base + j;
        }
      }
    }
    pos0 += cnt;
  }
  if (lane < 16) {
    const bool ok = lane < k;
    cd[w * 16 + lane] = ok ? kd : INFINITY;
    cp[w * 16 + lane] = ok ? kp : LLONG_MAX;
    cs[w * 16 + lane] = ok ? ks : -1;
  }
  __syncthreads();
  // merge the 4 wave lists (wave 0, one candidate per lane): select the k smallest (dist, pos)
  float md = 0.f;
  long long ms = -1, id = -1;
  bool sel = false;
  if (w == 0) {
    md = cd[lane];
    const long long mp = cp[lane];
    ms = cs[lane];
    int rank = 0;
    for (int j = 0; j < 64; ++j) rank += key_lt(cd[j], cp[j], md, mp) ? 1 : 0;
    sel = mp != LLONG_MAX && rank < k;
    id = sel ? ids[ms] : -1;
    sid_sh[lane] = id;
    sel_sh[lane] = sel ? 1 : 0;
  }
  __syncthreads();
  // order the selection by (dist, id); pad with (+inf, -1)
  if (w == 0) {
    int r2 = 0, nsel = 0;
    for (int j = 0; j < 64; ++j) {
      if (!sel_sh[j]) continue;
      ++nsel;
      if (key_lt(cd[j], sid_sh[j], md, id)) ++r2;
    }
    if (sel) {
      rd[r2] = md;
      ri[r2] = id;
    }
    if (lane >= nsel && lane < k) {
      rd[lane] = INFINITY;
      ri[lane] = -1;
    }
  }
  __syncthreads();
  if (dist_out && threadIdx.x < k) {
    dist_out[(long long)q * k + threadIdx.x] = rd[threadIdx.x];
    ids_out[(long long)q * k + threadIdx.x] = ri[threadIdx.x];
  }
  if (!out) return;
  if (threadIdx.x == 0) {
    for (int j = 0; j < k; ++j) {
      const float r = 1.0f / rd[j];
      rw[j] = r * r;
    }
    // numpy pairwise_sum (n < 8: sequential from -0.0; else 8 accumulators, tree, remainder), then
    // added to the reduction identity 0
    float sum;
    if (k < 8) {
      sum = -0.0f;
      for (int j = 0; j < k; ++j) sum = sum + rw[j];
    } else {
      float r0 = rw[0], r1 = rw[1], r2 = rw[2], r3 = rw[3], r4 = rw[4], r5 = rw[5], r6 = rw[6], r7 = rw[7];
      int j = 8;
      for (; j + 8 <= k; j += 8) {
        r0 = r0 + rw[j]; r1 = r1 + rw[j + 1]; r2 = r2 + rw[j + 2]; r3 = r3 + rw[j + 3];
        r4 = r4 + rw[j + 4]; r5 = r5 + rw[j + 5]; r6 = r6 + rw[j + 6]; r7 = r7 + rw[j + 7];
      }
      sum = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
      for (; j < k; ++j) sum = sum + rw[j];
    }
    sum = 0.0f + sum;
    for (int j = 0; j < k; ++j) {
      rw[j] = rw[j] / sum;
      // big_npy[ix]: ix = -1 is numpy's last row (weight 0 unless that row is non-finite)
      const long long bid = ri[j] < 0 ? ri[j] + ntotal : ri[j];
      rs[j] = slot_of_id[bid];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    float acc = vecs[rs[0] * d + c] * rw[0];
    for (int j = 1; j < k; ++j) acc = acc + vecs[rs[j] * d + c] * rw[j];
    out[(long long)q * d + c] = acc * rate + one_minus_rate * xq[c];
  }
}
#pragma clang fp contract(on)

// ------------------------------------------------------------------ launchers
size_t ivf_ws_floats(long long n, long long nlist, int nprobe) {
  return (size_t)n * nlist + (size_t)n * nprobe + 64;
}

hipError_t ivf_search(const IvfView& v, const float* x, long long n, int k, float* dist_out, long long* ids_out,
                      float rate, float one_minus_rate, float* out, float* ws, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  float* cd = ws;
  int* probe = reinterpret_cast<int*>(ws + (size_t)n * v.nlist);
  const size_t lds_c = (size_t)IVF_QB * v.d * sizeof(float);
  hipLaunchKernelGGL(k_ivf_coarse, dim3((unsigned)((v.nlist + 63) / 64), (unsigned)((n + IVF_QB - 1) / IVF_QB)),
                     dim3(256), lds_c, s, x, (int)n, v.d, v.cent, (int)v.nlist, cd);
  hipLaunchKernelGGL(k_ivf_probe, dim3((unsigned)n), dim3(64), 0, s, cd, (int)n, (int)v.nlist, v.nprobe, probe);
  const size_t lds_s = (size_t)v.d * sizeof(float) + 64 * sizeof(float) + 128 * sizeof(long long) +
                       16 * (2 * sizeof(float) + 2 * sizeof(long long));
  hipLaunchKernelGGL(k_ivf_scan, dim3((unsigned)n), dim3(256), lds_s, s, x, (int)n, v.d, v.vecs, v.off, v.ids,
                     probe, v.nprobe, k, dist_out, ids_out, v.slot_of_id, v.ntotal, rate, one_minus_rate, out);
  return hipGetLastError();
}

}  // namespace rvcx
