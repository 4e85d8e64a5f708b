// CREPE pitch estimator kernels (the "crepe" / "crepe-tiny" f0 methods): framing + per-frame normalisation,
// ReLU -> BatchNorm -> MaxPool(2) between the convs, the weighted-argmax decode and the 3-tap median / mean
// filters. The convs themselves run on the implicit-GEMM kernels (runtime_crepe.cpp).
// Reference: rvc_mlx/lib/mlx/crepe.py (CREPEModel :48-222, CREPE.get_f0 :282-325).
#include <algorithm>

#include "rvcx_kernels.h"

namespace rvcx {

namespace {
constexpr int CR_WIN = 1024, CR_HOP = 160, CR_PAD1 = 254, CR_BINS = 360;
constexpr int CR_T = 256;

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}
}  // namespace

// _frame_audio (crepe.py:327-359): frame f covers samples [f*160 - 512, f*160 + 512) of the reflect-padded
// signal; minus its mean, divided by its std when std > 1e-10 (mean and variance accumulated in fp64, the
// result rounded to fp32). Written with conv1's zero padding (crepe.py:196): row [254 | 1024 | 254].
// torch_sem: torchcrepe.preprocess instead (rvc/lib/predictors/f0.py:40-49 calls torchcrepe.predict with pad=True):
// zero padding of 512 per side, the unbiased std (n - 1), divided by max(1e-10, std).
__global__ __launch_bounds__(CR_T) void k_crepe_frames(const float* __restrict__ audio, long long n, long long f_first,
                                                        float* __restrict__ out, int ld, int torch_sem) {
  __shared__ double red[CR_T / 64];
  const long long f = f_first + blockIdx.x;
  float* row = out + (long long)blockIdx.x * ld;
  float v[CR_WIN / CR_T];
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < CR_WIN / CR_T; ++i) {
    long long src = f * CR_HOP - CR_WIN / 2 + threadIdx.x + i * CR_T;
    if (torch_sem) {
      v[i] = (src >= 0 && src < n) ? audio[src] : 0.f;
    } else {
      if (src < 0) src = -src;
      if (src > n - 1) src = 2 * (n - 1) - src;
      v[i] = audio[src];
    }
    s += v[i];
  }
  const float mean = (float)(block_sum_d(s, red) / CR_WIN);
  double s1 = 0.0;
#pragma unroll
  for (int i = 0; i < CR_WIN / CR_T; ++i) {
    v[i] = v[i] - mean;
    s1 += v[i];
  }
  const double m1 = block_sum_d(s1, red) / CR_WIN;  // np.std re-centres on the (tiny) mean of the centred frame
  double s2 = 0.0;
#pragma unroll
  for (int i = 0; i < CR_WIN / CR_T; ++i) {
    const double d = (double)v[i] - m1;
    s2 += d * d;
  }
  const float sd = (float)sqrt(block_sum_d(s2, red) / (torch_sem ? CR_WIN - 1 : CR_WIN));
  const float dv = fmaxf(sd, 1e-10f);
#pragma unroll
  for (int i = 0; i < CR_WIN / CR_T; ++i)
    row[CR_PAD1 + threadIdx.x + i * CR_T] = torch_sem ? v[i] / dv : (sd > 1e-10f ? v[i] / sd : v[i]);
  for (int i = threadIdx.x; i < CR_PAD1; i += CR_T) {
    row[i] = 0.f;
    row[CR_PAD1 + CR_WIN + i] = 0.f;
  }
}
hipError_t crepe_frames(const float* audio, long long n, long long f_first, int nf, float* out, int ld,
                        hipStream_t s, int torch_sem) {
  if (n <= (torch_sem ? 0 : CR_WIN / 2) || nf <= 0 || ld < CR_WIN + 2 * CR_PAD1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_crepe_frames, dim3(nf), dim3(CR_T), 0, s, audio, n, f_first, out, ld, torch_sem);
  return hipGetLastError();
}

// _layer tail (crepe.py:163-181): relu, BatchNorm (x - mean) * rsqrt(var + eps) * gamma + beta, max over row
// pairs. in [B][H][C] -> out [B][H/2][C]; 4 channels per thread.
__global__ void k_relu_bn_pool(const float* __restrict__ x, long long rows_out, int C, const float* __restrict__ bn,
                               float* __restrict__ y) {
  const int c4n = C >> 2;
  const long long n = rows_out * c4n;
  const float* mean = bn;
  const float* inv = bn + C;
  const float* gam = bn + 2 * C;
  const float* bet = bn + 3 * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % c4n) << 2;
    const long long r = i / c4n;
    const float4 a = *reinterpret_cast<const float4*>(x + (2 * r) * C + c);
    const float4 b = *reinterpret_cast<const float4*>(x + (2 * r + 1) * C + c);
    float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w}, o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float p = (fmaxf(av[j], 0.f) - mean[c + j]) * inv[c + j] * gam[c + j] + bet[c + j];
      const float q = (fmaxf(bv[j], 0.f) - mean[c + j]) * inv[c + j] * gam[c + j] + bet[c + j];
      o[j] = fmaxf(p, q);
    }
    *reinterpret_cast<float4*>(y + r * C + c) = make_float4(o[0], o[1], o[2], o[3]);
  }
}
hipError_t crepe_relu_bn_pool(const float* x, long long rows_in, int C, const float* bn, float* y, hipStream_t s) {
  if (C % 4 != 0 || rows_in % 2 != 0) return hipErrorInvalidValue;
  const long long n = rows_in / 2 * (C / 4);
  const long long nb = std::min<long long>((n + 255) / 256, 1 << 20);
  hipLaunchKernelGGL(k_relu_bn_pool, dim3((unsigned)nb), dim3(256), 0, s, x, rows_in / 2, C, bn, y);
  return hipGetLastError();
}

// numpy's pairwise summation order for n <= 9 (pairwise_sum: a plain loop below 8 elements, eight partial
// sums combined ((0+1)+(2+3))+((4+5)+(6+7)) then the remainder added in order)
template <class T>
__device__ __forceinline__ T np_sum9(const T* a, int n) {
  if (n < 8) {
    T r = 0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  T r = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  for (int i = 8; i < n; ++i) r += a[i];
  return r;
}

// _decode (crepe.py:387-441), one wave per frame: bins outside [lo, hi] cents zeroed, first argmax, periodicity
// = its probability, cents = sum(p * CENTS) (fp64) / sum(p) (fp32) over the +-4 bins, f0 = 10 * 2^(c/1200)
// in fp32 (numpy's float32 arithmetic, FMA contraction off).
#pragma clang fp contract(off)
__global__ void k_crepe_decode(const float* __restrict__ probs, int F, double lo, double hi, float* __restrict__ f0,
                               float* __restrict__ per) {
  const int lane = threadIdx.x & 63;
  const int fr = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (fr >= F) return;
  const float* p = probs + (long long)fr * CR_BINS;
  auto cents = [](int b) { return 20.0 * b + 1997.3794084376191; };
  auto pm = [&](int b) {
    const double cb = cents(b);
    return (cb >= lo && cb <= hi) ? p[b] : 0.f;
  };
  float best = -1.f;
  int bi = 0;
  for (int b = lane; b < CR_BINS; b += 64) {
    const float v = pm(b);
    if (v > best) {
      best = v;
      bi = b;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o);
    const int ob = __shfl_xor(bi, o);
    if (ov > best || (ov == best && ob < bi)) {
      best = ov;
      bi = ob;
    }
  }
  if (lane != 0) return;
  const int s = bi - 4 < 0 ? 0 : bi - 4, e = bi + 5 > CR_BINS ? CR_BINS : bi + 5;
  float w[9];
  double wc[9];
  for (int b = s; b < e; ++b) {
    w[b - s] = pm(b);
    wc[b - s] = (double)w[b - s] * cents(b);
  }
  const float tw = np_sum9(w, e - s);
  float c = 0.f;
  if (tw > 0.f) c = (float)(np_sum9(wc, e - s) / (double)tw);
  const float x = c / 1200.0f;
  f0[fr] = 10.0f * (float)pow(2.0, (double)x);
  per[fr] = best;
}

// get_f0 tail (crepe.py:313-323): median of 3 on the periodicity, mean of 3 on f0 (scipy.ndimage, mode
// 'reflect': x[-1] = x[0], x[F] = x[F-1]; the mean in fp64 as ndimage accumulates it), f0 = 0 where the
// filtered periodicity < threshold. Writes f0 (fp32), optionally f0 in fp64 and the filtered periodicity.
__global__ void k_crepe_filter(const float* __restrict__ f0r, const float* __restrict__ perr, int F, float thr,
                               float* __restrict__ f0, double* __restrict__ f0d, float* __restrict__ per) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F) return;
  const int a = i > 0 ? i - 1 : 0, b = i + 1 < F ? i + 1 : F - 1;
  const float p0 = perr[a], p1 = perr[i], p2 = perr[b];
  const float pmed = fmaxf(fminf(p0, p1), fminf(fmaxf(p0, p1), p2));
  float v = (float)(((double)f0r[a] + (double)f0r[i] + (double)f0r[b]) / 3.0);
  if (pmed < thr) v = 0.f;
  f0[i] = v;
  if (f0d) f0d[i] = (double)v;
  if (per) per[i] = pmed;
}
#pragma clang fp contract(on)

hipError_t crepe_decode(const float* probs, int F, double lo_cents, double hi_cents, float thr, float* f0_raw,
                        float* per_raw, float* f0, double* f0d, float* per, hipStream_t s) {
  if (F <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_crepe_decode, dim3((F + 3) / 4), dim3(256), 0, s, probs, F, lo_cents, hi_cents, f0_raw,
                     per_raw);
  hipLaunchKernelGGL(k_crepe_filter, dim3((F + 255) / 256), dim3(256), 0, s, f0_raw, per_raw, F, thr, f0, f0d, per);
  return hipGetLastError();
}

// ---- torchcrepe's decode (rvc/ semantics: rvc/lib/predictors/f0.py:40-53 -> torchcrepe.predict with its default
// decoder torchcrepe.decode.viterbi, then torchcrepe.filter.median(periodicity, 3), filter.mean(f0, 3) and
// f0[periodicity < 0.1] = 0). torchcrepe and librosa are not importable here: restated from their published source
// (torchcrepe.postprocess / decode.viterbi / convert, librosa.sequence.viterbi), parity unpinned.

constexpr int VT = 384;                 // threads of the decode blocks (six waves over the 360 bins)
constexpr int VBAND = 11;               // the transition matrix max(12 - |i - j|, 0) / row sum: +-11 bins nonzero
constexpr double V_TINY = 1.1754943508222875e-38;  // np.finfo(float32).tiny: librosa's epsilon for float32 probs

__device__ __forceinline__ float block_max_f(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < VT / 64; ++i) r = fmaxf(r, red[i]);
  return r;
}
__device__ __forceinline__ float block_sum_f(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < VT / 64; ++i) r += red[i];
  return r;
}

// postprocess + the viterbi decoder's input: bins outside [minidx, maxidx) -> -inf, softmax over the bins (the sigmoid
// outputs taken as logits, decode.viterbi), log(p + tiny) in fp32 (librosa.sequence.viterbi). One block per frame.
__global__ __launch_bounds__(VT) void k_crepe_logprob(const float* __restrict__ probs, int minidx, int maxidx,
                                                      float* __restrict__ lp) {
  __shared__ float red[VT / 64];
  const int j = threadIdx.x;
  const float* p = probs + (long long)blockIdx.x * CR_BINS;
  const bool in = j < CR_BINS && j >= minidx && j < maxidx;
  const float x = in ? p[j] : -INFINITY;
  const float mx = block_max_f(x, red);
  const float e = in ? expf(x - mx) : 0.f;
  const float sum = block_sum_f(e, red);
  if (j < CR_BINS) lp[(long long)blockIdx.x * CR_BINS + j] = logf(e / sum + 1.1754944e-38f);
}

// librosa.sequence.viterbi (_viterbi) on one block: value[t][j] = logp[t][j] + max_k (value[t-1][k] + log_trans[k][j])
// in fp64, first argmax; value[0] = logp[0] + log(1/360). log_trans[k][j] = log((12 - |k - j|) / S_k) inside the band
// (S_k the row sum) and log(tiny) outside it: the out-of-band candidates reduce to the global maximum of value[t-1]
// (its first index) plus log(tiny), which wins only when that index lies outside j's band. ptr [F][360]; the last
// state is the first argmax of value[F-1], then the back-pointers are followed (one lane).
// torchcrepe.predict decodes each batch of `seg` frames (rvc/lib/predictors/f0.py:38-49: batch_size 512) on its own --
// postprocess, and so decode.viterbi, runs once per batch from the uniform initial state -- so block b decodes frames
// [b seg, min(F, (b + 1) seg)) as an independent sequence (the segments also run in parallel).
__global__ __launch_bounds__(VT) void k_crepe_viterbi(const float* __restrict__ lp_all, int F_all, int seg,
                                                      int* __restrict__ ptr_all, int* __restrict__ bins_all) {
  const int t0 = blockIdx.x * seg;
  if (t0 >= F_all) return;
  const int F = min(seg, F_all - t0);
  const float* lp = lp_all + (long long)t0 * CR_BINS;
  int* ptr = ptr_all + (long long)t0 * CR_BINS;
  int* bins = bins_all + t0;
  __shared__ double val[2][CR_BINS];
  __shared__ double rv[VT / 64];
  __shared__ int ri[VT / 64];
  const int j = threadIdx.x, lane = j & 63, w = j >> 6;
  const bool act = j < CR_BINS;
  double lt[2 * VBAND + 1];  // log_trans[k = j - 11 + d][j]
#pragma unroll
  for (int d = 0; d <= 2 * VBAND; ++d) {
    const int k = j - VBAND + d;
    double sk = 0.0;
    for (int e = -VBAND; e <= VBAND; ++e)
      if (k + e >= 0 && k + e < CR_BINS) sk += (double)(12 - abs(e));
    lt[d] = (k >= 0 && k < CR_BINS) ? log((double)(12 - abs(d - VBAND)) / sk + V_TINY) : -INFINITY;
  }
  const double lout = log(V_TINY);
  const double lpi = log(1.0 / CR_BINS + V_TINY);
  // first argmax of the block's values: (value, index) pairs, larger value or equal value with the smaller index
  auto argmax = [&](double v, int i, double& bv, int& bi) {
    for (int o = 32; o > 0; o >>= 1) {
      const double ov = __shfl_xor(v, o);
      const int oi = __shfl_xor(i, o);
      if (ov > v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
      }
    }
    if (lane == 0) {
      rv[w] = v;
      ri[w] = i;
    }
    __syncthreads();
    bv = rv[0];
    bi = ri[0];
    for (int q = 1; q < VT / 64; ++q)
      if (rv[q] > bv || (rv[q] == bv && ri[q] < bi)) {
        bv = rv[q];
        bi = ri[q];
      }
    __syncthreads();
  };
  if (act) val[0][j] = (double)lp[j] + lpi;
  float nxt = (act && F > 1) ? lp[CR_BINS + j] : 0.f;
  __syncthreads();
  for (int t = 1; t < F; ++t) {
    const double* vp = val[(t - 1) & 1];
    double gm;
    int gk;
    argmax(act ? vp[j] : -INFINITY, act ? j : CR_BINS, gm, gk);
    const float cur = nxt;
    if (act && t + 1 < F) nxt = lp[(long long)(t + 1) * CR_BINS + j];
    if (act) {
      double best = -INFINITY;
      int arg = 0;
#pragma unroll
      for (int d = 0; d <= 2 * VBAND; ++d) {
        const int k = j - VBAND + d;
        if (k >= 0 && k < CR_BINS) {
          const double c = vp[k] + lt[d];
          if (c > best) {
            best = c;
            arg = k;
          }
        }
      }
      if (gk < j - VBAND || gk > j + VBAND) {
        const double c = gm + lout;
        if (c > best || (c == best && gk < arg)) {
          best = c;
          arg = gk;
        }
      }
      val[t & 1][j] = (double)cur + best;
      ptr[(long long)t * CR_BINS + j] = arg;
    }
    __syncthreads();
  }
  double gm;
  int st;
  argmax(act ? val[(F - 1) & 1][j] : -INFINITY, act ? j : CR_BINS, gm, st);
  __threadfence();
  __syncthreads();
  if (j == 0) {
    for (int t = F - 1; t > 0; --t) {
      bins[t] = st;
      st = __hip_atomic_load(&ptr[(long long)t * CR_BINS + st], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    bins[0] = st;
  }
}

// torchcrepe.convert.bins_to_frequency (cents = 20 bin + 1997.3794084376191 in fp32, plus the dither the caller
// passes -- torchcrepe draws it from scipy.stats.triang on [-20, 20] cents; NULL: none), f = 10 * 2^(cents / 1200);
// periodicity = the sigmoid output at the chosen bin (postprocess). Then f0.py:50-52: median of 3 on the periodicity
// and mean of 3 on f0 with torchcrepe.filter's edges (the window clipped to the 2 samples inside: the lower of the two
// / their mean), f0 = 0 where the filtered periodicity < thr.
__global__ void k_crepe_rvc_pitch(const float* __restrict__ probs, const int* __restrict__ bins,
                                  const float* __restrict__ dither, int F, float* __restrict__ f0r,
                                  float* __restrict__ perr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F) return;
  const int b = bins[i];
  float c = (float)(20 * b) + 1997.3794084376191f;
  if (dither) c = c + dither[i];
  f0r[i] = 10.0f * exp2f(c / 1200.0f);
  perr[i] = probs[(long long)i * CR_BINS + b];
}
__global__ void k_crepe_rvc_filter(const float* __restrict__ f0r, const float* __restrict__ perr, int F, float thr,
                                   float* __restrict__ f0, double* __restrict__ f0d, float* __restrict__ per) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F) return;
  float pmed, v;
  if (F == 1) {
    pmed = perr[0];
    v = f0r[0];
  } else if (i == 0 || i == F - 1) {
    const int o = i == 0 ? 1 : F - 2;
    pmed = fminf(perr[i], perr[o]);
    v = (i == 0 ? f0r[0] + f0r[1] : f0r[F - 2] + f0r[F - 1]) / 2.0f;
  } else {
    const float p0 = perr[i - 1], p1 = perr[i], p2 = perr[i + 1];
    pmed = fmaxf(fminf(p0, p1), fminf(fmaxf(p0, p1), p2));
    v = ((f0r[i - 1] + f0r[i]) + f0r[i + 1]) / 3.0f;
  }
  if (pmed < thr) v = 0.f;
  f0[i] = v;
  if (f0d) f0d[i] = (double)v;
  if (per) per[i] = pmed;
}

hipError_t crepe_decode_viterbi(const float* probs, int F, int minidx, int maxidx, const float* dither, float thr,
                                float* lp, int* ptr, int* bins, float* f0_raw, float* per_raw, float* f0, double* f0d,
                                float* per, hipStream_t s, int seg) {
  if (F <= 0) return hipSuccess;
  if (minidx < 0 || maxidx > CR_BINS || minidx >= maxidx || seg < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_crepe_logprob, dim3(F), dim3(VT), 0, s, probs, minidx, maxidx, lp);
  hipLaunchKernelGGL(k_crepe_viterbi, dim3((F + seg - 1) / seg), dim3(VT), 0, s, lp, F, seg, ptr, bins);
  hipLaunchKernelGGL(k_crepe_rvc_pitch, dim3((F + 255) / 256), dim3(256), 0, s, probs, bins, dither, F, f0_raw, per_raw);
  hipLaunchKernelGGL(k_crepe_rvc_filter, dim3((F + 255) / 256), dim3(256), 0, s, f0_raw, per_raw, F, thr, f0, f0d, per);
  return hipGetLastError();
}

}  // namespace rvcx
