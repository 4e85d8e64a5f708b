// Streaming (realtime) conversion kernels: B independent streams of identical geometry per launch
// (blockIdx.y = stream). Semantics of rvc/realtime/core.py (Realtime.inference :217-326,
// VoiceChanger.process_audio :404-451) and rvc/realtime/pipeline.py (get_f0 :122-212,
// voice_conversion :214-334). Buffers are ping-ponged (old -> new) so a circular write is a plain
// out-of-place copy with no intra-kernel read/write race.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rvcx_kernels.h"

namespace rvcx {

namespace {
constexpr int RT_TB = 256;

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0) {
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
    red[0] = t;
  }
  __syncthreads();
  t = red[0];
  __syncthreads();
  return t;
}
}  // namespace

// torchaudio sinc resample (polyphase FIR): y[f*new + p] = sum_k xpad[f*orig + k] * ker[p][k],
// xpad = zero-padded x shifted by `width` (functional.py _apply_sinc_resample_kernel). One thread per
// output sample; an optional per-stream multiplier `pre` is applied to x first (core.py:324:
// resample_out(audio_model * sqrt(vol))).
__global__ void k_rt_resample(const float* __restrict__ x, long long ldx, int n_in, const float* __restrict__ ker,
                              int K, int width, int orig, int nw, float* __restrict__ y, long long ldy, int n_out,
                              const float* __restrict__ pre) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_out) return;
  const int f = j / nw, p = j - f * nw;
  const float* xb = x + b * ldx;
  const float* kp = ker + (long long)p * K;
  const float m = pre ? pre[b] : 1.f;
  float acc = 0.f;
  const int base = f * orig - width;
  for (int k = 0; k < K; ++k) {
    const int i = base + k;
    if (i >= 0 && i < n_in) acc = fmaf(pre ? xb[i] * m : xb[i], kp[k], acc);
  }
  y[b * ldy + j] = acc;
}

// Realtime.inference input stage (core.py:232-267): circular_write(in16, audio_buffer);
// vol = sqrt(mean(audio_buffer^2)); gate = !(vol < sensitivity); if gate: circular_write(in16, convert_buffer).
// One block per stream. old/new buffers are distinct (ping-pong).
__global__ void __launch_bounds__(RT_TB) k_rt_ingest(const float* __restrict__ in16, int n16,
                                                     const float* __restrict__ abuf_old, float* __restrict__ abuf_new,
                                                     int na, const float* __restrict__ cbuf_old,
                                                     float* __restrict__ cbuf_new, int nc, double sensitivity,
                                                     float* __restrict__ vol, float* __restrict__ volsq,
                                                     int* __restrict__ gate) {
  __shared__ float red[RT_TB / 64];
  __shared__ int g_sh;
  const int b = blockIdx.x;
  const float* in = in16 + (long long)b * n16;
  const float* ao = abuf_old + (long long)b * na;
  float* an = abuf_new + (long long)b * na;
  float acc = 0.f;
  for (int i = threadIdx.x; i < na; i += blockDim.x) {
    const float v = i < na - n16 ? ao[i + n16] : in[i - (na - n16)];
    an[i] = v;
    acc = fmaf(v, v, acc);
  }
  const float tot = block_sum(acc, red);
  if (threadIdx.x == 0) {
    const float ms = tot / (float)na;
    const float v = sqrtf(ms);
    vol[b] = v;
    volsq[b] = sqrtf(v);  // torch.sqrt(vol_t): the output scale (core.py:324)
    const int g = !((double)v < sensitivity);
    gate[b] = g;
    g_sh = g;
  }
  __syncthreads();
  const int g = g_sh;
  const float* co = cbuf_old + (long long)b * nc;
  float* cn = cbuf_new + (long long)b * nc;
  for (int i = threadIdx.x; i < nc; i += blockDim.x)
    cn[i] = g ? (i < nc - n16 ? co[i + n16] : in[i - (nc - n16)]) : co[i];
}

// Realtime_Pipeline.get_f0 tail (rvc/realtime/pipeline.py:185-210): f0 *= 2^(key/12) (numpy fp64), then
// torch float32: mel = 1127 log(1 + f0/700); coarse = round(clip((mel - 50) * 254 / 1050 + 1, 1, 255));
// circular_write into the pitch / pitchf buffers (old -> new). One block per stream.
#pragma clang fp contract(off)
__global__ void k_rt_pitch(const double* __restrict__ f0, int F, const double* __restrict__ factor,
                           const int* __restrict__ pold, int* __restrict__ pnew, const float* __restrict__ fold,
                           float* __restrict__ fnew, int nbuf) {
  const int b = blockIdx.x;
  const double fac = factor[b];
  for (int i = threadIdx.x; i < nbuf; i += blockDim.x) {
    int pc;
    float pf;
    if (i < nbuf - F) {
      pc = pold[(long long)b * nbuf + i + F];
      pf = fold[(long long)b * nbuf + i + F];
    } else {
      const double fd = f0[(long long)b * F + (i - (nbuf - F))] * fac;
      pf = (float)fd;
      float mel = 1127.0f * logf(1.0f + pf / 700.0f);
      mel = (mel - 50.0f) * 254.0f / 1050.0f + 1.0f;
      mel = fminf(fmaxf(mel, 1.0f), 255.0f);
      pc = (int)rintf(mel);
    }
    pnew[(long long)b * nbuf + i] = pc;
    fnew[(long long)b * nbuf + i] = pf;
  }
}

// feats (retrieved) / feats0 [B][L][D] -> phone [B][T][D]: nearest x2 upsample of the L rows plus the
// repeated last frame (pipeline.py:261: cat(feats, feats[:, -1:])), [:p_len]; protect blend against
// pitchf (the last T entries of the pitchf buffer, times formant/return = `pscale`).
__global__ void k_rt_up2(const float* __restrict__ feats, const float* __restrict__ feats0, int L, int D,
                         float* __restrict__ phone, int T, const float* __restrict__ pitchf_buf, int nbuf, float pscale,
                         float protect, int use_protect, int* __restrict__ pitch_out, const int* __restrict__ pitch_buf,
                         float* __restrict__ pitchf_out) {
  const int b = blockIdx.y;
  const long long n = (long long)T * D;
  const float* fb = feats + (long long)b * L * D;
  const float* f0b = feats0 + (long long)b * L * D;
  const float* pfb = pitchf_buf + (long long)b * nbuf + (nbuf - T);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int t = (int)(i / D), c = (int)(i % D);
    const int src = (t >> 1) < L ? (t >> 1) : L - 1;
    const float f = fb[(long long)src * D + c];
    float v = f;
    if (use_protect) {
      const float pf = pfb[t] * pscale;
      const float p = pf < 1.f ? protect : (pf > 0.f ? 1.f : pf);
      v = f * p + f0b[(long long)src * D + c] * (1.f - p);
    }
    phone[(long long)b * n + i] = v;
    if (c == 0) {
      pitch_out[(long long)b * T + t] = pitch_buf[(long long)b * nbuf + (nbuf - T) + t];
      pitchf_out[(long long)b * T + t] = pfb[t] * pscale;
    }
  }
}

// clip(x, -1, 1) of RealtimeVoiceConverter.inference (pipeline.py:93). Silent hops are zeroed in k_rt_sola.
__global__ void k_rt_clip(float* __restrict__ x, long long ld, int n) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[b * ld + i];
  x[b * ld + i] = fminf(fmaxf(v, -1.0f), 1.0f);
}

// VoiceChanger.process_audio (core.py:404-451) for one stream per block:
// cor_nom[k] = sum_i a[k+i] sb[i]; cor_den[k] = sqrt(sum_i a[k+i]^2 + 1e-8); off = first argmax(nom/den);
// audio = a[off:]; audio[:cf] = audio[:cf]*fade_in + sb*fade_out; sb = audio[block:block+cf]; out = audio[:block].
// Silent hops (gate 0) see a zero `a` (core.py:285-288: zeros of the model output's shape).
__global__ void __launch_bounds__(RT_TB) k_rt_sola(const float* __restrict__ audio, long long lda,
                                                   const float* __restrict__ volsq, const int* __restrict__ gate,
                                                   float* __restrict__ sola_buf, int cf, int search,
                                                   const float* __restrict__ fade_in, float* __restrict__ out,
                                                   int block, int* __restrict__ offs) {
  extern __shared__ float sm[];
  float* ci = sm;                  // [cf + search]
  float* sb = ci + cf + search;    // [cf]
  float* ratio = sb + cf;          // [search + 1]
  const int b = blockIdx.x;
  const float* a = audio + b * lda;
  const int g = gate[b];
  const float m = volsq ? volsq[b] : 1.f;  // null when the output resample already applied sqrt(vol)
  float* sbg = sola_buf + (long long)b * cf;
  for (int i = threadIdx.x; i < cf + search; i += blockDim.x) ci[i] = g ? a[i] * m : 0.f;
  for (int i = threadIdx.x; i < cf; i += blockDim.x) sb[i] = sbg[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int k = w; k <= search; k += nw) {
    float nom = 0.f, den = 0.f;
    for (int i = lane; i < cf; i += 64) {
      const float v = ci[k + i];
      nom = fmaf(v, sb[i], nom);
      den = fmaf(v, v, den);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      nom += __shfl_xor(nom, o, 64);
      den += __shfl_xor(den, o, 64);
    }
    if (lane == 0) ratio[k] = nom / sqrtf(den + 1e-8f);
  }
  __syncthreads();
  __shared__ int off_sh;
  if (threadIdx.x == 0) {
    int best = 0;
    float bv = ratio[0];
    for (int k = 1; k <= search && bv == bv; ++k)  // torch.argmax: first maximum, NaN counts as maximal
      if (ratio[k] > bv || ratio[k] != ratio[k]) {
        bv = ratio[k];
        best = k;
      }
    off_sh = best;
    if (offs) offs[b] = best;
  }
  __syncthreads();
  const int off = off_sh;
  float* ob = out + (long long)b * block;
  for (int j = threadIdx.x; j < block; j += blockDim.x) {
    float v = g ? a[off + j] * m : 0.f;
    if (j < cf) v = v * fade_in[j] + sb[j] * (1.0f - fade_in[j]);
    ob[j] = v;
  }
  __syncthreads();  // every sb read above precedes the overwrite below
  for (int j = threadIdx.x; j < cf; j += blockDim.x) {
    const int idx = block + j;
    float v = g ? a[off + idx] * m : 0.f;
    if (idx < cf) v = v * fade_in[idx] + sb[idx] * (1.0f - fade_in[idx]);
    sbg[j] = v;
  }
}
#pragma clang fp contract(on)

// ------------------------------------------------------------------ launchers
hipError_t rt_resample(const float* x, long long ldx, int n_in, const float* ker, int K, int width, int orig, int nw,
                       float* y, long long ldy, int n_out, const float* pre, int B, hipStream_t s) {
  hipLaunchKernelGGL(k_rt_resample, dim3((n_out + RT_TB - 1) / RT_TB, B), dim3(RT_TB), 0, s, x, ldx, n_in, ker, K,
                     width, orig, nw, y, ldy, n_out, pre);
  return hipGetLastError();
}

hipError_t rt_ingest(const float* in16, int n16, const float* abuf_old, float* abuf_new, int na, const float* cbuf_old,
                     float* cbuf_new, int nc, double sensitivity, float* vol, float* volsq, int* gate, int B,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_rt_ingest, dim3(B), dim3(RT_TB), 0, s, in16, n16, abuf_old, abuf_new, na, cbuf_old, cbuf_new,
                     nc, sensitivity, vol, volsq, gate);
  return hipGetLastError();
}

hipError_t rt_pitch(const double* f0, int F, const double* factor, const int* pold, int* pnew, const float* fold,
                    float* fnew, int nbuf, int B, hipStream_t s) {
  hipLaunchKernelGGL(k_rt_pitch, dim3(B), dim3(RT_TB), 0, s, f0, F, factor, pold, pnew, fold, fnew, nbuf);
  return hipGetLastError();
}

hipError_t rt_up2(const float* feats, const float* feats0, int L, int D, float* phone, int T, const float* pitchf_buf,
                  int nbuf, float pscale, float protect, int use_protect, int* pitch_out, const int* pitch_buf,
                  float* pitchf_out, int B, hipStream_t s) {
  const long long n = (long long)T * D;
  const unsigned gx = (unsigned)std::min<long long>((n + RT_TB - 1) / RT_TB, 1024);
  hipLaunchKernelGGL(k_rt_up2, dim3(gx, B), dim3(RT_TB), 0, s, feats, feats0, L, D, phone, T, pitchf_buf, nbuf,
                     pscale, protect, use_protect, pitch_out, pitch_buf, pitchf_out);
  return hipGetLastError();
}

hipError_t rt_clip(float* x, long long ld, int n, int B, hipStream_t s) {
  hipLaunchKernelGGL(k_rt_clip, dim3((n + RT_TB - 1) / RT_TB, B), dim3(RT_TB), 0, s, x, ld, n);
  return hipGetLastError();
}

hipError_t rt_sola(const float* audio, long long lda, const float* volsq, const int* gate, float* sola_buf, int cf,
                   int search, const float* fade_in, float* out, int block, int* offs, int B, hipStream_t s) {
  const size_t lds = sizeof(float) * ((size_t)cf + search + cf + search + 1);
  hipLaunchKernelGGL(k_rt_sola, dim3(B), dim3(RT_TB), lds, s, audio, lda, volsq, gate, sola_buf, cf, search, fade_in,
                     out, block, offs);
  return hipGetLastError();
}

}  // namespace rvcx
