// Non-GEMM kernels of the RVC path: NSF source (SineGen), noise convs, conv_post, norms,
// softmax with relative-position bands, layout transforms, RNG, RMVPE front/back end.
// Elementwise / reduction work here is HBM- or latency-bound; every kernel keeps channels
// contiguous (time-major rows) so a wave reads whole 128-B lines.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "dd_math.h"
#include "rvcx_kernels.h"

namespace rvcx {

namespace {

constexpr int TB = 256;
typedef float f32x4v __attribute__((ext_vector_type(4)));

inline unsigned nblocks(long long n, int per = TB) {
  long long b = (n + per - 1) / per;
  if (b > 65535LL * 32) b = 65535LL * 32;
  return (unsigned)(b < 1 ? 1 : b);
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- Philox4x32-10 (counter-based; one 128-bit block per 4 normals)
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
__device__ __forceinline__ float normal_at(uint64_t seed, uint64_t idx) {
  uint32_t c[4] = {(uint32_t)(idx >> 1), (uint32_t)(idx >> 33), 0x52564358u, 0u};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float u1 = ((c[0] >> 8) + 1) * (1.0f / 16777217.0f);
  const float u2 = (c[1] >> 8) * (1.0f / 16777216.0f);
  const float r = sqrtf(-2.f * logf(u1));
  const float th = 6.283185307179586f * u2;
  return (idx & 1) ? r * sinf(th) : r * cosf(th);
}

}  // namespace

// ------------------------------------------------------------------ simple maps
__global__ void k_fill(float* p, float v, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = v;
}
hipError_t fill(float* p, float v, long long n, hipStream_t s) {
  hipLaunchKernelGGL(k_fill, dim3(nblocks(n)), dim3(TB), 0, s, p, v, n);
  return hipGetLastError();
}

__global__ void k_randn(float* y, long long n, uint64_t seed, uint64_t off) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] = normal_at(seed, off + i);
}
hipError_t randn(float* y, long long n, uint64_t seed, uint64_t offset, hipStream_t s) {
  hipLaunchKernelGGL(k_randn, dim3(nblocks(n)), dim3(TB), 0, s, y, n, seed, offset);
  return hipGetLastError();
}

__global__ void k_act(float* x, long long n, int act, float slope) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float v = x[i];
    switch (act) {
      case ACT_LRELU: v = v > 0.f ? v : v * slope; break;
      case ACT_RELU: v = v > 0.f ? v : 0.f; break;
      case ACT_GELU: v = 0.5f * v * (1.f + erff(v * 0.70710678118654752440f)); break;
      case ACT_TANH: v = tanhf(v); break;
      case ACT_SIGMOID: v = 1.f / (1.f + expf(-v)); break;
      default: break;
    }
    x[i] = v;
  }
}
hipError_t act_inplace(float* x, long long n, int act, float slope, hipStream_t s) {
  hipLaunchKernelGGL(k_act, dim3(nblocks(n)), dim3(TB), 0, s, x, n, act, slope);
  return hipGetLastError();
}

__global__ void k_affine(float* x, long long n, float a, float b) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    x[i] = x[i] * a + b;
}
hipError_t affine_inplace(float* x, long long n, float a, float b, hipStream_t s) {
  hipLaunchKernelGGL(k_affine, dim3(nblocks(n)), dim3(TB), 0, s, x, n, a, b);
  return hipGetLastError();
}

// [B][C][T] -> [B][T][C] and back, 32x32 LDS tiles
__global__ void k_tr(const float* x, float* y, int R, int Cc, long long ld_in, long long ld_out, long long bs_in,
                     long long bs_out) {
  __shared__ float t[32][33];
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const float* X = x + b * bs_in;
  float* Y = y + b * bs_out;
  for (int i = threadIdx.y; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + threadIdx.x;
    if (r < R && c < Cc) t[i][threadIdx.x] = X[(long long)r * ld_in + c];
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + threadIdx.x;
    if (r < R && c < Cc) Y[(long long)c * ld_out + r] = t[threadIdx.x][i];
  }
}
hipError_t transpose_bct_btc(const float* x, float* y, int B, int C, int T, hipStream_t s) {
  dim3 g((T + 31) / 32, (C + 31) / 32, B);
  hipLaunchKernelGGL(k_tr, g, dim3(32, 8), 0, s, x, y, C, T, (long long)T, (long long)C, (long long)C * T,
                     (long long)C * T);
  return hipGetLastError();
}
hipError_t transpose_btc_bct(const float* x, float* y, int B, int T, int C, int ldx, hipStream_t s) {
  dim3 g((C + 31) / 32, (T + 31) / 32, B);
  hipLaunchKernelGGL(k_tr, g, dim3(32, 8), 0, s, x, y, T, C, (long long)ldx, (long long)T, (long long)T * ldx,
                     (long long)C * T);
  return hipGetLastError();
}

__global__ void k_flip(const float* x, float* y, long long rows, int C) {
  const long long n = rows * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / C;
    const int c = (int)(i - r * C);
    y[i] = x[r * C + (C - 1 - c)];
  }
}
hipError_t channel_flip(const float* x, float* y, int rows, int C, hipStream_t s) {
  hipLaunchKernelGGL(k_flip, dim3(nblocks((long long)rows * C)), dim3(TB), 0, s, x, y, (long long)rows, C);
  return hipGetLastError();
}

__global__ void k_gather(const float* table, int ld, const int32_t* idx, float* y, long long rows, int C) {
  const long long n = rows * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / C;
    const int c = (int)(i - r * C);
    y[i] = table[(long long)idx[r] * ld + c];
  }
}
hipError_t gather_rows(const float* table, int ld_table, const int32_t* idx, float* y, int rows, int C,
                       hipStream_t s) {
  hipLaunchKernelGGL(k_gather, dim3(nblocks((long long)rows * C)), dim3(TB), 0, s, table, ld_table, idx, y,
                     (long long)rows, C);
  return hipGetLastError();
}

__global__ void k_seqmask(const int32_t* len, float* mask, int B, int T) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B * T) mask[i] = (i % T) < len[i / T] ? 1.f : 0.f;
}
hipError_t seq_mask(const int32_t* lengths, float* mask, int B, int T, hipStream_t s) {
  hipLaunchKernelGGL(k_seqmask, dim3(nblocks((long long)B * T)), dim3(TB), 0, s, lengths, mask, B, T);
  return hipGetLastError();
}

// ------------------------------------------------------------------ LayerNorm over rows (one wave per row)
__global__ void k_layernorm(const float* x, const float* r, float* y, const float* gamma, const float* beta,
                            int rows, int D, float eps, const float* mask) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= rows) return;
  const float* xr = x + (long long)wave * D;
  const float* rr = r ? r + (long long)wave * D : nullptr;
  float v[16];
  float s = 0.f;
  const int per = (D + 63) / 64;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int c = lane + j * 64;
    float t = 0.f;
    if (j < per && c < D) {
      t = xr[c];
      if (rr) t = t + rr[c];
    }
    v[j] = t;
    s += t;
  }
  const float mean = warp_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int c = lane + j * 64;
    if (j < per && c < D) {
      const float d = v[j] - mean;
      q += d * d;
    }
  }
  const float var = warp_sum(q) / (float)D;
  const float rstd = 1.f / sqrtf(var + eps);
  const float mk = mask ? mask[wave] : 1.f;
  float* yr = y + (long long)wave * D;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int c = lane + j * 64;
    if (j < per && c < D) {
      float o = (v[j] - mean) * rstd * gamma[c] + beta[c];
      if (mask) o *= mk;
      yr[c] = o;
    }
  }
}
hipError_t layernorm_rows(const float* x, const float* r, float* y, const float* gamma, const float* beta,
                          int rows, int D, float eps, const float* mask, hipStream_t s) {
  if (D > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_layernorm, dim3((rows + 3) / 4), dim3(256), 0, s, x, r, y, gamma, beta, rows, D, eps, mask);
  return hipGetLastError();
}

// ------------------------------------------------------------------ WaveNet gate
__global__ void k_gate(const float* xin, int ldx, const float* g, long long g_bs, float* acts, int B, int T,
                       int H) {
  const long long n = (long long)B * T * H;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % H);
    const long long bt = i / H;
    const int b = (int)(bt / T);
    const float* xr = xin + bt * ldx;
    const float* gb = g + b * g_bs;
    const float a = xr[c] + gb[c];
    const float z = xr[H + c] + gb[H + c];
    acts[i] = tanhf(a) * (1.f / (1.f + expf(-z)));
  }
}
hipError_t gate_tanh_sigmoid(const float* xin, int ldx, const float* g, long long g_bs, float* acts, int B,
                             int T, int H, hipStream_t s) {
  hipLaunchKernelGGL(k_gate, dim3(nblocks((long long)B * T * H)), dim3(TB), 0, s, xin, ldx, g, g_bs, acts, B, T, H);
  return hipGetLastError();
}


// ------------------------------------------------------------------ ConvTranspose2d 3x3 s2 p1 op1 as a 2x2-tap phase conv
// w [C][co][3][3] (torch layout) -> [tap = 2 dh + dw][4 co][C]: virtual column (ph 2 + pw) co + o of input offset (dh,
// dw) takes kernel tap (kmap[ph][dh], kmap[pw][dw]) with kmap = {{1, -1}, {2, 0}} (-1: no tap, zero); the runtime's
// packing of the U-Net decoder's up-conv (runtime_fe.cpp, BN scale 1)
__global__ void k_upconv_pack(const float* __restrict__ w, int C, int co, float* __restrict__ out) {
  const long long total = 4LL * 4 * co * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int ii = (int)(i % C);
    const long long r = i / C;
    const int n = (int)(r % (4 * co)), tap = (int)(r / (4 * co));
    const int dh = tap >> 1, dw = tap & 1, ph = n / (2 * co), pw = (n / co) & 1, o = n % co;
    const int kmap[2][2] = {{1, -1}, {2, 0}};
    const int kh = kmap[ph][dh], kw = kmap[pw][dw];
    out[i] = (kh < 0 || kw < 0) ? 0.f : w[(((long long)ii * co + o) * 3 + kh) * 3 + kw];
  }
}

hipError_t upconv_phase_pack(const float* w, int C, int co, float* out, hipStream_t s) {
  const long long total = 16LL * co * C;
  hipLaunchKernelGGL(k_upconv_pack, dim3((unsigned)std::min<long long>((total + 255) / 256, 8192)), dim3(256), 0, s,
                     w, C, co, out);
  return hipGetLastError();
}

// ------------------------------------------------------------------ NSF noise conv, accumulated into y
// One thread per 4 consecutive channels of one output row: the row's kk = taps * stride source samples are
// read once for the 4 channels, y is read and written as one float4 (coalesced along the row). The weights are
// staged once per block into LDS as [q][C] so each (q, 4 channels) is one 16-byte read. The per-channel sum runs
// over q in order as an fma chain, then + bias, then + y (the separate-launch order it replaces).
// STORE: y = sum + bias (the noise branch computed ahead into its own buffer, added later as the ConvTranspose's
// residual: y_up + (sum + bias), the same single addition)
constexpr int NOISE_LDS_FLOATS = 4096;
template <bool STORE>
__global__ __launch_bounds__(256) void k_noise_add(const float* __restrict__ har, long long har_bs, int stride,
                                                   int taps, const float* __restrict__ wf,
                                                   const float* __restrict__ nb, float* __restrict__ y, int B, int T,
                                                   int C) {
  __shared__ __attribute__((aligned(16))) float wq[NOISE_LDS_FLOATS];
  const int kk = taps * stride;
  for (int i = threadIdx.x; i < kk * C; i += blockDim.x) {
    const int q = i / C, c = i - q * C;
    const int tap = q / stride, j = q - tap * stride;
    wq[i] = wf[((long long)tap * C + c) * stride + j];
  }
  __syncthreads();
  // 32-bit index arithmetic (the launcher checks B * T * C / 4 < 2^31): 64-bit divisions cost more than the
  // whole per-element body
  const unsigned c4n = (unsigned)C >> 2;
  const unsigned n = (unsigned)B * (unsigned)T * c4n;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned bt = i / c4n;
    const int c = (int)(i - bt * c4n) << 2;
    const unsigned b = bt / (unsigned)T;
    const long long t = bt - b * (unsigned)T;
    const float* x = har + b * har_bs + t * stride;
    float xs[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) xs[q] = q < kk ? x[q] : 0.f;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (q < kk) {
        const float4 w = *reinterpret_cast<const float4*>(wq + q * C + c);
        acc.x = fmaf(w.x, xs[q], acc.x);
        acc.y = fmaf(w.y, xs[q], acc.y);
        acc.z = fmaf(w.z, xs[q], acc.z);
        acc.w = fmaf(w.w, xs[q], acc.w);
      }
    }
    float4* yp = reinterpret_cast<float4*>(y + (long long)bt * C + c);
    if constexpr (STORE) {
      *yp = make_float4(acc.x + nb[c], acc.y + nb[c + 1], acc.z + nb[c + 2], acc.w + nb[c + 3]);
    } else {
      float4 v = *yp;
      v.x = v.x + (acc.x + nb[c]);
      v.y = v.y + (acc.y + nb[c + 1]);
      v.z = v.z + (acc.z + nb[c + 2]);
      v.w = v.w + (acc.w + nb[c + 3]);
      *yp = v;
    }
  }
}
hipError_t noise_conv_add(const float* har, long long har_bs, int stride, int taps, const float* wf, const float* nb,
                          float* y, int B, int T, int C, hipStream_t s, bool store) {
  if (C % 4 != 0 || taps * stride > 16 || taps * stride < 1 || (reinterpret_cast<uintptr_t>(y) & 15) != 0 ||
      (long long)B * T * (C / 4) >= (1LL << 31) || taps * stride * C > NOISE_LDS_FLOATS)
    return hipErrorInvalidValue;
  // grid-stride over a capped grid: each block stages the weights once
  hipLaunchKernelGGL(store ? k_noise_add<true> : k_noise_add<false>,
                     dim3(std::min(nblocks((long long)B * T * (C / 4)), store ? 512u : 4096u)), dim3(TB), 0, s, har,
                     har_bs, stride,
                     taps, wf, nb, y, B, T, C);
  return hipGetLastError();
}

// ------------------------------------------------------------------ feature x2 upsample + protect blend
// pipeline.py:344-362: feats = interpolate(x2, nearest); pitchff = 1 if pitchf > 0 else protect;
// feats = feats * pitchff + feats0 * (1 - pitchff)   (feats0 == feats without index retrieval).
// x2 nearest upsample + protect blend (pipeline.py:344-362): feats = retrieved (or raw) features,
// feats0 = raw features; v = feats * p + feats0 * (1 - p) with each product and the sum rounded (torch).
#pragma clang fp contract(off)
__global__ void k_up2(const float* feats, const float* feats0, int L, int D, float* out, int T, const float* pitchf,
                      float protect) {
  const long long n = (long long)T * D;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int t = (int)(i / D), c = (int)(i % D);
    const int src = t >> 1 < L ? t >> 1 : L - 1;
    const float f = feats[(long long)src * D + c];
    float v = f;
    if (pitchf) {
      const float pf = pitchf[t];
      const float p = pf < 1.f ? protect : (pf > 0.f ? 1.f : pf);
      v = f * p + feats0[(long long)src * D + c] * (1.f - p);
    }
    out[i] = v;
  }
}
#pragma clang fp contract(on)
hipError_t upsample2_protect(const float* feats, const float* feats0, int L, int D, float* out, int T,
                             const float* pitchf, float protect, hipStream_t s) {
  hipLaunchKernelGGL(k_up2, dim3(nblocks((long long)T * D)), dim3(TB), 0, s, feats, feats0, L, D, out, T, pitchf,
                     protect);
  return hipGetLastError();
}

// ------------------------------------------------------------------ NSF harmonic source (SineGen, harmonic_num=0)
// generators/hifigan.py:156-228 + hifigan_nsf.py:48-52. Phase carry: rem[l] = fmod(f0[l]/sr*upp + .5, 1) - .5,
// cumsum accumulated in fp64 and rounded per element (torch CPU cumsum acc_type<float> = double), then fmod 1.
// SineGen phase prefix (generators/hifigan.py:156-228): rem[l] = fmod(f0[l]/sr*upp + 0.5, 1) - 0.5,
// cum = fmod(cumsum(rem), 1) with the cumsum accumulated in double (torch CPU acc type).
// Parallel scan, bit-identical to torch's sequential double loop: for f0 >= 0, inc + 0.5 >= 0.5 so every
// rem is a multiple of 2^-24 with |rem| <= 0.5, and any partial sum of fewer than 2^28 of them is a
// multiple of 2^-24 below 2^27 in magnitude (51 significant bits): every double addition is exact and the
// summation order cannot change a bit. One block per batch row: each thread sums a contiguous segment, a
// block scan of the segment sums gives each segment's start, and the segment is re-walked to emit
// fmod((float)acc, 1).
constexpr int SINE_T = 1024;
__global__ __launch_bounds__(SINE_T) void k_sine_cum(const float* __restrict__ f0, int B, int L, int upp, float sr,
                                                     double* __restrict__ cum) {
  __shared__ double wsum[SINE_T / 64];
  const int b = blockIdx.x;
  const float* fb = f0 + (long long)b * L;
  float* cf = reinterpret_cast<float*>(cum + (long long)b * L);
  const int n = L - 1;
  if (n <= 0) return;  // block-uniform
  const int per = (n + SINE_T - 1) / SINE_T;
  const int j0 = min(n, (int)threadIdx.x * per), j1 = min(n, j0 + per);
  auto rem_at = [&](int j) {
    const float inc = (fb[j] / sr) * (float)upp;
    return fmodf(inc + 0.5f, 1.0f) - 0.5f;
  };
  double s = 0.0;
  for (int j = j0; j < j1; ++j) s += (double)rem_at(j);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double v = s;  // inclusive scan over the wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double u = __shfl_up(v, d);
    if (lane >= d) v += u;
  }
  if (lane == 63) wsum[w] = v;
  __syncthreads();
  double acc = v - s;
  for (int k = 0; k < w; ++k) acc += wsum[k];
  for (int j = j0; j < j1; ++j) {
    acc += (double)rem_at(j);
    cf[j] = fmodf((float)acc, 1.0f);
  }
}
__global__ void k_sine(const float* f0, int B, int L, int upp, float sr, const double* cum, const float* eps,
                       uint64_t seed, float lin_w, float lin_b, float* har, long long har_ld) {
  const long long n = (long long)B * L * upp;
  const float two_pi = 6.283185307179586f;
  const float amp_unv = (float)(0.1 / 3.0);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int u = (int)(i % upp);
    const long long bl = i / upp;
    const int b = (int)(bl / L), l = (int)(bl % L);
    const float f = f0[bl];
    float ph = (f / sr) * (float)(u + 1);
    if (l > 0) ph = ph + reinterpret_cast<const float*>(cum + (long long)b * L)[l - 1];
    const float sine = sinf(two_pi * ph) * 0.1f;
    const float uv = f > 0.f ? 1.f : 0.f;
    const float amp = uv * 0.003f + (1.f - uv) * amp_unv;
    const float e = eps ? eps[i] : normal_at(seed, (uint64_t)i);
    const float merged = sine * uv + amp * e;
    har[(long long)b * har_ld + (long long)l * upp + u] = tanhf(merged * lin_w + lin_b);
  }
}
hipError_t sine_source(const float* f0, int B, int L, int upp, float sr, const float* eps, uint64_t seed,
                       float lin_w, float lin_b, double* cum_ws, float* har, long long har_ld, hipStream_t s) {
  hipLaunchKernelGGL(k_sine_cum, dim3(B), dim3(SINE_T), 0, s, f0, B, L, upp, sr, cum_ws);
  hipLaunchKernelGGL(k_sine, dim3(nblocks((long long)B * L * upp)), dim3(TB), 0, s, f0, B, L, upp, sr, cum_ws, eps,
                     seed, lin_w, lin_b, har, har_ld);
  return hipGetLastError();
}

// ------------------------------------------------------------------ noise_convs: y[b][t][c] += b[c] + sum_k har[t*s-p+k] w[c][k]
// ------------------------------------------------------------------ conv_post: tanh(conv1d(lrelu(x, 0.01), w[1][C][K], pad K/2)), no bias
// The C*K weights sit in LDS too: read from global inside the FMA loop (uniform address, possibly
// aliasing y) they were one dependent vector load per FMA (80 us at C2).
// LeakyReLU -> Conv1d(C -> 1, K taps) -> tanh over 256 output samples per block. The lrelu'd input tile (+ halo)
// is staged in LDS with an odd row stride (conflict-free column reads); it is fetched as float4 loads all issued
// before the first LDS store (CP_IT per thread), so a block waits for one load latency, not one per element.
constexpr int CP_T = 256, CP_IT = 24;  // C <= 92 at K = 7
__global__ __launch_bounds__(CP_T) void k_conv_post(const float* __restrict__ x, int T, int C,
                                                    const float* __restrict__ wg, int K, float slope,
                                                    float* __restrict__ y, float bias) {
  extern __shared__ float tile[];  // [(CP_T+K-1)][C+1], then w[C*K]
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * CP_T;
  const int pad = K / 2;
  const int rows = CP_T + K - 1;
  const int ldt = C + 1;
  const int C4 = C >> 2;
  float* w = tile + rows * ldt;
  for (int i = threadIdx.x; i < C * K; i += blockDim.x) w[i] = wg[i];
  const float* xb = x + (long long)b * T * C;
  f32x4v v[CP_IT];
#pragma unroll
  for (int it = 0; it < CP_IT; ++it) {
    const int idx = it * CP_T + threadIdx.x;
    const int r = idx / C4, c4 = (idx - r * C4) * 4;
    const int g = t0 - pad + r;
    v[it] = (r < rows && g >= 0 && g < T) ? *reinterpret_cast<const f32x4v*>(xb + (long long)g * C + c4)
                                          : f32x4v{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int it = 0; it < CP_IT; ++it) {
    const int idx = it * CP_T + threadIdx.x;
    const int r = idx / C4, c4 = (idx - r * C4) * 4;
    if (r < rows) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float u = v[it][e];
        tile[r * ldt + c4 + e] = u > 0.f ? u : u * slope;
      }
    }
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= T) return;
  float acc = 0.f;
  for (int c = 0; c < C; ++c)
    for (int k = 0; k < K; ++k) acc = fmaf(tile[(threadIdx.x + k) * ldt + c], w[c * K + k], acc);
  y[(long long)b * T + t] = tanhf(acc + bias);  // + 0 for the bias-free HiFi-GAN / RefineGAN conv_post
}
// The same conv_post at the HiFi-GAN-NSF / MRF shape (C = 32, K = 7: every RVC v2 rate): C and K at compile time,
// the lrelu'd tile in LDS with a 36-float row stride (16 consecutive rows' float4 reads hit 64 distinct banks), the
// weights as one float4 per (tap, 4 channels) broadcast, and the 224 products of an output in four independent fma
// chains per float4 lane (the generic kernel's single dependent chain of 224 LDS-fed fmas ran at 73 us for 744000
// samples, ~1/5 of the HBM rate for its 95 MB). Summation order: channel group c4 outer, tap inner per chain, the
// four chains added at the end: the result differs from the generic kernel's in the last bits only.
constexpr int CPF_C = 32, CPF_K = 7, CPF_LD = 36, CPF_ROWS = CP_T + CPF_K - 1;
__global__ __launch_bounds__(CP_T) void k_conv_post32(const float* __restrict__ x, int T,
                                                      const float* __restrict__ wg, float slope,
                                                      float* __restrict__ y, float bias) {
  __shared__ __attribute__((aligned(16))) float tile[CPF_ROWS * CPF_LD];
  __shared__ __attribute__((aligned(16))) float w[CPF_K * CPF_C];  // [k][c]
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * CP_T;
  constexpr int pad = CPF_K / 2;
  constexpr int C4 = CPF_C / 4;
  constexpr int IT = (CPF_ROWS * C4 + CP_T - 1) / CP_T;
  if (threadIdx.x < CPF_K * CPF_C) {
    const int k = threadIdx.x / CPF_C, c = threadIdx.x - k * CPF_C;
    w[threadIdx.x] = wg[c * CPF_K + k];
  }
  const float* xb = x + (long long)b * T * CPF_C;
  f32x4v v[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = it * CP_T + threadIdx.x;
    const int r = idx / C4, c4 = (idx - r * C4) * 4;
    const int g = t0 - pad + r;
    const bool ok = r < CPF_ROWS && g >= 0 && g < T;
    v[it] = *reinterpret_cast<const f32x4v*>(xb + (long long)(ok ? g : 0) * CPF_C + c4);
    if (!ok) v[it] = f32x4v{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = it * CP_T + threadIdx.x;
    const int r = idx / C4, c4 = (idx - r * C4) * 4;
    if (r < CPF_ROWS) {
      f32x4v u = v[it];
#pragma unroll
      for (int e = 0; e < 4; ++e) u[e] = u[e] > 0.f ? u[e] : u[e] * slope;
      *reinterpret_cast<f32x4v*>(&tile[r * CPF_LD + c4]) = u;
    }
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= T) return;
  f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c4 = 0; c4 < C4; ++c4)
#pragma unroll
    for (int k = 0; k < CPF_K; ++k) {
      const f32x4v xv = *reinterpret_cast<const f32x4v*>(&tile[(threadIdx.x + k) * CPF_LD + 4 * c4]);
      const f32x4v wv = *reinterpret_cast<const f32x4v*>(&w[k * CPF_C + 4 * c4]);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = fmaf(xv[e], wv[e], acc[e]);
    }
  y[(long long)b * T + t] = tanhf(((acc[0] + acc[1]) + (acc[2] + acc[3])) + bias);
}

hipError_t conv_post_tanh(const float* x, int B, int T, int C, const float* w, int K, float slope, float* y,
                          hipStream_t s, float bias) {
  if (C == CPF_C && K == CPF_K && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    hipLaunchKernelGGL(k_conv_post32, dim3((T + CP_T - 1) / CP_T, B), dim3(CP_T), 0, s, x, T, w, slope, y, bias);
    return hipGetLastError();
  }
  // the staged fetch covers (CP_T + K - 1) rows of C / 4 float4 in CP_IT rounds of CP_T threads
  if (C % 4 != 0 || (long long)(CP_T + K - 1) * (C / 4) > (long long)CP_IT * CP_T ||
      (reinterpret_cast<uintptr_t>(x) & 15) != 0)
    return hipErrorInvalidValue;
  const size_t smem = ((size_t)(CP_T + K - 1) * (C + 1) + (size_t)C * K) * sizeof(float);
  hipLaunchKernelGGL(k_conv_post, dim3((T + CP_T - 1) / CP_T, B), dim3(CP_T), smem, s, x, T, C, w, K, slope, y, bias);
  return hipGetLastError();
}

// ------------------------------------------------------------------ z_p = (m + exp(logs) * eps * 0.66666) * mask
// stats: [B][T][2I] (m | logs); eps (reference layout [B][I][T]) or generated.
__global__ void k_zp(const float* stats, int B, int T, int I, const float* eps, uint64_t seed, const float* mask,
                     float* zp) {
  const long long n = (long long)B * T * I;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % I);
    const long long bt = i / I;
    const int b = (int)(bt / T), t = (int)(bt % T);
    const float m = stats[bt * 2 * I + c];
    const float lg = stats[bt * 2 * I + I + c];
    const long long ei = ((long long)b * I + c) * T + t;
    const float e = eps ? eps[ei] : normal_at(seed, (uint64_t)ei);
    zp[i] = (m + expf(lg) * e * 0.66666f) * mask[bt];
  }
}
hipError_t zp_sample(const float* stats, int B, int T, int I, const float* eps, uint64_t seed, const float* mask,
                     float* zp, hipStream_t s) {
  hipLaunchKernelGGL(k_zp, dim3(nblocks((long long)B * T * I)), dim3(TB), 0, s, stats, B, T, I, eps, seed, mask, zp);
  return hipGetLastError();
}

// ------------------------------------------------------------------ GroupNorm(C groups of 1 channel) over time + GELU (HuBERT conv0)
__global__ void k_gn_stats(const float* x, int T, int C, int chunk, double* ws) {
  // grid (C/64, nchunks, B); block 256 = 64 channels x 4 row lanes
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int t0 = blockIdx.y * chunk;
  const int t1 = min(T, t0 + chunk);
  x += (long long)blockIdx.z * T * C;
  ws += (long long)blockIdx.z * gridDim.y * C * 2;
  double s = 0.0, q = 0.0;
  if (c < C) {
    for (int t = t0 + rl; t < t1; t += 4) {
      const double v = x[(long long)t * C + c];
      s += v;
      q += v * v;
    }
  }
  __shared__ double ss[4][64], qq[4][64];
  ss[rl][threadIdx.x & 63] = s;
  qq[rl][threadIdx.x & 63] = q;
  __syncthreads();
  if (rl == 0 && c < C) {
    s = ss[0][threadIdx.x] + ss[1][threadIdx.x] + ss[2][threadIdx.x] + ss[3][threadIdx.x];
    q = qq[0][threadIdx.x] + qq[1][threadIdx.x] + qq[2][threadIdx.x] + qq[3][threadIdx.x];
    ws[((long long)blockIdx.y * C + c) * 2] = s;
    ws[((long long)blockIdx.y * C + c) * 2 + 1] = q;
  }
}
// per-channel statistics -> affine form y = x * scale + shift (torch GroupNorm's ApplyScaleBias:
// scale = rstd * gamma, shift = beta - mean * scale), once per channel instead of per element.
// grid (C/256, B): sequence b's partials at ws + b*nchunks*C*2, its scale/shift at ss + b*2C
// grid (C/64, B), block 256 = 64 channels x 4 chunk lanes: lane r sums chunks r, r + 4, ... (coalesced over the 64
// channels), the 4 lane sums are added in order (one thread per channel looping over all 256 chunks took 66 us)
__global__ void k_gn_finalize(const double* ws, int nchunks, int T, int C, const float* gamma, const float* beta,
                              float eps, float* ss) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  ws += (long long)blockIdx.y * nchunks * C * 2;
  ss += (long long)blockIdx.y * 2 * C;
  double s = 0.0, q = 0.0;
  if (c < C) {
    for (int k = rl; k < nchunks; k += 4) {
      s += ws[((long long)k * C + c) * 2];
      q += ws[((long long)k * C + c) * 2 + 1];
    }
  }
  __shared__ double sp[4][64], qp[4][64];
  sp[rl][threadIdx.x & 63] = s;
  qp[rl][threadIdx.x & 63] = q;
  __syncthreads();
  if (rl != 0 || c >= C) return;
  s = ((sp[0][threadIdx.x] + sp[1][threadIdx.x]) + sp[2][threadIdx.x]) + sp[3][threadIdx.x];
  q = ((qp[0][threadIdx.x] + qp[1][threadIdx.x]) + qp[2][threadIdx.x]) + qp[3][threadIdx.x];
  const double mean = s / T;
  double var = q / T - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float scale = rstd * gamma[c];
  ss[c] = scale;
  ss[C + c] = beta[c] - (float)mean * scale;
}
// x: B sequences of T rows back to back; n4_per = T*C/4 float4 per sequence
// (32-bit indices: the launch checks n4 < 2^31; the 64-bit % and / per float4 were most of its instructions)
__global__ void k_gn_apply(float* __restrict__ x, unsigned n4, unsigned n4_per, unsigned C4, const float* __restrict__ ss,
                           int C) {
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    const float* sb = ss + (size_t)(i / n4_per) * 2 * C;
    f32x4v v = reinterpret_cast<f32x4v*>(x)[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float t = v[j] * sb[c + j] + sb[C + c + j];
      v[j] = 0.5f * t * (1.f + erff(t * 0.70710678118654752440f));
    }
    reinterpret_cast<f32x4v*>(x)[i] = v;
  }
}
hipError_t groupnorm_time_gelu(float* x, int T, int C, const float* gamma, const float* beta, float eps, double* ws,
                               hipStream_t s, int B) {
  // ws (groupnorm_ws_doubles(C, B)): B * GN_CHUNKS * C * 2 doubles of partial sums, then B * 2C floats
  const int nchunks = GN_CHUNKS;
  const int chunk = (T + nchunks - 1) / nchunks;
  if (C % 4 || B < 1) return hipErrorInvalidValue;
  float* ss = reinterpret_cast<float*>(ws + (size_t)B * nchunks * C * 2);
  hipLaunchKernelGGL(k_gn_stats, dim3((C + 63) / 64, nchunks, B), dim3(256), 0, s, x, T, C, chunk, ws);
  hipLaunchKernelGGL(k_gn_finalize, dim3((C + 63) / 64, B), dim3(256), 0, s, ws, nchunks, T, C, gamma, beta, eps,
                     ss);
  const long long n4p = (long long)T * C / 4;
  if (n4p * B >= (1LL << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gn_apply, dim3(nblocks(n4p * B)), dim3(TB), 0, s, x, (unsigned)(n4p * B), (unsigned)n4p,
                     (unsigned)(C / 4), ss, C);
  return hipGetLastError();
}

// ------------------------------------------------------------------ HuBERT conv0 + GroupNorm + GELU, fused
// conv_layers.0 (modeling_hubert.py HubertGroupNormConvLayer: Conv1d(1, C, 10, stride 5, bias=False) -> GroupNorm(C, C)
// -> GELU). The conv is 10 MACs per output, so the statistics pass recomputes it instead of reading a stored copy, and
// the apply pass computes it a third time and writes the normalized, activated output once: no conv output in HBM,
// no read-modify-write pass (round 6; before: the conv on the 3-plane MFMA kernel at K = 5 x 2 taps, 65 us, then
// k_gn_stats / k_gn_finalize / k_gn_apply over the stored 101 MB, 96 us). Every pass evaluates hconv0_at, one fp32 fma
// chain over the 10 taps, so the statistics are those of the values the apply pass normalizes.
__device__ __forceinline__ float hconv0_at(const float* __restrict__ xr, const float (&wr)[10]) {
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < 10; ++k) v = fmaf(wr[k], xr[k], v);
  return v;
}
// grid (C/64, nchunks, B), block 256 = 64 channels x 4 row lanes: k_gn_stats's partial-sum layout (k_gn_finalize reads it)
__global__ __launch_bounds__(256) void k_hconv0_stats(const float* __restrict__ x, long long ldx, const float* __restrict__ w,
                                                      int T, int C, int chunk, double* __restrict__ ws) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int t0 = blockIdx.y * chunk;
  const int t1 = min(T, t0 + chunk);
  x += (long long)blockIdx.z * ldx;
  ws += (long long)blockIdx.z * gridDim.y * C * 2;
  float wr[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) wr[k] = w[(long long)c * 10 + k];
  double s = 0.0, q = 0.0;
  for (int t = t0 + rl; t < t1; t += 4) {
    const double v = hconv0_at(x + 5LL * t, wr);
    s += v;
    q += v * v;
  }
  __shared__ double ss[4][64], qq[4][64];
  ss[rl][threadIdx.x & 63] = s;
  qq[rl][threadIdx.x & 63] = q;
  __syncthreads();
  if (rl == 0) {
    s = ss[0][threadIdx.x] + ss[1][threadIdx.x] + ss[2][threadIdx.x] + ss[3][threadIdx.x];
    q = qq[0][threadIdx.x] + qq[1][threadIdx.x] + qq[2][threadIdx.x] + qq[3][threadIdx.x];
    ws[((long long)blockIdx.y * C + c) * 2] = s;
    ws[((long long)blockIdx.y * C + c) * 2 + 1] = q;
  }
}
// block C/4 threads (thread = 4 channels, its 40 weights in registers), grid (rows, B): rows t = blockIdx.x + k gridDim.x
__global__ void k_hconv0_apply(const float* __restrict__ x, long long ldx, const float* __restrict__ w, int T, int C,
                               const float* __restrict__ ss, float* __restrict__ y) {
  const int c0 = threadIdx.x * 4;
  x += (long long)blockIdx.y * ldx;
  y += (long long)blockIdx.y * T * C;
  ss += (long long)blockIdx.y * 2 * C;
  float wr[4][10];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 10; ++k) wr[j][k] = w[(long long)(c0 + j) * 10 + k];
  const f32x4v sc = *reinterpret_cast<const f32x4v*>(ss + c0);
  const f32x4v sh = *reinterpret_cast<const f32x4v*>(ss + C + c0);
  for (int t = blockIdx.x; t < T; t += gridDim.x) {
    const float* xr = x + 5LL * t;
    f32x4v v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float u = hconv0_at(xr, wr[j]) * sc[j] + sh[j];  // k_gn_apply's arithmetic
      v[j] = 0.5f * u * (1.f + erff(u * 0.70710678118654752440f));
    }
    *reinterpret_cast<f32x4v*>(y + (long long)t * C + c0) = v;
  }
}
hipError_t hubert_conv0_gn_gelu(const float* x, long long ldx, const float* w10, int T, int C, const float* gamma,
                                const float* beta, float eps, double* ws, float* y, hipStream_t s, int B) {
  // ws: groupnorm_ws_doubles(C, B); x row b at x + b ldx holds >= 5 (T - 1) + 10 samples; y [B][T][C]
  if (C % 64 || C > 1024 || B < 1 || B > 65535 || T < 1 || (reinterpret_cast<uintptr_t>(y) & 15)) return hipErrorInvalidValue;
  const int nchunks = GN_CHUNKS;
  const int chunk = (T + nchunks - 1) / nchunks;
  float* ss = reinterpret_cast<float*>(ws + (size_t)B * nchunks * C * 2);
  hipLaunchKernelGGL(k_hconv0_stats, dim3(C / 64, nchunks, B), dim3(256), 0, s, x, ldx, w10, T, C, chunk, ws);
  hipLaunchKernelGGL(k_gn_finalize, dim3(C / 64, B), dim3(256), 0, s, ws, nchunks, T, C, gamma, beta, eps, ss);
  hipLaunchKernelGGL(k_hconv0_apply, dim3((unsigned)std::min(T, 2048), B), dim3(C / 4), 0, s, x, ldx, w10, T, C, ss, y);
  return hipGetLastError();
}

// ------------------------------------------------------------------ RMVPE front end
// grid.y = sequence: x rows of stride ldx, y rows of stride ldy
// (a row stride ldy past the padded length gets its tail zeroed here: no fill launch before)
__global__ void k_reflect1d(const float* x, int n, int pl, int pr, float* y, long long ldx, long long ldy) {
  const int m = n + pl + pr;
  const int mz = ldy > m ? (int)ldy : m;
  x += blockIdx.y * ldx;
  y += blockIdx.y * ldy;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < mz; i += gridDim.x * blockDim.x) {
    int j = i - pl;
    if (j < 0) j = -j;
    if (j >= n) j = 2 * (n - 1) - j;
    y[i] = i < m ? x[j] : 0.f;
  }
}
hipError_t reflect_pad_1d(const float* x, int n, int pad_l, int pad_r, float* y, hipStream_t s, int B, long long ldx,
                          long long ldy) {
  if (pad_l >= n || pad_r >= n) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_reflect1d, dim3(std::min(nblocks(n + pad_l + pad_r), 2048u), B), dim3(TB), 0, s, x, n, pad_l,
                     pad_r, y, ldx, ldy);
  return hipGetLastError();
}
// grid.y = image: x [B][rows][C] -> y [B][rows + pr][C]
__global__ void k_reflect_rows(const float* x, int rows, int C, int pr, float* y) {
  const long long n = (long long)(rows + pr) * C;
  x += (long long)blockIdx.y * rows * C;
  y += (long long)blockIdx.y * n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / C), c = (int)(i % C);
    const int src = r < rows ? r : 2 * (rows - 1) - r;
    y[i] = x[(long long)src * C + c];
  }
}
hipError_t reflect_pad_rows(const float* x, int rows, int C, int pad_r, float* y, hipStream_t s, int B) {
  if (pad_r >= rows) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_reflect_rows, dim3(std::min(nblocks((long long)(rows + pad_r) * C), 2048u), B), dim3(TB), 0,
                     s, x, rows, C, pad_r, y);
  return hipGetLastError();
}
// |STFT| rows of ldm floats: bins 0 .. nb - 1, then zeros up to ldm (the mel GEMM's contraction runs over whole
// 32-bin chunks)
__global__ void k_stftmag(const float* spec, int F, int nb, float* mag, int ldm) {
  const long long n = (long long)F * ldm;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int f = (int)(i / ldm), k = (int)(i % ldm);
    float v = 0.f;
    if (k < nb) {
      const float re = spec[(long long)f * 2 * nb + k];
      const float im = spec[(long long)f * 2 * nb + nb + k];
      v = sqrtf(re * re + im * im);
    }
    mag[i] = v;
  }
}
hipError_t stft_magnitude(const float* spec, int F, int nbins, float* mag, int ldm, hipStream_t s) {
  if (ldm < nbins) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_stftmag, dim3(nblocks((long long)F * ldm)), dim3(TB), 0, s, spec, F, nbins, mag, ldm);
  return hipGetLastError();
}

__global__ void k_avgpool2(const float* x, int H, int W, int C, int ldx, float* y) {
  const int Ho = H / 2, Wo = W / 2;
  const long long n = (long long)Ho * Wo * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long p = i / C;
    const int h = (int)(p / Wo), w = (int)(p % Wo);
    const float* a = x + ((long long)(2 * h) * W + 2 * w) * ldx + c;
    const float* bb = a + (long long)W * ldx;
    y[i] = (((a[0] + a[ldx]) + bb[0]) + bb[ldx]) / 4.f;
  }
}
hipError_t avgpool2(const float* x, int H, int W, int C, int ldx, float* y, hipStream_t s) {
  hipLaunchKernelGGL(k_avgpool2, dim3(nblocks((long long)(H / 2) * (W / 2) * C)), dim3(TB), 0, s, x, H, W, C, ldx, y);
  return hipGetLastError();
}

__global__ void k_nhwc_hcw(const float* x, int H, int W, int C, float* y) {
  const long long n = (long long)H * W * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int h = (int)(i / (W * C));
    const int rem = (int)(i % (W * C));
    const int c = rem / W, w = rem % W;
    y[i] = x[((long long)h * W + w) * C + c];
  }
}
hipError_t nhwc_to_hcw(const float* x, int H, int W, int C, float* y, hipStream_t s) {
  hipLaunchKernelGGL(k_nhwc_hcw, dim3(nblocks((long long)H * W * C)), dim3(TB), 0, s, x, H, W, C, y);
  return hipGetLastError();
}

// ------------------------------------------------------------------ RMVPE decode (RMVPE.py:484-540), fp64 like numpy
// rows of B sequences: frame f of sequence b reads sal[(b*Fs + f)][.] and writes f0[b*F + f]
__global__ void k_decode(const float* sal, int F, int Fs, int nrows, int ncls, float thred, double* f0) {
#pragma clang fp contract(off)  // numpy rounds every product and sum separately
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= nrows) return;
  const int f = row;
  const float* s = sal + ((long long)(row / F) * Fs + row % F) * ncls;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int k = lane; k < ncls; k += 64) {
    const float v = s[k];
    if (v > best) {
      best = v;
      bi = k;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) {
      best = ov;
      bi = oi;
    }
  }
  if (lane == 0) {
    // numpy reduces each 9-wide row with its pairwise kernel: 8 partials seeded by a[0..7], combined
    // ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then + a[8]. weight_sum stays float32 (salience dtype),
    // product_sum is float64 (float32 * float64 cents map). Out-of-range slots are the zero padding.
    float wv[9];
    double pv[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int k = bi - 4 + j;
      const bool in = k >= 0 && k < ncls;
      wv[j] = in ? s[k] : 0.f;
      pv[j] = in ? (double)wv[j] * (20.0 * k + 1997.3794084376191) : 0.0;
    }
    const float wsf = (((wv[0] + wv[1]) + (wv[2] + wv[3])) + ((wv[4] + wv[5]) + (wv[6] + wv[7]))) + wv[8];
    const double ps = (((pv[0] + pv[1]) + (pv[2] + pv[3])) + ((pv[4] + pv[5]) + (pv[6] + pv[7]))) + pv[8];
    const double ws = (double)wsf;
    double cents = ps / ws;
    if ((double)best <= (double)thred) cents = 0.0;
    double v = 10.0 * pow(2.0, cents / 1200.0);
    if (v == 10.0) v = 0.0;
    f0[f] = v;
  }
}
hipError_t rmvpe_decode(const float* sal, int F, int ncls, float thred, double* f0, hipStream_t s, int B, int Fs) {
  if (Fs <= 0) Fs = F;
  const int nrows = B * F;
  hipLaunchKernelGGL(k_decode, dim3((nrows + 3) / 4), dim3(256), 0, s, sal, F, Fs, nrows, ncls, thred, f0);
  return hipGetLastError();
}

// ------------------------------------------------------------------ f0 shift + coarse quantisation (pipeline.py:280-291)
__global__ void k_f0post(const double* f0, int F, double shift, int32_t* coarse, float* pitchf, double* f0_out) {
#pragma clang fp contract(off)  // numpy rounds every product and sum separately
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F) return;
  const double f = f0[i] * shift;
  // self.f0_mel_min / f0_mel_max = 1127 * np.log(1 + 50/700), 1127 * np.log(1 + 1100/700) (pipeline.py:195-196):
  // numpy, glibc and the correctly rounded log agree on both
  constexpr double mel_min = 0x1.370515d9beb10p+6;
  constexpr double mel_max = 0x1.0a1a207dfdbe5p+10;
  // log correctly rounded (dd_math.h): the coarse pitch is integer output; every other step is one IEEE op
  double m = 1127.0 * dd::log_cr(1.0 + f / 700.0);
  if (m > 0) m = (m - mel_min) * 254.0 / (mel_max - mel_min) + 1.0;
  if (m <= 1) m = 1;
  if (m > 255) m = 255;
  coarse[i] = (int32_t)rint(m);
  pitchf[i] = (float)f;
  if (f0_out) f0_out[i] = f;
}
hipError_t f0_post(const double* f0, int F, double shift, int32_t* coarse, float* pitchf, double* f0_out,
                   hipStream_t s) {
  hipLaunchKernelGGL(k_f0post, dim3(nblocks(F)), dim3(TB), 0, s, f0, F, shift, coarse, pitchf, f0_out);
  return hipGetLastError();
}

}  // namespace rvcx

// =================================================================== pipeline DSP on device
namespace rvcx {

// scipy.signal.filtfilt(b, a, x) with padtype='odd', padlen = 3*max(len(a), len(b)) (pipeline.py:439),
// lfilter in direct form II transposed, fp64. The 5th-order 48 Hz high-pass has poles at |p| <= 0.9942
// and a highly non-normal DF2T state matrix (||F^256|| ~ 4e7), so chunk-state propagation
// (s_{c+1} = F^L s_c + e_c) is numerically unstable. Instead each chunk of IIR_L outputs re-runs
// IIR_W samples of history from a zero state (||F^10240|| ~ 1e-18, so the truncated history is below
// fp64 resolution); chunks that reach the signal start run from lfilter_zi * x[0] exactly as scipy.
// Measured vs scipy on the 13.5 s reference clip: max |diff| 3.4e-8 (below the fp32 ulp the models see).
constexpr int IIR_L = 512;
constexpr int IIR_W = 8192;  // ||F^8192|| ~ 2e-14: truncated history far below the DF2T's own rounding noise

struct IirCoef {
  double b[IIR_MAXO + 1], a[IIR_MAXO + 1], zi[IIR_MAXO];
  int order;
};

template <int O>
__device__ __forceinline__ double iir_step(const IirCoef& c, double* z, double x) {
  const double y = c.b[0] * x + z[0];
#pragma unroll
  for (int i = 0; i < O - 1; ++i) z[i] = c.b[i + 1] * x + z[i + 1] - c.a[i + 1] * y;
  z[O - 1] = c.b[O] * x - c.a[O] * y;
  return y;
}

// odd extension of x by padlen on both sides (scipy _arraytools.odd_ext)
__global__ void k_odd_ext(const double* x, long long n, int padlen, double* e) {
  const long long ne = n + 2 * padlen;
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < ne; j += (long long)gridDim.x * blockDim.x) {
    const long long k = j - padlen;
    double v;
    if (k < 0) v = 2.0 * x[0] - x[-k];
    else if (k >= n) v = 2.0 * x[n - 1] - x[2 * (n - 1) - k];
    else v = x[k];
    e[j] = v;
  }
}

// one pass of lfilter over seq (read reversed when rev): chunk ch writes outputs [ch*L, ch*L+L)
template <int O>
__global__ void k_iir_warm(const IirCoef c, const double* seq, long long ne, int rev, double* out) {
  const long long ch = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long nch = (ne + IIR_L - 1) / IIR_L;
  if (ch >= nch) return;
  const long long j0 = ch * IIR_L, j1 = min(ne, j0 + IIR_L);
  long long js = j0 - IIR_W;
  double z[O];
  auto at = [&](long long j) { return rev ? seq[ne - 1 - j] : seq[j]; };
  if (js <= 0) {
    js = 0;
    const double x0 = at(0);
#pragma unroll
    for (int i = 0; i < O; ++i) z[i] = c.zi[i] * x0;
  } else {
#pragma unroll
    for (int i = 0; i < O; ++i) z[i] = 0.0;
  }
  // warm-up over history (no outputs), 16 inputs fetched per batch ahead of the recurrence
  constexpr int NB = 16;
  long long j = js;
  for (; j + NB <= j0; j += NB) {
    double xb[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) xb[i] = at(j + i);
#pragma unroll
    for (int i = 0; i < NB; ++i) (void)iir_step<O>(c, z, xb[i]);
  }
  for (; j < j0; ++j) (void)iir_step<O>(c, z, at(j));
  for (; j + NB <= j1; j += NB) {
    double xb[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) xb[i] = at(j + i);
#pragma unroll
    for (int i = 0; i < NB; ++i) out[j + i] = iir_step<O>(c, z, xb[i]);
  }
  for (; j < j1; ++j) out[j] = iir_step<O>(c, z, at(j));
}

// audio_pad[k] = y[reflect(k - t_pad)] with y the filtfilt output (backward pass result yb reversed, trimmed)
__global__ void k_filt_pad(const double* yb, long long ne, int padlen, long long n, long long t_pad, double* pad64,
                           float* pad32) {
  const long long m = n + 2 * t_pad;
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < m; k += (long long)gridDim.x * blockDim.x) {
    long long j = k - t_pad;
    if (j < 0) j = -j;
    if (j >= n) j = 2 * (n - 1) - j;
    const double v = yb[ne - 1 - (j + padlen)];
    if (pad64) pad64[k] = v;
    pad32[k] = (float)v;
  }
}

hipError_t filtfilt_pad(const double* x, long long n, const double* b, const double* a, const double* zi,
                        const double* /*FL*/, int order, long long t_pad, double* ws, double* pad64, float* pad32,
                        hipStream_t s) {
  if (order < 1 || order > IIR_MAXO) return hipErrorInvalidValue;
  const int padlen = 3 * (order + 1);
  if (n <= padlen || t_pad >= n) return hipErrorInvalidValue;
  IirCoef c;
  c.order = order;
  for (int i = 0; i <= order; ++i) {
    c.b[i] = b[i];
    c.a[i] = a[i];
  }
  for (int i = 0; i < order; ++i) c.zi[i] = zi[i];
  const long long ne = n + 2 * padlen;
  const long long nch = (ne + IIR_L - 1) / IIR_L;
  double* ext = ws;
  double* yf = ext + ne;
  double* yb = yf + ne;
  hipLaunchKernelGGL(k_odd_ext, dim3(nblocks(ne)), dim3(TB), 0, s, x, n, padlen, ext);
  const unsigned g = (unsigned)((nch + 63) / 64);
  for (int rev = 0; rev < 2; ++rev) {
    const double* in = rev ? yf : ext;
    double* o = rev ? yb : yf;
    switch (order) {
#define RVCX_IIR_CASE(O_) \
  case O_: hipLaunchKernelGGL(k_iir_warm<O_>, dim3(g), dim3(64), 0, s, c, in, ne, rev, o); break;
      RVCX_IIR_CASE(1) RVCX_IIR_CASE(2) RVCX_IIR_CASE(3) RVCX_IIR_CASE(4)
      RVCX_IIR_CASE(5) RVCX_IIR_CASE(6) RVCX_IIR_CASE(7) RVCX_IIR_CASE(8)
#undef RVCX_IIR_CASE
      default: return hipErrorInvalidValue;
    }
  }
  hipLaunchKernelGGL(k_filt_pad, dim3(nblocks(n + 2 * t_pad)), dim3(TB), 0, s, yb, ne, padlen, n, t_pad, pad64,
                     pad32);
  return hipGetLastError();
}

hipError_t filtfilt_sos_pad(const SosPlan& p, int order, const double* x, long long n, long long t_pad, double* ws,
                            double* pad64, float* pad32, hipStream_t s) {
  const int padlen = 3 * (order + 1);
  if (n <= padlen || t_pad >= n || p.nsec < 1) return hipErrorInvalidValue;
  const long long ne = n + 2 * padlen;
  if (!p.casc) return hipErrorInvalidValue;
  double* ext = ws;
  hipLaunchKernelGGL(k_odd_ext, dim3(nblocks(ne)), dim3(TB), 0, s, x, n, padlen, ext);
  return casc_filtfilt_pad(p, ext, ne, padlen, n, t_pad, ext + ne, pad64, pad32, s);
}

size_t filtfilt_sos_ws_doubles(long long n, int order, int L) {
  const long long ne = n + 2 * 3 * (order + 1);
  (void)L;
  return (size_t)(3 * ne) + casc_ws_doubles(ne, 64);
}

size_t filtfilt_ws_doubles(long long n, int order) {
  const long long ne = n + 2 * 3 * (order + 1);
  return (size_t)(3 * ne);
}

// peak normalisation (pipeline.py:550-552): m = max|x| / 0.99 ; if m > 1: x /= m. Fused with the trim copy
// (pipeline.py:494 audio_opt slices): dst = src / m read from the un-trimmed buffer. Two launches for all B rows
// and no fill: each absmax block writes its own maximum to ws[row][block], the scale pass reduces those <= 256
// partials per block before it scales (no atomics, nothing to zero between calls).
constexpr int PEAK_BLOCKS = 256;
__global__ void k_absmax(const float* x, long long n, long long ldx, float* part) {
  __shared__ float wm[TB / 64];
  x += blockIdx.y * ldx;
  float m = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(x[i]));
  m = warp_max(m);
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) m = fmaxf(m, wm[w]);
    part[blockIdx.y * PEAK_BLOCKS + blockIdx.x] = m;
  }
}
__global__ void k_peak_scale(const float* src, long long lds, float* dst, long long ldd, long long n, const float* part,
                             int nparts) {
  __shared__ float wm[TB / 64];
  src += blockIdx.y * lds;
  dst += blockIdx.y * ldd;
  float m = threadIdx.x < nparts ? part[blockIdx.y * PEAK_BLOCKS + threadIdx.x] : 0.f;
  m = warp_max(m);
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  m = wm[0];
  for (int w = 1; w < TB / 64; ++w) m = fmaxf(m, wm[w]);
  m = m / 0.99f;
  const bool scale = m > 1.f;
  if (!scale && src == dst) return;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    dst[i] = scale ? src[i] / m : src[i];
}
hipError_t peak_normalize(const float* src, float* dst, long long n, float* ws, hipStream_t s, int B, long long lds,
                          long long ldd) {
  if (n <= 0 || B < 1) return hipSuccess;
  const int nparts = (int)std::min<long long>(PEAK_BLOCKS, (n + TB - 1) / TB);
  hipLaunchKernelGGL(k_absmax, dim3(nparts, B), dim3(TB), 0, s, src, n, lds, ws);
  hipLaunchKernelGGL(k_peak_scale, dim3(std::min(nblocks(n), 4096u), B), dim3(TB), 0, s, src, lds, dst, ldd, n, ws,
                     nparts);
  return hipGetLastError();
}
size_t peak_normalize_ws_floats(int B) { return (size_t)B * PEAK_BLOCKS; }

// ------------------------------------------------------------------ get_f0 adjustments
// Autotune.autotune_f0 (rvc/infer/pipeline.py:151-162): snap to the nearest of 54 note
// frequencies (first minimum wins, like Python's min()), blend by strength. The rvc/ path snaps
// every frame (f0 = 0 -> 49 Hz * strength); rvc_mlx (pipeline_mlx.py:72-80) leaves f0 <= 0 alone.
__constant__ double c_notes[54] = {
    49.00,  51.91,  55.00,  58.27,  61.74,  65.41,  69.30,  73.42,  77.78,  82.41,  87.31,  92.50,  98.00,  103.83,
    110.00, 116.54, 123.47, 130.81, 138.59, 146.83, 155.56, 164.81, 174.61, 185.00, 196.00, 207.65, 220.00, 233.08,
    246.94, 261.63, 277.18, 293.66, 311.13, 329.63, 349.23, 369.99, 392.00, 415.30, 440.00, 466.16, 493.88, 523.25,
    554.37, 587.33, 622.25, 659.25, 698.46, 739.99, 783.99, 830.61, 880.00, 932.33, 987.77, 1046.50};

__global__ void k_autotune(double* f0, int F, double strength, int skip_unvoiced) {
#pragma clang fp contract(off)  // numpy rounds every product and sum separately
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F) return;
  const double f = f0[i];
  if (skip_unvoiced && f <= 0.0) return;
  double best = c_notes[0], bd = fabs(c_notes[0] - f);
  for (int j = 1; j < 54; ++j) {
    const double d = fabs(c_notes[j] - f);
    if (d < bd) {
      bd = d;
      best = c_notes[j];
    }
  }
  f0[i] = f + (best - f) * strength;
}
hipError_t f0_autotune(double* f0, int F, double strength, int skip_unvoiced, hipStream_t s) {
  hipLaunchKernelGGL(k_autotune, dim3(nblocks(F)), dim3(TB), 0, s, f0, F, strength, skip_unvoiced);
  return hipGetLastError();
}

// ------------------------------------------------------------------ long-input split points
// Pipeline.pipeline opt_ts search (rvc/infer/pipeline.py:440-452): with xp = reflect-pad(x, w/2),
// audio_sum[p] = sum_{i<w} xp[p+i] accumulated in i order (numpy's `audio_sum += audio_pad[i:i-w]`,
// so the fp64 result is bit-identical), then for every t = t_center, 2 t_center, ... < n the split
// is t - t_query + first argmin |audio_sum[t - t_query : t + t_query]|.
__global__ void k_window_sum(const double* x, long long n, int w, double* sum) {
  const long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (p >= n) return;
  const long long h = w / 2;
  double acc = 0.0;
  for (int i = 0; i < w; ++i) {
    long long q = p + i - h;
    if (q < 0) q = -q;
    if (q >= n) q = 2 * (n - 1) - q;
    acc += x[q];
  }
  sum[p] = acc;
}
__global__ void k_split_argmin(const double* sum, long long n, long long t_center, long long t_query,
                               long long* ts) {
  const long long t = t_center * (blockIdx.x + 1);
  const long long lo = t - t_query;
  const long long hi = t + t_query < n ? t + t_query : n;
  double bv = INFINITY;
  long long bi = hi;
  for (long long p = lo + threadIdx.x; p < hi; p += blockDim.x) {
    const double v = fabs(sum[p]);
    if (v < bv) {  // ascending p per thread: keeps the first minimum
      bv = v;
      bi = p;
    }
  }
  __shared__ double sv[TB];
  __shared__ long long si[TB];
  sv[threadIdx.x] = bv;
  si[threadIdx.x] = bi;
  __syncthreads();
  for (int o = TB / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      const double v2 = sv[threadIdx.x + o];
      const long long i2 = si[threadIdx.x + o];
      if (v2 < sv[threadIdx.x] || (v2 == sv[threadIdx.x] && i2 < si[threadIdx.x])) {
        sv[threadIdx.x] = v2;
        si[threadIdx.x] = i2;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) ts[blockIdx.x] = si[0];
}
hipError_t split_points(const double* x, long long n, int window, long long t_center, long long t_query,
                        double* sum_ws, long long* ts, int nts, hipStream_t s) {
  hipLaunchKernelGGL(k_window_sum, dim3(nblocks(n)), dim3(TB), 0, s, x, n, window, sum_ws);
  if (nts > 0) hipLaunchKernelGGL(k_split_argmin, dim3(nts), dim3(TB), 0, s, sum_ws, n, t_center, t_query, ts);
  return hipGetLastError();
}

// ------------------------------------------------------------------ volume envelope
// AudioProcessor.change_rms (rvc/infer/pipeline.py:35-82): librosa.feature.rms (center=True, zero pad
// frame/2, mean |x|^2 per frame, sqrt) of source and target, both linearly interpolated
// (F.interpolate mode='linear', align_corners=False) to the target length, then
// y *= rms1^(1-rate) * max(rms2, 1e-6)^(rate-1). One block per RMS frame, fp64 sums.
template <class T>
__global__ void k_rms_frames(const T* x, long long n, int frame, int hop, float* rms) {
  const long long start = (long long)blockIdx.x * hop - frame / 2;
  double acc = 0.0;
  for (int j = threadIdx.x; j < frame; j += blockDim.x) {
    const long long q = start + j;
    if (q >= 0 && q < n) {
      const double v = (double)x[q];
      acc += v * v;
    }
  }
  __shared__ double red[TB];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = TB / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) rms[blockIdx.x] = (float)sqrt(red[0] / frame);
}
// librosa.feature.rms (center=True, zero pad frame/2) kept in fp64 for librosa.effects.split's power_to_db test
// (rvc/lib/tools/split_audio.py:19-24): rms[k] = sqrt(mean over the frame of x^2), frame k centred at k*hop.
__global__ void k_rms_frames_f64(const double* x, long long n, int frame, int hop, double* rms) {
  const long long start = (long long)blockIdx.x * hop - frame / 2;
  double acc = 0.0;
  for (int j = threadIdx.x; j < frame; j += blockDim.x) {
    const long long q = start + j;
    if (q >= 0 && q < n) acc += x[q] * x[q];
  }
  __shared__ double red[TB];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = TB / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) rms[blockIdx.x] = sqrt(red[0] / frame);
}
hipError_t rms_frames_f64(const double* x, long long n, int frame, int hop, double* rms, int nframes, hipStream_t s) {
  if (frame <= 0 || hop <= 0 || nframes <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_rms_frames_f64, dim3(nframes), dim3(TB), 0, s, x, n, frame, hop, rms);
  return hipGetLastError();
}
__device__ __forceinline__ float interp_linear(const float* r, int n_in, long long i, long long n_out) {
  const float scale = (float)n_in / (float)n_out;
  float src = scale * ((float)i + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  int i0 = (int)src;
  if (i0 > n_in - 1) i0 = n_in - 1;
  const int i1 = i0 + (i0 < n_in - 1 ? 1 : 0);
  float l1 = src - (float)i0;
  l1 = fminf(fmaxf(l1, 0.f), 1.f);
  return (1.f - l1) * r[i0] + l1 * r[i1];
}
__global__ void k_apply_rms(float* y, long long n, const float* r1, int n1, const float* r2, int n2, float rate) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float a = interp_linear(r1, n1, i, n);
    const float b = fmaxf(interp_linear(r2, n2, i, n), 1e-6f);
    y[i] = y[i] * (powf(a, 1.f - rate) * powf(b, rate - 1.f));
  }
}
int rms_frame_count(long long n, int sr) { return (int)(1 + n / (sr / 2)); }
hipError_t change_rms(const double* src, long long n_src, int sr_src, float* y, long long n_y, int sr_y, float rate,
                      float* ws, hipStream_t s) {
  const int n1 = rms_frame_count(n_src, sr_src), n2 = rms_frame_count(n_y, sr_y);
  hipLaunchKernelGGL(k_rms_frames<double>, dim3(n1), dim3(TB), 0, s, src, n_src, sr_src / 2 * 2, sr_src / 2, ws);
  hipLaunchKernelGGL(k_rms_frames<float>, dim3(n2), dim3(TB), 0, s, (const float*)y, n_y, sr_y / 2 * 2, sr_y / 2,
                     ws + n1);
  hipLaunchKernelGGL(k_apply_rms, dim3(nblocks(n_y)), dim3(TB), 0, s, y, n_y, ws, n1, ws + n1, n2, rate);
  return hipGetLastError();
}
// change_rms with a float32 source (the streaming path's 16 kHz convert buffer, rvc/realtime/pipeline.py:303-310)
hipError_t change_rms_f32src(const float* src, long long n_src, int sr_src, float* y, long long n_y, int sr_y,
                             float rate, float* ws, hipStream_t s) {
  const int n1 = rms_frame_count(n_src, sr_src), n2 = rms_frame_count(n_y, sr_y);
  hipLaunchKernelGGL(k_rms_frames<float>, dim3(n1), dim3(TB), 0, s, src, n_src, sr_src / 2 * 2, sr_src / 2, ws);
  hipLaunchKernelGGL(k_rms_frames<float>, dim3(n2), dim3(TB), 0, s, (const float*)y, n_y, sr_y / 2 * 2, sr_y / 2,
                     ws + n1);
  hipLaunchKernelGGL(k_apply_rms, dim3(nblocks(n_y)), dim3(TB), 0, s, y, n_y, ws, n1, ws + n1, n2, rate);
  return hipGetLastError();
}

}  // namespace rvcx
