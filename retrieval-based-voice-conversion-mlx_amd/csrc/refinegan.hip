// Elementwise / resampling kernels of the RefineGAN decoder (rvc/lib/algorithm/generators/refinegan.py):
// torchaudio's kaiser-sinc downsampling of the source branch, linear x-rate upsampling fused with the skip
// concatenation, and AdaIN (noise injection + LeakyReLU 0.2). Time-major [T][C] rows throughout; the heavy
// contractions (every Conv1d) run on the MFMA conv kernels. These are HBM / L2 bound.
#include <cmath>

#include "rvcx_kernels.h"

#pragma clang fp contract(off)

namespace rvcx {

namespace {

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
  uint32_t c[4] = {(uint32_t)(idx >> 1), (uint32_t)(idx >> 33), 0x41444149u, 2u};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float u1 = ((c[0] >> 8) + 1) * (1.0f / 16777217.0f);
  const float u2 = (c[1] >> 8) * (1.0f / 16777216.0f);
  const float r = sqrtf(-2.f * logf(u1));
  const float th = 6.283185307179586f * u2;
  return (idx & 1) ? r * sinf(th) : r * cosf(th);
}

__device__ __forceinline__ float lrelu(float v, float s) { return v > 0.f ? v : v * s; }

// y[b][t][c] = sum_k x[b][t*orig + k - width][c] * ker[k]  (zero outside the input): the new_freq = 1 case of
// torchaudio's _apply_sinc_resample_kernel (pad (width, width + orig), conv1d stride orig). One thread per output
// element, channels fastest; the kernel sits in LDS.
__global__ void k_resample_dw(const float* __restrict__ x, int T_in, int C, const float* __restrict__ ker, int K,
                              int orig, int width, float* __restrict__ y, int T_out, int B) {
  extern __shared__ float sk[];
  for (int i = threadIdx.x; i < K; i += blockDim.x) sk[i] = ker[i];
  __syncthreads();
  const long long total = (long long)B * T_out * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long bt = i / C;
    const int b = (int)(bt / T_out), t = (int)(bt % T_out);
    const float* xb = x + (long long)b * T_in * C + c;
    const int r0 = t * orig - width;
    const int k0 = r0 < 0 ? -r0 : 0;
    const int k1 = min(K, T_in - r0);
    float acc = 0.f;
    for (int k = k0; k < k1; ++k) acc = fmaf(xb[(long long)(r0 + k) * C], sk[k], acc);
    y[i] = acc;
  }
}

// y[b][t][0:C] = linear(lrelu(x, slope)) at t (align_corners=False, scale = 1/rate, nn.Upsample semantics),
// y[b][t][C:C+Cd] = skip[b][t]; rows of y are ldy floats
__global__ void k_lerp_up_cat(const float* __restrict__ x, int T, int C, int ldx, int rate, float slope,
                              const float* __restrict__ skip, int Cd, float* __restrict__ y, int ldy, int B) {
  const long long To = (long long)T * rate;
  const long long total = (long long)B * To * (C + Cd);
  const float scale = 1.0f / (float)rate;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % (C + Cd));
    const long long bt = i / (C + Cd);
    const int b = (int)(bt / To);
    const long long t = bt % To;
    float v;
    if (c < C) {
      float src = scale * ((float)t + 0.5f) - 0.5f;
      if (src < 0.f) src = 0.f;
      const int i0 = (int)src;
      const int i1 = i0 + (i0 < T - 1 ? 1 : 0);
      const float l1 = src - (float)i0, l0 = 1.f - l1;
      const float* xb = x + (long long)b * T * ldx + c;
      v = l0 * lrelu(xb[(long long)i0 * ldx], slope) + l1 * lrelu(xb[(long long)i1 * ldx], slope);
    } else {
      v = skip[((long long)b * To + t) * Cd + (c - C)];
    }
    y[((long long)b * To + t) * ldy + c] = v;
  }
}

// AdaIN (refinegan.py:74-94): v = lrelu(x + eps * w[c], 0.2); eps injected in the reference layout [B][C][T] or
// Philox(seed). mode 0: y = v; 1: y += v; 2: y = (y + v) / div
__global__ void k_adain(const float* __restrict__ x, int B, int T, int C, const float* __restrict__ w,
                        const float* __restrict__ eps, uint64_t seed, float slope, float* __restrict__ y, int mode,
                        float div) {
  const long long total = (long long)B * T * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long bt = i / C;
    const int b = (int)(bt / T), t = (int)(bt % T);
    const long long ei = ((long long)b * C + c) * T + t;
    const float e = eps ? eps[ei] : normal_at(seed, (uint64_t)ei);
    const float v = lrelu(x[i] + e * w[c], slope);
    if (mode == 0) y[i] = v;
    else if (mode == 1) y[i] = y[i] + v;
    else y[i] = (y[i] + v) / div;
  }
}

inline unsigned nb(long long n) {
  long long b = (n + 255) / 256;
  if (b > 65535LL * 16) b = 65535LL * 16;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace

hipError_t resample_dw(const float* x, int B, int T_in, int C, const float* ker, int K, int orig, int width, float* y,
                       int T_out, hipStream_t s) {
  hipLaunchKernelGGL(k_resample_dw, dim3(nb((long long)B * T_out * C)), dim3(256), (size_t)K * sizeof(float), s, x,
                     T_in, C, ker, K, orig, width, y, T_out, B);
  return hipGetLastError();
}

hipError_t lerp_up_cat(const float* x, int B, int T, int C, int ldx, int rate, float slope, const float* skip, int Cd,
                       float* y, int ldy, hipStream_t s) {
  hipLaunchKernelGGL(k_lerp_up_cat, dim3(nb((long long)B * T * rate * (C + Cd))), dim3(256), 0, s, x, T, C, ldx, rate,
                     slope, skip, Cd, y, ldy, B);
  return hipGetLastError();
}

hipError_t adain(const float* x, int B, int T, int C, const float* w, const float* eps, uint64_t seed, float slope,
                 float* y, int mode, float div, hipStream_t s) {
  hipLaunchKernelGGL(k_adain, dim3(nb((long long)B * T * C)), dim3(256), 0, s, x, B, T, C, w, eps, seed, slope, y,
                     mode, div);
  return hipGetLastError();
}

}  // namespace rvcx
