// Per-sample harmonic source of the MRF HiFi-GAN and RefineGAN decoders: SineGenerator._f02sine + forward +
// the merging Linear + tanh (rvc/lib/algorithm/generators/hifigan_mrf.py:120-230, refinegan.py:158-236).
//
// Per batch row and harmonic h (H = harmonic_num + 1), over the N = L * upp upsampled samples:
//   rad[n]   = (f0_up[n] * (h + 1) / sr) % 1          (+ rand_ini[h] at n = 0, rand_ini[0] = 0)
//   c1       = cumsum(rad)                             (torch CPU cumsum: double accumulation, float output)
//   shift[n] = -1 where (c1[n] % 1) - (c1[n-1] % 1) < 0, else 0   (n >= 1)
//   c2       = cumsum(rad + shift)
//   sine     = sin(c2 * 2 * pi) * 0.1 ; uv = f0_up > 0 ; amp = uv * 0.003 + (1 - uv) * 0.1 / 3
//   x[h]     = sine * uv + amp * eps[n][h]
// har[n] = tanh(sum_h x[h] * w[h] + b).
//
// Exactness: every rad (and rad + shift, rounded to float first as torch does) is a multiple of 2^-33 for
// f0 >= 50 Hz at sr >= 16 kHz (and 0 when unvoiced), and every partial sum is below 2^20, so each double
// addition is exact: a chunked parallel scan (per-chunk sums -> chunk prefix -> in-chunk block scan) is
// bit-identical to torch's sequential loop. Elementwise float ops keep torch's rounding (no FMA contraction).
#include <cmath>

#include "rvcx_kernels.h"

#pragma clang fp contract(off)

namespace rvcx {

namespace {

constexpr int SH_T = 256;   // threads per block
constexpr int SH_V = 4;     // consecutive samples per thread
constexpr int SH_CHUNK = SH_T * SH_V;

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
  uint32_t c[4] = {(uint32_t)(idx >> 1), (uint32_t)(idx >> 33), 0x48524d53u, 0u};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float u1 = ((c[0] >> 8) + 1) * (1.0f / 16777217.0f);
  const float u2 = (c[1] >> 8) * (1.0f / 16777216.0f);
  const float r = sqrtf(-2.f * logf(u1));
  const float th = 6.283185307179586f * u2;
  return (idx & 1) ? r * sinf(th) : r * cosf(th);
}
__device__ __forceinline__ float uniform_at(uint64_t seed, uint64_t idx) {
  uint32_t c[4] = {(uint32_t)idx, (uint32_t)(idx >> 32), 0x494e4954u, 1u};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return (c[0] >> 8) * (1.0f / 16777216.0f);  // [0, 1)
}

struct Src {
  const float* f0;  // [B][L] frame f0
  int B, L, upp, H, linear;
  float sr;
  const float* eps;   // [B][N][H] or null (Philox normals)
  const float* ini;   // [B][H] or null (Philox uniforms); element 0 forced to 0
  uint64_t seed;
};

// f0 upsampled to sample n: nearest (nn.Upsample, hifigan_mrf.py:276) or linear with align_corners=False
// (F.interpolate(..., mode="linear"), refinegan.py:402)
__device__ __forceinline__ float f0_at(const Src& s, const float* fb, long long n) {
  if (!s.linear) return fb[n / s.upp];
  const float scale = (float)s.L / (float)((long long)s.L * s.upp);
  float x = ((float)n + 0.5f) * scale - 0.5f;
  if (x < 0.f) x = 0.f;
  const int x0 = (int)x;
  const int x1 = x0 + (x0 < s.L - 1 ? 1 : 0);
  const float l1 = x - (float)x0, l0 = 1.f - l1;
  return l0 * fb[x0] + l1 * fb[x1];
}

__device__ __forceinline__ float rad_at(const Src& s, const float* fb, long long n, int h, float ini) {
  const float f = f0_at(s, fb, n) * (float)(h + 1);  // f0_buf[..., h] = f0 * (h + 1) (float)
  const float q = f / s.sr;
  float r = q - floorf(q);  // torch.remainder(q, 1)
  if (n == 0) r = r + ini;
  return r;
}

__device__ __forceinline__ float ini_at(const Src& s, int b, int h) {
  if (h == 0) return 0.f;  // rand_ini[:, 0] = 0
  return s.ini ? s.ini[b * s.H + h] : uniform_at(s.seed, (uint64_t)b * s.H + h);
}

// exclusive block scan of one double per thread; returns this thread's exclusive prefix and the block total
__device__ __forceinline__ double block_exscan(double v, double* wsum, double& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double u = __shfl_up(inc, d);
    if (lane >= d) inc += u;
  }
  __syncthreads();
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  double pre = inc - v;
  total = 0.0;
  for (int k = 0; k < SH_T / 64; ++k) {
    if (k < w) pre += wsum[k];
    total += wsum[k];
  }
  return pre;
}

// pass 1 (stage 0): chunk sums of rad; pass 2 (stage 1): chunk sums of rad + shift
template <int STAGE>
__global__ __launch_bounds__(SH_T) void k_harm_sums(Src s, const double* pre1, double* sums, int nchunk) {
  __shared__ double wsum[SH_T / 64];
  const int c = blockIdx.x, b = blockIdx.y;
  const long long N = (long long)s.L * s.upp;
  const float* fb = s.f0 + (long long)b * s.L;
  const long long n0 = (long long)c * SH_CHUNK + (long long)threadIdx.x * SH_V;
  for (int h = 0; h < s.H; ++h) {
    const float ini = ini_at(s, b, h);
    float r[SH_V];
    double ts = 0.0;
#pragma unroll
    for (int v = 0; v < SH_V; ++v) {
      r[v] = (n0 + v < N) ? rad_at(s, fb, n0 + v, h, ini) : 0.f;
      ts += (double)r[v];
    }
    double total;
    if (STAGE == 1) {
      // c1 at every sample: chunk prefix + in-chunk prefix; shift from consecutive (c1 % 1)
      const double cpre = pre1[((long long)b * s.H + h) * nchunk + c];
      double acc = cpre + block_exscan(ts, wsum, total);
      float prev = (float)acc;  // c1[n0 - 1] (the exclusive prefix)
      prev = prev - floorf(prev);
      double ts2 = 0.0;
#pragma unroll
      for (int v = 0; v < SH_V; ++v) {
        if (n0 + v >= N) break;
        acc += (double)r[v];
        float cf = (float)acc;
        cf = cf - floorf(cf);
        const float shift = (n0 + v > 0 && cf - prev < 0.f) ? -1.f : 0.f;
        prev = cf;
        ts2 += (double)(r[v] + shift);
      }
      ts = ts2;
    }
    block_exscan(ts, wsum, total);
    if (threadIdx.x == 0) sums[((long long)b * s.H + h) * nchunk + c] = total;
  }
}

// exclusive prefix of each (b, h) row of chunk sums, in place (exact in any order; one thread per row)
__global__ void k_harm_rowscan(double* sums, int rows, int nchunk) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  double* p = sums + (long long)r * nchunk;
  double acc = 0.0;
  for (int c = 0; c < nchunk; ++c) {
    const double v = p[c];
    p[c] = acc;
    acc += v;
  }
}

__global__ __launch_bounds__(SH_T) void k_harm_emit(Src s, const double* pre1, const double* pre2, int nchunk,
                                                    const float* lin_w, float lin_b, float* har, long long har_ld) {
  __shared__ double wsum[SH_T / 64];
  const int c = blockIdx.x, b = blockIdx.y;
  const long long N = (long long)s.L * s.upp;
  const float* fb = s.f0 + (long long)b * s.L;
  const long long n0 = (long long)c * SH_CHUNK + (long long)threadIdx.x * SH_V;
  float mix[SH_V];
  float uvv[SH_V];
#pragma unroll
  for (int v = 0; v < SH_V; ++v) {
    mix[v] = 0.f;
    uvv[v] = (n0 + v < N && f0_at(s, fb, n0 + v) > 0.f) ? 1.f : 0.f;
  }
  const float amp_v = 0.003f, amp_u = (0.1f) / 3.0f;  // (1 - uv) * sine_amp / 3 with uv = 0
  const float two_pi_a = 2.0f, two_pi_b = 3.14159265358979323846f;
  for (int h = 0; h < s.H; ++h) {
    const float ini = ini_at(s, b, h);
    const long long row = (long long)b * s.H + h;
    float r[SH_V];
    double ts = 0.0;
#pragma unroll
    for (int v = 0; v < SH_V; ++v) {
      r[v] = (n0 + v < N) ? rad_at(s, fb, n0 + v, h, ini) : 0.f;
      ts += (double)r[v];
    }
    double total;
    double acc = pre1[row * nchunk + c] + block_exscan(ts, wsum, total);
    float prev = (float)acc;
    prev = prev - floorf(prev);
    float x[SH_V];
    double ts2 = 0.0;
#pragma unroll
    for (int v = 0; v < SH_V; ++v) {
      x[v] = 0.f;
      if (n0 + v >= N) continue;
      acc += (double)r[v];
      float cf = (float)acc;
      cf = cf - floorf(cf);
      const float shift = (n0 + v > 0 && cf - prev < 0.f) ? -1.f : 0.f;
      prev = cf;
      x[v] = r[v] + shift;
      ts2 += (double)x[v];
    }
    double acc2 = pre2[row * nchunk + c] + block_exscan(ts2, wsum, total);
    const float w = lin_w[h];
#pragma unroll
    for (int v = 0; v < SH_V; ++v) {
      if (n0 + v >= N) continue;
      acc2 += (double)x[v];
      const float ph = ((float)acc2 * two_pi_a) * two_pi_b;  // cumsum(...) * 2 * np.pi
      const float sine = sinf(ph) * 0.1f;
      const float uv = uvv[v];
      const float amp = uv * amp_v + (1.f - uv) * 0.1f / 3.0f;
      const long long ei = ((long long)b * N + n0 + v) * s.H + h;
      const float e = s.eps ? s.eps[ei] : normal_at(s.seed, (uint64_t)ei);
      const float xv = sine * uv + amp * e;
      mix[v] = (h == 0) ? xv * w : mix[v] + xv * w;
    }
    (void)amp_u;
  }
#pragma unroll
  for (int v = 0; v < SH_V; ++v)
    if (n0 + v < N) har[(long long)b * har_ld + n0 + v] = tanhf(mix[v] + lin_b);
}

}  // namespace

size_t harm_source_ws_doubles(int B, int L, int upp, int H) {
  const long long N = (long long)L * upp;
  const long long nchunk = (N + SH_CHUNK - 1) / SH_CHUNK;
  return (size_t)2 * B * H * nchunk;
}

hipError_t harm_source(const float* f0, int B, int L, int upp, float sr, int H, int linear_up, const float* eps,
                       const float* ini, uint64_t seed, const float* lin_w, float lin_b, double* ws, float* har,
                       long long har_ld, hipStream_t st) {
  if (B <= 0 || L <= 0 || upp <= 0 || H <= 0) return hipErrorInvalidValue;
  const long long N = (long long)L * upp;
  const int nchunk = (int)((N + SH_CHUNK - 1) / SH_CHUNK);
  Src s{f0, B, L, upp, H, linear_up, sr, eps, ini, seed};
  double* p1 = ws;
  double* p2 = ws + (size_t)B * H * nchunk;
  const dim3 grid(nchunk, B);
  const int rows = B * H;
  hipLaunchKernelGGL(k_harm_sums<0>, grid, dim3(SH_T), 0, st, s, nullptr, p1, nchunk);
  hipLaunchKernelGGL(k_harm_rowscan, dim3((rows + 63) / 64), dim3(64), 0, st, p1, rows, nchunk);
  hipLaunchKernelGGL(k_harm_sums<1>, grid, dim3(SH_T), 0, st, s, p1, p2, nchunk);
  hipLaunchKernelGGL(k_harm_rowscan, dim3((rows + 63) / 64), dim3(64), 0, st, p2, rows, nchunk);
  hipLaunchKernelGGL(k_harm_emit, grid, dim3(SH_T), 0, st, s, p1, p2, nchunk, lin_w, lin_b, har, har_ld);
  return hipGetLastError();
}

}  // namespace rvcx
