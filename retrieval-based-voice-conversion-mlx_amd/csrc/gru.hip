// RMVPE BiGRU recurrence (RMVPE.py:543-564: nn.GRU(384, 256, bidirectional, batch_first)).
//
// The input projection gi = x W_ih^T + b_ih (both directions, [T][1536]) is one MFMA GEMM
// launched before this kernel. What is left is 2 x T dependent steps of h' = GRUCell(gi_t, h)
// with W_hh = 768 x 256 fp32 (786 KB per direction: more than one CU's VGPRs + LDS can hold).
//
// Design: one launch of 4 workgroups = 2 directions x 2 halves of the hidden units. A workgroup
// owns 128 hidden units = 384 rows of W_hh (its units' r, z, n rows) and keeps ALL of them in
// VGPRs: 768 threads, thread (g, r) holds row r's 128 columns of column-half g (128 floats).
//   g = 0 : columns of the workgroup's OWN units  -> dot with h_own (known locally)
//   g = 1 : columns of the PARTNER's units        -> dot with h_partner (received)
// Per step the two column halves run concurrently in different waves, so the partner hand-off
// latency overlaps the own-half dot products; the gate threads then add both halves.
// Hand-off: 8-byte {tag = step + 1, value} granules stored with agent-scope relaxed atomics (the
// data IS the flag; MI355X_MICROARCH.md, hand-off "R2"), double-buffered by step parity; every
// partner-half wave polls all 128 granules (2 per lane) with agent-scope relaxed loads (sc1,
// L1-bypassing). Spins are bounded: on timeout *status is set and the kernel exits (no hang).
// The granule buffer is zeroed before every launch (hipMemsetAsync in gru_bidir).
//
// Cell arithmetic follows ATen GRUCell: r = sig(hg_r + ig_r), z = sig(hg_z + ig_z),
// n = tanh(ig_n + hg_n * r), h' = (h - n) * z + n, with hg = W_hh h + b_hh.
#include "rvcx_kernels.h"

namespace rvcx {

namespace {
constexpr int H = 256;
constexpr int UNITS = 128;  // hidden units per workgroup
constexpr int ROWS = 3 * UNITS;
constexpr int NT = 2 * ROWS;  // 768 threads
constexpr unsigned SPIN_LIMIT = 1u << 22;

__device__ __forceinline__ float sigm(float v) { return 1.f / (1.f + expf(-v)); }
}  // namespace

__global__ __launch_bounds__(NT, 1) void k_gru_bidir(const float* __restrict__ gi, const float* whh_f,
                                                     const float* bhh_f, const float* whh_b, const float* bhh_b,
                                                     int T, float* out, unsigned long long* xchg,
                                                     unsigned* status) {
  __shared__ __attribute__((aligned(16))) float h_own[UNITS];
  __shared__ __attribute__((aligned(16))) float h_par[NT / 64][UNITS];  // per-wave copy of the partner half
  __shared__ float part[2][ROWS];
  __shared__ float bias_h[ROWS];
  __shared__ int abort_flag;

  const int d = blockIdx.x >> 1;  // direction
  const int q = blockIdx.x & 1;   // half
  // blockIdx.y = independent sequence (batched streams / utterances of one length)
  gi += (long long)blockIdx.y * T * 6 * H;
  out += (long long)blockIdx.y * T * 2 * H;
  xchg += (long long)blockIdx.y * 4 * 2 * UNITS;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int grp = tid / ROWS;     // 0: own columns, 1: partner columns (wave-uniform: ROWS % 64 == 0)
  const int r = tid - grp * ROWS; // local row: gate r / 128, unit r % 128
  const float* whh = d ? whh_b : whh_f;
  const float* bhh = d ? bhh_b : bhh_f;
  unsigned long long* mine = xchg + ((long long)(d * 2 + q) * 2) * UNITS;          // [2][128]
  unsigned long long* theirs = xchg + ((long long)(d * 2 + (1 - q)) * 2) * UNITS;  // [2][128]

  const int gate = r / UNITS, unit = r % UNITS;
  const int grow = gate * H + q * UNITS + unit;
  const int colbase = (grp == 0 ? q : 1 - q) * UNITS;
  float w[UNITS];
#pragma unroll
  for (int k = 0; k < UNITS; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(&whh[(long long)grow * H + colbase + k]);
    w[k] = v.x;
    w[k + 1] = v.y;
    w[k + 2] = v.z;
    w[k + 3] = v.w;
  }
  if (tid < UNITS) h_own[tid] = 0.f;
  if (tid == 0) abort_flag = 0;
  const int gunit = q * UNITS + tid;  // gate threads: tid < 128
  if (tid < ROWS) bias_h[tid] = bhh[(tid / UNITS) * H + q * UNITS + tid % UNITS];
  float* hp = h_par[wave];
  __syncthreads();

  for (int s = 0; s < T; ++s) {
    const int t = d ? (T - 1 - s) : s;
    // ---- phase A: half dot products (own half uses h_own(s-1); partner half waits for it)
    const float* hv;
    if (grp == 0) {
      hv = h_own;
    } else {
      if (s > 0) {
        const unsigned epoch = (unsigned)s;  // partner's h(s-1), published with tag s
        const unsigned long long* slot = theirs + ((s - 1) & 1) * UNITS;
#pragma unroll
        for (int rep = 0; rep < 2; ++rep) {
          const int jj = lane + rep * 64;
          unsigned spins = 0;
          unsigned long long gv;
          while (true) {
            gv = __hip_atomic_load(&slot[jj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((unsigned)(gv >> 32) == epoch) break;
            if (++spins > SPIN_LIMIT) {
              abort_flag = 1;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          hp[jj] = __uint_as_float((unsigned)gv);
        }
      } else {
        hp[lane] = 0.f;
        hp[lane + 64] = 0.f;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      hv = hp;
    }
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int k = 0; k < UNITS; k += 16) {
      const float4 x0 = *reinterpret_cast<const float4*>(&hv[k]);
      const float4 x1 = *reinterpret_cast<const float4*>(&hv[k + 4]);
      const float4 x2 = *reinterpret_cast<const float4*>(&hv[k + 8]);
      const float4 x3 = *reinterpret_cast<const float4*>(&hv[k + 12]);
      a0 = fmaf(w[k], x0.x, a0); a0 = fmaf(w[k + 1], x0.y, a0); a0 = fmaf(w[k + 2], x0.z, a0); a0 = fmaf(w[k + 3], x0.w, a0);
      a1 = fmaf(w[k + 4], x1.x, a1); a1 = fmaf(w[k + 5], x1.y, a1); a1 = fmaf(w[k + 6], x1.z, a1); a1 = fmaf(w[k + 7], x1.w, a1);
      a2 = fmaf(w[k + 8], x2.x, a2); a2 = fmaf(w[k + 9], x2.y, a2); a2 = fmaf(w[k + 10], x2.z, a2); a2 = fmaf(w[k + 11], x2.w, a2);
      a3 = fmaf(w[k + 12], x3.x, a3); a3 = fmaf(w[k + 13], x3.y, a3); a3 = fmaf(w[k + 14], x3.z, a3); a3 = fmaf(w[k + 15], x3.w, a3);
    }
    part[grp][r] = (a0 + a1) + (a2 + a3);
    float ig_r = 0.f, ig_z = 0.f, ig_n = 0.f;
    if (tid < UNITS) {  // input gates for this step (issued before the barrier)
      const float* g = gi + (long long)t * (6 * H) + d * 3 * H;
      ig_r = g[gunit];
      ig_z = g[H + gunit];
      ig_n = g[2 * H + gunit];
    }
    __syncthreads();
    if (abort_flag) {
      if (tid == 0) atomicOr(status, 1u);
      return;
    }
    // ---- phase B: gates for the 128 own units, publish h(s)
    if (tid < UNITS) {
      const float hr = (part[0][tid] + part[1][tid]) + bias_h[tid];
      const float hz = (part[0][UNITS + tid] + part[1][UNITS + tid]) + bias_h[UNITS + tid];
      const float hn = (part[0][2 * UNITS + tid] + part[1][2 * UNITS + tid]) + bias_h[2 * UNITS + tid];
      const float rr = sigm(hr + ig_r);
      const float zz = sigm(hz + ig_z);
      const float nn = tanhf(ig_n + hn * rr);
      const float hprev = h_own[tid];
      const float hnew = (hprev - nn) * zz + nn;
      h_own[tid] = hnew;
      out[(long long)t * (2 * H) + d * H + gunit] = hnew;
      const unsigned long long g =
          ((unsigned long long)(unsigned)(s + 1) << 32) | (unsigned long long)__float_as_uint(hnew);
      __hip_atomic_store(&mine[(s & 1) * UNITS + tid], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
}

hipError_t gru_bidir(const float* gi, const float* whh_f, const float* bhh_f, const float* whh_b,
                     const float* bhh_b, int T, float* out, unsigned long long* xchg, unsigned* status,
                     hipStream_t s, int B) {
  // the two halves of a direction spin on each other: all 4B workgroups (1 per CU) must be co-resident
  if (B < 1 || 4 * B > 256) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(xchg, 0, sizeof(unsigned long long) * gru_xchg_words(B), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_gru_bidir, dim3(4, B), dim3(NT), 0, s, gi, whh_f, bhh_f, whh_b, bhh_b, T, out, xchg, status);
  return hipGetLastError();
}

}  // namespace rvcx
