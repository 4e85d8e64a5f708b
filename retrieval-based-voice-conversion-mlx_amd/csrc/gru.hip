// RMVPE BiGRU recurrence (RMVPE.py:543-564: nn.GRU(384, 256, bidirectional, batch_first)).
//
// The input projection gi = x W_ih^T + b_ih (both directions, [T][1536]) is one MFMA GEMM
// launched before this kernel. What is left is 2 x T dependent steps of h' = GRUCell(gi_t, h)
// with W_hh = 768 x 256 fp32 (786 KB per direction: more than one CU's LDS + VGPRs can hold).
//
// Design: one launch, 4 workgroups of 1024 threads = 2 directions x 2 halves of the hidden
// units. Each workgroup owns 128 hidden units = 384 rows of W_hh (r, z, n rows of its units):
// the 256 r/z rows live in VGPRs (64 weights per thread, 4 threads per row), the 128 n rows in
// LDS (128 KB). Per step a workgroup computes its 128 new h values and hands them to the
// partner half through 8-byte {tag = step+1, value} granules written with agent-scope relaxed
// atomic stores (the data IS the flag; MI355X_MICROARCH.md "R2"), double-buffered by step parity;
// the partner polls them with agent-scope relaxed loads (sc1, L1-bypassing). Spins are bounded:
// on timeout the kernel sets *status and stops (no hang). The granule buffer must be zeroed
// before every launch (the caller's hipMemsetAsync).
//
// Cell arithmetic follows ATen GRUCell: r = sig(hg_r + ig_r), z = sig(hg_z + ig_z),
// n = tanh(ig_n + hg_n * r), h' = (h - n) * z + n, with hg = W_hh h + b_hh.
#include "rvcx_kernels.h"

namespace rvcx {

namespace {
constexpr int H = 256;
constexpr int UNITS = 128;     // hidden units per workgroup
constexpr int NT = 1024;
constexpr int LDS_LD = 260;    // padded LDS row for the n-gate rows
constexpr unsigned SPIN_LIMIT = 1u << 22;

__device__ __forceinline__ float sigm(float v) { return 1.f / (1.f + expf(-v)); }
}  // namespace

__global__ __launch_bounds__(NT, 1) void k_gru_bidir(const float* __restrict__ gi, const float* whh_f,
                                                     const float* bhh_f, const float* whh_b, const float* bhh_b,
                                                     int T, float* out, unsigned long long* xchg,
                                                     unsigned* status) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* wn = sm;                          // [128][LDS_LD] n-gate rows
  float* hbuf = wn + UNITS * LDS_LD;       // [2][256] h double buffer
  float* hg = hbuf + 2 * H;                // [384] hidden-gate pre-activations
  int& abort_flag = *reinterpret_cast<int*>(hg + 3 * UNITS);

  const int d = blockIdx.x >> 1;   // direction
  const int q = blockIdx.x & 1;    // half
  const int tid = threadIdx.x;
  const float* whh = d ? whh_b : whh_f;
  const float* bhh = d ? bhh_b : bhh_f;
  unsigned long long* mine = xchg + ((long long)(d * 2 + q) * 2) * UNITS;          // [2][128]
  unsigned long long* theirs = xchg + ((long long)(d * 2 + (1 - q)) * 2) * UNITS;  // [2][128]

  // register rows: local row lr = tid/4 in [0,256): lr<128 -> r gate unit lr ; else z gate unit lr-128
  const int lr = tid >> 2, seg = tid & 3;
  const int grow = (lr < UNITS) ? (q * UNITS + lr) : (H + q * UNITS + (lr - UNITS));
  float wr[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) wr[k] = whh[(long long)grow * H + seg * 64 + k];
  // LDS rows: n gate rows 512 + q*128 + j
  for (int idx = tid; idx < UNITS * H; idx += NT) {
    const int j = idx / H, k = idx % H;
    wn[j * LDS_LD + k] = whh[(long long)(2 * H + q * UNITS + j) * H + k];
  }
  for (int k = tid; k < 2 * H; k += NT) hbuf[k] = 0.f;
  if (tid == 0) abort_flag = 0;
  // per-unit constants for the gate threads
  float b_r = 0.f, b_z = 0.f, b_n = 0.f;
  const int unit = q * UNITS + tid;  // valid for tid < 128
  if (tid < UNITS) {
    b_r = bhh[unit];
    b_z = bhh[H + unit];
    b_n = bhh[2 * H + unit];
  }
  __syncthreads();

  const int nrow = tid >> 3, nseg = tid & 7;  // LDS part: row nrow (0..127), 32 columns nseg*32..
  int cur = 0;
  for (int s = 0; s < T; ++s) {
    const int t = d ? (T - 1 - s) : s;
    // prefetch input gates for this step (gate threads)
    float ig_r = 0.f, ig_z = 0.f, ig_n = 0.f;
    if (tid < UNITS) {
      const float* g = gi + (long long)t * (6 * H) + d * 3 * H;
      ig_r = g[unit];
      ig_z = g[H + unit];
      ig_n = g[2 * H + unit];
    }
    const float* h = hbuf + cur * H;
    // register rows: 64-column segment
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 64; k += 4) {
      const float4 hv = *reinterpret_cast<const float4*>(&h[seg * 64 + k]);
      acc = fmaf(wr[k], hv.x, acc);
      acc = fmaf(wr[k + 1], hv.y, acc);
      acc = fmaf(wr[k + 2], hv.z, acc);
      acc = fmaf(wr[k + 3], hv.w, acc);
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    if (seg == 0) hg[lr] = acc;
    // LDS rows: 32-column segment
    float acc2 = 0.f;
    const float* wrow = wn + nrow * LDS_LD + nseg * 32;
#pragma unroll
    for (int k = 0; k < 32; k += 4) {
      const float4 wv = *reinterpret_cast<const float4*>(&wrow[k]);
      const float4 hv = *reinterpret_cast<const float4*>(&h[nseg * 32 + k]);
      acc2 = fmaf(wv.x, hv.x, acc2);
      acc2 = fmaf(wv.y, hv.y, acc2);
      acc2 = fmaf(wv.z, hv.z, acc2);
      acc2 = fmaf(wv.w, hv.w, acc2);
    }
    acc2 += __shfl_xor(acc2, 1, 64);
    acc2 += __shfl_xor(acc2, 2, 64);
    acc2 += __shfl_xor(acc2, 4, 64);
    if (nseg == 0) hg[2 * UNITS + nrow] = acc2;
    __syncthreads();
    float* hn = hbuf + (cur ^ 1) * H;
    const unsigned epoch = (unsigned)s + 1u;
    unsigned long long* slot_m = mine + (s & 1) * UNITS;
    unsigned long long* slot_t = theirs + (s & 1) * UNITS;
    if (tid < UNITS) {
      const float hr = hg[tid] + b_r;
      const float hz = hg[UNITS + tid] + b_z;
      const float hnn = hg[2 * UNITS + tid] + b_n;
      const float r = sigm(hr + ig_r);
      const float z = sigm(hz + ig_z);
      const float n = tanhf(ig_n + hnn * r);
      const float hp = (h[unit] - n) * z + n;
      hn[unit] = hp;
      out[(long long)t * (2 * H) + d * H + unit] = hp;
      const unsigned long long g = ((unsigned long long)epoch << 32) | (unsigned long long)__float_as_uint(hp);
      __hip_atomic_store(&slot_m[tid], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (tid < 2 * UNITS) {
      // one wave polls the partner's 128 granules (2 per lane)
      if (tid < UNITS + 64) {
        const int j = tid - UNITS;
#pragma unroll
        for (int rep = 0; rep < 2; ++rep) {
          const int jj = j + rep * 64;
          unsigned spins = 0;
          unsigned long long g;
          while (true) {
            g = __hip_atomic_load(&slot_t[jj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((unsigned)(g >> 32) == epoch) break;
            if (++spins > SPIN_LIMIT) {
              abort_flag = 1;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          hn[(1 - q) * UNITS + jj] = __uint_as_float((unsigned)g);
        }
      }
    }
    __syncthreads();
    if (abort_flag) {
      if (tid == 0) atomicOr(status, 1u);
      return;
    }
    cur ^= 1;
  }
}

hipError_t gru_bidir(const float* gi, const float* whh_f, const float* bhh_f, const float* whh_b,
                     const float* bhh_b, int T, float* out, unsigned long long* xchg, unsigned* status,
                     hipStream_t s) {
  const size_t smem = (size_t)(UNITS * LDS_LD + 2 * H + 3 * UNITS + 4) * sizeof(float);
  hipError_t e = hipMemsetAsync(xchg, 0, sizeof(unsigned long long) * 4 * 2 * UNITS, s);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_gru_bidir), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)smem);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_gru_bidir, dim3(4), dim3(NT), smem, s, gi, whh_f, bhh_f, whh_b, bhh_b, T, out, xchg, status);
  return hipGetLastError();
}

}  // namespace rvcx
