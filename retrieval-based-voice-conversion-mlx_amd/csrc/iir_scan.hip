// Zero-phase high-pass (scipy.signal.filtfilt, rvc/infer/pipeline.py:22-27, :439) as a chunk-parallel
// linear scan over second-order sections.
//
// The pipeline's 5th-order 48 Hz Butterworth is designed by scipy and handed over as SOS (exact zpk
// sections, scipy butter(..., output='sos')): each section is a 2-state DF2T biquad whose state matrix
// A = [[-a1, 1], [-a2, 0]] has |eigenvalues| <= 0.9942 and mild transient growth, so chunk-state
// propagation is stable (the order-5 companion form of (b, a) is not: ||F^512|| ~ 3e11 in fp64).
// The sections of one pass run as ONE cascaded linear system over n samples, chunks of L:
//   local  : every chunk from a zero state -> zero-state outputs y0 and end state e_c
//   carry  : S_0 = w * x0 (steady state for the constant input x0, scipy's zi semantics),
//            S_{c+1} = A^L S_c + e_c  as a two-level scan of affine maps
//   fix    : y_t = y0_t + (C A^k) S_c, k = t - cL  (fused into the next pass's local pass / the final pad)
// (Round 3-4's per-section form, one local / carry / fix round per section, measured slower and is gone.)
// fp64 throughout. Error vs scipy.sosfiltfilt ~1e-12; vs filtfilt(b, a) (the TF form the reference
// runs) ~6e-8 of the peak, which is the TF form's own rounding (tests/test_gpu_models.py).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rvcx_kernels.h"

namespace rvcx {

// ---------------------------------------------------------------- the whole cascade as one linear system
// The sections of one pass form one 2 nsec-state system (block lower-triangular, as stable as its sections), so a pass
// is ONE local / carry / fix round instead of one per section, and filtfilt is six launches: the backward local pass
// applies the forward pass's fix-up while it reads its input, and the last kernel applies the backward one while it
// reflect-pads. Tables (SosPlan::casc): coef [nsec][5] at 0, w [NS] at 40, pow[s] = A^(L 2^s) [NS][NS] at 48 + 64 s
// (s < 12), CA[k] = C A^k [NS] at 816 + 8 k (k < L); NS = 2 nsec <= 8.
namespace {
constexpr int CASC_W = 40, CASC_POW = 48, CASC_CA = 48 + 64 * 12;

// value t of a pass's final output, from its zero-state output y0 and chunk start states S (NS per chunk)
template <int NS>
__device__ __forceinline__ double casc_fixed(const double* y0, const double* S, const double* ca, int L, long long t) {
  const long long c = t / L;
  const int k = (int)(t - c * L);
  double v = y0[t];
#pragma unroll
  for (int i = 0; i < NS; ++i) v = fma(ca[CASC_CA + 8 * k + i], S[NS * c + i], v);
  return v;
}

// zero-state pass of the cascade over chunk c. Input: x (read reversed when rev), or -- when S_in is set -- the
// previous pass's final output y0_in + C A^k S_in evaluated on the fly (casc_fixed's arithmetic). A block of 64 lanes
// (one chunk each) stages its 64 L consecutive inputs through LDS: read coalesced (consecutive threads, consecutive
// samples; every load of the block in flight at once) into rows of L + 1 doubles, then each lane runs its chunk's
// recurrence from its row and leaves the outputs in place, written back coalesced. (One lane reading its own chunk
// from global memory waited out a load latency per sample or per batch of samples: 25-61 us per pass at C2, r05i-s.)
constexpr int CASC_LC = 128, CASC_B = 64;  // chunk length (SosPlan::casc_L, compile-time here), chunks per block
constexpr int CASC_LD = CASC_LC + 1;        // LDS row stride (doubles): lanes 0-31 / 32-63 each cover all banks
constexpr int CASC_NT = 256;                // threads per block: 4 waves stage, wave 0 runs the 64 recurrences
template <int NSEC>
__global__ __launch_bounds__(CASC_NT) void k_casc_local(const double* __restrict__ x, const double* __restrict__ S_in,
                                                        long long n, int rev, const double* __restrict__ tab,
                                                        double* __restrict__ y0, double* __restrict__ e) {
  constexpr int NS = 2 * NSEC, L = CASC_LC;
  extern __shared__ double smem_casc[];  // rows [CASC_B][CASC_LD], the C A^k rows [L][NS], the input states [65][NS]
  __shared__ double wsc[NS][CASC_B];     // the block scan of the chunk end states
  __shared__ double pw6[6 * 64];         // A^(L 2^s), s < 6, for that scan
  double* rows = smem_casc;
  double* ca_s = rows + CASC_B * CASC_LD;
  double* s_s = ca_s + L * NS;
  const int tid = threadIdx.x;
  const long long nch = (n + L - 1) / L;
  const long long tb0 = (long long)blockIdx.x * CASC_B * L;  // the block's first sample (processing order)
  const int cnt = (int)min((long long)CASC_B * L, n - tb0);  // samples of the block
  // the previous pass's chunks the block's samples come from: ti in [ta, tb], chunks ci0 .. ci0 + 64 at most
  const long long ta = rev ? n - 1 - (tb0 + cnt - 1) : tb0;
  const long long ci0 = ta / L;
  for (int i = tid; i < 6 * 64; i += CASC_NT) pw6[i] = tab[CASC_POW + i];
  if (S_in) {
    for (int i = tid; i < L * NS; i += CASC_NT) {
      const int k = i / NS, q = i - k * NS;
      ca_s[i] = tab[CASC_CA + 8 * k + q];
    }
    const long long nci = min((long long)CASC_B + 1, nch - ci0);
    for (int i = tid; i < nci * NS; i += CASC_NT) s_s[i] = S_in[NS * ci0 + i];
  }
  __syncthreads();
  auto input = [&](long long t) -> double {
    const long long ti = rev ? n - 1 - t : t;
    if (!S_in) return x[ti];
    const long long ci = ti / L;
    const int k = (int)(ti - ci * L);
    const double* sv = s_s + (ci - ci0) * NS;
    double v = x[ti];
#pragma unroll
    for (int i = 0; i < NS; ++i) v = fma(ca_s[k * NS + i], sv[i], v);
    return v;
  };
  // staging: element i of the block (row i / L, column i % L); 16 loads per thread in flight per group
  for (int i0 = 0; i0 < cnt; i0 += 16 * CASC_NT) {
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = i0 + u * CASC_NT + tid;
      v[u] = i < cnt ? input(tb0 + i) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = i0 + u * CASC_NT + tid;
      if (i < cnt) rows[(i / L) * CASC_LD + (i % L)] = v[u];
    }
  }
  __syncthreads();
  const long long c = (long long)blockIdx.x * CASC_B + tid;
  if (tid < CASC_B && c < nch) {
    double b0[NSEC], b1[NSEC], b2[NSEC], a1[NSEC], a2[NSEC], z0[NSEC], z1[NSEC];
#pragma unroll
    for (int j = 0; j < NSEC; ++j) {
      b0[j] = tab[5 * j], b1[j] = tab[5 * j + 1], b2[j] = tab[5 * j + 2], a1[j] = tab[5 * j + 3],
      a2[j] = tab[5 * j + 4];
      z0[j] = z1[j] = 0.0;
    }
    double* row = rows + tid * CASC_LD;
    const int len = (int)min((long long)L, n - c * L);
    auto step = [&](double u) -> double {
#pragma unroll
      for (int j = 0; j < NSEC; ++j) {
        const double y = b0[j] * u + z0[j];
        z0[j] = b1[j] * u - a1[j] * y + z1[j];
        z1[j] = b2[j] * u - a2[j] * y;
        u = y;
      }
      return u;
    };
    int t = 0;
    for (; t + 16 <= len; t += 16) {  // 16 inputs read ahead of their dependent chain, outputs written in place
      double u[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) u[k] = row[t + k];
#pragma unroll
      for (int k = 0; k < 16; ++k) u[k] = step(u[k]);
#pragma unroll
      for (int k = 0; k < 16; ++k) row[t + k] = u[k];
    }
    for (; t < len; ++t) row[t] = step(row[t]);
#pragma unroll
    for (int j = 0; j < NSEC; ++j) {
      wsc[2 * j][tid] = z0[j];
      wsc[2 * j + 1][tid] = z1[j];
    }
  } else if (tid < CASC_B) {
#pragma unroll
    for (int i = 0; i < NS; ++i) wsc[i][tid] = 0.0;
  }
  // the block's chunk end states e_k (zero past the last chunk) -> W_k = sum_{j <= k} A^(L (k - j)) e_j, the end state
  // of chunk k when the block starts from a zero state: a Hillis-Steele scan over the 64 chunk lanes of wave 0 with
  // the A^(L 2^s) tables (k_casc_carry then adds the block's start state)
  if (tid < CASC_B) {
    double a[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) a[i] = wsc[i][tid];
    for (int sidx = 0; (1 << sidx) < CASC_B; ++sidx) {
      const int d = 1 << sidx;
      double u[NS];
#pragma unroll
      for (int i = 0; i < NS; ++i) u[i] = tid >= d ? wsc[i][tid - d] : 0.0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (tid >= d) {
        const double* M = pw6 + 64 * sidx;
#pragma unroll
        for (int r = 0; r < NS; ++r) {
          double acc = a[r];
#pragma unroll
          for (int q = 0; q < NS; ++q) acc = fma(M[8 * r + q], u[q], acc);
          a[r] = acc;
        }
      }
#pragma unroll
      for (int i = 0; i < NS; ++i) wsc[i][tid] = a[i];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (c < nch) {
#pragma unroll
      for (int i = 0; i < NS; ++i) e[NS * c + i] = a[i];
    }
  }
  __syncthreads();
  for (int i = tid; i < cnt; i += CASC_NT) y0[tb0 + i] = rows[(i / L) * CASC_LD + (i % L)];
}

// chunk start states S_0 = w x0, S_{c+1} = A^L S_c + e_c, from k_casc_local's block scans (e holds W_k, the end state of
// chunk k of its 64-chunk block from a zero block start). Block b of this launch (64 threads, one per chunk of local
// block b) first walks the earlier blocks serially, S_start(j+1) = A^(64 L) S_start(j) + W_63(j) (NS lanes, one row
// each), then sets S_(c0+k) = A^(L k) S_start(b) + W_(k-1), the power by binary decomposition over the A^(L 2^s) tables.
// (Round 4's single-block Hillis-Steele scan over all chunks: 26 us per pass at C2; x0 = the pass input's first sample:
// x[0] / x[n - 1] (rev), or the previous pass's output there (S_in set).)
template <int NS>
__global__ void __launch_bounds__(CASC_B) k_casc_carry(const double* __restrict__ e, long long nch,
                                                       const double* __restrict__ tab, const double* __restrict__ x,
                                                       const double* __restrict__ S_in, long long n, int L, int rev,
                                                       double* __restrict__ S) {
  __shared__ double st[NS];
  const int tid = threadIdx.x;
  const long long b = blockIdx.x, c0 = b * CASC_B;
  if (tid < NS) {
    const long long i0 = rev ? n - 1 : 0;
    const double x0 = S_in ? casc_fixed<NS>(x, S_in, tab, L, i0) : x[i0];
    st[tid] = tab[CASC_W + tid] * x0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // the earlier blocks' aggregates W_63 come in groups of 256 (all loads of a group in flight), the A^(64 L) row of
  // lane r in registers: the serial walk then touches only LDS
  __shared__ double agg[256][NS];
  double p64[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) p64[q] = tid < NS ? tab[CASC_POW + 64 * 6 + 8 * tid + q] : 0.0;
  for (long long j0 = 0; j0 < b; j0 += 256) {
    const int cnt = (int)min((long long)256, b - j0);
    for (int i = tid; i < cnt * NS; i += CASC_B) {
      const int jj = i / NS, q = i - jj * NS;
      agg[jj][q] = e[NS * ((j0 + jj) * CASC_B + CASC_B - 1) + q];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int jj = 0; jj < cnt; ++jj) {
      double nv = 0.0;
      if (tid < NS) {
        double acc = agg[jj][tid];
#pragma unroll
        for (int q = 0; q < NS; ++q) acc = fma(p64[q], st[q], acc);
        nv = acc;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (tid < NS) st[tid] = nv;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  const long long c = c0 + tid;
  if (c >= nch) return;
  double v[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) v[i] = st[i];
  for (int sidx = 0; (1 << sidx) <= tid; ++sidx) {
    if (tid & (1 << sidx)) {
      const double* M = tab + CASC_POW + 64 * sidx;
      double r[NS];
#pragma unroll
      for (int rr = 0; rr < NS; ++rr) {
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < NS; ++q) acc = fma(M[8 * rr + q], v[q], acc);
        r[rr] = acc;
      }
#pragma unroll
      for (int i = 0; i < NS; ++i) v[i] = r[i];
    }
  }
  if (tid > 0) {
#pragma unroll
    for (int i = 0; i < NS; ++i) v[i] += e[NS * (c - 1) + i];
  }
#pragma unroll
  for (int i = 0; i < NS; ++i) S[NS * c + i] = v[i];
}

// the backward pass's final output (its fix-up applied on the fly), un-reversed, trimmed of the odd extension and
// reflect-padded by t_pad (k_filt_pad's indexing)
template <int NS>
__global__ void k_casc_final_pad(const double* __restrict__ y0b, const double* __restrict__ Sb,
                                 const double* __restrict__ tab, int L, long long ne, int padlen, long long n,
                                 long long t_pad, double* __restrict__ pad64, float* __restrict__ pad32) {
  const long long m = n + 2 * t_pad;
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < m; k += (long long)gridDim.x * blockDim.x) {
    long long j = k - t_pad;
    if (j < 0) j = -j;
    if (j >= n) j = 2 * (n - 1) - j;
    const double v = casc_fixed<NS>(y0b, Sb, tab, L, ne - 1 - (j + padlen));
    if (pad64) pad64[k] = v;
    pad32[k] = (float)v;
  }
}

template <int NSEC>
hipError_t casc_filtfilt(const SosPlan& p, const double* ext, long long ne, int padlen, long long n, long long t_pad,
                         double* ws, double* pad64, float* pad32, hipStream_t s) {
  constexpr int NS = 2 * NSEC;
  const int L = p.casc_L;
  if (L != CASC_LC) return hipErrorInvalidValue;  // k_casc_local's compile-time chunk length
  const long long nch = (ne + L - 1) / L;
  double* y0f = ws;
  double* y0b = y0f + ne;
  double* e = y0b + ne;
  double* Sf = e + NS * nch;
  double* Sb = Sf + NS * nch;
  const unsigned g = (unsigned)((nch + CASC_B - 1) / CASC_B);
  const size_t lds = sizeof(double) * ((size_t)CASC_B * CASC_LD + (size_t)CASC_LC * NS + (size_t)(CASC_B + 1) * NS);
  static bool lds_set = false;  // per instantiation: allow the ~72 KB of dynamic LDS once
  if (!lds_set) {
    hipError_t er = hipFuncSetAttribute(reinterpret_cast<const void*>(k_casc_local<NSEC>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (er != hipSuccess) return er;
    lds_set = true;
  }
  hipLaunchKernelGGL(k_casc_local<NSEC>, dim3(g), dim3(CASC_NT), lds, s, ext, nullptr, ne, 0, p.casc, y0f, e);
  hipLaunchKernelGGL(k_casc_carry<NS>, dim3(g), dim3(CASC_B), 0, s, e, nch, p.casc, ext, nullptr, ne, L, 0, Sf);
  // backward over the reversed forward output (y0f fixed up with Sf on the fly)
  hipLaunchKernelGGL(k_casc_local<NSEC>, dim3(g), dim3(CASC_NT), lds, s, y0f, Sf, ne, 1, p.casc, y0b, e);
  hipLaunchKernelGGL(k_casc_carry<NS>, dim3(g), dim3(CASC_B), 0, s, e, nch, p.casc, y0f, Sf, ne, L, 1, Sb);
  const long long m = n + 2 * t_pad;
  const unsigned gb = (unsigned)std::min<long long>((m + 255) / 256, 4096);
  hipLaunchKernelGGL(k_casc_final_pad<NS>, dim3(gb), dim3(256), 0, s, y0b, Sb, p.casc, L, ne, padlen, n, t_pad, pad64,
                     pad32);
  return hipGetLastError();
}
}  // namespace

hipError_t casc_filtfilt_pad(const SosPlan& p, const double* ext, long long ne, int padlen, long long n,
                             long long t_pad, double* ws, double* pad64, float* pad32, hipStream_t s) {
  switch (p.nsec) {
    case 1: return casc_filtfilt<1>(p, ext, ne, padlen, n, t_pad, ws, pad64, pad32, s);
    case 2: return casc_filtfilt<2>(p, ext, ne, padlen, n, t_pad, ws, pad64, pad32, s);
    case 3: return casc_filtfilt<3>(p, ext, ne, padlen, n, t_pad, ws, pad64, pad32, s);
    case 4: return casc_filtfilt<4>(p, ext, ne, padlen, n, t_pad, ws, pad64, pad32, s);
    default: return hipErrorInvalidValue;
  }
}

size_t casc_ws_doubles(long long ne, int L) {
  const long long nch = (ne + L - 1) / L;
  return (size_t)(2 * ne + 3 * 8 * nch + 16);
}

}  // namespace rvcx
