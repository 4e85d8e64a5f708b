// Zero-phase high-pass (scipy.signal.filtfilt, rvc/infer/pipeline.py:22-27, :439) as a chunk-parallel
// linear scan over second-order sections.
//
// The pipeline's 5th-order 48 Hz Butterworth is designed by scipy and handed over as SOS (exact zpk
// sections, scipy butter(..., output='sos')): each section is a 2-state DF2T biquad whose state matrix
// A = [[-a1, 1], [-a2, 0]] has |eigenvalues| <= 0.9942 and mild transient growth, so chunk-state
// propagation is stable (the order-5 companion form of (b, a) is not: ||F^512|| ~ 3e11 in fp64).
// One pass of one section over n samples, chunks of L:
//   local  : every chunk from a zero state -> zero-state outputs y0 and end state e_c   (thread/chunk)
//   carry  : S_0 = w * x0 (steady state for the constant input x0, scipy's zi semantics),
//            S_{c+1} = A^L S_c + e_c  as a Hillis-Steele scan of affine maps            (one block)
//   fix    : y_t = y0_t + (C A^k) S_c, k = t - cL                                         (fused into the
//            next section's local pass, or the last section's output)
// fp64 throughout. Error vs scipy.sosfiltfilt ~1e-12; vs filtfilt(b, a) (the TF form the reference
// runs) ~6e-8 of the peak, which is the TF form's own rounding (tests/test_gpu_models.py).
#include <hip/hip_runtime.h>

#include "rvcx_kernels.h"

namespace rvcx {

namespace {
constexpr int SCAN_T = 1024;

__device__ __forceinline__ double in_at(const double* x, long long n, int rev, long long t) {
  return rev ? x[n - 1 - t] : x[t];
}
}  // namespace

// One lane per chunk; inputs are fetched NB at a time ahead of the recurrence (each lane's NB samples
// are one 128-B line) so the load latency overlaps the dependent fp64 chain of the previous batch.
constexpr int NB = 16;

// zero-state pass of section (coef: b0 b1 b2 a1 a2) over chunk c; input read reversed when rev
__global__ void k_sos_local(const double* __restrict__ x, long long n, int rev, const double* __restrict__ coef,
                            int L, double* __restrict__ y0, double* __restrict__ e) {
  const long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long nch = (n + L - 1) / L;
  if (c >= nch) return;
  const double b0 = coef[0], b1 = coef[1], b2 = coef[2], a1 = coef[3], a2 = coef[4];
  double z0 = 0.0, z1 = 0.0;
  const long long t0 = c * L, t1 = min(n, t0 + L);
  long long t = t0;
  double xb[NB];
  if (t + NB <= t1) {
#pragma unroll
    for (int i = 0; i < NB; ++i) xb[i] = in_at(x, n, rev, t + i);
  }
  for (; t + NB <= t1; t += NB) {
    double cur[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) cur[i] = xb[i];
    if (t + 2 * NB <= t1) {
#pragma unroll
      for (int i = 0; i < NB; ++i) xb[i] = in_at(x, n, rev, t + NB + i);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const double y = b0 * cur[i] + z0;
      z0 = b1 * cur[i] - a1 * y + z1;
      z1 = b2 * cur[i] - a2 * y;
      y0[t + i] = y;
    }
  }
  for (; t < t1; ++t) {
    const double xv = in_at(x, n, rev, t);
    const double y = b0 * xv + z0;
    z0 = b1 * xv - a1 * y + z1;
    z1 = b2 * xv - a2 * y;
    y0[t] = y;
  }
  e[2 * c] = z0;
  e[2 * c + 1] = z1;
}

// chunk start states: S_0 = w * x0, S_{c+1} = A^L S_c + e_c. One block of SCAN_T threads walks the chunks in
// segments of SCAN_T: an inclusive Hillis-Steele scan of e with the operator (u, v) -> P_s u + v, P_s =
// A^{L 2^s}, then S_{c+1} = A^{L (t+1)} S_seg + v_t with the power taken by binary decomposition.
__global__ void __launch_bounds__(SCAN_T) k_sos_carry(const double* __restrict__ e, long long nch,
                                                      const double* __restrict__ P, const double* __restrict__ w,
                                                      const double* __restrict__ x, long long n, int rev,
                                                      double* __restrict__ S) {
  __shared__ double v0[SCAN_T], v1[SCAN_T];
  __shared__ double seg[2];
  const int t = threadIdx.x;
  if (t == 0) {
    const double x0 = in_at(x, n, rev, 0);
    seg[0] = w[0] * x0;
    seg[1] = w[1] * x0;
    S[0] = seg[0];
    S[1] = seg[1];
  }
  __syncthreads();
  for (long long c0 = 0; c0 + 1 < nch; c0 += SCAN_T) {
    const long long c = c0 + t;  // this thread produces S_{c+1} from e_c
    const bool act = c + 1 < nch;
    double a = act ? e[2 * c] : 0.0, b = act ? e[2 * c + 1] : 0.0;
    for (int s = 0; (1 << s) < SCAN_T; ++s) {
      v0[t] = a;
      v1[t] = b;
      __syncthreads();
      const int d = 1 << s;
      if (t >= d) {
        const double* M = P + 4 * s;
        const double u0 = v0[t - d], u1 = v1[t - d];
        a = M[0] * u0 + M[1] * u1 + a;
        b = M[2] * u0 + M[3] * u1 + b;
      }
      __syncthreads();
    }
    // + A^{L (t+1)} S_seg
    double s0 = seg[0], s1 = seg[1];
    const int pw = t + 1;
    for (int s = 0; (1 << s) <= pw; ++s) {
      if (pw & (1 << s)) {
        const double* M = P + 4 * s;
        const double r0 = M[0] * s0 + M[1] * s1, r1 = M[2] * s0 + M[3] * s1;
        s0 = r0;
        s1 = r1;
      }
    }
    a += s0;
    b += s1;
    if (act) {
      S[2 * (c + 1)] = a;
      S[2 * (c + 1) + 1] = b;
    }
    __syncthreads();
    const long long last = min(nch - 2, c0 + SCAN_T - 1);  // the segment's last produced state
    if (c == last) {
      seg[0] = a;
      seg[1] = b;
    }
    __syncthreads();
  }
}

// final output of section j for chunk c (y0 + (C A^k) S_c), then, when next_coef is set, the zero-state
// pass of section j+1 over it (y0n, en); otherwise the final samples go to out.
__global__ void k_sos_fix(const double* __restrict__ y0, long long n, int L, const double* __restrict__ S,
                          const double* __restrict__ CA, const double* __restrict__ next_coef,
                          double* __restrict__ y0n, double* __restrict__ en, double* __restrict__ out) {
  const long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long nch = (n + L - 1) / L;
  if (c >= nch) return;
  const double s0 = S[2 * c], s1 = S[2 * c + 1];
  const long long t0 = c * L, t1 = min(n, t0 + L);
  double b0 = 0, b1 = 0, b2 = 0, a1 = 0, a2 = 0;
  if (next_coef) b0 = next_coef[0], b1 = next_coef[1], b2 = next_coef[2], a1 = next_coef[3], a2 = next_coef[4];
  double* dst = next_coef ? y0n : out;
  double z0 = 0.0, z1 = 0.0;
  long long t = t0;
  double xb[NB];
  if (t + NB <= t1) {
#pragma unroll
    for (int i = 0; i < NB; ++i) xb[i] = y0[t + i];
  }
  for (; t + NB <= t1; t += NB) {
    double cur[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) cur[i] = xb[i];
    if (t + 2 * NB <= t1) {
#pragma unroll
      for (int i = 0; i < NB; ++i) xb[i] = y0[t + NB + i];
    }
    const int k0 = (int)(t - t0);
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const double xv = cur[i] + (CA[2 * (k0 + i)] * s0 + CA[2 * (k0 + i) + 1] * s1);
      if (next_coef) {
        const double y = b0 * xv + z0;
        z0 = b1 * xv - a1 * y + z1;
        z1 = b2 * xv - a2 * y;
        dst[t + i] = y;
      } else {
        dst[t + i] = xv;
      }
    }
  }
  for (; t < t1; ++t) {
    const int k = (int)(t - t0);
    const double xv = y0[t] + (CA[2 * k] * s0 + CA[2 * k + 1] * s1);
    if (next_coef) {
      const double y = b0 * xv + z0;
      z0 = b1 * xv - a1 * y + z1;
      z1 = b2 * xv - a2 * y;
      dst[t] = y;
    } else {
      dst[t] = xv;
    }
  }
  if (next_coef) {
    en[2 * c] = z0;
    en[2 * c + 1] = z1;
  }
}

size_t sos_ws_doubles(long long n_ext, int L) {
  const long long nch = (n_ext + L - 1) / L;
  return (size_t)(2 * n_ext + 4 * nch + 16);
}

// one lfilter pass over x (read reversed when rev) through all sections -> out (processing order)
hipError_t sos_pass(const SosPlan& p, const double* x, long long n, int rev, double* out, double* ws, hipStream_t s) {
  const int L = p.L;
  const long long nch = (n + L - 1) / L;
  double* ya = ws;
  double* yb = ya + n;
  double* e = yb + n;
  double* S = e + 2 * nch;
  const unsigned g = (unsigned)((nch + 63) / 64);
  hipLaunchKernelGGL(k_sos_local, dim3(g), dim3(64), 0, s, x, n, rev, p.coef(0), L, ya, e);
  for (int j = 0; j < p.nsec; ++j) {
    hipLaunchKernelGGL(k_sos_carry, dim3(1), dim3(SCAN_T), 0, s, e, nch, p.pow(j), p.w(j), x, n, rev, S);
    const bool last = j + 1 == p.nsec;
    hipLaunchKernelGGL(k_sos_fix, dim3(g), dim3(64), 0, s, ya, n, L, S, p.ca(j), last ? nullptr : p.coef(j + 1),
                       yb, e, last ? out : nullptr);
    std::swap(ya, yb);
  }
  return hipGetLastError();
}

}  // namespace rvcx
