// Correctly rounded double-precision natural log on the device, for the integer coarse-pitch
// quantisation of Pipeline.get_f0 (rvc/infer/pipeline.py:283-289: rint(f(log(1 + f0/700)))).
//
// Why: the coarse pitch is integer output, so a 1-ulp difference in log can flip rint() when the
// scaled mel value lands on a half-integer. OCML's log is faithful (<= 1 ulp), not correctly rounded.
// The reference evaluates np.log on the host (glibc or numpy's own SIMD kernels, which differ from each
// other by an ulp on ~0.2% of inputs); the only machine-independent target is the correctly rounded log,
// which every one of them returns on the vast majority of inputs (tests/test_gpu_f0_post.py measures it).
//
// Method: y = 2^e * m with m in [sqrt(1/2), sqrt(2)); log(m) = 2 atanh(s), s = (m-1)/(m+1), |s| <= 0.1716,
// evaluated in double-double (~104 bits) with 24 series terms (s^49/49 < 2^-130 relative), plus e * ln2 in
// double-double; the sum rounded once to double. Products that need an fma are explicit fma calls, and every
// function turns contraction off: a contracted a*b + c next to the rounded a*b breaks the error-free
// transformations (measured: HIP's default fp-contract=fast made 17% of the sweep 1 ulp off on the device).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

namespace rvcx {
namespace dd {

struct D2 {
  double hi, lo;
};

__host__ __device__ __forceinline__ D2 two_sum(double a, double b) {
#pragma clang fp contract(off)
  const double s = a + b;
  const double bb = s - a;
  const double e = (a - (s - bb)) + (b - bb);
  return {s, e};
}
__host__ __device__ __forceinline__ D2 quick_two_sum(double a, double b) {
#pragma clang fp contract(off)
  const double s = a + b;
  return {s, b - (s - a)};
}
__host__ __device__ __forceinline__ D2 two_prod(double a, double b) {
#pragma clang fp contract(off)
  const double p = a * b;
  return {p, __builtin_fma(a, b, -p)};
}
__host__ __device__ __forceinline__ D2 add(D2 a, D2 b) {
#pragma clang fp contract(off)
  D2 s = two_sum(a.hi, b.hi);
  D2 t = two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = quick_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return quick_two_sum(s.hi, s.lo);
}
__host__ __device__ __forceinline__ D2 mul(D2 a, D2 b) {
#pragma clang fp contract(off)
  D2 p = two_prod(a.hi, b.hi);
  p.lo += __builtin_fma(a.hi, b.lo, a.lo * b.hi);
  return quick_two_sum(p.hi, p.lo);
}
__host__ __device__ __forceinline__ D2 mul_d(D2 a, double b) {
#pragma clang fp contract(off)
  D2 p = two_prod(a.hi, b);
  p.lo += a.lo * b;
  return quick_two_sum(p.hi, p.lo);
}
// (a.hi + a.lo) / (b.hi + b.lo): one long-division correction step (relative error ~2^-104)
__host__ __device__ __forceinline__ D2 div(D2 a, D2 b) {
#pragma clang fp contract(off)
  const double q1 = a.hi / b.hi;
  D2 r = add(a, mul_d(b, -q1));
  const double q2 = r.hi / b.hi;
  r = add(r, mul_d(b, -q2));
  const double q3 = r.hi / b.hi;
  D2 q = quick_two_sum(q1, q2);
  return add(q, D2{q3, 0.0});
}

// log(y) for finite y > 0, correctly rounded (barring a true value within ~2^-100 relative of a rounding
// midpoint). y <= 0 / inf / nan follow IEEE log.
__host__ __device__ inline double log_cr(double y) {
#pragma clang fp contract(off)
  if (!(y > 0.0) || y == HUGE_VAL) return log(y);
  int e = 0;
  double m = frexp(y, &e);  // m in [0.5, 1)
  if (m < 0.70710678118654752440) {
    m *= 2.0;
    e -= 1;
  }
  // s = (m - 1) / (m + 1); m - 1 is exact (Sterbenz), m + 1 carried as a double-double
  const D2 num{m - 1.0, 0.0};
  const D2 den = two_sum(m, 1.0);
  const D2 s = div(num, den);
  const D2 s2 = mul(s, s);
  // atanh(s)/s = sum_k s^(2k) / (2k + 1), Horner from k = 24 down; 1/(2k+1) as double-doubles
  constexpr int K = 24;
  D2 p{1.0 / (2 * K + 1), 0.0};
  {
    const double d = 2 * K + 1;
    p.lo = __builtin_fma(-p.hi, d, 1.0) / d;
  }
  for (int k = K - 1; k >= 0; --k) {
    const double d = 2 * k + 1;
    const double h = 1.0 / d;
    const D2 c{h, __builtin_fma(-h, d, 1.0) / d};
    p = add(mul(p, s2), c);
  }
  D2 r = mul(s, p);
  r.hi *= 2.0;  // exact scaling
  r.lo *= 2.0;
  // + e * ln2 (ln2 = LN2_HI + LN2_LO to ~2^-107)
  constexpr double LN2_HI = 0x1.62e42fefa39efp-1;
  constexpr double LN2_LO = 0x1.abc9e3b39803fp-56;
  const D2 el = add(two_prod((double)e, LN2_HI), D2{(double)e * LN2_LO, 0.0});
  const D2 t = add(el, r);
  return t.hi + t.lo;
}

}  // namespace dd
}  // namespace rvcx
