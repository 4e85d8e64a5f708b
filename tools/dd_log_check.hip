// Diagnostic: dd::log_cr and the coarse-pitch chain on the device vs the same code compiled for the host.
// Build: hipcc -x hip --offload-arch=gfx950 -O3 -I<csrc> tools/dd_log_check.hip -o build/dd_log_check
// Input: hex doubles on stdin. Output: mismatch counts (and the first few values).
#include <cstdio>
#include <vector>

#include "dd_math.h"

__host__ __device__ double chain(double f) {
#pragma clang fp contract(off)
  constexpr double mel_min = 0x1.370515d9beb10p+6;
  constexpr double mel_max = 0x1.0a1a207dfdbe5p+10;
  double m = 1127.0 * rvcx::dd::log_cr(1.0 + f / 700.0);
  if (m > 0) m = (m - mel_min) * 254.0 / (mel_max - mel_min) + 1.0;
  return m;
}

__global__ void k(const double* x, double* lg, double* ch, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    lg[i] = rvcx::dd::log_cr(1.0 + x[i] / 700.0);
    ch[i] = chain(x[i]);
  }
}

int main() {
  std::vector<double> x;
  double v;
  while (scanf("%la", &v) == 1) x.push_back(v);
  int n = (int)x.size();
  double *dx, *dl, *dc;
  hipMalloc(&dx, n * 8);
  hipMalloc(&dl, n * 8);
  hipMalloc(&dc, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dl, dc, n);
  std::vector<double> l(n), c(n);
  hipMemcpy(l.data(), dl, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(c.data(), dc, n * 8, hipMemcpyDeviceToHost);
  int bl = 0, bc = 0;
  for (int i = 0; i < n; ++i) {
    const double hl = rvcx::dd::log_cr(1.0 + x[i] / 700.0), hc = chain(x[i]);
    if (hl != l[i]) {
      if (bl < 5) printf("log mismatch f0=%a host %a dev %a\n", x[i], hl, l[i]);
      ++bl;
    }
    if (hc != c[i]) {
      if (bc < 5) printf("chain mismatch f0=%a host %a dev %a\n", x[i], hc, c[i]);
      ++bc;
    }
  }
  printf("n=%d log mismatches %d chain mismatches %d\n", n, bl, bc);
  return 0;
}
