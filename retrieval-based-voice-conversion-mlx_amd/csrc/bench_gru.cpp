// Standalone timing of the BiGRU recurrence kernel (not part of librvcx.so): gru_bidir at the C2 length.
// Build: make bench_gru ; run on the GPU box: build/bench_gru [T] [B] [iters].
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rvcx_kernels.h"

using namespace rvcx;

#define CK_(x)                                                                          \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 1568;
  const int B = argc > 2 ? atoi(argv[2]) : 1;
  const int iters = argc > 3 ? atoi(argv[3]) : 5;
  const int H = 256;
  std::vector<float> hgi((size_t)B * T * 6 * H), hw(3 * H * H), hb(3 * H);
  srand(7);
  for (auto& v : hgi) v = ((float)rand() / (float)RAND_MAX * 2.f - 1.f);
  for (auto& v : hw) v = ((float)rand() / (float)RAND_MAX * 2.f - 1.f) * 0.0625f;
  for (auto& v : hb) v = ((float)rand() / (float)RAND_MAX * 2.f - 1.f) * 0.1f;
  float *gi, *w, *b, *out;
  unsigned long long* xchg;
  unsigned* status;
  CK_(hipMalloc(&gi, hgi.size() * 4));
  CK_(hipMalloc(&w, hw.size() * 4));
  CK_(hipMalloc(&b, hb.size() * 4));
  CK_(hipMalloc(&out, (size_t)B * T * 2 * H * 4));
  CK_(hipMalloc(&xchg, gru_xchg_words(B) * 8));
  CK_(hipMemset(xchg, 0, gru_xchg_words(B) * 8));
  CK_(hipMalloc(&status, 4));
  CK_(hipMemset(status, 0, 4));
  CK_(hipMemcpy(gi, hgi.data(), hgi.size() * 4, hipMemcpyHostToDevice));
  CK_(hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK_(hipMemcpy(b, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  unsigned tag = 0;
  CK_(gru_bidir(gi, w, b, w, b, T, out, xchg, status, &tag, 0, B));
  CK_(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK_(hipEventCreate(&e0));
  CK_(hipEventCreate(&e1));
  CK_(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK_(gru_bidir(gi, w, b, w, b, T, out, xchg, status, &tag, 0, B));
  CK_(hipEventRecord(e1, 0));
  CK_(hipEventSynchronize(e1));
  float ms = 0;
  CK_(hipEventElapsedTime(&ms, e0, e1));
  unsigned st = 0;
  CK_(hipMemcpy(&st, status, 4, hipMemcpyDeviceToHost));
  std::vector<float> ho((size_t)B * T * 2 * H);
  CK_(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
  double cs = 0;
  for (float v : ho) cs += v;
  // fp64 host reference of sequence 0 (both directions; ATen GRUCell), checked on the first min(T, 400) steps of each
  double maxerr = 0.0;
  const int Tc = T < 400 ? T : 400;
  for (int dd = 0; dd < 2; ++dd) {
    std::vector<double> h(H, 0.0), hg(3 * H);
    for (int s = 0; s < Tc; ++s) {
      const int t = dd ? T - 1 - s : s;
      for (int r = 0; r < 3 * H; ++r) {
        double a = hb[r];
        for (int c = 0; c < H; ++c) a += (double)hw[(size_t)r * H + c] * h[c];
        hg[r] = a;
      }
      const float* ig = &hgi[(size_t)t * 6 * H + dd * 3 * H];
      for (int u = 0; u < H; ++u) {
        const double rr = 1.0 / (1.0 + std::exp(-(hg[u] + ig[u])));
        const double zz = 1.0 / (1.0 + std::exp(-(hg[H + u] + ig[H + u])));
        const double nn = std::tanh(ig[2 * H + u] + hg[2 * H + u] * rr);
        h[u] = (h[u] - nn) * zz + nn;
        maxerr = std::max(maxerr, std::fabs(h[u] - (double)ho[(size_t)t * 2 * H + dd * H + u]));
      }
    }
  }
  printf("T=%d B=%d: %.3f ms/call = %.3f us/step  status=%u checksum=%.6f  max|h - fp64| (first %d steps) %.2e\n", T, B,
         ms / iters, 1000.0 * ms / iters / T, st, cs, Tc, maxerr);
  return 0;
}
