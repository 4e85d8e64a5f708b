// Micro-benchmark of the gather-streamed split kernel (conv_gs.hip) on the C2 step's short contractions (not part of
// librvcx.so). Build: make bench_gs ; run on the GPU box: bench_gs [iters] [flush]
// Per shape and split-K count: warm time (the same launch back to back) and, with flush=1, cold time (a 512 MB buffer
// rewritten before every timed launch, so weights and activations come from HBM as in the pipeline).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rvcx_kernels.h"

using namespace rvcx;

#define CK_(x)                                                                                  \
  do {                                                                                          \
    hipError_t e = (x);                                                                         \
    if (e != hipSuccess) {                                                                      \
      fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__);         \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

struct Shape {
  const char* name;
  int two_d, H, W, C, N, taps;  // 1-D: H = rows, W = 0
};

__global__ void k_touch(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  const int flush = argc > 2 ? atoi(argv[2]) : 1;
  const int only = argc > 3 ? atoi(argv[3]) : -1;
  const int plan_only = argc > 4 ? atoi(argv[4]) : 0;  // 1: only the library's split plan (PMC passes)
  std::vector<Shape> shapes = {
      {"unet L5 196px 512->512 3x3", 1, 49, 4, 512, 512, 9},   {"unet L4 784px 256->256 3x3", 1, 98, 8, 256, 256, 9},
      {"unet L3 3136px 128->128", 1, 196, 16, 128, 128, 9},    {"unet L2 12544px 64->64", 1, 392, 32, 64, 64, 9},
      {"hubert qkv 775 768->2304", 0, 775, 0, 768, 2304, 1},   {"hubert ffn1 775 768->3072", 0, 775, 0, 768, 3072, 1},
      {"hubert ffn2 775 3072->768", 0, 775, 0, 3072, 768, 1},  {"hubert o 775 768->768", 0, 775, 0, 768, 768, 1},
      {"te 1x1 1550 192->192", 0, 1550, 0, 192, 192, 1},       {"flow in 1550 k5 192->384", 0, 1550, 0, 192, 384, 5},
      {"te ffn1 1550 k3 192->768", 0, 1550, 0, 192, 768, 3},   {"te ffn2 1550 k3 768->192", 0, 1550, 0, 768, 192, 3},
  };
  float* junk = nullptr;
  const size_t njunk = (size_t)128 << 20;  // 512 MB: more than the 256 MB Infinity Cache
  if (flush) CK_(hipMalloc(&junk, njunk * 4));
  hipEvent_t e0, e1;
  CK_(hipEventCreate(&e0));
  CK_(hipEventCreate(&e1));
  for (size_t si = 0; si < shapes.size(); ++si) {
    if (only >= 0 && (int)si != only) continue;
    const Shape& sh = shapes[si];
    const long long rows = sh.two_d ? (long long)sh.H * sh.W : sh.H;
    const size_t nx = (size_t)rows * sh.C, nw = (size_t)sh.taps * sh.N * sh.C, ny = (size_t)rows * sh.N;
    float *x, *w, *b, *y;
    CK_(hipMalloc(&x, nx * 4));
    CK_(hipMalloc(&w, nw * 4));
    CK_(hipMalloc(&b, sh.N * 4));
    CK_(hipMalloc(&y, ny * 4));
    {
      std::vector<float> h(std::max(nx, nw));
      for (auto& v : h) v = (float)rand() / RAND_MAX - 0.5f;
      CK_(hipMemcpy(x, h.data(), nx * 4, hipMemcpyHostToDevice));
      CK_(hipMemcpy(w, h.data(), nw * 4, hipMemcpyHostToDevice));
      CK_(hipMemset(b, 0, sh.N * 4));
    }
    const double flops = 2.0 * rows * sh.N * (double)sh.C * sh.taps;
    printf("%-30s", sh.name);
    for (int ks : {0, 1, 2, 4, 8, 16, 32}) {
      if (plan_only && ks != 0) continue;
      ConvArgs a;
      a.x = x; a.ldx = sh.C; a.C_in = sh.C;
      a.w = w; a.ldw = sh.C; a.w_ts = (long long)sh.N * sh.C; a.taps = sh.taps;
      a.y = y; a.ldy = sh.N; a.N = sh.N; a.bias = b; a.act = ACT_RELU;
      if (sh.two_d) {
        a.T_in = sh.H; a.W_in = sh.W; a.T_out = sh.H; a.W_out = sh.W; a.KH = 3; a.KW = 3; a.padh = 1; a.padw = 1;
      } else {
        a.T_in = sh.H; a.T_out = sh.H; a.pad = (sh.taps - 1) / 2;
      }
      a.math = 2; a.w_static = 1; a.wsb = 2;
      a.force_cfg = 30;
      void* wsb = nullptr;
      CK_(hipMalloc(&wsb, conv_wsplit_bytes(a)));
      CK_(conv_wsplit_build(a, wsb, 0));
      a.wsplit = wsb; a.wsplit_npad = conv_wsplit_npad(a.N);
      long long need = conv_plan_splitk(a, sh.two_d != 0);
      const int plan_ks = a.ksplit;
      if (ks > 0) {  // forced split count
        const int steps = (sh.C / 32) * sh.taps;
        if (ks > steps) { printf("  ks%-2d:   -   ", ks); (void)hipFree(wsb); continue; }
        a.ksplit = ks;
        a.ws_rows = rows;
        need = ks > 1 ? (long long)ks * rows * sh.N : 0;
      }
      float* ws = nullptr;
      if (need > 0) {
        CK_(hipMalloc(&ws, need * 4));
        a.ws = ws;
      }
      auto run = [&]() { return sh.two_d ? conv2d(a, 0) : conv1d(a, 0); };
      CK_(run());
      CK_(hipDeviceSynchronize());
      // warm: back to back
      CK_(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) CK_(run());
      CK_(hipEventRecord(e1, 0));
      CK_(hipEventSynchronize(e1));
      float ms = 0;
      CK_(hipEventElapsedTime(&ms, e0, e1));
      const double warm_us = ms * 1e3 / iters;
      double cold_us = 0;
      if (flush) {
        double tot = 0;
        for (int i = 0; i < iters; ++i) {
          hipLaunchKernelGGL(k_touch, dim3(4096), dim3(256), 0, 0, junk, njunk, (float)i);
          CK_(hipEventRecord(e0, 0));
          CK_(run());
          CK_(hipEventRecord(e1, 0));
          CK_(hipEventSynchronize(e1));
          CK_(hipEventElapsedTime(&ms, e0, e1));
          tot += ms;
        }
        cold_us = tot * 1e3 / iters;
      }
      if (ks == 0)
        printf("  plan ks%-2d %6.1f/%6.1fus %5.1fTF", plan_ks, warm_us, cold_us, flops / (cold_us > 0 ? cold_us : warm_us) / 1e6);
      else
        printf("  ks%-2d %6.1f/%6.1f", ks, warm_us, cold_us);
      if (ws) (void)hipFree(ws);
      (void)hipFree(wsb);
    }
    printf("\n");
    fflush(stdout);
    (void)hipFree(x); (void)hipFree(w); (void)hipFree(b); (void)hipFree(y);
  }
  return 0;
}
