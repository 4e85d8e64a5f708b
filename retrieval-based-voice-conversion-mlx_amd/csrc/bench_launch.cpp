// Kernel-boundary floor on one stream (not part of librvcx.so). Build: make bench_launch.
// Times chains of dependent launches with hipEvents (no profiler) and prints the cost per launch for:
//   nop1      1 workgroup of 64 threads writing one word
//   nop256    256 workgroups of 256 threads, one word each
//   dirty X   1024 workgroups writing X bytes (float4 stores) that the next launch reads one line of
//   graph     the nop256 chain captured once and replayed as a hipGraph
//   busy      nop256 while a second stream keeps a long kernel resident on part of the chip (the step's HuBERT /
//             BiGRU overlap)
//   ahead     the nop256 chain (and one with a 512-byte kernel argument, the size of ConvArgs) enqueued behind a
//             5 ms single-workgroup kernel, timed from that kernel's end: the GPU-side cost per launch with the host
//             far ahead (the eager nop chains above are host-bound: ~3.6 us of enqueue per launch)
// Run it bare and under `rocprofv3 --kernel-trace --stats` to compare the tracer's per-kernel duration with the
// event-timed cost per launch.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#define CK_(x)                                                                       \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ void k_nop(int* p, int v) {
  if (threadIdx.x == 0) p[blockIdx.x] = v + p[blockIdx.x + 4096];
}

struct BigArg {
  int v[128];
};
__global__ void k_nop_big(int* p, BigArg a) {
  if (threadIdx.x == 0) p[blockIdx.x] = a.v[blockIdx.x & 127] + p[blockIdx.x + 4096];
}

// writes n float4 (dirty bytes for the next launch) and reads one line of the previous launch's output
__global__ void k_dirty(float4* dst, const float4* prev, long long n, int v) {
  const long long i0 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const float add = prev[(i0 * 64) % n].x;
  for (long long i = i0; i < n; i += (long long)gridDim.x * blockDim.x)
    dst[i] = make_float4((float)v + add, 0.f, 0.f, 0.f);
}

// a long resident kernel: each workgroup spins on arithmetic for `iters` rounds (bounded: every wave exits)
__global__ void k_busy(float* out, int iters) {
  float x = threadIdx.x * 1e-3f, y = 1.f;
  for (int i = 0; i < iters; ++i) {
    x = fmaf(x, 1.0000001f, 1e-7f);
    y = fmaf(y, 0.9999999f, x);
  }
  if (x + y == -1.f) out[blockIdx.x] = x;
}

static double chain_us(hipStream_t s, int n, const std::function<void()>& launch) {
  for (int i = 0; i < 20; ++i) launch();
  CK_(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK_(hipEventCreate(&e0));
  CK_(hipEventCreate(&e1));
  CK_(hipEventRecord(e0, s));
  for (int i = 0; i < n; ++i) launch();
  CK_(hipEventRecord(e1, s));
  CK_(hipEventSynchronize(e1));
  float ms = 0.f;
  CK_(hipEventElapsedTime(&ms, e0, e1));
  CK_(hipEventDestroy(e0));
  CK_(hipEventDestroy(e1));
  return ms * 1e3 / n;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 400;
  hipStream_t s, s2;
  CK_(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK_(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  int* w;
  CK_(hipMalloc(&w, 65536 * sizeof(int)));
  CK_(hipMemset(w, 0, 65536 * sizeof(int)));
  const long long big = 64ll << 20;  // bytes
  float4 *d0, *d1;
  CK_(hipMalloc(&d0, big));
  CK_(hipMalloc(&d1, big));
  CK_(hipMemset(d0, 0, big));
  CK_(hipMemset(d1, 0, big));
  float* bo;
  CK_(hipMalloc(&bo, 4096 * sizeof(float)));

  int v = 0;
  const double nop1 = chain_us(s, n, [&] { hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s, w, ++v); });
  const double nop256 = chain_us(s, n, [&] { hipLaunchKernelGGL(k_nop, dim3(256), dim3(256), 0, s, w, ++v); });
  // host enqueue rate of the same chain (no GPU wait inside the loop)
  CK_(hipStreamSynchronize(s));
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_nop, dim3(256), dim3(256), 0, s, w, ++v);
  auto t1 = std::chrono::steady_clock::now();
  CK_(hipStreamSynchronize(s));
  const double host_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
  printf("nop1     %7.2f us per launch\n", nop1);
  printf("nop256   %7.2f us per launch (host enqueue %.2f us per launch)\n", nop256, host_us);
  for (long long bytes : {1ll << 20, 8ll << 20, 32ll << 20, 64ll << 20}) {
    int flip = 0;
    const long long nf4 = bytes / 16;
    const double us = chain_us(s, n / 2, [&] {
      float4* dst = flip ? d1 : d0;
      const float4* src = flip ? d0 : d1;
      flip ^= 1;
      hipLaunchKernelGGL(k_dirty, dim3(1024), dim3(256), 0, s, dst, src, nf4, ++v);
    });
    printf("dirty %3lld MB %7.2f us per launch (%.2f us at 6 TB/s for the bytes alone)\n", bytes >> 20, us,
           bytes / 6e12 * 1e6);
  }
  {
    // graph replay of the nop256 chain
    hipGraph_t g;
    hipGraphExec_t ge;
    CK_(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_nop, dim3(256), dim3(256), 0, s, w, i);
    CK_(hipStreamEndCapture(s, &g));
    CK_(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK_(hipGraphLaunch(ge, s));
    CK_(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK_(hipEventCreate(&e0));
    CK_(hipEventCreate(&e1));
    CK_(hipEventRecord(e0, s));
    CK_(hipGraphLaunch(ge, s));
    CK_(hipEventRecord(e1, s));
    CK_(hipEventSynchronize(e1));
    float ms = 0.f;
    CK_(hipEventElapsedTime(&ms, e0, e1));
    printf("graph    %7.2f us per launch (nop256 chain replayed)\n", ms * 1e3 / n);
    CK_(hipGraphExecDestroy(ge));
    CK_(hipGraphDestroy(g));
  }
  {
    // a long kernel resident on part of the chip on a second stream, the nop256 chain beside it
    for (int wgs : {64, 512}) {
      hipLaunchKernelGGL(k_busy, dim3(wgs), dim3(256), 0, s2, bo, 2000000);
      const double us = chain_us(s, n, [&] { hipLaunchKernelGGL(k_nop, dim3(256), dim3(256), 0, s, w, ++v); });
      CK_(hipStreamSynchronize(s2));
      printf("busy%-4d %7.2f us per launch (nop256 beside %d resident workgroups)\n", wgs, us, wgs);
    }
  }
  {
    // host far ahead: a 5 ms one-workgroup kernel first, then the chain; events around the chain only
    for (int big = 0; big < 2; ++big) {
      BigArg ba;
      for (int i = 0; i < 128; ++i) ba.v[i] = i;
      hipEvent_t e0, e1;
      CK_(hipEventCreate(&e0));
      CK_(hipEventCreate(&e1));
      for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s, bo, 3000000);
        CK_(hipEventRecord(e0, s));
        auto h0 = std::chrono::steady_clock::now();
        for (int i = 0; i < n; ++i) {
          if (big) hipLaunchKernelGGL(k_nop_big, dim3(256), dim3(256), 0, s, w, ba);
          else hipLaunchKernelGGL(k_nop, dim3(256), dim3(256), 0, s, w, ++v);
        }
        auto h1 = std::chrono::steady_clock::now();
        CK_(hipEventRecord(e1, s));
        CK_(hipEventSynchronize(e1));
        float ms = 0.f, busy_ms = 0.f;
        CK_(hipEventElapsedTime(&ms, e0, e1));
        const double host = std::chrono::duration<double, std::micro>(h1 - h0).count() / n;
        if (rep == 1)
          printf("ahead%s %7.2f us per launch on the GPU (host enqueue %.2f us per launch, %s)\n", big ? "512" : "   ",
                 ms * 1e3 / n, host, ms * 1e3 > host * n ? "host ahead" : "HOST-BOUND: lengthen the busy kernel");
        (void)busy_ms;
      }
      CK_(hipEventDestroy(e0));
      CK_(hipEventDestroy(e1));
    }
  }
  {
    // marginal cost of a trivial launch between real kernels (host ahead): a chain of 2 MB-writing kernels with and
    // without a nop256 after each
    for (int with_nop = 0; with_nop < 2; ++with_nop) {
      hipEvent_t e0, e1;
      CK_(hipEventCreate(&e0));
      CK_(hipEventCreate(&e1));
      int flip = 0;
      for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s, bo, 3000000);
        CK_(hipEventRecord(e0, s));
        for (int i = 0; i < n / 2; ++i) {
          float4* dst = flip ? d1 : d0;
          const float4* src = flip ? d0 : d1;
          flip ^= 1;
          hipLaunchKernelGGL(k_dirty, dim3(1024), dim3(256), 0, s, dst, src, (2ll << 20) / 16, ++v);
          if (with_nop) hipLaunchKernelGGL(k_nop, dim3(256), dim3(256), 0, s, w, ++v);
        }
        CK_(hipEventRecord(e1, s));
        CK_(hipEventSynchronize(e1));
        float ms = 0.f;
        CK_(hipEventElapsedTime(&ms, e0, e1));
        if (rep == 1)
          printf("real2MB%s %7.2f us per real kernel%s\n", with_nop ? "+nop" : "    ", ms * 1e3 / (n / 2),
                 with_nop ? " (with a nop256 after each)" : "");
      }
      CK_(hipEventDestroy(e0));
      CK_(hipEventDestroy(e1));
    }
  }
  CK_(hipDeviceSynchronize());
  return 0;
}
