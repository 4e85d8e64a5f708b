// Standalone micro-benchmark + correctness check of the implicit-GEMM conv kernel
// (not part of librvcx.so). Build: make bench_conv ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "rvcx_kernels.h"

using namespace rvcx;

#define CK_(x)                                                                      \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ void naive_conv1d(const float* x, const float* w, const float* b, float* y, int Tin, int Cin, int Tout,
                             int N, int taps, int dil, int pad, int stride) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)Tout * N) return;
  const int t = (int)(i / N), n = (int)(i % N);
  double acc = 0.0;
  for (int k = 0; k < taps; ++k) {
    const int r = t * stride - pad + k * dil;
    if (r < 0 || r >= Tin) continue;
    for (int c = 0; c < Cin; ++c) {
      float xv = x[(long long)r * Cin + c];
      xv = xv > 0.f ? xv : 0.1f * xv;
      acc += (double)xv * w[((long long)k * N + n) * Cin + c];
    }
  }
  y[i] = (float)acc + b[n];
}

static void fill_rand(std::vector<float>& v, unsigned seed) {
  srand(seed);
  for (auto& x : v) x = (float)rand() / RAND_MAX * 2.f - 1.f;
}

struct Case {
  const char* name;
  int T, Cin, N, taps, dil;
  int res = 0;  // ResBlock convs2 epilogue: + residual (separate buffer), accumulated into y, no activation
};

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  // bench_conv ITERS CASE CFG: time one case with one forced config (10.. = split kernel), no checks (PMC passes)
  const int only_case = argc > 3 ? atoi(argv[2]) : -1;
  const int only_cfg = argc > 3 ? atoi(argv[3]) : -2;
  if (only_case < 0) {
  // correctness on a small shape for every forced config x pipe
  // shape 0: every config; the others (ragged T, odd chunk counts, k = 5 / 11): the fp16 image on cfg 23
  struct Shape { int T, C, N, taps, dil; };
  const Shape shapes[] = {{1000, 128, 128, 7, 3}, {777, 96, 64, 11, 5}, {777, 96, 64, 5, 1}, {500, 64, 192, 11, 1},
                          {300, 32, 64, 7, 5}};
  for (int si = 0; si < (int)(sizeof(shapes) / sizeof(shapes[0])); ++si) {
    const int T = shapes[si].T, C = shapes[si].C, N = shapes[si].N, taps = shapes[si].taps, dil = shapes[si].dil;
    const int pad = (taps * dil - dil) / 2;
    std::vector<float> hx((size_t)T * C), hw((size_t)taps * N * C), hb(N);
    fill_rand(hx, 1);
    fill_rand(hw, 2);
    fill_rand(hb, 3);
    float *x, *w, *b, *y, *yr;
    CK_(hipMalloc(&x, hx.size() * 4));
    CK_(hipMalloc(&w, hw.size() * 4));
    CK_(hipMalloc(&b, N * 4));
    CK_(hipMalloc(&y, (size_t)T * N * 4));
    CK_(hipMalloc(&yr, (size_t)T * N * 4));
    CK_(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CK_(hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    CK_(hipMemcpy(b, hb.data(), N * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(naive_conv1d, dim3((T * N + 255) / 256), dim3(256), 0, 0, x, w, b, yr, T, C, T, N, taps, dil,
                       pad, 1);
    std::vector<float> ref((size_t)T * N), out((size_t)T * N);
    CK_(hipMemcpy(ref.data(), yr, ref.size() * 4, hipMemcpyDeviceToHost));
    // fmt 1: the two-plane fp16 image (math 3), fmt 2: its reduced-precision hi-plane mode
    for (int cfg : {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 23, 24, 25, 27})
      for (int fmt : {0, 1, 2}) {
        if (fmt && cfg != 23 && cfg != 24 && cfg != 25 && cfg != 27) continue;
        if (si > 0 && (cfg != 23 || fmt == 0)) continue;
        const int pipe = -1;
        ConvArgs a;
        a.x = x; a.ldx = C; a.T_in = T; a.C_in = C;
        a.w = w; a.ldw = C; a.w_ts = (long long)N * C; a.taps = taps; a.dil = dil; a.pad = pad;
        a.y = y; a.ldy = N; a.T_out = T; a.N = N; a.bias = b;
        a.pre_act = ACT_LRELU; a.pre_slope = 0.1f;
        a.force_cfg = cfg; a.pipe = pipe;
        void* wsb = nullptr;
        if (cfg >= 20) {  // weight-streamed split kernel: pre-split weight image
          a.wsplit_fmt = fmt ? WSPLIT_H16 : WSPLIT_BF16;
          a.lowp = fmt == 2;
          CK_(hipMalloc(&wsb, conv_wsplit_bytes(a)));
          CK_(conv_wsplit_build(a, wsb, 0));
          a.wsplit = wsb; a.wsplit_npad = conv_wsplit_npad(a.N); a.math = fmt ? 3 : 2; a.wsb = 1;
        }
        CK_(hipMemset(y, 0, (size_t)T * N * 4));
        CK_(conv1d(a, 0));
        if (wsb) (void)hipFree(wsb);
        CK_(hipDeviceSynchronize());
        CK_(hipMemcpy(out.data(), y, out.size() * 4, hipMemcpyDeviceToHost));
        double md = 0, mr = 0, se = 0;
        for (size_t i = 0; i < out.size(); ++i) {
          md = std::max(md, (double)fabsf(out[i] - ref[i]));
          mr = std::max(mr, (double)fabsf(ref[i]));
          se += (double)(out[i] - ref[i]) * (out[i] - ref[i]);
        }
        const double tol = fmt == 2 ? 2e-2 : 1e-5;
        printf("check T=%d C=%d N=%d k=%d d=%d cfg=%d (%s) pipe=%d max|diff|/max|ref| = %.3e rms diff %.3e %s\n", T, C,
               N, taps, dil, cfg,
               fmt == 2 ? "h16 lowp" : (fmt ? "h16x2" : (cfg >= 10 ? "split" : "f32")), pipe, md / mr,
               std::sqrt(se / out.size()), md / mr < tol ? "OK" : "FAIL");
      }
    (void)hipFree(x); (void)hipFree(w); (void)hipFree(b); (void)hipFree(y); (void)hipFree(yr);
  }
  // split-K correctness on small-M shapes
  {
    const int T = 150, C = 512, N = 384, taps = 1, dil = 1, pad = 0;
    std::vector<float> hx((size_t)T * C), hw((size_t)taps * N * C), hb(N);
    fill_rand(hx, 11);
    fill_rand(hw, 12);
    fill_rand(hb, 13);
    float *x, *w, *b, *y, *yr, *ws;
    CK_(hipMalloc(&x, hx.size() * 4));
    CK_(hipMalloc(&w, hw.size() * 4));
    CK_(hipMalloc(&b, N * 4));
    CK_(hipMalloc(&y, (size_t)T * N * 4));
    CK_(hipMalloc(&yr, (size_t)T * N * 4));
    CK_(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CK_(hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    CK_(hipMemcpy(b, hb.data(), N * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(naive_conv1d, dim3((T * N + 255) / 256), dim3(256), 0, 0, x, w, b, yr, T, C, T, N, taps, dil,
                       pad, 1);
    std::vector<float> ref((size_t)T * N), out((size_t)T * N);
    CK_(hipMemcpy(ref.data(), yr, ref.size() * 4, hipMemcpyDeviceToHost));
    for (int pipe : {-1, 1})
    for (int math : {1, 2}) {
      ConvArgs a;
      a.math = math;
      a.x = x; a.ldx = C; a.T_in = T; a.C_in = C;
      a.w = w; a.ldw = C; a.w_ts = (long long)N * C; a.taps = taps; a.dil = dil; a.pad = pad;
      a.y = y; a.ldy = N; a.T_out = T; a.N = N; a.bias = b;
      a.pre_act = ACT_LRELU; a.pre_slope = 0.1f; a.pipe = pipe;
      const long long need = conv_plan_splitk(a, false);
      CK_(hipMalloc(&ws, (need > 0 ? need : 1) * 4));
      a.ws = ws;
      CK_(hipMemset(y, 0, (size_t)T * N * 4));
      CK_(conv1d(a, 0));
      CK_(hipDeviceSynchronize());
      CK_(hipMemcpy(out.data(), y, out.size() * 4, hipMemcpyDeviceToHost));
      double md = 0, mr = 0;
      for (size_t i = 0; i < out.size(); ++i) {
        md = std::max(md, (double)fabsf(out[i] - ref[i]));
        mr = std::max(mr, (double)fabsf(ref[i]));
      }
      printf("check splitk math=%d ksplit=%d pipe=%d max|diff|/max|ref| = %.3e %s\n", math, a.ksplit, pipe, md / mr,
             md / mr < 1e-5 ? "OK" : "FAIL");
      (void)hipFree(ws);
    }
  }
  }
  // timing
  std::vector<Case> cases = {
      {"gen.s1 C256 k11 d5", 18600, 256, 256, 11, 5}, {"gen.s2 C128 k3 d1", 186000, 128, 128, 3, 1},
      {"gen.s2 C128 k7 d3", 186000, 128, 128, 7, 3},  {"gen.s2 C128 k11 d5", 186000, 128, 128, 11, 5},
      {"gen.s3 C64 k11 d5", 372000, 64, 64, 11, 5},   {"gen.s4 C32 k11 d5", 744000, 32, 32, 11, 5},
      {"hubert ffn1 775x768->3072", 775, 768, 3072, 1, 1}, {"hubert qkv 775x768->2304", 775, 768, 2304, 1, 1},
      {"hubert conv1 24808 k3 s2", 24808, 512, 512, 3, 1},
      {"hubert ffn2 775x3072->768", 775, 3072, 768, 1, 1}, {"te ffn1 1550 k3 192->768", 1550, 192, 768, 3, 1},
      {"te qkv 1550x192->576", 1550, 192, 576, 1, 1}, {"flow in 1550 k5 192->384", 1550, 192, 384, 5, 1},
      {"gen.s4 C32 k3 d1", 744000, 32, 32, 3, 1},      {"gen.s4 C32 k3 d1 res", 744000, 32, 32, 3, 1, 1},
      {"gen.s3 C64 k3 d1 res", 372000, 64, 64, 3, 1, 1}, {"gen.s4 C32 k7 d3 res", 744000, 32, 32, 7, 3, 1},
      {"gen.s2 C128 k3 d1 res", 186000, 128, 128, 3, 1, 1},
      {"gen.up1 1550 512->12x256 t2", 1550, 512, 3072, 2, 1}, {"gen.up2 18600 256->10x128 t2", 18600, 256, 1280, 2, 1},
      {"gen.up3 186000 128->2x64 t2", 186000, 128, 128, 2, 1},
      {"gen.s1 C256 k3 d1 res", 18600, 256, 256, 3, 1, 1}, {"gen.up2 18600 256->10x128 t3", 18600, 256, 1280, 3, 1},
  };
  for (size_t ci = 0; ci < cases.size(); ++ci) {
    if (only_case >= 0 && (int)ci != only_case) continue;
    auto& cs = cases[ci];
    const size_t nx = (size_t)cs.T * cs.Cin, nw = (size_t)cs.taps * cs.N * cs.Cin, ny = (size_t)cs.T * cs.N;
    float *x, *w, *b, *y, *rb = nullptr;
    if (cs.res) {
      CK_(hipMalloc(&rb, ny * 4));
      CK_(hipMemset(rb, 0, ny * 4));
    }
    CK_(hipMalloc(&x, nx * 4));
    CK_(hipMalloc(&w, nw * 4));
    CK_(hipMalloc(&b, cs.N * 4));
    CK_(hipMalloc(&y, ny * 4));
    std::vector<float> hx(nx), hw(nw);
    fill_rand(hx, 5);
    fill_rand(hw, 6);
    CK_(hipMemcpy(x, hx.data(), nx * 4, hipMemcpyHostToDevice));
    CK_(hipMemcpy(w, hw.data(), nw * 4, hipMemcpyHostToDevice));
    CK_(hipMemset(b, 0, cs.N * 4));
    const double flops = 2.0 * cs.T * cs.N * (double)cs.Cin * cs.taps;
    // variants: (cfg, math, pipe); cfg -1 = the library's policy for that math
    struct V { int cfg, math, pipe; };
    std::vector<V> vars = {{-1, 2, 0}, {23, 2, -1}, {24, 2, -1}, {27, 2, -1}, {23, 3, -1}, {24, 3, -1}, {40, 3, -1}, {-1, 3, -1},
                           {27, 3, -1}, {25, 3, -1}, {23, 4, -1}, {27, 4, -1}, {13, 2, -1}, {1, 1, -1}};
    if (cs.taps == 1)
      for (int c : {10, 12, 13, 14, 15}) vars.push_back({c, 2, 1});
    printf("%-28s", cs.name);
    for (size_t vi = 0; vi < vars.size(); ++vi) {
      const V& vv = vars[vi];
      if (only_case >= 0 && (vv.cfg != only_cfg || vv.pipe > 0)) continue;
      double best = 0;
      int ksp = 1;
      for (int round = 0; round < (only_case >= 0 ? 1 : 2); ++round) {
        ConvArgs a;
        a.x = x; a.ldx = cs.Cin; a.T_in = cs.T; a.C_in = cs.Cin;
        a.w = w; a.ldw = cs.Cin; a.w_ts = (long long)cs.N * cs.Cin; a.taps = cs.taps; a.dil = cs.dil;
        a.pad = (cs.taps * cs.dil - cs.dil) / 2;
        a.y = y; a.ldy = cs.N; a.T_out = cs.T; a.N = cs.N; a.bias = b;
        a.pre_act = ACT_LRELU; a.pre_slope = 0.1f; a.act = ACT_LRELU; a.slope = 0.1f;
        if (cs.res) {
          a.act = ACT_NONE;
          a.res = rb; a.ldr = cs.N; a.res_mode = RES_ADD_POST; a.acc_mode = ACC_ADD;
        }
        a.force_cfg = vv.cfg; a.pipe = vv.pipe; a.math = vv.math == 4 ? 3 : vv.math;
        a.wsplit_fmt = vv.math >= 3 ? WSPLIT_H16 : WSPLIT_BF16;
        a.lowp = vv.math == 4;
        float* wsp = nullptr;
        void* wsb = nullptr;
        if (vv.cfg >= 20) {
          if (!conv_wsb_eligible(a)) break;
          CK_(hipMalloc(&wsb, conv_wsplit_bytes(a)));
          CK_(conv_wsplit_build(a, wsb, 0));
          a.wsplit = wsb; a.wsplit_npad = conv_wsplit_npad(a.N); a.wsb = 1;
        }
        if (vv.cfg < 0) {
          const long long need = conv_plan_splitk(a, false);
          if (need > 0) { CK_(hipMalloc(&wsp, need * 4)); a.ws = wsp; }
        }
        if (conv1d(a, 0) != hipSuccess) {
          (void)hipGetLastError();
          if (wsp) (void)hipFree(wsp);
          if (wsb) (void)hipFree(wsb);
          break;
        }
        for (int i = 0; i < 3; ++i) CK_(conv1d(a, 0));
        CK_(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        CK_(hipEventCreate(&e0));
        CK_(hipEventCreate(&e1));
        CK_(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) CK_(conv1d(a, 0));
        CK_(hipEventRecord(e1, 0));
        CK_(hipEventSynchronize(e1));
        float ms = 0;
        CK_(hipEventElapsedTime(&ms, e0, e1));
        ms /= iters;
        best = std::max(best, flops / ms / 1e9);
        ksp = a.ksplit;
        if (wsp) (void)hipFree(wsp);
        if (wsb) (void)hipFree(wsb);
      }
      printf(" %s%d%s:%6.1f%s", vv.math == 2 ? "e" : (vv.math == 3 ? "h" : (vv.math == 4 ? "l" : "f")), vv.cfg,
             vv.pipe > 0 ? "p" : "", best, ksp > 1 ? "*" : " ");
    }
    printf("\n");
    fflush(stdout);
    (void)hipFree(x); (void)hipFree(w); (void)hipFree(b); (void)hipFree(y);
    if (rb) (void)hipFree(rb);
  }
  return 0;
}
