// RefineGAN decoder on device (rvc/lib/algorithm/generators/refinegan.py:240-436; selected by
// Synthesizer(vocoder="RefineGAN"), synthesizers.py:99-107): 1-harmonic source on the linearly upsampled f0,
// pre_conv, a downsampling source branch (LeakyReLU 0.2 -> torchaudio kaiser-sinc resampling -> conv) whose
// stages are kept as skips, mel_conv + cond, then per upsampling stage LeakyReLU -> linear x rate -> concat skip
// -> ParallelResBlock (input_conv, three AdaIN -> ResBlock(slope 0.2) -> AdaIN branches, mean) -> conv_post.
// Every Conv1d is an implicit-GEMM launch (conv_gemm / conv_emu); refinegan.hip holds the resampler, the
// upsample+concat and AdaIN kernels; source_harm.hip the source.
#include <cmath>

#include "runtime.h"

namespace rvcx {

namespace {

constexpr int RG_C0 = 512;   // RefineGANGenerator upsample_initial_channel (default, not from the config)
constexpr int RG_START = 16; // start_channels
constexpr float RG_SLOPE = 0.2f;
constexpr int RG_K[3] = {3, 7, 11};
constexpr int RG_D[3] = {1, 3, 5};

const HostTensor& rg_get(Ctx& c, const std::string& n, std::vector<int64_t> shape) {
  auto it = c.host[0].find(n);
  if (it == c.host[0].end()) throw Error(RVCX_E_STATE, "missing weight: " + n);
  if (it->second.shape != shape) throw Error(RVCX_E_SHAPE, "weight " + n + " has an unexpected shape");
  return it->second;
}

std::vector<float> rg_pack(const HostTensor& t) {  // [O][I][K] -> [K][O][I]
  const int64_t O = t.shape[0], I = t.shape[1], K = t.shape[2];
  std::vector<float> out(t.v.size());
  for (int64_t o = 0; o < O; ++o)
    for (int64_t i = 0; i < I; ++i)
      for (int64_t k = 0; k < K; ++k) out[(k * O + o) * I + i] = t.v[(o * I + i) * K + k];
  return out;
}

// modified Bessel function of the first kind, order 0 (series; the kernel is computed once at finalize)
double bessel_i0(double x) {
  double sum = 1.0, term = 1.0;
  const double q = 0.25 * x * x;
  for (int k = 1; k < 200; ++k) {
    term *= q / ((double)k * k);
    sum += term;
    if (term < 1e-17 * sum) break;
  }
  return sum;
}

// torchaudio.functional._get_sinc_resample_kernel(orig, 1, ..., lowpass_filter_width 64, rolloff 0.9475937167399596,
// "sinc_interp_kaiser", beta 14.769656459379492) in float32 as the waveform dtype requests (refinegan.py:410-419)
std::vector<float> kaiser_kernel(int orig, int& width) {
  const double lw = 64.0, rolloff = 0.9475937167399596, beta = 14.769656459379492;
  const double base = 1.0 * rolloff;
  width = (int)std::ceil(lw * orig / base);
  const int K = 2 * width + orig;
  std::vector<float> k(K);
  const float bf = (float)base, pi = (float)M_PI, fbeta = (float)beta;
  const float i0b = (float)bessel_i0((double)fbeta);
  for (int j = 0; j < K; ++j) {
    float t = (float)(j - width) / (float)orig;  // idx (float32 arange / orig) + 0 / new
    t = t * bf;
    t = std::fmin(std::fmax(t, -(float)lw), (float)lw);
    const float r = t / (float)lw;
    const float win = (float)bessel_i0((double)(fbeta * std::sqrt(1.f - r * r))) / i0b;
    t = t * pi;
    const float sc = (float)(base / orig);
    const float sinc = t == 0.f ? 1.f : std::sin(t) / t;
    k[j] = sinc * (win * sc);
  }
  return k;
}

}  // namespace

void finalize_refinegan(Ctx& c) {
  const SynthCfg& g = c.scfg;
  const int nu = (int)g.ups.size();
  c.alloc_weight("rg.merge", rg_get(c, "dec.m_source.merge.0.weight", {1, 1}).v);
  c.alloc_weight("rg.pre.w", rg_pack(rg_get(c, "dec.pre_conv.weight", {RG_START, 1, 7})));
  c.alloc_weight("rg.pre.b", rg_get(c, "dec.pre_conv.bias", {RG_START}).v);
  int ch = RG_START;
  for (int i = 0; i < nu; ++i) {
    const std::string n = "dec.downsample_blocks." + std::to_string(i);
    c.alloc_weight("rg.down" + std::to_string(i) + ".w", rg_pack(rg_get(c, n + ".weight", {2 * ch, ch, 7})));
    c.alloc_weight("rg.down" + std::to_string(i) + ".b", rg_get(c, n + ".bias", {2 * ch}).v);
    int width = 0;
    const int r = g.ups[nu - 1 - i];
    c.alloc_weight("rg.rs" + std::to_string(i), kaiser_kernel(r, width));
    c.host[0]["__rg_rs_width" + std::to_string(i) + "__"] = HostTensor{{(float)width}, {1}};
    ch *= 2;
  }
  if (ch != RG_C0 / 2) throw Error(RVCX_E_SHAPE, "RefineGAN: the source branch must end at 256 channels");
  c.alloc_weight("rg.mel.w", rg_pack(rg_get(c, "dec.mel_conv.weight", {RG_C0 / 2, g.I, 7})));
  c.alloc_weight("rg.mel.b", rg_get(c, "dec.mel_conv.bias", {RG_C0 / 2}).v);
  c.alloc_weight("rg.cond.w", rg_get(c, "dec.cond.weight", {RG_C0 / 2, g.gin, 1}).v);
  c.alloc_weight("rg.cond.b", rg_get(c, "dec.cond.bias", {RG_C0 / 2}).v);
  int C = RG_C0;
  for (int i = 0; i < nu; ++i) {
    const int out = C / 2, cin = C + C / 4;
    const std::string p = "dec.upsample_conv_blocks." + std::to_string(i);
    const std::string q = "rg.up" + std::to_string(i);
    c.alloc_weight(q + ".in.w", rg_pack(rg_get(c, p + ".input_conv.weight", {out, cin, 7})));
    c.alloc_weight(q + ".in.b", rg_get(c, p + ".input_conv.bias", {out}).v);
    for (int j = 0; j < 3; ++j) {
      const std::string b = p + ".blocks." + std::to_string(j);
      const std::string d = q + ".b" + std::to_string(j);
      c.alloc_weight(d + ".ain", rg_get(c, b + ".0.weight", {out}).v);
      c.alloc_weight(d + ".aout", rg_get(c, b + ".2.weight", {out}).v);
      for (int m = 0; m < 3; ++m)
        for (int v = 1; v <= 2; ++v) {
          const std::string n = b + ".1.convs" + std::to_string(v) + "." + std::to_string(m);
          const std::string e = d + ".c" + std::to_string(v) + "." + std::to_string(m);
          c.alloc_weight(e + ".w", rg_pack(rg_get(c, n + ".weight", {out, out, RG_K[j]})));
          c.alloc_weight(e + ".b", rg_get(c, n + ".bias", {out}).v);
        }
    }
    C = out;
  }
  c.alloc_weight("rg.post.w", rg_get(c, "dec.conv_post.weight", {1, C, 7}).v);
}

long long SynthCfg::src_noise_total(int B, long long T) const {
  if (!f0) return 0;
  if (vocoder == 2) return refinegan_noise_floats(*this, B, T);
  return B * src_noise_row(T) + B * src_noise_tail();
}

long long refinegan_noise_floats(const SynthCfg& g, int B, long long T) {
  long long n = (long long)B * T * g.upp() + B;  // source randn [B][N][1] + torch.rand [B][1]
  long long ch = RG_C0, t = T;
  for (int r : g.ups) {
    ch /= 2;
    t *= r;
    n += 6LL * B * ch * t;  // 3 branches x (AdaIN in, AdaIN out) [B][C][T_stage]
  }
  return n;
}

static ConvArgs rg_conv(const float* x, int ldx, int Tin, int Cin, const float* w, int N, int taps, int pad,
                        const float* bias, float* y, int ldy, int Tout, int B, int dil = 1) {
  ConvArgs a;
  a.x = x;
  a.ldx = ldx;
  a.T_in = Tin;
  a.C_in = Cin;
  a.x_bs = (long long)Tin * ldx;
  a.w = w;
  a.ldw = Cin;
  a.w_ts = (long long)N * Cin;
  a.taps = taps;
  a.dil = dil;
  a.pad = pad;
  a.y = y;
  a.ldy = ldy;
  a.y_bs = (long long)Tout * ldy;
  a.T_out = Tout;
  a.N = N;
  a.bias = bias;
  a.batch = B;
  return a;
}

void refinegan_forward(Ctx& c, int B, int T, const float* z_btc, const float* mask, const float* f0, const float* g,
                       const float* eps_src, uint64_t seed, float* out, hipStream_t s) {
  const SynthCfg& cf = c.scfg;
  const int nu = (int)cf.ups.size(), upp = cf.upp(), I = cf.I;
  const long long N = (long long)T * upp;
  auto nseed = [&](int k) {
    uint64_t x = seed + 0x9E3779B97F4A7C15ull * (uint64_t)(k + 1);
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
  };
  // 1. source on the linearly upsampled f0 (refinegan.py:402-403)
  float* har = c.buf<float>("rg.har", (size_t)B * N, s);
  {
    double* ws = c.buf<double>("rg.harm_ws", harm_source_ws_doubles(B, T, upp, 1), s);
    check(harm_source(f0, B, T, upp, (float)cf.sr, 1, 1, eps_src, eps_src ? eps_src + (size_t)B * N : nullptr,
                      nseed(0), c.W("rg.merge"), 0.f, ws, har, N, s),
          "rg.source");
  }
  const float* eps_ada = eps_src ? eps_src + (size_t)B * N + B : nullptr;
  // 2. pre_conv + downsampling branch (:404-419); downs[i] = lrelu(x) before stage i's resample
  std::vector<float*> downs(nu);
  std::vector<int> dch(nu);
  std::vector<long long> dlen(nu);
  float* catb = c.buf<float>("rg.cat0", (size_t)B * T * RG_C0, s);  // [mel_conv | source branch] (:424-425)
  {
    float* x = c.buf<float>("rg.down0", (size_t)B * N * RG_START, s);
    launch_conv(c, rg_conv(har, 1, (int)N, 1, c.W("rg.pre.w"), RG_START, 7, 3, c.W("rg.pre.b"), x, RG_START, (int)N, B),
                false, s);
    long long len = N;
    int ch = RG_START;
    for (int i = 0; i < nu; ++i) {
      check(act_inplace(x, (long long)B * len * ch, ACT_LRELU, RG_SLOPE, s), "rg.lrelu");
      downs[i] = x;
      dch[i] = ch;
      dlen[i] = len;
      const int r = cf.ups[nu - 1 - i];
      const int width = (int)c.host[0].at("__rg_rs_width" + std::to_string(i) + "__").v[0];
      const int K = 2 * width + r;
      const long long lout = (len + r - 1) / r;
      float* xr = c.buf<float>("rg.rs", (size_t)B * lout * ch, s);
      check(resample_dw(x, B, (int)len, ch, c.W("rg.rs" + std::to_string(i)), K, r, width, xr, (int)lout, s),
            "rg.resample");
      const bool last = i + 1 == nu;
      float* y = last ? catb + RG_C0 / 2 : c.buf<float>("rg.down" + std::to_string(i + 1), (size_t)B * lout * 2 * ch, s);
      ConvArgs a = rg_conv(xr, ch, (int)lout, ch, c.W("rg.down" + std::to_string(i) + ".w"), 2 * ch, 7, 3,
                           c.W("rg.down" + std::to_string(i) + ".b"), y, last ? RG_C0 : 2 * ch, (int)lout, B);
      launch_conv(c, a, false, s);
      x = y;
      len = lout;
      ch *= 2;
    }
    if (len != T) throw Error(RVCX_E_SHAPE, "RefineGAN: source branch length != frames");
  }
  // 3. mel_conv(z * mask) + cond(g) into the first half of the concat (:421-423)
  {
    float* cv = c.buf<float>("rg.cvec", (size_t)B * (RG_C0 / 2), s);
    ConvArgs l = rg_conv(g, cf.gin, 1, cf.gin, c.W("rg.cond.w"), RG_C0 / 2, 1, 0, c.W("rg.cond.b"), cv, RG_C0 / 2, 1,
                         B);
    launch_conv(c, l, false, s);
    ConvArgs a = rg_conv(z_btc, I, T, I, c.W("rg.mel.w"), RG_C0 / 2, 7, 3, c.W("rg.mel.b"), catb, RG_C0, T, B);
    a.pre_mask = mask;
    a.pre_mask_bs = T;
    a.res = cv;
    a.ldr = 0;
    a.res_bs = RG_C0 / 2;
    a.res_mode = RES_ADD_PRE;
    launch_conv(c, a, false, s);
  }
  // 4. upsampling stages (:426-434)
  const float* x = catb;
  int C = RG_C0, ldx = RG_C0;
  long long Tc = T;
  long long eoff = 0;
  int draw = 1;
  size_t maxe = 0;
  {
    long long t = T;
    int ch = RG_C0;
    for (int r : cf.ups) {
      t *= r;
      maxe = std::max(maxe, (size_t)t * (ch + ch / 4));
      ch /= 2;
    }
  }
  float* U = c.buf<float>("rg.u", (size_t)B * maxe, s);
  float* X0 = c.buf<float>("rg.x0", (size_t)B * maxe, s);
  float* A = c.buf<float>("rg.a", (size_t)B * maxe, s);
  float* T1 = c.buf<float>("rg.t1", (size_t)B * maxe, s);
  float* RR = c.buf<float>("rg.rr", (size_t)B * maxe, s);
  float* RL = c.buf<float>("rg.rl", (size_t)B * maxe, s);
  float* S[2] = {c.buf<float>("rg.s0", (size_t)B * maxe, s), c.buf<float>("rg.s1", (size_t)B * maxe, s)};
  for (int i = 0; i < nu; ++i) {
    const int r = cf.ups[i];
    const int d = nu - 1 - i;
    const int Cd = dch[d], out = C / 2, cin = C + Cd;
    const long long Tn = Tc * r;
    if (Tn != dlen[d]) throw Error(RVCX_E_SHAPE, "RefineGAN: skip length mismatch");
    check(lerp_up_cat(x, B, (int)Tc, C, ldx, r, RG_SLOPE, downs[d], Cd, U, cin, s), "rg.up_cat");
    const std::string q = "rg.up" + std::to_string(i);
    launch_conv(c, rg_conv(U, cin, (int)Tn, cin, c.W(q + ".in.w"), out, 7, 3, c.W(q + ".in.b"), X0, out, (int)Tn, B),
                false, s);
    float* Sx = S[i & 1];
    const long long nel = (long long)B * Tn * out;
    for (int j = 0; j < 3; ++j) {
      const std::string bj = q + ".b" + std::to_string(j);
      check(adain(X0, B, (int)Tn, out, c.W(bj + ".ain"), eps_ada ? eps_ada + eoff : nullptr, nseed(draw), RG_SLOPE, A,
                  0, 1.f, s),
            "rg.adain_in");
      eoff += nel;
      ++draw;
      const float* r_in = A;
      for (int m = 0; m < 3; ++m) {
        const int k = RG_K[j], dil = RG_D[m];
        const std::string e = bj + ".c1." + std::to_string(m), e2 = bj + ".c2." + std::to_string(m);
        ConvArgs a1 = rg_conv(r_in, out, (int)Tn, out, c.W(e + ".w"), out, k, (k * dil - dil) / 2, c.W(e + ".b"), T1,
                              out, (int)Tn, B, dil);
        a1.pre_act = ACT_LRELU;
        a1.pre_slope = RG_SLOPE;
        a1.act = ACT_LRELU;
        a1.slope = RG_SLOPE;
        launch_conv(c, a1, false, s);
        float* dst = (m == 2) ? RL : RR;
        ConvArgs a2 = rg_conv(T1, out, (int)Tn, out, c.W(e2 + ".w"), out, k, (k - 1) / 2, c.W(e2 + ".b"), dst, out,
                              (int)Tn, B);
        a2.res = r_in;
        a2.ldr = out;
        a2.res_bs = Tn * out;
        a2.res_mode = RES_ADD_POST;
        launch_conv(c, a2, false, s);
        r_in = RR;
      }
      check(adain(RL, B, (int)Tn, out, c.W(bj + ".aout"), eps_ada ? eps_ada + eoff : nullptr, nseed(draw), RG_SLOPE,
                  Sx, j == 0 ? 0 : (j == 2 ? 2 : 1), 3.f, s),
            "rg.adain_out");
      eoff += nel;
      ++draw;
    }
    x = Sx;
    C = out;
    ldx = out;
    Tc = Tn;
  }
  // 5. LeakyReLU(0.2) -> conv_post (no bias) -> tanh (:435-437)
  check(conv_post_tanh(x, B, (int)Tc, C, c.W("rg.post.w"), 7, RG_SLOPE, out, s, 0.f), "rg.conv_post");
}

}  // namespace rvcx
