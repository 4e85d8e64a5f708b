// CREPE pitch estimator on device (f0 methods "crepe" / "crepe-tiny"): rvc_mlx/lib/mlx/crepe.py (the network is
// torchcrepe's, called by rvc/lib/predictors/f0.py:25-57). Frames are batched through the six convs on the
// implicit-GEMM kernels, time-major [frame][row][channel]:
//   conv1 (1 -> C1, k 512, stride 4 over the 254-zero-padded 1024-sample frame) is a contraction over 512 samples
//   per output row. Read as rows of 32 samples that start every 4 samples (ldx = 4 < C_in = 32: overlapping
//   rows of the same frame buffer), it becomes 16 taps x 32 channels at dilation 8 (tap t reads samples
//   4m + 32t .. 4m + 32t + 31), so the MFMA tile contracts full 32-channel chunks instead of 1-channel ones.
//   conv2..6 (k 64, zero pad 31 / 32) are ordinary 1-D convs; relu -> BatchNorm -> MaxPool(2) follow each.
// The classifier (Linear + sigmoid) gives the [F][360] probabilities; decode + median/mean filters finish.
#include <cmath>

#include "runtime.h"

namespace rvcx {

namespace {
constexpr int M = 3;  // model slot (RVCX_MODEL_CREPE)
constexpr int WIN = 1024, HOP = 160, FRAME_LD = WIN + 2 * 254, K1 = 512, BINS = 360;
constexpr int CHUNK = 256;  // frames per pass: bounds conv1's [CHUNK][256][C1] activation (256 MB at full)
constexpr int KC = 64;      // conv2..6 kernel
constexpr double BN_EPS = 1e-3;

const HostTensor& getc(Ctx& c, const std::string& n, std::vector<int64_t> shape) {
  auto it = c.host[M].find(n);
  if (it == c.host[M].end()) throw Error(RVCX_E_STATE, "missing weight: " + n);
  if (it->second.shape != shape) {
    std::string got, want;
    for (auto s : it->second.shape) got += std::to_string(s) + ",";
    for (auto s : shape) want += std::to_string(s) + ",";
    throw Error(RVCX_E_SHAPE, "weight " + n + " has shape (" + got + ") expected (" + want + ")");
  }
  return it->second;
}

int crepe_cap(const Ctx& c, int i) { return (int)c.host[M].at("__cap__").v[i]; }

ConvArgs conv1d_args(const float* x, int ldx, int Tin, int Cin, const float* w, int N, int taps, int dil, int pad,
                     const float* bias, float* y, int Tout, int B) {
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
  a.ldy = N;
  a.y_bs = (long long)Tout * N;
  a.T_out = Tout;
  a.N = N;
  a.bias = bias;
  a.batch = B;
  return a;
}
}  // namespace

// Validates torchcrepe-named weights (conv{i}.weight [O][I][K][1], conv{i}.bias, conv{i}_BN.*, classifier.*),
// packs conv weights to [tap][O][I] (conv1 to its 16 x 32 framed form) and BatchNorm to (mean, 1/sqrt(var +
// eps), gamma, beta) per channel.
void finalize_crepe(Ctx& c) {
  auto it = c.host[M].find("conv1.weight");
  if (it == c.host[M].end() || it->second.shape.size() != 4) throw Error(RVCX_E_STATE, "missing weight: conv1.weight");
  const int c1 = (int)it->second.shape[0];
  int cap[6];
  if (c1 == 1024) {
    const int f[6] = {1024, 128, 128, 128, 256, 512};
    std::copy(f, f + 6, cap);
  } else if (c1 == 128) {
    const int t[6] = {128, 16, 16, 16, 32, 64};
    std::copy(t, t + 6, cap);
  } else {
    throw Error(RVCX_E_SHAPE, "conv1.weight: CREPE full (1024) or tiny (128) filters expected");
  }
  for (int i = 0; i < 6; ++i) {
    const std::string p = "conv" + std::to_string(i + 1);
    const int O = cap[i], I = i == 0 ? 1 : cap[i - 1], K = i == 0 ? K1 : KC;
    const auto& w = getc(c, p + ".weight", {O, I, K, 1}).v;
    std::vector<float> pk((size_t)O * I * K);
    if (i == 0) {  // [tap t][o][ch j] = w[o][0][32 t + j]
      for (int t = 0; t < K1 / 32; ++t)
        for (int o = 0; o < O; ++o)
          for (int j = 0; j < 32; ++j) pk[((size_t)t * O + o) * 32 + j] = w[(size_t)o * K1 + 32 * t + j];
    } else {
      for (int o = 0; o < O; ++o)
        for (int ci = 0; ci < I; ++ci)
          for (int k = 0; k < K; ++k) pk[((size_t)k * O + o) * I + ci] = w[((size_t)o * I + ci) * K + k];
    }
    c.alloc_weight("cr." + p + ".w", pk);
    c.alloc_weight("cr." + p + ".b", getc(c, p + ".bias", {O}).v);
    const auto& mu = getc(c, p + "_BN.running_mean", {O}).v;
    const auto& var = getc(c, p + "_BN.running_var", {O}).v;
    const auto& gam = getc(c, p + "_BN.weight", {O}).v;
    const auto& bet = getc(c, p + "_BN.bias", {O}).v;
    std::vector<float> bn((size_t)4 * O);
    for (int o = 0; o < O; ++o) {
      bn[o] = mu[o];
      bn[O + o] = (float)(1.0 / std::sqrt((double)var[o] + BN_EPS));  // rsqrt(var + eps) (crepe.py:174)
      bn[2 * O + o] = gam[o];
      bn[3 * O + o] = bet[o];
    }
    c.alloc_weight("cr." + p + ".bn", bn);
  }
  const int feat = 4 * cap[5];  // 1024 / 4 / 2^6 = 4 rows x C6 (crepe.py:70, :76)
  c.alloc_weight("cr.fc.w", getc(c, "classifier.weight", {BINS, feat}).v);
  c.alloc_weight("cr.fc.b", getc(c, "classifier.bias", {BINS}).v);
  std::vector<float> capv(cap, cap + 6);
  c.host[M]["__cap__"] = HostTensor{capv, {6}};
}

// CREPE.get_f0 (crepe.py:282-325) over audio [n] fp32 @16 kHz: F = 1 + n/160 frames. Writes the filtered f0
// (fp32 [F]; fp64 copy when f0d), the filtered periodicity and the raw probabilities [F][360] when asked.
// sem 1: rvc/'s CREPE.get_f0 instead (rvc/lib/predictors/f0.py:31-55): torchcrepe.predict's framing (zero padding,
// unbiased std) and viterbi decode (dither [F] cents from the caller, or none), median / mean of 3, f0 = 0 where the
// periodicity < thr.
int64_t crepe_forward(Ctx& c, const float* audio, int64_t n, double f0_min, double f0_max, float thr, float* f0,
                      double* f0d, float* per, float* probs_out, hipStream_t s, int sem, const float* dither) {
  if (!c.ready[M]) throw Error(RVCX_E_STATE, "crepe weights not finalized");
  if (sem == 0 && n <= WIN / 2) throw Error(RVCX_E_INVALID, "crepe: input shorter than 513 samples (reflect pad of 512)");
  if (!(f0_min > 0.0) || !(f0_max >= f0_min)) throw Error(RVCX_E_INVALID, "crepe: need 0 < f0_min <= f0_max");
  const int64_t F = 1 + n / HOP;
  int cap[6];
  for (int i = 0; i < 6; ++i) cap[i] = crepe_cap(c, i);
  const int feat = 4 * cap[5];
  float* probs = probs_out ? probs_out : c.buf<float>("cr.probs", (size_t)F * BINS, s);
  const int nb = (int)std::min<int64_t>(CHUNK, F);
  float* fr = c.buf<float>("cr.frames", (size_t)nb * FRAME_LD, s);
  // ping-pong activations: conv output [nb][H][C] then the pooled [nb][H/2][C]
  size_t big = (size_t)nb * 256 * cap[0];
  for (int i = 1, H = 128; i < 6; ++i, H /= 2) big = std::max(big, (size_t)nb * H * cap[i]);
  float* hc = c.buf<float>("cr.conv", big, s);
  float* hp = c.buf<float>("cr.pool", (size_t)nb * 128 * cap[0], s);
  for (int64_t f0i = 0; f0i < F; f0i += nb) {
    const int B = (int)std::min<int64_t>(nb, F - f0i);
    check(crepe_frames(audio, n, f0i, B, fr, FRAME_LD, s, sem), "crepe_frames");
    {  // conv1: rows of 32 samples every 4 (376 rows cover the 1532-sample padded frame), 16 taps at dilation 8
      ConvArgs a = conv1d_args(fr, 4, (FRAME_LD - 32) / 4 + 1, 32, c.W("cr.conv1.w"), cap[0], K1 / 32, 8, 0,
                               c.W("cr.conv1.b"), hc, 256, B);
      a.x_bs = FRAME_LD;
      launch_conv(c, a, false, s, 2.0 * B * 256.0 * cap[0] * K1);
    }
    check(crepe_relu_bn_pool(hc, (long long)B * 256, cap[0], c.W("cr.conv1.bn"), hp, s), "crepe_bn1");
    int H = 128;
    for (int i = 1; i < 6; ++i) {
      const std::string p = "cr.conv" + std::to_string(i + 1);
      ConvArgs a = conv1d_args(hp, cap[i - 1], H, cap[i - 1], c.W(p + ".w"), cap[i], KC, 1, KC / 2 - 1, c.W(p + ".b"),
                               hc, H, B);
      launch_conv(c, a, false, s);
      check(crepe_relu_bn_pool(hc, (long long)B * H, cap[i], c.W(p + ".bn"), hp, s), "crepe_bn");
      H /= 2;
    }
    // classifier over the flattened [4][C6] rows (H-major then channel, crepe.py:214-220) + sigmoid
    ConvArgs a;
    a.x = hp;
    a.ldx = feat;
    a.T_in = B;
    a.C_in = feat;
    a.w = c.W("cr.fc.w");
    a.ldw = feat;
    a.y = probs + (size_t)f0i * BINS;
    a.ldy = BINS;
    a.T_out = B;
    a.N = BINS;
    a.bias = c.W("cr.fc.b");
    a.act = ACT_SIGMOID;
    launch_conv(c, a, false, s);
  }
  float* f0r = c.buf<float>("cr.f0raw", (size_t)F, s);
  float* pr = c.buf<float>("cr.perraw", (size_t)F, s);
  if (sem == 1) {
    // torchcrepe.postprocess: bins below frequency_to_bins(fmin) (floor) and from frequency_to_bins(fmax, ceil) on
    // are masked (clamped to the 360 bins here)
    const double off = 1997.3794084376191;
    const int minidx = (int)std::min(360.0, std::max(0.0, std::floor((1200.0 * std::log2(f0_min / 10.0) - off) / 20.0)));
    const int maxidx = (int)std::min(360.0, std::max(0.0, std::ceil((1200.0 * std::log2(f0_max / 10.0) - off) / 20.0)));
    if (minidx >= maxidx) throw Error(RVCX_E_INVALID, "crepe: [f0_min, f0_max] covers no pitch bin");
    float* lp = c.buf<float>("cr.lp", (size_t)F * BINS, s);
    int* ptr = c.buf<int>("cr.ptr", (size_t)F * BINS, s);
    int* bins = c.buf<int>("cr.bins", (size_t)F, s);
    check(crepe_decode_viterbi(probs, (int)F, minidx, maxidx, dither, thr, lp, ptr, bins, f0r, pr, f0, f0d, per, s),
          "crepe_decode_viterbi");
    return F;
  }
  const double lo = 1200.0 * std::log2(f0_min / 10.0), hi = 1200.0 * std::log2(f0_max / 10.0);
  check(crepe_decode(probs, (int)F, lo, hi, thr, f0r, pr, f0, f0d, per, s), "crepe_decode");
  return F;
}

}  // namespace rvcx
