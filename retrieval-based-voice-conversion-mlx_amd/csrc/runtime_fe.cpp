// Front end of the pipeline on device: HuBERT/ContentVec features and the RMVPE pitch predictor.
//   HuBERT: transformers modeling_hubert.py HubertModel (contentvec config:
//           rvc_mlx/models/embedders/contentvec/config.json); MLX rvc_mlx/lib/mlx/hubert.py.
//   RMVPE : rvc/lib/predictors/RMVPE.py (E2E U-Net + BiGRU, MelSpectrogram, decode);
//           MLX rvc_mlx/lib/mlx/rmvpe.py.
#include <cmath>

#include "runtime.h"

namespace rvcx {

namespace {

const HostTensor& getw(Ctx& c, int model, const std::string& n, std::vector<int64_t> shape) {
  auto it = c.host[model].find(n);
  if (it == c.host[model].end()) throw Error(RVCX_E_STATE, "missing weight: " + n);
  if (it->second.shape != shape) {
    std::string got, want;
    for (auto s : it->second.shape) got += std::to_string(s) + ",";
    for (auto s : shape) want += std::to_string(s) + ",";
    throw Error(RVCX_E_SHAPE, "weight " + n + " has shape (" + got + ") expected (" + want + ")");
  }
  return it->second;
}

std::vector<float> pack_conv1d(const HostTensor& t) {
  const int64_t O = t.shape[0], I = t.shape[1], K = t.shape[2];
  std::vector<float> out(t.v.size());
  for (int64_t o = 0; o < O; ++o)
    for (int64_t i = 0; i < I; ++i)
      for (int64_t k = 0; k < K; ++k) out[(k * O + o) * I + i] = t.v[(o * I + i) * K + k];
  return out;
}

ConvArgs lin(const float* x, int ldx, int rows, int K, const float* w, int N, const float* bias, float* y, int ldy) {
  ConvArgs a;
  a.x = x;
  a.ldx = ldx;
  a.T_in = rows;
  a.C_in = K;
  a.w = w;
  a.ldw = K;
  a.taps = 1;
  a.y = y;
  a.ldy = ldy;
  a.T_out = rows;
  a.N = N;
  a.bias = bias;
  return a;
}


void run1(Ctx& c, const ConvArgs& a, hipStream_t s, double flops = -1.0) { launch_conv(c, a, false, s, flops); }
void run2(Ctx& c, const ConvArgs& a, hipStream_t s, double flops = -1.0) { launch_conv(c, a, true, s, flops); }

constexpr int HD = 768, HHEADS = 12, HFF = 3072, HCONV = 512;
const int HK[7] = {10, 3, 3, 3, 3, 2, 2};
const int HS[7] = {5, 2, 2, 2, 2, 2, 2};
constexpr int POS_K = 128, POS_G = 16;

}  // namespace

// ================================================================== HuBERT
void finalize_hubert(Ctx& c) {
  const int M = 1;
  // conv0 (C_in 1, k 10, s 5): [512][1][10] as is, the fused conv + GroupNorm + GELU kernel's [c][k] layout
  c.alloc_weight("hb.conv0", getw(c, M, "feature_extractor.conv_layers.0.conv.weight", {HCONV, 1, HK[0]}).v);
  for (int i = 1; i < 7; ++i)
    c.alloc_weight("hb.conv" + std::to_string(i),
                   pack_conv1d(getw(c, M, "feature_extractor.conv_layers." + std::to_string(i) + ".conv.weight",
                                    {HCONV, HCONV, HK[i]})));
  c.alloc_weight("hb.gn.g", getw(c, M, "feature_extractor.conv_layers.0.layer_norm.weight", {HCONV}).v);
  c.alloc_weight("hb.gn.b", getw(c, M, "feature_extractor.conv_layers.0.layer_norm.bias", {HCONV}).v);
  c.alloc_weight("hb.fp.ln.g", getw(c, M, "feature_projection.layer_norm.weight", {HCONV}).v);
  c.alloc_weight("hb.fp.ln.b", getw(c, M, "feature_projection.layer_norm.bias", {HCONV}).v);
  c.alloc_weight("hb.fp.w", getw(c, M, "feature_projection.projection.weight", {HD, HCONV}).v);
  c.alloc_weight("hb.fp.b", getw(c, M, "feature_projection.projection.bias", {HD}).v);
  {  // grouped positional conv: [768][48][128] -> [group][tap][48 out][48 in]
    const int cg = HD / POS_G;
    auto& w = getw(c, M, "encoder.pos_conv_embed.conv.weight", {HD, cg, POS_K});
    std::vector<float> v((size_t)POS_G * POS_K * cg * cg);
    for (int g = 0; g < POS_G; ++g)
      for (int t = 0; t < POS_K; ++t)
        for (int o = 0; o < cg; ++o)
          for (int i = 0; i < cg; ++i)
            v[(((size_t)g * POS_K + t) * cg + o) * cg + i] = w.v[((size_t)(g * cg + o) * cg + i) * POS_K + t];
    c.alloc_weight("hb.pos.w", v);
    c.alloc_weight("hb.pos.b", getw(c, M, "encoder.pos_conv_embed.conv.bias", {HD}).v);
  }
  c.alloc_weight("hb.enc.ln.g", getw(c, M, "encoder.layer_norm.weight", {HD}).v);
  c.alloc_weight("hb.enc.ln.b", getw(c, M, "encoder.layer_norm.bias", {HD}).v);
  for (int i = 0; i < 12; ++i) {
    const std::string p = "encoder.layers." + std::to_string(i);
    const std::string q = "hb." + std::to_string(i);
    std::vector<float> w, b;
    for (const char* n : {"q_proj", "k_proj", "v_proj"}) {
      auto& tw = getw(c, M, p + ".attention." + n + ".weight", {HD, HD}).v;
      auto& tb = getw(c, M, p + ".attention." + n + ".bias", {HD}).v;
      w.insert(w.end(), tw.begin(), tw.end());
      b.insert(b.end(), tb.begin(), tb.end());
    }
    c.alloc_weight(q + ".qkv.w", w);
    c.alloc_weight(q + ".qkv.b", b);
    c.alloc_weight(q + ".o.w", getw(c, M, p + ".attention.out_proj.weight", {HD, HD}).v);
    c.alloc_weight(q + ".o.b", getw(c, M, p + ".attention.out_proj.bias", {HD}).v);
    c.alloc_weight(q + ".ln1.g", getw(c, M, p + ".layer_norm.weight", {HD}).v);
    c.alloc_weight(q + ".ln1.b", getw(c, M, p + ".layer_norm.bias", {HD}).v);
    c.alloc_weight(q + ".ff1.w", getw(c, M, p + ".feed_forward.intermediate_dense.weight", {HFF, HD}).v);
    c.alloc_weight(q + ".ff1.b", getw(c, M, p + ".feed_forward.intermediate_dense.bias", {HFF}).v);
    c.alloc_weight(q + ".ff2.w", getw(c, M, p + ".feed_forward.output_dense.weight", {HD, HFF}).v);
    c.alloc_weight(q + ".ff2.b", getw(c, M, p + ".feed_forward.output_dense.bias", {HD}).v);
    c.alloc_weight(q + ".ln2.g", getw(c, M, p + ".final_layer_norm.weight", {HD}).v);
    c.alloc_weight(q + ".ln2.b", getw(c, M, p + ".final_layer_norm.bias", {HD}).v);
  }
  if (c.host[M].count("final_proj.weight")) {
    c.alloc_weight("hb.final_proj.w", getw(c, M, "final_proj.weight", {256, HD}).v);
    c.alloc_weight("hb.final_proj.b", getw(c, M, "final_proj.bias", {256}).v);
  }
}

int64_t hubert_frames(int64_t n) {
  int64_t t = n;
  for (int i = 0; i < 7; ++i) {
    if (t < HK[i]) return 0;
    t = (t - HK[i]) / HS[i] + 1;
  }
  return t;
}

// B equal-length sequences: audio row b at audio + b*lda; feats row block b at feats + b*L*outD.
// Row-wise ops (LayerNorm, Linear, FFN) run over all B*L rows at once; convolutions, GroupNorm and
// attention take the sequence as their batch index.
HubertRun hubert_front(Ctx& c, const float* audio, int64_t n, int64_t lda, int B, int version, float* feats,
                       int64_t cap, hipStream_t s) {
  if (B < 1) throw Error(RVCX_E_INVALID, "hubert: batch < 1");
  int64_t T[8];
  T[0] = n;
  for (int i = 0; i < 7; ++i) {
    if (T[i] < HK[i]) throw Error(RVCX_E_SHAPE, "hubert: input too short (" + std::to_string(n) + " samples)");
    T[i + 1] = (T[i] - HK[i]) / HS[i] + 1;
  }
  const int L = (int)T[7];
  const int BL = B * L;
  if (L > cap) throw Error(RVCX_E_CAPACITY, "hubert: output needs " + std::to_string(L) + " rows");
  float* a = c.buf<float>("hb.a", (size_t)B * T[1] * HCONV, s);
  float* b = c.buf<float>("hb.b", (size_t)B * T[2] * HCONV, s);
  double* gnws = c.buf<double>("hb.gnws", groupnorm_ws_doubles(HCONV, B), s);
  // conv0 -> GroupNorm(512, 512) -> GELU in three launches (statistics, finalize, apply), the conv recomputed by each
  check(hubert_conv0_gn_gelu(audio, lda, c.W("hb.conv0"), (int)T[1], HCONV, c.W("hb.gn.g"), c.W("hb.gn.b"), 1e-5f, gnws,
                             a, s, B),
        "hubert_conv0");
  float* cur = a;
  float* nxt = b;
  for (int i = 1; i < 7; ++i) {
    ConvArgs ci = lin(cur, HCONV, (int)T[i], HCONV, c.W("hb.conv" + std::to_string(i)), HCONV, nullptr, nxt, HCONV);
    ci.taps = HK[i];
    ci.stride = HS[i];
    ci.w_ts = (long long)HCONV * HCONV;
    ci.T_out = (int)T[i + 1];
    ci.act = ACT_GELU;
    ci.batch = B;
    ci.x_bs = T[i] * HCONV;
    ci.y_bs = T[i + 1] * HCONV;
    run1(c, ci, s);
    std::swap(cur, nxt);
  }
  // feature projection: LayerNorm(512) -> Linear(512, 768)
  float* hs = c.buf<float>("hb.hs", (size_t)BL * HD, s);
  float* hs2 = c.buf<float>("hb.hs2", (size_t)BL * HD, s);
  check(layernorm_rows(cur, nullptr, nxt, c.W("hb.fp.ln.g"), c.W("hb.fp.ln.b"), BL, HCONV, 1e-5f, nullptr, s),
        "fp_ln");
  run1(c, lin(nxt, HCONV, BL, HCONV, c.W("hb.fp.w"), HD, c.W("hb.fp.b"), hs, HD), s);
  {  // hs + gelu(pos_conv(hs)) (groups as inner batch, sequences as outer batch), then encoder LayerNorm
    const int cg = HD / POS_G;
    ConvArgs p = lin(hs, HD, L, cg, c.W("hb.pos.w"), cg, c.W("hb.pos.b"), hs2, HD);
    p.taps = POS_K;
    p.pad = POS_K / 2;
    p.ldw = cg;
    p.w_ts = (long long)cg * cg;
    p.batch_inner = POS_G;
    p.x_bs2 = cg;
    p.w_bs2 = (long long)POS_K * cg * cg;
    p.y_bs2 = cg;
    p.bias_bs2 = cg;
    p.act = ACT_GELU;
    p.res = hs;
    p.ldr = HD;
    p.res_bs2 = cg;
    p.res_mode = RES_ADD_POST;
    p.batch = B;
    p.x_bs = p.y_bs = p.res_bs = (long long)L * HD;
    run1(c, p, s);
    check(layernorm_rows(hs2, nullptr, hs, c.W("hb.enc.ln.g"), c.W("hb.enc.ln.b"), BL, HD, 1e-5f, nullptr, s),
          "enc_ln");
  }
  HubertRun r;
  r.B = B;
  r.L = L;
  r.version = version;
  r.feats = feats;
  return r;
}

// encoder layers [l0, l1) on the hidden states the front end left in "hb.hs" (modeling_hubert.py
// HubertEncoderLayer: post-LN attention + FFN)
void hubert_layers(Ctx& c, const HubertRun& run, int l0, int l1, hipStream_t s) {
  const int B = run.B, L = run.L, BL = B * L;
  float* hs = c.buf<float>("hb.hs", (size_t)BL * HD, s);
  float* qkv = c.buf<float>("hb.qkv", (size_t)BL * 3 * HD, s);
  const int nsplit = flash_attn_splits(B, HHEADS, L);
  float* part_o = c.buf<float>("hb.fa_o", (size_t)flash_attn_ws_floats(B, HHEADS, L, HD / HHEADS, nsplit), s);
  float* part_ml = c.buf<float>("hb.fa_ml", (size_t)nsplit * B * HHEADS * L * 2, s);
  float* att = c.buf<float>("hb.att", (size_t)BL * HD, s);
  float* ff = c.buf<float>("hb.ff", (size_t)BL * HFF, s);
  const int hd = HD / HHEADS;
  for (int i = l0; i < l1; ++i) {
    const std::string q = "hb." + std::to_string(i);
    run1(c, lin(hs, HD, BL, HD, c.W(q + ".qkv.w"), 3 * HD, c.W(q + ".qkv.b"), qkv, 3 * HD), s);
    // softmax((q * hd^-0.5) k^T) v per head in one pass (flash_attn.hip): no [B][12][L][L] scores
    check(flash_attn(qkv, 3 * HD, B, L, HHEADS, hd, (float)std::pow((double)hd, -0.5), nullptr, nullptr, 0, nullptr,
                     part_o, part_ml, nsplit, att, HD, s),
          "flash_attn");
    {  // hs = LN(hs + out_proj(att)) (layer_norm) in the split-K combine, in place: one combine block per row reads
       // the row's residual before it writes the row (round 6: the combine + a separate LayerNorm pass before)
      ConvArgs a3 = lin(att, HD, BL, HD, c.W(q + ".o.w"), HD, c.W(q + ".o.b"), hs, HD);
      a3.res = hs;
      a3.ldr = HD;
      a3.ln_g = c.W(q + ".ln1.g");
      a3.ln_b = c.W(q + ".ln1.b");
      run1(c, a3, s);
    }
    {
      ConvArgs f1 = lin(hs, HD, BL, HD, c.W(q + ".ff1.w"), HFF, c.W(q + ".ff1.b"), ff, HFF);
      f1.act = ACT_GELU;
      run1(c, f1, s);
      // v2's output is the last layer's LN itself: written straight into the caller's buffer (no tail copy)
      float* dst = (run.version != 1 && i == HUBERT_LAYERS - 1) ? run.feats : hs;
      // dst = LN(hs + ff2(ff)) in the split-K combine (final_layer_norm): no hs2 round trip, no separate pass
      ConvArgs f2 = lin(ff, HFF, BL, HFF, c.W(q + ".ff2.w"), HD, c.W(q + ".ff2.b"), dst, HD);
      f2.res = hs;
      f2.ldr = HD;
      f2.ln_g = c.W(q + ".ln2.g");
      f2.ln_b = c.W(q + ".ln2.b");
      run1(c, f2, s);
    }
  }
}

// v2: last_hidden_state; v1: final_proj (pipeline.py:331-334)
int64_t hubert_tail(Ctx& c, const HubertRun& run, hipStream_t s) {
  const int BL = run.B * run.L;
  const int version = run.version, outD = version == 1 ? 256 : HD;
  float* hs = c.buf<float>("hb.hs", (size_t)BL * HD, s);
  float* feats = run.feats;
  if (version == 1) {
    if (!c.dev.count("hb.final_proj.w")) throw Error(RVCX_E_STATE, "hubert: v1 needs final_proj weights");
    run1(c, lin(hs, HD, BL, HD, c.W("hb.final_proj.w"), 256, c.W("hb.final_proj.b"), feats, 256), s);
  }  // v2: the last layer wrote feats (hubert_layers)
  (void)outD;
  return run.L;
}

int64_t hubert_forward_b(Ctx& c, const float* audio, int64_t n, int64_t lda, int B, int version, float* feats,
                         int64_t cap, hipStream_t s) {
  const HubertRun r = hubert_front(c, audio, n, lda, B, version, feats, cap, s);
  hubert_layers(c, r, 0, HUBERT_LAYERS, s);
  return hubert_tail(c, r, s);
}

int64_t hubert_forward(Ctx& c, const float* audio, int64_t n, int version, float* feats, int64_t cap,
                       hipStream_t s) {
  return hubert_forward_b(c, audio, n, n, 1, version, feats, cap, s);
}

// ================================================================== RMVPE
namespace {

constexpr int NMEL = 128, NFFT = 1024, HOP = 160, NBIN = NFFT / 2 + 1, NCLS = 360;
// the mel projection's contraction padded to whole 32-bin chunks (zero magnitudes x zero weights): K = 513 kept it off
// the streamed fp16 kernels (the three-plane LDS kernel + a split-K combine: 60 + 16 us at C2, r05i)
constexpr int NBIN_P = 544;
constexpr int LEVELS = 5, INTER = 4, NBLK = 4, C_BASE = 16, GRU_H = 256;

// librosa.filters.mel(sr=16000, n_fft=1024, n_mels=128, fmin=30, fmax=8000, htk=True, norm='slaney')
std::vector<float> mel_basis() {
  const int n = NMEL + 2;
  auto hz2mel = [](double f) { return 2595.0 * std::log10(1.0 + f / 700.0); };
  auto mel2hz = [](double m) { return 700.0 * (std::pow(10.0, m / 2595.0) - 1.0); };
  const double lo = hz2mel(30.0), hi = hz2mel(8000.0);
  const double step = (hi - lo) / (n - 1);
  std::vector<double> mel_f(n);
  for (int i = 0; i < n; ++i) mel_f[i] = mel2hz(i == n - 1 ? hi : lo + i * step);
  std::vector<float> w((size_t)NMEL * NBIN_P, 0.f);  // [mel][bin], rows of NBIN_P (bins >= NBIN zero)
  for (int i = 0; i < NMEL; ++i) {
    const double fd0 = mel_f[i + 1] - mel_f[i], fd1 = mel_f[i + 2] - mel_f[i + 1];
    const double enorm = 2.0 / (mel_f[i + 2] - mel_f[i]);
    for (int k = 0; k < NBIN; ++k) {
      const double f = k * (16000.0 / NFFT);
      const double lower = -(mel_f[i] - f) / fd0;
      const double upper = (mel_f[i + 2] - f) / fd1;
      const float tri = (float)std::max(0.0, std::min(lower, upper));
      w[(size_t)i * NBIN_P + k] = (float)((double)tri * enorm);
    }
  }
  return w;
}

// STFT as a conv over 32-sample rows: W[tap][n][c], sample k = 32*tap + c; n < 513 real, else imag.
std::vector<float> stft_weights() {
  std::vector<float> w((size_t)32 * 2 * NBIN * 32);
  const double pi = 3.14159265358979323846;
  for (int t = 0; t < 32; ++t)
    for (int nn = 0; nn < 2 * NBIN; ++nn)
      for (int cc = 0; cc < 32; ++cc) {
        const int k = 32 * t + cc;
        const double win = 0.5 - 0.5 * std::cos(2.0 * pi * k / NFFT);
        const int f = nn < NBIN ? nn : nn - NBIN;
        const double ang = 2.0 * pi * (double)((long long)k * f % NFFT) / NFFT;
        const double v = nn < NBIN ? std::cos(ang) : -std::sin(ang);
        w[((size_t)t * 2 * NBIN + nn) * 32 + cc] = (float)(win * v);
      }
  return w;
}

struct BN {
  std::vector<double> a, b;
};
BN bn_fold(Ctx& c, const std::string& p, int C) {
  auto& g = getw(c, 2, p + ".weight", {C}).v;
  auto& bb = getw(c, 2, p + ".bias", {C}).v;
  auto& m = getw(c, 2, p + ".running_mean", {C}).v;
  auto& v = getw(c, 2, p + ".running_var", {C}).v;
  BN r;
  r.a.resize(C);
  r.b.resize(C);
  for (int i = 0; i < C; ++i) {
    const double inv = 1.0 / std::sqrt((double)v[i] + 1e-5);
    r.a[i] = inv * g[i];
    r.b[i] = (double)bb[i] - (double)m[i] * r.a[i];
  }
  return r;
}

// Conv2d [O][I][3][3] + BN -> [9][O][I], bias [O]
void conv_bn(Ctx& c, const std::string& wname, const std::string& bnname, int O, int I, const std::string& dst) {
  auto& w = getw(c, 2, wname, {O, I, 3, 3}).v;
  BN bn = bn_fold(c, bnname, O);
  std::vector<float> v((size_t)9 * O * I), bias(O);
  for (int o = 0; o < O; ++o) {
    for (int i = 0; i < I; ++i)
      for (int t = 0; t < 9; ++t) v[((size_t)t * O + o) * I + i] = (float)((double)w[((size_t)o * I + i) * 9 + t] * bn.a[o]);
    bias[o] = (float)bn.b[o];
  }
  c.alloc_weight(dst + ".w", v);
  c.alloc_weight(dst + ".b", bias);
}

void block_weights(Ctx& c, const std::string& p, const std::string& q, int cin, int cout) {
  conv_bn(c, p + ".conv.0.weight", p + ".conv.1", cout, cin, q + ".c1");
  conv_bn(c, p + ".conv.3.weight", p + ".conv.4", cout, cout, q + ".c2");
  if (cin != cout) {
    c.alloc_weight(q + ".sc.w", getw(c, 2, p + ".shortcut.weight", {cout, cin, 1, 1}).v);
    c.alloc_weight(q + ".sc.b", getw(c, 2, p + ".shortcut.bias", {cout}).v);
  }
}

ConvArgs c2d(const float* x, int ldx, int H, int W, int Cin, const float* w, int N, const float* bias, float* y,
             int ldy, int B = 1) {
  ConvArgs a;
  a.batch = B;  // B images of H x W pixels back to back
  a.x_bs = (long long)H * W * ldx;
  a.y_bs = (long long)H * W * ldy;
  a.x = x;
  a.ldx = ldx;
  a.T_in = H;
  a.W_in = W;
  a.C_in = Cin;
  a.w = w;
  a.ldw = Cin;
  a.w_ts = (long long)N * Cin;
  a.taps = 9;
  a.KH = 3;
  a.KW = 3;
  a.padh = 1;
  a.padw = 1;
  a.y = y;
  a.ldy = ldy;
  a.T_out = H;
  a.W_out = W;
  a.N = N;
  a.bias = bias;
  return a;
}

// ConvBlockRes (RMVPE.py:13-57): relu(bn(conv)) x2 + shortcut(x) (or x)
// B images back to back (NHWC, row stride ldx / ldy per pixel)
void conv_block(Ctx& c, const std::string& q, const float* x, int ldx, int H, int W, int cin, int cout, float* y,
                int ldy, hipStream_t s, int B = 1) {
  const size_t P = (size_t)H * W;
  float* t = c.buf<float>("rm.blk.t", (size_t)B * P * cout, s);
  ConvArgs a = c2d(x, ldx, H, W, cin, c.W(q + ".c1.w"), cout, c.W(q + ".c1.b"), t, cout, B);
  a.act = ACT_RELU;
  run2(c, a, s);
  const float* res = x;
  int ldr = ldx;
  if (cin != cout) {
    float* sc = c.buf<float>("rm.blk.sc", (size_t)B * P * cout, s);
    run1(c, lin(x, ldx, (int)(B * P), cin, c.W(q + ".sc.w"), cout, c.W(q + ".sc.b"), sc, cout), s);
    res = sc;
    ldr = cout;
  }
  ConvArgs b = c2d(t, cout, H, W, cout, c.W(q + ".c2.w"), cout, c.W(q + ".c2.b"), y, ldy, B);
  b.act = ACT_RELU;
  b.res = res;
  b.ldr = ldr;
  b.res_bs = (long long)P * ldr;
  b.res_mode = RES_ADD_POST;
  run2(c, b, s);
}

}  // namespace

void finalize_rmvpe(Ctx& c) {
  c.alloc_weight("rm.stft", stft_weights());
  c.alloc_weight("rm.mel", mel_basis());
  {
    BN bn = bn_fold(c, "unet.encoder.bn", 1);
    c.host[2]["__bn0__"] = HostTensor{{(float)bn.a[0], (float)bn.b[0]}, {2}};
  }
  int cin = 1, cout = C_BASE;
  for (int i = 0; i < LEVELS; ++i) {
    for (int b = 0; b < NBLK; ++b)
      block_weights(c, "unet.encoder.layers." + std::to_string(i) + ".conv." + std::to_string(b),
                    "rm.enc" + std::to_string(i) + "." + std::to_string(b), b == 0 ? cin : cout, cout);
    cin = cout;
    cout *= 2;
  }
  const int top = C_BASE << LEVELS;  // 512
  int ci = top / 2;
  for (int i = 0; i < INTER; ++i) {
    for (int b = 0; b < NBLK; ++b)
      block_weights(c, "unet.intermediate.layers." + std::to_string(i) + ".conv." + std::to_string(b),
                    "rm.int" + std::to_string(i) + "." + std::to_string(b), b == 0 ? ci : top, top);
    ci = top;
  }
  int C = top;
  for (int i = 0; i < LEVELS; ++i) {
    const int co = C / 2;
    const std::string p = "unet.decoder.layers." + std::to_string(i);
    const std::string q = "rm.dec" + std::to_string(i);
    {  // ConvTranspose2d 3x3 s2 p1 op1 + BN as a 2x2-tap phase conv with 4*co virtual outputs
      auto& w = getw(c, 2, p + ".conv1.0.weight", {C, co, 3, 3}).v;
      BN bn = bn_fold(c, p + ".conv1.1", co);
      std::vector<float> v((size_t)4 * 4 * co * C, 0.f), bias((size_t)4 * co);
      const int kmap[2][2] = {{1, -1}, {2, 0}};  // [phase][input offset] -> kernel index
      for (int dh = 0; dh < 2; ++dh)
        for (int dw = 0; dw < 2; ++dw)
          for (int ph = 0; ph < 2; ++ph)
            for (int pw = 0; pw < 2; ++pw) {
              const int kh = kmap[ph][dh], kw = kmap[pw][dw];
              if (kh < 0 || kw < 0) continue;
              const int tap = dh * 2 + dw;
              for (int o = 0; o < co; ++o) {
                const int n = (ph * 2 + pw) * co + o;
                for (int ii = 0; ii < C; ++ii)
                  v[((size_t)tap * 4 * co + n) * C + ii] =
                      (float)((double)w[(((size_t)ii * co + o) * 3 + kh) * 3 + kw] * bn.a[o]);
              }
            }
      for (int ph = 0; ph < 4; ++ph)
        for (int o = 0; o < co; ++o) bias[(size_t)ph * co + o] = (float)bn.b[o];
      c.alloc_weight(q + ".up.w", v);
      c.alloc_weight(q + ".up.b", bias);
    }
    for (int b = 0; b < NBLK; ++b)
      block_weights(c, p + ".conv2." + std::to_string(b), q + "." + std::to_string(b), b == 0 ? 2 * co : co, co);
    C = co;
  }
  c.alloc_weight("rm.cnn.w", [&] {
    auto& w = getw(c, 2, "cnn.weight", {3, C_BASE, 3, 3}).v;
    std::vector<float> v((size_t)9 * 3 * C_BASE);
    for (int o = 0; o < 3; ++o)
      for (int i = 0; i < C_BASE; ++i)
        for (int t = 0; t < 9; ++t) v[((size_t)t * 3 + o) * C_BASE + i] = w[((size_t)o * C_BASE + i) * 9 + t];
    return v;
  }());
  c.alloc_weight("rm.cnn.b", getw(c, 2, "cnn.bias", {3}).v);
  {
    const int nin = 3 * NMEL;
    auto& wf = getw(c, 2, "fc.0.gru.weight_ih_l0", {3 * GRU_H, nin}).v;
    auto& wb = getw(c, 2, "fc.0.gru.weight_ih_l0_reverse", {3 * GRU_H, nin}).v;
    std::vector<float> w(wf);
    w.insert(w.end(), wb.begin(), wb.end());
    c.alloc_weight("rm.gru.wih", w);
    auto& bf = getw(c, 2, "fc.0.gru.bias_ih_l0", {3 * GRU_H}).v;
    auto& bb = getw(c, 2, "fc.0.gru.bias_ih_l0_reverse", {3 * GRU_H}).v;
    std::vector<float> b(bf);
    b.insert(b.end(), bb.begin(), bb.end());
    c.alloc_weight("rm.gru.bih", b);
    c.alloc_weight("rm.gru.whh_f", getw(c, 2, "fc.0.gru.weight_hh_l0", {3 * GRU_H, GRU_H}).v);
    c.alloc_weight("rm.gru.whh_b", getw(c, 2, "fc.0.gru.weight_hh_l0_reverse", {3 * GRU_H, GRU_H}).v);
    c.alloc_weight("rm.gru.bhh_f", getw(c, 2, "fc.0.gru.bias_hh_l0", {3 * GRU_H}).v);
    c.alloc_weight("rm.gru.bhh_b", getw(c, 2, "fc.0.gru.bias_hh_l0_reverse", {3 * GRU_H}).v);
  }
  c.alloc_weight("rm.fc.w", getw(c, 2, "fc.1.weight", {NCLS, 2 * GRU_H}).v);
  c.alloc_weight("rm.fc.b", getw(c, 2, "fc.1.bias", {NCLS}).v);
}

// E2E on B mel chunk images [B][Fc][128] (already padded to a multiple of 32 frames) -> sal [B][Fc][360].
// Pooling and the per-row transforms run on the B images stacked along time (every level's height is
// even, so no 2x2 window straddles two images); convolutions take the image as their batch index.
static void e2e_chunk(Ctx& c, float* img, int Fc, float* sal, hipStream_t s, int B = 1) {
  int H = Fc, W = NMEL;
  // encoder: level outputs go to the second half of the decoder concat buffers
  float* catb[LEVELS];
  int cin = 1, cout = C_BASE;
  const float* x = img;
  int ldx = 1;
  for (int i = 0; i < LEVELS; ++i) {
    catb[i] = c.buf<float>("rm.cat" + std::to_string(i), (size_t)B * H * W * 2 * cout, s);
    float* pa = c.buf<float>("rm.pa", (size_t)B * Fc * NMEL * C_BASE * 2, s);
    float* pb = c.buf<float>("rm.pb", (size_t)B * Fc * NMEL * C_BASE * 2, s);
    const float* in = x;
    int ldi = ldx, ci = cin;
    for (int b = 0; b < NBLK; ++b) {
      const bool last = b == NBLK - 1;
      float* out = last ? catb[i] + cout : (b % 2 == 0 ? pa : pb);
      conv_block(c, "rm.enc" + std::to_string(i) + "." + std::to_string(b), in, ldi, H, W, ci, cout, out,
                 last ? 2 * cout : cout, s, B);
      in = out;
      ldi = last ? 2 * cout : cout;
      ci = cout;
    }
    float* pooled = c.buf<float>("rm.pool" + std::to_string(i), (size_t)B * (H / 2) * (W / 2) * cout, s);
    check(avgpool2(catb[i] + cout, B * H, W, cout, 2 * cout, pooled, s), "avgpool");
    x = pooled;
    ldx = cout;
    H /= 2;
    W /= 2;
    cin = cout;
    cout *= 2;
  }
  // intermediate (4 x ResEncoderBlock without pooling)
  const int top = C_BASE << LEVELS;
  {
    float* ia = c.buf<float>("rm.ia", (size_t)B * H * W * top, s);
    float* ib = c.buf<float>("rm.ib", (size_t)B * H * W * top, s);
    const float* in = x;
    int ci = cin, ldi = ldx, k = 0;
    for (int i = 0; i < INTER; ++i)
      for (int b = 0; b < NBLK; ++b, ++k) {
        float* out = (k % 2 == 0) ? ia : ib;
        conv_block(c, "rm.int" + std::to_string(i) + "." + std::to_string(b), in, ldi, H, W, ci, top, out, top, s,
                   B);
        in = out;
        ci = top;
        ldi = top;
      }
    x = in;
    ldx = top;
  }
  // decoder
  int C = top;
  for (int i = 0; i < LEVELS; ++i) {
    const int co = C / 2;
    const std::string q = "rm.dec" + std::to_string(i);
    float* cb = catb[LEVELS - 1 - i];
    {
      ConvArgs a;
      a.x = x;
      a.ldx = ldx;
      a.T_in = H;
      a.W_in = W;
      a.C_in = C;
      a.w = c.W(q + ".up.w");
      a.ldw = C;
      a.w_ts = (long long)4 * co * C;
      a.taps = 4;
      a.KH = 2;
      a.KW = 2;
      a.y = cb;
      a.ldy = 2 * co;
      a.T_out = H;
      a.W_out = W;
      a.N = 4 * co;
      a.out_map = OUT_UPSAMPLE2D;
      a.out_cv = co;
      a.bias = c.W(q + ".up.b");
      a.act = ACT_RELU;
      a.batch = B;
      a.x_bs = (long long)H * W * ldx;
      a.y_bs = (long long)(2 * H) * (2 * W) * 2 * co;
      run2(c, a, s, 2.0 * B * H * W * (double)C * co * 9);
    }
    H *= 2;
    W *= 2;
    float* da = c.buf<float>("rm.da", (size_t)B * Fc * NMEL * C_BASE, s);
    float* db = c.buf<float>("rm.db", (size_t)B * Fc * NMEL * C_BASE, s);
    const float* in = cb;
    int ci = 2 * co, ldi = 2 * co;
    for (int b = 0; b < NBLK; ++b) {
      float* out = (b % 2 == 0) ? da : db;
      conv_block(c, q + "." + std::to_string(b), in, ldi, H, W, ci, co, out, co, s, B);
      in = out;
      ci = co;
      ldi = co;
    }
    x = in;
    ldx = co;
    C = co;
  }
  // cnn (16 -> 3, 3x3, bias) -> [Fc][3*128] (index c*128 + w) -> BiGRU -> Linear + sigmoid
  float* cn = c.buf<float>("rm.cnn", (size_t)B * Fc * NMEL * 3, s);
  run2(c, c2d(x, ldx, H, W, C_BASE, c.W("rm.cnn.w"), 3, c.W("rm.cnn.b"), cn, 3, B), s);
  float* feat = c.buf<float>("rm.feat", (size_t)B * Fc * 3 * NMEL, s);
  check(nhwc_to_hcw(cn, B * Fc, NMEL, 3, feat, s), "nhwc_to_hcw");
  float* gi = c.buf<float>("rm.gi", (size_t)B * Fc * 6 * GRU_H, s);
  run1(c, lin(feat, 3 * NMEL, B * Fc, 3 * NMEL, c.W("rm.gru.wih"), 6 * GRU_H, c.W("rm.gru.bih"), gi, 6 * GRU_H), s);
  float* go = c.buf<float>("rm.gruout", (size_t)B * Fc * 2 * GRU_H, s);
  unsigned long long* xchg = c.buf<unsigned long long>("rm.xchg", gru_xchg_words(B), s);
  // a new (or regrown) allocation holds garbage tags: zeroed once, and the tag counters of its slices restart
  if (c.zero_once("rm.xchg", xchg, sizeof(unsigned long long) * gru_xchg_words(B), (long long)B, s))
    c.gru_tags.clear();
  unsigned* status = c.device_status();  // sticky until the host reads it (Ctx::check_device_status)
  // work the caller wants issued beside the BiGRU (which occupies 4 CUs): the gate event marks this point of the
  // stream, the BiGRU goes out first and the hook's (many) launches after it, so the host time spent issuing
  // them overlaps the BiGRU instead of delaying its launch
  std::function<void(hipStream_t)> hook = std::move(c.before_gru);
  c.before_gru = nullptr;
  if (hook && c.ev_gate) RVCX_HIP(hipEventRecord(c.ev_gate, s));
  for (int g0 = 0; g0 < B; g0 += 16)  // at most 16 sequences per launch (16 x 4 working workgroups co-resident)
    check(gru_bidir(gi + (size_t)g0 * Fc * 6 * GRU_H, c.W("rm.gru.whh_f"), c.W("rm.gru.bhh_f"), c.W("rm.gru.whh_b"),
                    c.W("rm.gru.bhh_b"), Fc, go + (size_t)g0 * Fc * 2 * GRU_H, xchg + gru_xchg_words(g0), status,
                    &c.gru_tags[xchg + gru_xchg_words(g0)], s, std::min(16, B - g0)),
          "gru");
  if (hook) hook(s);
  ConvArgs f = lin(go, 2 * GRU_H, B * Fc, 2 * GRU_H, c.W("rm.fc.w"), NCLS, c.W("rm.fc.b"), sal, NCLS);
  f.act = ACT_SIGMOID;
  run1(c, f, s);
}

// B equal-length sequences: audio row b at audio + b*lda; f0 row b at f0 + b*F; hidden row b at hidden + b*F*360.
int64_t rmvpe_forward_b(Ctx& c, const float* audio, int64_t n, int64_t lda, int B, float thred, double* f0,
                        int64_t cap, float* hidden, hipStream_t s) {
  if (B < 1) throw Error(RVCX_E_INVALID, "rmvpe: batch < 1");
  if (n < NFFT / 2 + 1) throw Error(RVCX_E_SHAPE, "rmvpe: input shorter than 513 samples");
  const int F = (int)(1 + n / HOP);
  if (F > cap) throw Error(RVCX_E_CAPACITY, "rmvpe: output needs " + std::to_string(F) + " frames");
  // MelSpectrogram (RMVPE.py:388-417): reflect pad 512, |STFT| (Hann 1024, hop 160), mel, log(clamp(1e-5))
  const int64_t np = n + NFFT;
  const int64_t rows = (np + 31) / 32;
  float* xp = c.buf<float>("rm.xp", (size_t)B * rows * 32, s);
  check(reflect_pad_1d(audio, (int)n, NFFT / 2, NFFT / 2, xp, s, B, lda, rows * 32), "reflect_pad");
  float* spec = c.buf<float>("rm.spec", (size_t)B * F * 2 * NBIN, s);
  {
    ConvArgs a = lin(xp, 32, (int)rows, 32, c.W("rm.stft"), 2 * NBIN, nullptr, spec, 2 * NBIN);
    a.taps = 32;
    a.stride = 5;
    a.w_ts = (long long)2 * NBIN * 32;
    a.T_out = F;
    a.batch = B;
    a.x_bs = rows * 32;
    a.y_bs = (long long)F * 2 * NBIN;
    run1(c, a, s, 0.0);
  }
  const int ldm = NBIN_P;
  float* mag = c.buf<float>("rm.mag", (size_t)B * F * ldm, s);
  check(stft_magnitude(spec, B * F, NBIN, mag, ldm, s), "stft_mag");
  float* mel = c.buf<float>("rm.melout", (size_t)B * F * NMEL, s);
  {
    ConvArgs a = lin(mag, ldm, B * F, NBIN_P, c.W("rm.mel"), NMEL, nullptr, mel, NMEL);
    a.act = ACT_LOGCLAMP;
    a.slope = 1e-5f;
    run1(c, a, s);
  }
  // mel2hidden (RMVPE.py:445-482): reflect-pad frames to a multiple of 32, E2E per 32000-frame chunk
  const int Fp = 32 * ((F - 1) / 32 + 1);
  float* img = c.buf<float>("rm.img", (size_t)B * Fp * NMEL, s);
  if (Fp > F) {
    check(reflect_pad_rows(mel, F, NMEL, Fp - F, img, s, B), "pad_frames");
  } else {
    RVCX_HIP(hipMemcpyAsync(img, mel, (size_t)B * F * NMEL * sizeof(float), hipMemcpyDeviceToDevice, s));
  }
  const auto& bn0 = c.host[2].at("__bn0__").v;
  check(affine_inplace(img, (long long)B * Fp * NMEL, bn0[0], bn0[1], s), "bn0");
  float* sal = c.buf<float>("rm.sal", (size_t)B * Fp * NCLS, s);
  const int chunk = 32000;
  if (Fp <= chunk) {
    for (int b0 = 0; b0 < B; b0 += 64) {  // the BiGRU keeps 4 co-resident workgroups per sequence
      const int nb = std::min(64, B - b0);
      e2e_chunk(c, img + (size_t)b0 * Fp * NMEL, Fp, sal + (size_t)b0 * Fp * NCLS, s, nb);
    }
  } else {
    // every chunk is an independent E2E pass (RMVPE.py:459-481: the U-Net pads each chunk's edges, the BiGRU
    // restarts); a sequence's full 32000-frame chunks lie back to back, so they go through as one batch (as the
    // short branch batches sequences), the shorter tail chunk as a second pass
    const int nfull = Fp / chunk, tail = Fp - nfull * chunk;
    for (int b = 0; b < B; ++b) {
      for (int k0 = 0; k0 < nfull; k0 += 8) {  // <= 8 chunks per pass: ~13 GB of U-Net activations
        const int nb = std::min(8, nfull - k0);
        const size_t r0 = (size_t)b * Fp + (size_t)k0 * chunk;
        e2e_chunk(c, img + r0 * NMEL, chunk, sal + r0 * NCLS, s, nb);
      }
      if (tail > 0) {
        const size_t r0 = (size_t)b * Fp + (size_t)nfull * chunk;
        e2e_chunk(c, img + r0 * NMEL, tail, sal + r0 * NCLS, s);
      }
    }
  }
  if (hidden)
    for (int b = 0; b < B; ++b)
      RVCX_HIP(hipMemcpyAsync(hidden + (size_t)b * F * NCLS, sal + (size_t)b * Fp * NCLS, (size_t)F * NCLS * sizeof(float),
                              hipMemcpyDeviceToDevice, s));
  check(rmvpe_decode(sal, F, NCLS, thred, f0, s, B, Fp), "decode");
  return F;
}

int64_t rmvpe_forward(Ctx& c, const float* audio, int64_t n, float thred, double* f0, int64_t cap, float* hidden,
                      hipStream_t s) {
  return rmvpe_forward_b(c, audio, n, n, 1, thred, f0, cap, hidden, s);
}

}  // namespace rvcx
