// Synthesizer (TextEncoder -> flow reverse -> HiFiGAN-NSF) on device: weight repacking and
// the forward pass as a sequence of MFMA conv-GEMM launches plus small fused kernels.
// Reference semantics: rvc/lib/algorithm/{synthesizers,encoders,attentions,modules,residuals}.py,
// generators/{hifigan_nsf,hifigan}.py (see each block's comment for file:line).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "runtime.h"

namespace rvcx {

namespace {
constexpr long long HAR_PAD = 64;  // >= max(noise-conv pad, stride - pad) of every stage

uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

const HostTensor& get(Ctx& c, int model, const std::string& n, std::vector<int64_t> shape) {
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

// torch Conv1d weight [O][I][K] -> [K][O][I]
std::vector<float> pack_conv1d(const HostTensor& t) {
  const int64_t O = t.shape[0], I = t.shape[1], K = t.shape[2];
  std::vector<float> out(t.v.size());
  for (int64_t o = 0; o < O; ++o)
    for (int64_t i = 0; i < I; ++i)
      for (int64_t k = 0; k < K; ++k) out[(k * O + o) * I + i] = t.v[(o * I + i) * K + k];
  return out;
}

std::vector<float> cat(std::initializer_list<const std::vector<float>*> parts) {
  std::vector<float> out;
  for (auto* p : parts) out.insert(out.end(), p->begin(), p->end());
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

// 1-D conv over B independent sequences of T rows ([B][T][ld]); weights packed [taps][N][Cin].
ConvArgs conv(const float* x, int ldx, int Tin, int Cin, const float* w, int N, int taps, int dil, int pad,
              const float* bias, float* y, int ldy, int Tout, int B) {
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
  a.stride = 1;
  a.y = y;
  a.ldy = ldy;
  a.y_bs = (long long)Tout * ldy;
  a.T_out = Tout;
  a.N = N;
  a.bias = bias;
  a.batch = B;
  return a;
}


}  // namespace

static void run(Ctx& c, const ConvArgs& a, hipStream_t s, double flops = -1.0) {
  launch_conv(c, a, false, s, flops);
}

float* Ctx::W(const std::string& name) const {
  auto it = dev.find(name);
  if (it == dev.end()) throw Error(RVCX_E_STATE, "packed weight not found: " + name);
  return static_cast<float*>(it->second->p);
}

float* Ctx::alloc_weight(const std::string& name, const std::vector<float>& data) {
  std::unique_ptr<DevBuf> b(new DevBuf());
  size_t bytes = data.size() * sizeof(float);
  if (bytes == 0) bytes = 16;
  if (hipMalloc(&b->p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    throw Error(RVCX_E_OOM, "weight allocation failed: " + name);
  }
  b->bytes = bytes;
  RVCX_HIP(hipMemcpy(b->p, data.data(), data.size() * sizeof(float), hipMemcpyHostToDevice));
  float* p = static_cast<float*>(b->p);
  auto old = dev.find(name);
  if (old != dev.end()) {
    const uintptr_t o = reinterpret_cast<uintptr_t>(old->second->p);
    wranges.erase(o);
    drop_splits(o, o + old->second->bytes);  // the replaced tensor's split images
  }
  const uintptr_t u = reinterpret_cast<uintptr_t>(p);
  drop_splits(u, u + bytes);  // images cached for an earlier tensor at a reused address
  wranges[u] = u + bytes;
  dev[name] = std::move(b);
  return p;
}

void Ctx::drop_splits(uintptr_t lo, uintptr_t hi) {
  for (auto it = wsplit_cache.begin(); it != wsplit_cache.end();) {
    const uintptr_t u = reinterpret_cast<uintptr_t>(std::get<0>(it->first));
    it = (u >= lo && u < hi) ? wsplit_cache.erase(it) : std::next(it);
  }
  for (auto it = rb_wsplit_cache.begin(); it != rb_wsplit_cache.end();) {
    const uintptr_t u = reinterpret_cast<uintptr_t>(it->first.first);
    it = (u >= lo && u < hi) ? rb_wsplit_cache.erase(it) : std::next(it);
  }
}

bool Ctx::is_weight(const void* q) const {
  const uintptr_t u = reinterpret_cast<uintptr_t>(q);
  auto it = wranges.upper_bound(u);
  if (it == wranges.begin()) return false;
  --it;
  return u < it->second;
}

// ------------------------------------------------------------------ weight repacking
void finalize_synth(Ctx& c) {
  const SynthCfg& g = c.scfg;
  const int H = g.H, I = g.I, F = g.F, E = g.emb_dim, dk = H / g.n_heads, nw = 2 * g.window + 1;
  const int M = 0;
  // TextEncoder (encoders.py:88-144)
  c.alloc_weight("te.emb_phone.w", get(c, M, "enc_p.emb_phone.weight", {H, E}).v);
  c.alloc_weight("te.emb_phone.b", get(c, M, "enc_p.emb_phone.bias", {H}).v);
  if (g.f0) c.alloc_weight("te.emb_pitch", get(c, M, "enc_p.emb_pitch.weight", {256, H}).v);
  for (int i = 0; i < g.n_layers; ++i) {
    const std::string p = "enc_p.encoder.attn_layers." + std::to_string(i);
    const std::string q = "te." + std::to_string(i);
    auto& wq = get(c, M, p + ".conv_q.weight", {H, H, 1}).v;
    auto& wk = get(c, M, p + ".conv_k.weight", {H, H, 1}).v;
    auto& wv = get(c, M, p + ".conv_v.weight", {H, H, 1}).v;
    c.alloc_weight(q + ".qkv.w", cat({&wq, &wk, &wv}));
    auto& bq = get(c, M, p + ".conv_q.bias", {H}).v;
    auto& bk = get(c, M, p + ".conv_k.bias", {H}).v;
    auto& bv = get(c, M, p + ".conv_v.bias", {H}).v;
    c.alloc_weight(q + ".qkv.b", cat({&bq, &bk, &bv}));
    c.alloc_weight(q + ".o.w", get(c, M, p + ".conv_o.weight", {H, H, 1}).v);
    c.alloc_weight(q + ".o.b", get(c, M, p + ".conv_o.bias", {H}).v);
    c.alloc_weight(q + ".rel_k", get(c, M, p + ".emb_rel_k", {1, nw, dk}).v);
    c.alloc_weight(q + ".rel_v", get(c, M, p + ".emb_rel_v", {1, nw, dk}).v);
    const std::string n1 = "enc_p.encoder.norm_layers_1." + std::to_string(i);
    const std::string n2 = "enc_p.encoder.norm_layers_2." + std::to_string(i);
    c.alloc_weight(q + ".ln1.g", get(c, M, n1 + ".gamma", {H}).v);
    c.alloc_weight(q + ".ln1.b", get(c, M, n1 + ".beta", {H}).v);
    c.alloc_weight(q + ".ln2.g", get(c, M, n2 + ".gamma", {H}).v);
    c.alloc_weight(q + ".ln2.b", get(c, M, n2 + ".beta", {H}).v);
    const std::string f = "enc_p.encoder.ffn_layers." + std::to_string(i);
    c.alloc_weight(q + ".ffn1.w", pack_conv1d(get(c, M, f + ".conv_1.weight", {F, H, g.ksize})));
    c.alloc_weight(q + ".ffn1.b", get(c, M, f + ".conv_1.bias", {F}).v);
    c.alloc_weight(q + ".ffn2.w", pack_conv1d(get(c, M, f + ".conv_2.weight", {H, F, g.ksize})));
    c.alloc_weight(q + ".ffn2.b", get(c, M, f + ".conv_2.bias", {H}).v);
  }
  c.alloc_weight("te.proj.w", get(c, M, "enc_p.proj.weight", {2 * I, H, 1}).v);
  c.alloc_weight("te.proj.b", get(c, M, "enc_p.proj.bias", {2 * I}).v);
  // flow (residuals.py:103-258, modules.py:5-117). A coupling's WaveNet state lives in one [T][2H] buffer: the
  // residual stream h in columns [0, H), the skip sum in [H, 2H). `pre` is packed with H zero rows appended, so its
  // launch also clears the skip sum; the cond layers of all couplings are one [flow_n * cl][gin] GEMM.
  // The Flip before each coupling of the reverse pass (residuals.py:233-258) is folded into the weights when there is an
  // even number of them: the reverse loop's k-th coupling (k = flow_n - 1 - f) with k even sees the channels reversed,
  // so its `pre` reads the upper half with its input columns reversed and its `post` writes the lower half with its
  // output rows (and bias) reversed; after the last (odd k) coupling the layout is the reference's again.
  std::vector<float> condw, condb;
  for (int f = 0; f < g.flow_n; ++f) {
    const std::string p = "flow.flows." + std::to_string(2 * f);
    const std::string q = "flow." + std::to_string(f);
    const bool rev = g.flow_n % 2 == 0 && (g.flow_n - 1 - f) % 2 == 0;
    std::vector<float> prew = get(c, M, p + ".pre.weight", {H, I / 2, 1}).v, preb = get(c, M, p + ".pre.bias", {H}).v;
    if (rev)
      for (int o = 0; o < H; ++o) std::reverse(prew.begin() + (size_t)o * (I / 2), prew.begin() + (size_t)(o + 1) * (I / 2));
    prew.resize((size_t)2 * H * (I / 2), 0.f);
    preb.resize((size_t)2 * H, 0.f);
    c.alloc_weight(q + ".pre.w", prew);
    c.alloc_weight(q + ".pre.b", preb);
    const int cl = 2 * H * g.flow_layers;
    const auto& cw = get(c, M, p + ".enc.cond_layer.weight", {cl, g.gin, 1}).v;
    const auto& cb = get(c, M, p + ".enc.cond_layer.bias", {cl}).v;
    condw.insert(condw.end(), cw.begin(), cw.end());
    condb.insert(condb.end(), cb.begin(), cb.end());
    for (int L = 0; L < g.flow_layers; ++L) {
      const std::string l = std::to_string(L);
      c.alloc_weight(q + ".in" + l + ".w",
                     pack_conv1d(get(c, M, p + ".enc.in_layers." + l + ".weight", {2 * H, H, g.flow_k})));
      c.alloc_weight(q + ".in" + l + ".b", get(c, M, p + ".enc.in_layers." + l + ".bias", {2 * H}).v);
      const int rs = (L == g.flow_layers - 1) ? H : 2 * H;
      c.alloc_weight(q + ".rs" + l + ".w", get(c, M, p + ".enc.res_skip_layers." + l + ".weight", {rs, H, 1}).v);
      c.alloc_weight(q + ".rs" + l + ".b", get(c, M, p + ".enc.res_skip_layers." + l + ".bias", {rs}).v);
    }
    std::vector<float> postw = get(c, M, p + ".post.weight", {I / 2, H, 1}).v, postb = get(c, M, p + ".post.bias", {I / 2}).v;
    if (rev) {
      for (int o = 0; o < I / 4; ++o)
        std::swap_ranges(postw.begin() + (size_t)o * H, postw.begin() + (size_t)(o + 1) * H,
                         postw.begin() + (size_t)(I / 2 - 1 - o) * H);
      std::reverse(postb.begin(), postb.end());
    }
    c.alloc_weight(q + ".post.w", postw);
    c.alloc_weight(q + ".post.b", postb);
  }
  c.alloc_weight("flow.cond.w", condw);
  c.alloc_weight("flow.cond.b", condb);
  c.alloc_weight("emb_g", get(c, M, "emb_g.weight", {g.n_spk, g.gin}).v);
  if (g.f0 && g.vocoder == 2) {  // RefineGAN (generators/refinegan.py), its own weight tree
    finalize_refinegan(c);
    return;
  }
  // HiFiGAN-NSF (generators/hifigan_nsf.py:55-171); without pitch guidance the plain HiFiGANGenerator
  // (generators/hifigan.py:9-104): the same conv_pre / cond / ups / resblocks / conv_post, no source module
  const int C0 = g.C0;
  c.alloc_weight("dec.pre.w", pack_conv1d(get(c, M, "dec.conv_pre.weight", {C0, I, 7})));
  c.alloc_weight("dec.pre.b", get(c, M, "dec.conv_pre.bias", {C0}).v);
  c.alloc_weight("dec.cond.w", get(c, M, "dec.cond.weight", {C0, g.gin, 1}).v);
  c.alloc_weight("dec.cond.b", get(c, M, "dec.cond.bias", {C0}).v);
  // MRF HiFi-GAN (generators/hifigan_mrf.py:234-330) has the same dataflow under other names: upsamples.i for
  // ups.i, mrfs.i.j.layers.m.conv1/conv2 for resblocks.(i*nk+j).convs1/convs2.m, a 9-harmonic source and a
  // conv_post bias; its weights are packed under the NSF decoder's device names
  const bool mrf = g.vocoder == 1;
  const int Hs = g.src_harmonics();
  if (g.f0) {
    auto& lw = get(c, M, "dec.m_source.l_linear.weight", {1, Hs}).v;
    auto& lb = get(c, M, "dec.m_source.l_linear.bias", {1}).v;
    c.alloc_weight("dec.src.w", lw);
    c.host[M]["__src_lin__"] = HostTensor{{lw[0], lb[0]}, {2}};
  }
  c.ups.clear();
  const int nu = (int)g.ups.size();
  for (int i = 0; i < nu; ++i) {
    const int cin = C0 >> i, cout = C0 >> (i + 1), u = g.ups[i], k = g.up_k[i];
    // NSF: padding (k - u) / 2 or u / 2 + u % 2 with output_padding u % 2 (hifigan_nsf.py:88-103);
    // HiFiGANGenerator: padding (k - u) / 2, no output_padding (hifigan.py:46-58)
    const int p = (!g.f0 || u % 2 == 0) ? (k - u) / 2 : u / 2 + u % 2;
    const int op = g.f0 ? u % 2 : 0;
    if (k + op - 2 * p != u)
      throw Error(RVCX_E_SHAPE, "ConvTranspose1d stage " + std::to_string(i) + ": output length != T*u unsupported");
    const std::string n = "dec.ups." + std::to_string(i);
    const std::string nref = (mrf ? "dec.upsamples." : "dec.ups.") + std::to_string(i);
    auto& w = get(c, M, nref + ".weight", {cin, cout, k});
    auto& b = get(c, M, nref + ".bias", {cout});
    auto fdiv = [](int a, int bb) { return (a >= 0) ? a / bb : -((-a + bb - 1) / bb); };
    int smin = 1 << 30, smax = -(1 << 30);
    for (int r = 0; r < u; ++r) {
      const int lo = -fdiv(r + p, u);                // ceil(-(r+p)/u)
      const int hi = fdiv(k - 1 - r - p, u);         // floor((k-1-r-p)/u)
      smin = std::min(smin, lo);
      smax = std::max(smax, hi);
    }
    UpsLayer L;
    L.cin = cin;
    L.cout = cout;
    L.u = u;
    L.k = k;
    L.taps = smax - smin + 1;
    L.pad = smax;
    std::vector<float> wv((size_t)L.taps * u * cout * cin, 0.f), bv((size_t)u * cout);
    for (int tau = 0; tau < L.taps; ++tau) {
      const int s = smax - tau;
      for (int r = 0; r < u; ++r) {
        const int kk = s * u + r + p;
        if (kk < 0 || kk >= k) continue;
        for (int co = 0; co < cout; ++co)
          for (int ci = 0; ci < cin; ++ci)
            wv[(((size_t)tau * u + r) * cout + co) * cin + ci] = w.v[((size_t)ci * cout + co) * k + kk];
      }
    }
    for (int r = 0; r < u; ++r)
      for (int co = 0; co < cout; ++co) bv[(size_t)r * cout + co] = b.v[co];
    L.w = c.alloc_weight(n + ".vw", wv);
    L.b = c.alloc_weight(n + ".vb", bv);
    c.ups.push_back(L);
    if (!g.f0) continue;
    // noise conv (C_in = 1)
    int stride = 1;
    for (int j = i + 1; j < nu; ++j) stride *= g.ups[j];
    const int kern = stride == 1 ? 1 : stride * 2 - stride % 2;
    const std::string nn = "dec.noise_convs." + std::to_string(i);
    // framed form for the implicit GEMM: the source is read as rows of `stride` samples, so the
    // kern = 2*stride conv becomes 2 taps x stride channels: wf[tap][co][ci] = w[co][0][tap*stride + ci]
    // (kern = 1 when stride = 1: one tap, one channel)
    const HostTensor& wn = get(c, M, nn + ".weight", {cout, 1, kern});
    const int ntap = kern == 1 ? 1 : 2;
    std::vector<float> wf((size_t)ntap * cout * stride, 0.f);
    for (int tp = 0; tp < ntap; ++tp)
      for (int co = 0; co < cout; ++co)
        for (int ci = 0; ci < stride; ++ci) {
          const int kk = tp * stride + ci;
          if (kk < kern) wf[((size_t)tp * cout + co) * stride + ci] = wn.v[(size_t)co * kern + kk];
        }
    c.alloc_weight(nn + ".wf", wf);
    c.alloc_weight(nn + ".b", get(c, M, nn + ".bias", {cout}).v);
  }
  const int nk = (int)g.rb_k.size();
  for (int i = 0; i < nu; ++i) {
    const int C = C0 >> (i + 1);
    for (int j = 0; j < nk; ++j) {
      const int k = g.rb_k[j];
      const std::string rb = "dec.resblocks." + std::to_string(i * nk + j);
      for (size_t m = 0; m < g.rb_d[j].size(); ++m) {
        for (int q = 0; q < 2; ++q) {
          const std::string n = rb + (q ? ".convs2." : ".convs1.") + std::to_string(m);
          const std::string nref = mrf ? "dec.mrfs." + std::to_string(i) + "." + std::to_string(j) + ".layers." +
                                             std::to_string(m) + (q ? ".conv2" : ".conv1")
                                       : n;
          c.alloc_weight(n + ".w", pack_conv1d(get(c, M, nref + ".weight", {C, C, k})));
          c.alloc_weight(n + ".b", get(c, M, nref + ".bias", {C}).v);
        }
      }
    }
  }
  const int Cl = C0 >> nu;
  c.alloc_weight("dec.post.w", get(c, M, "dec.conv_post.weight", {1, Cl, 7}).v);
  const float post_b = mrf ? get(c, M, "dec.conv_post.bias", {1}).v[0] : 0.f;  // weight_norm(Conv1d(ch, 1, 7))
  c.host[M]["__post_b__"] = HostTensor{{post_b}, {1}};
}

// ------------------------------------------------------------------ generator
// HiFiGANNSFGenerator.forward (generators/hifigan_nsf.py:173-212); z_btc [B][T][I] time-major.
namespace {
// noise_convs[i]'s framing for stage i (hifigan_nsf.py:184-199): stride = the product of the later upsample rates,
// kernel 2 stride - stride % 2 (1 at the last stage), read from har at HAR_PAD - npad; ntap taps of `stride` samples
struct NoiseFrame {
  int stride = 1, kern = 1, npad = 0, ntap = 1;
};
NoiseFrame noise_frame(const SynthCfg& cf, size_t i) {
  NoiseFrame f;
  for (size_t j = i + 1; j < cf.ups.size(); ++j) f.stride *= cf.ups[j];
  f.kern = f.stride == 1 ? 1 : f.stride * 2 - f.stride % 2;
  f.npad = f.stride == 1 ? 0 : (f.kern - f.stride) / 2;
  f.ntap = f.kern == 1 ? 1 : 2;
  if (f.npad > HAR_PAD || f.ntap * f.stride - f.npad > HAR_PAD + f.stride)
    throw Error(RVCX_E_SHAPE, "noise conv stride too large for the source padding");
  return f;
}
bool noise_row_kernel(const NoiseFrame& f, int B, long long Ti, int C) {  // k_noise_add's limits
  return f.ntap * f.stride <= 16 && C % 4 == 0 && (long long)B * Ti * (C / 4) < (1LL << 31) && f.ntap * f.stride * C <= 4096;
}
// NSF source (SineGen + l_linear + tanh) into the zero-padded rows of "dec.har"
float* dec_source(Ctx& c, int B, int T, const float* f0, const float* eps_src, uint64_t seed, hipStream_t s) {
  const SynthCfg& cf = c.scfg;
  const int upp = cf.upp();
  const long long Nh = (long long)T * upp;
  // har rows carry HAR_PAD zeros on both sides so every framed noise-conv read stays in its row
  const long long har_ld = Nh + 2 * HAR_PAD;
  float* har = c.buf<float>("dec.har", (size_t)(B * har_ld), s);
  // the pad columns stay zero from call to call (the sources write the interior only)
  c.zero_once("dec.har", har, sizeof(float) * (size_t)(B * har_ld), har_ld * 65536 + B, s);
  const auto& lin_wb = c.host[0].at("__src_lin__").v;
  const uint64_t sseed = splitmix(seed ^ 0x5352434e4f495345ull);
  if (cf.vocoder == 0) {  // NSF SineGen, harmonic_num 0 (hifigan.py:156-228)
    double* cum = c.buf<double>("dec.cum", (size_t)B * T, s);
    check(sine_source(f0, B, T, upp, (float)cf.sr, eps_src, sseed, lin_wb[0], lin_wb[1], cum, har + HAR_PAD, har_ld, s),
          "sine_source");
  } else {  // MRF: 9 harmonics, per-sample phase accumulation (hifigan_mrf.py:120-230)
    const int Hs = cf.src_harmonics();
    double* ws = c.buf<double>("dec.harm_ws", harm_source_ws_doubles(B, T, upp, Hs), s);
    const float* ini = eps_src ? eps_src + (size_t)B * cf.src_noise_row(T) : nullptr;
    check(harm_source(f0, B, T, upp, (float)cf.sr, Hs, 0, eps_src, ini, sseed, c.W("dec.src.w"), lin_wb[1], ws,
                      har + HAR_PAD, har_ld, s),
          "harm_source");
  }
  return har;
}
}  // namespace

bool dec_noise_prepare(Ctx& c, int B, int T, const float* f0, const float* eps_src, uint64_t seed, hipStream_t s) {
  const SynthCfg& cf = c.scfg;
  if (!cf.f0 || cf.vocoder == 2 || !f0) return false;
  const long long har_ld = (long long)T * cf.upp() + 2 * HAR_PAD;
  float* har = dec_source(c, B, T, f0, eps_src, seed, s);
  long long Ti = T;
  for (size_t i = 0; i < cf.ups.size(); ++i) {
    const int C = c.ups[i].cout;
    Ti *= cf.ups[i];
    const NoiseFrame f = noise_frame(cf, i);
    if (f.ntap * f.stride == 1) continue;  // the one-tap stage stays in its ConvTranspose's epilogue (dec_forward)
    const std::string nn = "dec.noise_convs." + std::to_string(i);
    float* nz = c.buf<float>("dec.nz" + std::to_string(i), (size_t)B * Ti * C, s);
    if (noise_row_kernel(f, B, Ti, C)) {
      check(noise_conv_add(har + HAR_PAD - f.npad, har_ld, f.stride, f.ntap, c.W(nn + ".wf"), c.W(nn + ".b"), nz, B,
                           (int)Ti, C, s, true),
            "noise_conv");
    } else {
      ConvArgs an = conv(har + HAR_PAD - f.npad, f.stride, (int)Ti + f.ntap - 1, f.stride, c.W(nn + ".wf"), C, f.ntap, 1,
                         0, c.W(nn + ".b"), nz, C, (int)Ti, B);
      an.x_bs = har_ld;
      an.lds_pad = 64 * 1024;  // beside the flow's latency-bound chain: at most two of its workgroups per CU
      run(c, an, s, 2.0 * B * (double)Ti * C * f.kern);
    }
  }
  return true;
}

// ------------------------------------------------------------------ generator
// HiFiGANNSFGenerator.forward (generators/hifigan_nsf.py:173-212); z_btc [B][T][I] time-major.
void dec_forward(Ctx& c, int B, int T, const float* z_btc, const float* mask, const float* f0, const float* g,
                 const float* eps_src, uint64_t seed, float* out, hipStream_t s, int gen_lowp, bool noise_pre) {
  const SynthCfg& cf = c.scfg;
  if (cf.f0 && cf.vocoder == 2) {
    refinegan_forward(c, B, T, z_btc, mask, f0, g, eps_src, seed, out, s);
    return;
  }
  const int I = cf.I, C0 = cf.C0;
  const long long har_ld = (long long)T * cf.upp() + 2 * HAR_PAD;
  float* har = nullptr;
  if (cf.f0) {
    if (noise_pre) {
      har = c.buf<float>("dec.har", (size_t)(B * har_ld), s);  // written by dec_noise_prepare
    } else {
      har = dec_source(c, B, T, f0, eps_src, seed, s);
    }
  }
  // conv_pre + cond(g)
  float* cv = c.buf<float>("dec.cvec", (size_t)B * C0, s);
  run(c, lin(g, cf.gin, B, cf.gin, c.W("dec.cond.w"), C0, c.W("dec.cond.b"), cv, C0), s);
  // stage buffers sized for the largest stage
  size_t maxe = (size_t)T * C0;
  {
    long long t = T;
    for (size_t i = 0; i < cf.ups.size(); ++i) {
      t *= cf.ups[i];
      maxe = std::max(maxe, (size_t)t * (C0 >> (i + 1)));
    }
  }
  float* xin = c.buf<float>("dec.x", (size_t)B * maxe, s);
  float* y = c.buf<float>("dec.y", (size_t)B * maxe, s);
  float* R = c.buf<float>("dec.r", (size_t)B * maxe, s);
  float* t1 = c.buf<float>("dec.t", (size_t)B * maxe, s);
  {
    ConvArgs a = conv(z_btc, I, T, I, c.W("dec.pre.w"), C0, 7, 1, 3, c.W("dec.pre.b"), xin, C0, T, B);
    a.pre_mask = mask;
    a.pre_mask_bs = T;
    a.res = cv;
    a.ldr = 0;
    a.res_bs = C0;
    a.res_mode = RES_ADD_PRE;
    run(c, a, s);
  }
  float* cur = xin;
  int curT = T, Cin = C0;
  const int nk = (int)cf.rb_k.size();
  for (size_t i = 0; i < cf.ups.size(); ++i) {
    const UpsLayer& L = c.ups[i];
    const int C = L.cout, u = L.u, Ti = curT * u;
    // LeakyReLU(0.1) -> ConvTranspose1d (polyphase) ; output [B][curT][u*C] == [B][Ti][C]
    ConvArgs a = conv(cur, Cin, curT, Cin, L.w, u * C, L.taps, 1, L.pad, L.b, y, u * C, curT, B);
    a.w_static = 1;
    a.lowp = gen_lowp;
    a.pre_act = ACT_LRELU;
    a.pre_slope = 0.1f;
    // + noise_convs[i](har) (hifigan_nsf.py:196-199): the last stage's one-tap noise conv in the ConvTranspose's own
    // epilogue where that runs on the weight-streamed fp16 kernel (ConvArgs::nz_*, k_noise_add's arithmetic:
    // bit-identical, and y is not read back and rewritten by a second pass: 70 + 34 -> 97 us at C2); the other short
    // kernels (<= 16 taps) by a coalesced row kernel after it, one pass over y (in the epilogue, their 4 / 8 taps of
    // per-element loads cost more than the pass: stage 1 120 + 39 -> 173 us, stage 2 93 + 37 -> 130, r05q); the
    // long first-stage kernel as a framed implicit GEMM
    NoiseFrame nf;
    int& stride = nf.stride;
    int& kern = nf.kern;
    int& npad = nf.npad;
    int& ntap = nf.ntap;
    std::string nn;
    bool nz_fused = false;
    if (cf.f0) {
      nf = noise_frame(cf, i);
      nn = "dec.noise_convs." + std::to_string(i);
      const int kk = ntap * stride;
      if (noise_pre && kk > 1) {
        // computed ahead (dec_noise_prepare): y = ups(x) + nz, the residual of this ConvTranspose's epilogue -- the
        // same single addition as the accumulate pass after it (k_noise_add / the ACC_ADD conv), bit-identical
        a.res = c.buf<float>("dec.nz" + std::to_string(i), (size_t)B * Ti * C, s);
        a.ldr = u * C;
        a.res_bs = (long long)Ti * C;
        a.res_mode = RES_ADD_POST;
        nz_fused = true;
      } else if (kk == 1 && conv_routes_wsb16(c, a)) {
        a.nz_har = har + HAR_PAD - npad;
        a.nz_bs = har_ld;
        a.nz_stride = stride;
        a.nz_kk = ntap * stride;
        a.nz_u = u;
        a.nz_C = C;
        a.nz_w = c.W(nn + ".wf");
        a.nz_b = c.W(nn + ".b");
        nz_fused = true;
      }
    }
    run(c, a, s, 2.0 * B * curT * (double)Cin * C * L.k);
    if (cf.f0 && !nz_fused) {
      if (noise_row_kernel(nf, B, Ti, C)) {
        check(noise_conv_add(har + HAR_PAD - npad, har_ld, stride, ntap, c.W(nn + ".wf"), c.W(nn + ".b"), y, B, Ti,
                             C, s),
              "noise_conv_add");
      } else {
        ConvArgs an = conv(har + HAR_PAD - npad, stride, Ti + ntap - 1, stride, c.W(nn + ".wf"), C, ntap, 1, 0,
                           c.W(nn + ".b"), y, C, Ti, B);
        an.x_bs = har_ld;
        an.acc_mode = ACC_ADD;
        run(c, an, s, 2.0 * B * (double)Ti * C * kern);
      }
    }
    // mean of the ResBlocks (residuals.py:71-80) accumulated into S. `cur` (= xin) is dead once the
    // ConvTranspose above has consumed it, so S reuses it and becomes the next stage's input.
    float* S = xin;
    float* T1 = t1;
    float* RR = R;
    for (int j = 0; j < nk; ++j) {
      const int k = cf.rb_k[j];
      const auto& dil = cf.rb_d[j];
      const std::string rb = "dec.resblocks." + std::to_string(i * nk + j);
      const float* r_in = y;
      // widest stage taking the fused pair: 32 channels (same-box A/B of C2: fused 32 + weight-streamed 64 21.97 ms,
      // fused 32 + 64 22.46, weight-streamed both 23.07; again +0.1 ms at 64 in round 5)
      bool fuse = C <= 32;
      for (int d : dil) fuse = fuse && rb_pair_fits(C, k, d);
      if (fuse) {
        // each dilation pair as one fused kernel (resblock_fused.hip); pairs ping-pong between RR and T1 (a pair
        // reads its neighbours' halo rows, so it never writes its own input), the last one accumulates into S
        for (size_t m = 0; m < dil.size(); ++m) {
          const std::string n1 = rb + ".convs1." + std::to_string(m);
          const std::string n2 = rb + ".convs2." + std::to_string(m);
          const bool last = (m + 1 == dil.size());
          float* dst = last ? S : (m % 2 == 0 ? RR : T1);
          RbPairArgs p;
          p.x = r_in;
          p.x_bs = (long long)Ti * C;
          p.wfmt = (gen_lowp || c.conv_math_default() == 3) ? RB_WF16 : RB_WBF16;
          p.w1s = c.rb_wsplit_for(c.W(n1 + ".w"), C, k, p.wfmt, s);
          p.b1 = c.W(n1 + ".b");
          p.w2s = c.rb_wsplit_for(c.W(n2 + ".w"), C, k, p.wfmt, s);
          p.b2 = c.W(n2 + ".b");
          p.C = C;
          p.k = k;
          p.d = dil[m];
          p.T = Ti;
          p.B = B;
          p.y = dst;
          p.y_bs = (long long)Ti * C;
          p.lowp = gen_lowp;
          if (last) {
            p.acc_mode = (j == 0) ? ACC_STORE : ((j + 1 == nk) ? ACC_ADD_DIV : ACC_ADD);
            p.acc_div = (float)nk;
          }
          launch_rb_pair(c, p, s);
          r_in = dst;
        }
        continue;
      }
      // (c1 handing its output to c2 as a two-plane fp16 image, so that c2's halo staging is a copy instead of a split,
      // measured within noise of the fp32 hand-off in round 5: 13.03 / 13.06 ms vs 12.996 / 12.954; removed)
      for (size_t m = 0; m < dil.size(); ++m) {
        const int d = dil[m];
        const std::string n1 = rb + ".convs1." + std::to_string(m);
        const std::string n2 = rb + ".convs2." + std::to_string(m);
        ConvArgs a1 = conv(r_in, C, Ti, C, c.W(n1 + ".w"), C, k, d, (k * d - d) / 2, c.W(n1 + ".b"), T1, C, Ti, B);
        a1.w_static = 1;
        a1.lowp = gen_lowp;
        a1.pre_act = ACT_LRELU;
        a1.pre_slope = 0.1f;
        a1.act = ACT_LRELU;
        a1.slope = 0.1f;
        const bool last = (m + 1 == dil.size());
        float* dst = last ? S : RR;
        ConvArgs a2 = conv(T1, C, Ti, C, c.W(n2 + ".w"), C, k, 1, (k - 1) / 2, c.W(n2 + ".b"), dst, C, Ti, B);
        a2.w_static = 1;
        a2.lowp = gen_lowp;
        run(c, a1, s);
        a2.res = r_in;
        a2.ldr = C;
        a2.res_bs = (long long)Ti * C;
        a2.res_mode = RES_ADD_POST;
        if (last) {
          a2.acc_mode = (j == 0) ? ACC_STORE : ((j + 1 == nk) ? ACC_ADD_DIV : ACC_ADD);
          a2.acc_div = (float)nk;
        }
        run(c, a2, s);
        r_in = RR;
      }
    }
    cur = S;
    curT = Ti;
    Cin = C;
  }
  // LeakyReLU(0.01) -> conv_post (no bias) -> tanh
  check(conv_post_tanh(cur, B, curT, Cin, c.W("dec.post.w"), 7, 0.01f, out, s, c.host[0].at("__post_b__").v[0]),
        "conv_post");
}

// ------------------------------------------------------------------ Synthesizer.infer
void synth_forward(Ctx& c, int B, int T, const float* phone, const int32_t* lengths, const int32_t* pitch,
                   const float* pitchf, const int32_t* sid, const float* eps_z, const float* eps_src, uint64_t seed,
                   float* out, float* zp_out, float* z_out, hipStream_t s, int gen_lowp, int head, float* mp_out,
                   float* logsp_out) {
  const SynthCfg& cf = c.scfg;
  const int H = cf.H, I = cf.I, F = cf.F, E = cf.emb_dim, nh = cf.n_heads, dk = H / nh;
  const long long BT = (long long)B * T;
  float* mask = c.buf<float>("te.mask", BT, s);
  check(seq_mask(lengths, mask, B, T, s), "seq_mask");
  float* g = c.buf<float>("spk.g", (size_t)B * cf.gin, s);
  check(gather_rows(c.W("emb_g"), cf.gin, sid, g, B, cf.gin, s), "emb_g");
  // ---- TextEncoder (encoders.py:128-144)
  // x = emb_phone(phone) [+ emb_pitch(pitch) when pitch-guided, encoders.py:131-133]
  float* pe = nullptr;
  if (cf.f0) {
    pe = c.buf<float>("te.pe", BT * H, s);
    check(gather_rows(c.W("te.emb_pitch"), H, pitch, pe, (int)BT, H, s), "emb_pitch");
  }
  float* x = c.buf<float>("te.x", BT * H, s);
  {
    ConvArgs a = lin(phone, E, (int)BT, E, c.W("te.emb_phone.w"), H, c.W("te.emb_phone.b"), x, H);
    a.res = pe;
    a.ldr = H;
    a.res_mode = pe ? RES_ADD_PRE : RES_NONE;
    a.alpha = (float)std::sqrt((double)H);
    a.act = ACT_LRELU;
    a.slope = 0.1f;
    a.mask = mask;
    run(c, a, s);
  }
  float* qkv = c.buf<float>("te.qkv", BT * 3 * H, s);
  const int nsplit = flash_attn_splits(B, nh, T);
  float* part_o = c.buf<float>("te.fa_o", (size_t)flash_attn_ws_floats(B, nh, T, dk, nsplit), s);
  float* part_ml = c.buf<float>("te.fa_ml", (size_t)nsplit * B * nh * T * 2, s);
  float* att = c.buf<float>("te.att", BT * H, s);
  float* h1 = c.buf<float>("te.h1", BT * F, s);
  const float qscale = (float)(1.0 / std::sqrt((double)dk));
  for (int i = 0; i < cf.n_layers; ++i) {
    const std::string q = "te." + std::to_string(i);
    run(c, lin(x, H, (int)BT, H, c.W(q + ".qkv.w"), 3 * H, c.W(q + ".qkv.b"), qkv, 3 * H), s);
    // attentions.py:79-185 in one pass per query block (flash_attn.hip): no [B][nh][T][T] scores. The key mask only
    // where a row is shorter than T: with every length T it is all ones, and its per-element loads in the key loop
    // cost the TextEncoder's attention ~1/3 of its time (the fill never fires: identical results)
    check(flash_attn(qkv, 3 * H, B, T, nh, dk, qscale, c.W(q + ".rel_k"), c.W(q + ".rel_v"), cf.window,
                     c.synth_full_lengths ? nullptr : mask, part_o, part_ml, nsplit, att, H, s),
          "flash_attn");
    {  // x = LN(x + conv_o(att)) (norm_layers_1, attentions.py:57-62) in the split-K combine, in place (one combine
       // block per row reads the row's residual before writing it): one launch instead of the GEMM + a LayerNorm pass
      ConvArgs a = lin(att, H, (int)BT, H, c.W(q + ".o.w"), H, c.W(q + ".o.b"), x, H);
      a.res = x;
      a.ldr = H;
      a.ln_g = c.W(q + ".ln1.g");
      a.ln_b = c.W(q + ".ln1.b");
      run(c, a, s);
    }
    {  // FFN (attentions.py:221-231): conv_1(pad(x*mask)) -> relu -> conv_2(pad(.*mask)) * mask
      ConvArgs a = conv(x, H, T, H, c.W(q + ".ffn1.w"), F, cf.ksize, 1, (cf.ksize - 1) / 2, c.W(q + ".ffn1.b"), h1,
                        F, T, B);
      a.pre_mask = mask;
      a.pre_mask_bs = T;
      a.act = ACT_RELU;
      run(c, a, s);
      // x = LN(x + conv_2(.) * mask) in the split-K combine (norm_layers_2, attentions.py:63-66): no separate pass
      ConvArgs b = conv(h1, F, T, F, c.W(q + ".ffn2.w"), H, cf.ksize, 1, (cf.ksize - 1) / 2, c.W(q + ".ffn2.b"), x,
                        H, T, B);
      b.pre_mask = mask;
      b.pre_mask_bs = T;
      b.mask = mask;
      b.mask_bs = T;
      b.res = x;
      b.ldr = H;
      b.res_bs = (long long)T * H;
      b.ln_g = c.W(q + ".ln2.g");
      b.ln_b = c.W(q + ".ln2.b");
      run(c, b, s);
    }
  }
  float* stats = c.buf<float>("te.stats", BT * 2 * I, s);
  {
    ConvArgs a = lin(x, H, (int)BT, H, c.W("te.proj.w"), 2 * I, c.W("te.proj.b"), stats, 2 * I);
    a.pre_mask = mask;
    a.mask = mask;
    run(c, a, s);
  }
  // m_p / logs_p [B][T][I] for the caller (the return tuple of Synthesizer.infer, synthesizers.py:243)
  if (mp_out)
    RVCX_HIP(hipMemcpy2DAsync(mp_out, (size_t)I * 4, stats, (size_t)2 * I * 4, (size_t)I * 4, (size_t)BT,
                              hipMemcpyDeviceToDevice, s));
  if (logsp_out)
    RVCX_HIP(hipMemcpy2DAsync(logsp_out, (size_t)I * 4, stats + I, (size_t)2 * I * 4, (size_t)I * 4, (size_t)BT,
                              hipMemcpyDeviceToDevice, s));
  // ---- z_p = (m + exp(logs) * eps * 0.66666) * mask   (synthesizers.py:228)
  float* z = c.buf<float>("flow.z", BT * I, s);
  float* xf = c.buf<float>("flow.xf", BT * I, s);
  check(zp_sample(stats, B, T, I, eps_z, splitmix(seed ^ 0x5a505f4e4f495345ull), mask, z, s), "zp_sample");
  // rate (synthesizers.py:230-234): z_p, x_mask and nsff0 from frame head on; the noise was drawn over all T frames
  const int Tf = T - head;
  const long long BTf = (long long)B * Tf;
  const float* maskf = mask;
  const float* pitchff = pitchf;
  if (head > 0) {
    if (head >= T) throw Error(RVCX_E_SHAPE, "synthesizer: rate leaves no frames");
    float* z2 = c.buf<float>("flow.z_rate", (size_t)BTf * I, s);
    RVCX_HIP(hipMemcpy2DAsync(z2, (size_t)Tf * I * 4, z + (size_t)head * I, (size_t)T * I * 4, (size_t)Tf * I * 4,
                              (size_t)B, hipMemcpyDeviceToDevice, s));
    float* m2 = c.buf<float>("te.mask_rate", (size_t)BTf, s);
    RVCX_HIP(hipMemcpy2DAsync(m2, (size_t)Tf * 4, mask + head, (size_t)T * 4, (size_t)Tf * 4, (size_t)B,
                              hipMemcpyDeviceToDevice, s));
    if (pitchf) {
      float* p2 = c.buf<float>("dec.pitchf_rate", (size_t)BTf, s);
      RVCX_HIP(hipMemcpy2DAsync(p2, (size_t)Tf * 4, pitchf + head, (size_t)T * 4, (size_t)Tf * 4, (size_t)B,
                                hipMemcpyDeviceToDevice, s));
      pitchff = p2;
    }
    z = z2;
    maskf = m2;
  }
  if (zp_out) RVCX_HIP(hipMemcpyAsync(zp_out, z, BTf * I * sizeof(float), hipMemcpyDeviceToDevice, s));
  // the decoder's NSF source and multi-tap noise convs depend on f0 alone: issued now on the aux stream, beside the
  // flow's latency-bound chain, instead of between the decoder's ConvTransposes (kernel timing and RVCX_NO_OVERLAP
  // keep them on this stream, fork_aux)
  hipStream_t nax = s;
  bool noise_pre = false;
  if (cf.f0 && cf.vocoder != 2 && pitchff) {
    nax = fork_aux(c, s);
    noise_pre = dec_noise_prepare(c, B, Tf, pitchff, eps_src, seed, nax);
  }
  // ---- flow reverse (residuals.py:151-164, 233-258; modules.py:78-109)
  // hs [BTf][2H]: the WaveNet residual stream h (columns [0, H)) and its skip sum (columns [H, 2H))
  float* hs = c.buf<float>("flow.hs", BTf * 2 * H, s);
  float* acts = c.buf<float>("flow.acts", BTf * H, s);
  const int cl = 2 * H * cf.flow_layers;
  float* gc = c.buf<float>("flow.gc", (size_t)B * cf.flow_n * cl, s);
  // g -> every coupling's cond_layer(g) in one GEMM (modules.py:32-35, :92-93)
  run(c, lin(g, cf.gin, B, cf.gin, c.W("flow.cond.w"), cf.flow_n * cl, c.W("flow.cond.b"), gc, cf.flow_n * cl), s);
  const bool fold = cf.flow_n % 2 == 0;  // the flips folded into the couplings' weights (finalize)
  for (int f = cf.flow_n - 1; f >= 0; --f) {
    const std::string q = "flow." + std::to_string(f);
    // this coupling's x0 (pre's input) and x1 (post's residual and output) columns of the state
    float* x0 = xf;
    float* x1 = xf + I / 2;
    if (fold) {
      const bool rev = (cf.flow_n - 1 - f) % 2 == 0;
      x0 = rev ? z + I / 2 : z;
      x1 = rev ? z : z + I / 2;
    } else {
      check(channel_flip(z, xf, (int)BTf, I, s), "flip");
    }
    {  // h = pre(x0) * mask, and the skip sum cleared (the zero rows of the packed pre weight)
      ConvArgs a = lin(x0, I, (int)BTf, I / 2, c.W(q + ".pre.w"), 2 * H, c.W(q + ".pre.b"), hs, 2 * H);
      a.mask = maskf;
      run(c, a, s);
    }
    for (int L = 0; L < cf.flow_layers; ++L) {
      const std::string l = std::to_string(L);
      {  // acts = tanh(in(h)[:H] + g_l[:H]) * sigmoid(in(h)[H:] + g_l[H:])  (commons.py:88-103), in the split-K combine
        ConvArgs a = conv(hs, 2 * H, Tf, H, c.W(q + ".in" + l + ".w"), 2 * H, cf.flow_k, 1, (cf.flow_k - 1) / 2,
                          c.W(q + ".in" + l + ".b"), acts, H, Tf, B);
        a.x_bs = (long long)Tf * 2 * H;
        a.gate_h = H;
        a.gate_g = gc + (size_t)f * cl + (size_t)L * 2 * H;
        a.gate_g_bs = (long long)cf.flow_n * cl;
        run(c, a, s);
      }
      const float* wrs = c.W(q + ".rs" + l + ".w");
      const float* brs = c.W(q + ".rs" + l + ".b");
      // h = (h + res(acts)) * mask and skip += skip(acts) as one GEMM over both halves (modules.py:95-107); the skip
      // sum is masked at every layer instead of once at the end: the same values, the mask being exactly 0 / 1
      const bool last = L == cf.flow_layers - 1;
      ConvArgs a = lin(acts, H, (int)BTf, H, wrs, last ? H : 2 * H, brs, last ? hs + H : hs, 2 * H);
      a.acc_mode = ACC_ADD;
      a.mask = maskf;
      run(c, a, s);
    }
    {  // x1 = (x1 - m) * mask, m = post(h) * mask
      ConvArgs a = lin(hs + H, 2 * H, (int)BTf, H, c.W(q + ".post.w"), I / 2, c.W(q + ".post.b"), x1, I);
      a.res = x1;
      a.ldr = I;
      a.res_mode = RES_RSUB_POST;
      a.mask = maskf;
      run(c, a, s);
    }
    if (!fold) std::swap(z, xf);
  }
  if (z_out) RVCX_HIP(hipMemcpyAsync(z_out, z, BTf * I * sizeof(float), hipMemcpyDeviceToDevice, s));
  // ---- dec(z * mask, nsff0, g)
  join_aux(c, s, nax);
  dec_forward(c, B, Tf, z, maskf, pitchff, g, eps_src, seed, out, s, gen_lowp, noise_pre);
}

}  // namespace rvcx
