// Streaming voice conversion (config C5): a group of B concurrent streams of one buffer geometry,
// converted together per hop on the caller's stream.
//
// Reference: rvc/realtime/core.py -- VoiceChanger (:329-484), Realtime.realloc (:165-216),
// Realtime.inference (:217-326) -- and rvc/realtime/pipeline.py Realtime_Pipeline.get_f0 (:122-212) /
// voice_conversion (:214-334) / _retrieve_speaker_embeddings (:336-352). The MLX port of this path is
// not functional, so the PyTorch semantics are followed.
//
// Per hop, all on device: 48k -> 16k resample (torchaudio sinc kernel), circular audio/convert buffers
// and the RMS gate, RMVPE f0 + realtime quantisation into the circular pitch buffers, HuBERT (+ repeated
// last frame), optional index retrieval from skip_head // 2, x2 upsample + protect, one batched
// Synthesizer.infer over the B streams, clip, [volume envelope], * sqrt(vol), [tgt -> 48k resample],
// SOLA offset search + crossfade. The host only plans (and syncs once per hop for proposed_pitch).
#include <cmath>
#include <cstring>

#include "runtime.h"

namespace rvcx {

namespace {

// torchaudio.functional.functional._get_sinc_resample_kernel (sinc_interp_hann, width 6, rolloff 0.99),
// evaluated in float32 like Resample(..., dtype=torch.float32) (core.py:99-108).
struct SincKernel {
  int orig = 1, nw = 1, width = 0, K = 0;
  std::vector<float> k;  // [nw][K]
};

SincKernel sinc_kernel(int orig_freq, int new_freq) {
  auto gcd = [](int a, int b) {
    while (b) {
      const int t = a % b;
      a = b;
      b = t;
    }
    return a;
  };
  const int g = gcd(orig_freq, new_freq);
  SincKernel r;
  r.orig = orig_freq / g;
  r.nw = new_freq / g;
  const float lpw = 6.0f;
  const double base_d = (double)std::min(r.orig, r.nw) * 0.99;
  r.width = (int)std::ceil(6.0 * r.orig / base_d);
  r.K = 2 * r.width + r.orig;
  r.k.resize((size_t)r.nw * r.K);
  const float base = (float)base_d;
  const float pi = (float)M_PI;
  for (int p = 0; p < r.nw; ++p) {
    for (int i = 0; i < r.K; ++i) {
      const float idx = (float)(i - r.width) / (float)r.orig;
      float t = (-(float)p) / (float)r.nw + idx;
      t = t * base;
      t = std::min(std::max(t, -lpw), lpw);
      const float c = std::cos(t * pi / lpw / 2.0f);
      const float window = c * c;
      t = t * pi;
      const float scale = (float)(base_d / r.orig);
      const float kv = t == 0.0f ? 1.0f : std::sin(t) / t;
      r.k[(size_t)p * r.K + i] = kv * (window * scale);
    }
  }
  return r;
}

template <class T>
void dev_alloc(DevBuf& b, size_t count) {
  const size_t bytes = std::max<size_t>(count * sizeof(T), 16);
  if (hipMalloc(&b.p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    throw Error(RVCX_E_OOM, "stream state allocation failed");
  }
  b.bytes = bytes;
  RVCX_HIP(hipMemset(b.p, 0, bytes));
}

}  // namespace

struct RtState {
  int B = 0;
  int block48 = 0, cross48 = 0, extra48 = 0, sola48 = 0;
  int block16 = 0, cross16 = 0, sola16 = 0, extra16 = 0;
  int conv16 = 0, feat = 0, skip_head = 0, return_length = 0, silence_front = 0;
  int n16 = 0;      // resampled input length per hop (ceil(block48 / 3))
  int abuf_n = 0, pbuf_n = 0;
  double sensitivity = 1.0;
  int tgt_sr = 48000;
  SincKernel kin, kout;
  bool out_identity = true;
  DevBuf d_kin, d_kout, abuf[2], cbuf[2], pbuf[2], fbuf[2], sola, fade_in, offs, vol, volsq, gate, factor, meta;
  int cur = 0;
};

RtState* rt_create(Ctx& c, const rvcx_rt_desc& d) {
  if (!c.ready[0] || !c.ready[1] || !c.ready[2]) throw Error(RVCX_E_STATE, "stream: synth, hubert and rmvpe must be finalized");
  if (d.n_streams < 1 || d.n_streams > 4096) throw Error(RVCX_E_INVALID, "stream: n_streams out of range");
  if (d.read_chunk_size < 1) throw Error(RVCX_E_INVALID, "stream: read_chunk_size < 1");
  auto r = std::make_unique<RtState>();
  RtState& s = *r;
  const double AUDIO_SR = 48000.0, SR = 16000.0;
  const int window = 160;
  s.B = d.n_streams;
  // VoiceChanger.__init__ (core.py:351-354)
  s.block48 = d.read_chunk_size * 128;
  s.cross48 = (int)(d.cross_fade_overlap_size * AUDIO_SR);
  s.extra48 = (int)(d.extra_convert_size * AUDIO_SR);
  s.sola48 = 48000 / 100;
  // Realtime.realloc (core.py:172-199)
  s.block16 = (int)((double)s.block48 / AUDIO_SR * SR);
  s.cross16 = (int)((double)s.cross48 / AUDIO_SR * SR);
  s.sola16 = (int)((double)s.sola48 / AUDIO_SR * SR);
  s.extra16 = (int)((double)s.extra48 / AUDIO_SR * SR);
  int conv = s.block16 + s.sola16 + s.extra16 + s.cross16;
  if (conv % window) conv += window - conv % window;
  s.conv16 = conv;
  s.feat = conv / window;
  s.skip_head = s.extra16 / window;
  s.return_length = s.feat - s.skip_head;
  s.silence_front = 0;  // Realtime.__init__ sets 0, so realloc keeps 0 (core.py:57, :200-202)
  s.abuf_n = s.block16 + s.cross16;
  s.pbuf_n = s.feat + 1;
  s.sensitivity = std::pow(10.0, d.silent_threshold / 20.0);
  s.tgt_sr = c.scfg.sr;
  s.kin = sinc_kernel(48000, 16000);
  s.n16 = (int)std::ceil((double)s.kin.nw * s.block48 / s.kin.orig);
  if (s.n16 > s.abuf_n || s.n16 > s.conv16) throw Error(RVCX_E_INVALID, "stream: block larger than its buffers");
  s.out_identity = s.tgt_sr == 48000;
  if (!s.out_identity) s.kout = sinc_kernel(s.tgt_sr, 48000);
  const int upp = c.scfg.upp();
  const int64_t n_model = (int64_t)s.feat * upp;
  const int64_t n48 = s.out_identity ? n_model : (int64_t)std::ceil((double)s.kout.nw * n_model / s.kout.orig);
  if (n48 < (int64_t)s.sola48 + s.block48 + s.cross48)
    throw Error(RVCX_E_INVALID, "stream: model output shorter than sola search + block + crossfade");
  const int64_t L = hubert_frames(s.conv16);
  if (L < 1 || 2 * L + 1 < s.feat) throw Error(RVCX_E_INVALID, "stream: convert buffer too short for HuBERT");
  if (s.skip_head / 2 >= L) throw Error(RVCX_E_INVALID, "stream: skip_head beyond the feature frames");
  RVCX_HIP(hipSetDevice(c.device));
  dev_alloc<float>(s.d_kin, s.kin.k.size());
  RVCX_HIP(hipMemcpy(s.d_kin.p, s.kin.k.data(), s.kin.k.size() * sizeof(float), hipMemcpyHostToDevice));
  if (!s.out_identity) {
    dev_alloc<float>(s.d_kout, s.kout.k.size());
    RVCX_HIP(hipMemcpy(s.d_kout.p, s.kout.k.data(), s.kout.k.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  for (int i = 0; i < 2; ++i) {
    dev_alloc<float>(s.abuf[i], (size_t)s.B * s.abuf_n);
    dev_alloc<float>(s.cbuf[i], (size_t)s.B * s.conv16);
    dev_alloc<int>(s.pbuf[i], (size_t)s.B * s.pbuf_n);
    dev_alloc<float>(s.fbuf[i], (size_t)s.B * s.pbuf_n);
  }
  dev_alloc<float>(s.sola, (size_t)s.B * s.cross48);
  // fade_in = sin(0.5*pi*linspace(0, 1, cf))**2 in float32 (core.py:376-396; torch linspace's
  // two-sided formula)
  std::vector<float> fi((size_t)std::max(1, s.cross48));
  const int cf = s.cross48;
  if (cf == 1) {
    fi[0] = 0.f;
  } else if (cf > 1) {
    const float step = 1.0f / (float)(cf - 1);
    const int half = cf / 2;
    const float hp = (float)(0.5 * M_PI);
    for (int i = 0; i < cf; ++i) {
      const float x = i < half ? step * (float)i : 1.0f - step * (float)(cf - i - 1);
      const float v = std::sin(hp * x);
      fi[i] = v * v;
    }
  }
  dev_alloc<float>(s.fade_in, fi.size());
  RVCX_HIP(hipMemcpy(s.fade_in.p, fi.data(), fi.size() * sizeof(float), hipMemcpyHostToDevice));
  dev_alloc<int>(s.offs, s.B);
  dev_alloc<float>(s.vol, s.B);
  dev_alloc<float>(s.volsq, s.B);
  dev_alloc<int>(s.gate, s.B);
  dev_alloc<double>(s.factor, s.B);
  dev_alloc<int32_t>(s.meta, 2 * (size_t)s.B);
  return r.release();
}

void rt_destroy(RtState* s) { delete s; }

void rt_geometry(const RtState& s, int64_t* g) {
  const int64_t v[12] = {s.B,        s.block48,       s.block16,       s.conv16,     s.feat,    s.skip_head,
                         s.return_length, s.cross48, s.sola48, s.extra48, s.n16, s.silence_front};
  std::memcpy(g, v, sizeof(v));
}

void rt_reset(Ctx& c, RtState& s, hipStream_t st) {
  (void)c;
  for (int i = 0; i < 2; ++i) {
    RVCX_HIP(hipMemsetAsync(s.abuf[i].p, 0, s.abuf[i].bytes, st));
    RVCX_HIP(hipMemsetAsync(s.cbuf[i].p, 0, s.cbuf[i].bytes, st));
    RVCX_HIP(hipMemsetAsync(s.pbuf[i].p, 0, s.pbuf[i].bytes, st));
    RVCX_HIP(hipMemsetAsync(s.fbuf[i].p, 0, s.fbuf[i].bytes, st));
  }
  RVCX_HIP(hipMemsetAsync(s.sola.p, 0, s.sola.bytes, st));
  s.cur = 0;
}

void rt_process(Ctx& c, RtState& s, const float* in48, const int32_t* sids, const rvcx_rt_opts& o,
                const float* eps_z, const float* eps_src, uint64_t seed, float* out48, float* vol_out, int* offs_out,
                hipStream_t st) {
  const int B = s.B, E = c.scfg.emb_dim, upp = c.scfg.upp(), I = c.scfg.I;
  for (int b = 0; b < B; ++b)
    if (sids[b] < 0 || sids[b] >= c.scfg.n_spk) throw Error(RVCX_E_INVALID, "stream: sid out of range");
  if (o.index_rate > 0 && !c.ivf) throw Error(RVCX_E_STATE, "stream: index_rate > 0 but no feature index loaded");
  if (o.gen_precision < 0 || o.gen_precision > 1)
    throw Error(RVCX_E_INVALID, "stream: gen_precision must be 0 (fp32) or 1 (fp16 generator)");
  if (o.index_rate > 0 && c.ivf->view.d != E) throw Error(RVCX_E_SHAPE, "stream: index dimension mismatch");
  const int nxt = 1 - s.cur;
  // 1. input resample 48k -> 16k, circular buffers, RMS gate (core.py:227-267)
  float* in16 = c.buf<float>("rt.in16", (size_t)B * s.n16, st);
  check(rt_resample(in48, s.block48, s.block48, static_cast<const float*>(s.d_kin.p), s.kin.K, s.kin.width, s.kin.orig,
                    s.kin.nw, in16, s.n16, s.n16, nullptr, B, st),
        "rt_resample_in");
  check(rt_ingest(in16, s.n16, static_cast<float*>(s.abuf[s.cur].p), static_cast<float*>(s.abuf[nxt].p), s.abuf_n,
                  static_cast<float*>(s.cbuf[s.cur].p), static_cast<float*>(s.cbuf[nxt].p), s.conv16, s.sensitivity,
                  static_cast<float*>(s.vol.p), static_cast<float*>(s.volsq.p), static_cast<int*>(s.gate.p), B, st),
        "rt_ingest");
  const float* conv = static_cast<const float*>(s.cbuf[nxt].p);
  // 2. f0 on the convert buffer (pipeline.py:233-245 -> get_f0 :122-212)
  const int nf = s.conv16 - s.silence_front;
  const int F = 1 + nf / 160;
  if (F > s.pbuf_n) throw Error(RVCX_E_SHAPE, "stream: f0 track longer than the pitch buffer");
  double* f0 = c.buf<double>("rt.f0", (size_t)B * F, st);
  const int64_t L = hubert_frames(s.conv16);
  float* feats = c.buf<float>("rt.feats", (size_t)B * L * E, st);
  hipStream_t ax = fork_aux(c, st);  // batched HuBERT beside batched RMVPE (pipeline.py:233-254)
  hubert_forward_b(c, conv, s.conv16, s.conv16, B, hubert_version_for(c), feats, L, ax);
  const bool guided = c.scfg.f0;  // no get_f0, pitch or protect without pitch guidance (pipeline.py:242-293)
  if (guided) {
  rmvpe_forward_b(c, conv + s.silence_front, nf, s.conv16, B, 0.03f, f0, F, nullptr, st);
  std::vector<double> fac(B, std::pow(2.0, o.f0_up_key / 12.0));
  if (o.f0_autotune) {
    check(f0_autotune(f0, B * F, o.f0_autotune_strength, 0, st), "f0_autotune");
    std::fill(fac.begin(), fac.end(), 1.0);  // autotune replaces the shift (pipeline.py:157-158)
  } else if (o.proposed_pitch) {
    std::vector<double> h((size_t)B * F);
    RVCX_HIP(hipMemcpyAsync(h.data(), f0, sizeof(double) * h.size(), hipMemcpyDeviceToHost, st));
    RVCX_HIP(hipStreamSynchronize(st));
    c.check_device_status();
    for (int b = 0; b < B; ++b) {
      std::vector<double> one(h.begin() + (size_t)b * F, h.begin() + (size_t)(b + 1) * F);
      fac[b] = std::pow(2.0, (o.f0_up_key + proposed_key(one, o.proposed_pitch_threshold)) / 12.0);
    }
  }
  RVCX_HIP(hipMemcpyAsync(s.factor.p, fac.data(), sizeof(double) * B, hipMemcpyHostToDevice, st));
  check(rt_pitch(f0, F, static_cast<const double*>(s.factor.p), static_cast<const int*>(s.pbuf[s.cur].p),
                 static_cast<int*>(s.pbuf[nxt].p), static_cast<const float*>(s.fbuf[s.cur].p),
                 static_cast<float*>(s.fbuf[nxt].p), s.pbuf_n, B, st),
        "rt_pitch");
  }
  // 3. HuBERT over the B convert buffers (pipeline.py:248-254), rows [B][L][E]
  join_aux(c, st, ax);
  // 4. index retrieval of rows skip_head // 2 .. (pipeline.py:264-268, :336-352)
  const float* fx = feats;
  if (o.index_rate > 0) {
    float* fr = c.buf<float>("rt.feats_idx", (size_t)B * L * E, st);
    const int64_t off = s.skip_head / 2;
    for (int b = 0; b < B; ++b) {
      const float* src = feats + (size_t)b * L * E;
      float* dst = fr + (size_t)b * L * E;
      if (off > 0) RVCX_HIP(hipMemcpyAsync(dst, src, sizeof(float) * off * E, hipMemcpyDeviceToDevice, st));
      index_retrieve(c, src + off * E, L - off, E, o.index_rate, dst + off * E, st);
    }
    fx = fr;
  }
  // 5. x2 upsample [:p_len] + protect; pitch tails (pipeline.py:270-293)
  const int T = s.feat;
  float* phone = c.buf<float>("rt.phone", (size_t)B * T * E, st);
  int32_t* pitch = c.buf<int32_t>("rt.pitch", (size_t)B * T, st);
  float* pitchf = c.buf<float>("rt.pitchf", (size_t)B * T, st);
  const double formant = std::ceil(s.return_length * 1.0);
  const float pscale = (float)(formant / (double)s.return_length);
  check(rt_up2(fx, feats, (int)L, E, phone, T, static_cast<const float*>(s.fbuf[nxt].p), s.pbuf_n, pscale, o.protect,
               (guided && o.protect < 0.5f) ? 1 : 0, pitch, static_cast<const int*>(s.pbuf[nxt].p), pitchf, B, st),
        "rt_up2");
  // 6. one batched Synthesizer.infer over the B streams (pipeline.py:295-297), clip (:93)
  std::vector<int32_t> meta(2 * (size_t)B);
  for (int b = 0; b < B; ++b) {
    meta[b] = T;
    meta[B + b] = sids[b];
  }
  int32_t* dmeta = static_cast<int32_t*>(s.meta.p);
  RVCX_HIP(hipMemcpyAsync(dmeta, meta.data(), sizeof(int32_t) * meta.size(), hipMemcpyHostToDevice, st));
  const int64_t n_model = (int64_t)T * upp;
  float* model = c.buf<float>("rt.model", (size_t)B * n_model, st);
  {
    ScopedFullLengths full(c);  // every stream's hop is T frames (meta above)
    synth_forward(c, B, T, phone, dmeta, guided ? pitch : nullptr, guided ? pitchf : nullptr, dmeta + B, eps_z,
                  eps_src, seed, model, nullptr, nullptr, st, o.gen_precision);
  }
  (void)I;
  check(rt_clip(model, n_model, (int)n_model, B, st), "rt_clip");
  if (o.volume_envelope != 1.0) {  // pipeline.py:299-307 (source = the 16 kHz convert buffer)
    const int n1 = rms_frame_count(s.conv16, 16000), n2 = rms_frame_count(n_model, s.tgt_sr);
    float* ws = c.buf<float>("rt.rms", (size_t)(n1 + n2), st);
    for (int b = 0; b < B; ++b)
      check(change_rms_f32src(conv + (size_t)b * s.conv16, s.conv16, 16000, model + (size_t)b * n_model, n_model,
                              s.tgt_sr, (float)o.volume_envelope, ws, st),
            "change_rms");
  }
  // 7. * sqrt(vol) [-> 48 kHz], SOLA crossfade (core.py:324, :404-451)
  const float* a48 = model;
  int64_t lda = n_model;
  const float* scale = static_cast<const float*>(s.volsq.p);
  if (!s.out_identity) {
    const int64_t n48 = (int64_t)std::ceil((double)s.kout.nw * n_model / s.kout.orig);
    float* r48 = c.buf<float>("rt.model48", (size_t)B * n48, st);
    check(rt_resample(model, n_model, (int)n_model, static_cast<const float*>(s.d_kout.p), s.kout.K, s.kout.width,
                      s.kout.orig, s.kout.nw, r48, n48, (int)n48, scale, B, st),
          "rt_resample_out");
    a48 = r48;
    lda = n48;
    scale = nullptr;
  }
  check(rt_sola(a48, lda, scale, static_cast<const int*>(s.gate.p), static_cast<float*>(s.sola.p), s.cross48,
                s.sola48, static_cast<const float*>(s.fade_in.p), out48, s.block48,
                offs_out ? offs_out : static_cast<int*>(s.offs.p), B, st),
        "rt_sola");
  if (vol_out) RVCX_HIP(hipMemcpyAsync(vol_out, s.vol.p, sizeof(float) * B, hipMemcpyDeviceToDevice, st));
  s.cur = nxt;
}

}  // namespace rvcx
