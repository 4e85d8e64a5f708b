// Whole-utterance pipeline on device: Pipeline.pipeline (rvc/infer/pipeline.py:390-558;
// rvc_mlx/infer/pipeline_mlx.py:263-373) = filtfilt -> reflect pad -> RMVPE -> get_f0 adjustments ->
// [split at quiet points when longer than t_max] -> per chunk HuBERT -> x2 upsample + protect ->
// Synthesizer.infer -> trim -> concatenate -> change_rms -> peak normalise.
//
// Everything that touches samples runs as HIP kernels on the caller's stream. The host only plans:
// it reads back the split points (long inputs) and, for proposed_pitch, the f0 track whose median
// sets the key offset (pipeline.py:250-277) -- both are a few KB and need one stream sync each.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "runtime.h"

namespace rvcx {

void set_highpass(Ctx& c, const double* b, const double* a, const double* zi, int order) {
  if (order < 1 || order > IIR_MAXO) throw Error(RVCX_E_INVALID, "highpass order out of range");
  if (!(a[0] != 0.0)) throw Error(RVCX_E_INVALID, "highpass a[0] == 0");
  c.hp_order = order;
  c.hp_sos = SosPlan();  // a new (b, a) filter drops any section form set for the previous one
  c.hp_b.assign(b, b + order + 1);
  c.hp_a.assign(a, a + order + 1);
  c.hp_zi.assign(zi, zi + order);
  const double a0 = a[0];
  for (auto& v : c.hp_b) v /= a0;
  for (auto& v : c.hp_a) v /= a0;
}

// SOS plan (iir_scan.hip): per section the DF2T biquad, its steady state for a unit pass input (scipy
// filtfilt's zi * x0: the whole cascade at rest on the constant x0, DC gains of the preceding sections
// included), A^(L 2^s) for the carry scan and the rows C A^k of the chunk fix-up.
void set_highpass_sos(Ctx& c, const double* sos, int nsec) {
  if (nsec < 1 || nsec > IIR_MAXO) throw Error(RVCX_E_INVALID, "highpass: bad section count");
  SosPlan p;
  p.nsec = nsec;
  p.L = 256;
  if (nsec > 4) throw Error(RVCX_E_INVALID, "highpass: more than 4 sections");
  std::vector<double> tab((size_t)nsec * p.stride(), 0.0);
  double gain = 1.0;  // DC gain of the sections before j
  for (int j = 0; j < nsec; ++j) {
    const double* q = sos + 6 * j;
    if (!(q[3] != 0.0)) throw Error(RVCX_E_INVALID, "highpass: section a0 == 0");
    const double b0 = q[0] / q[3], b1 = q[1] / q[3], b2 = q[2] / q[3], a1 = q[4] / q[3], a2 = q[5] / q[3];
    double* t = tab.data() + (size_t)j * p.stride();
    t[0] = b0, t[1] = b1, t[2] = b2, t[3] = a1, t[4] = a2;
    // steady state z = (I - A)^-1 B u with A = [[-a1, 1], [-a2, 0]], B = [b1 - a1 b0, b2 - a2 b0], u = gain
    const double B0 = b1 - a1 * b0, B1 = b2 - a2 * b0;
    const double det = (1.0 + a1) * 1.0 + a2;  // det(I - A) = (1 + a1) * 1 - (-1) * (a2)
    if (!(std::fabs(det) > 1e-300)) throw Error(RVCX_E_INVALID, "highpass: section has a pole at z = 1");
    // (I - A) = [[1 + a1, -1], [a2, 1]] -> inverse = [[1, 1], [-a2, 1 + a1]] / det
    t[8] = (B0 + B1) / det * gain;
    t[9] = (-a2 * B0 + (1.0 + a1) * B1) / det * gain;
    gain *= (b0 + b1 + b2) / (1.0 + a1 + a2);
    // A^L then squarings: pow[s] = A^(L 2^s), s = 0..10
    double M[4] = {1, 0, 0, 1};
    double* ca = t + 64;
    for (int k = 0; k < p.L; ++k) {
      ca[2 * k] = M[0];
      ca[2 * k + 1] = M[1];
      const double n0 = -a1 * M[0] + M[2], n1 = -a1 * M[1] + M[3], n2 = -a2 * M[0], n3 = -a2 * M[1];
      M[0] = n0, M[1] = n1, M[2] = n2, M[3] = n3;  // M <- A M
    }
    for (int sidx = 0; sidx < 11; ++sidx) {
      double* P = t + 16 + 4 * sidx;
      P[0] = M[0], P[1] = M[1], P[2] = M[2], P[3] = M[3];
      const double n0 = M[0] * M[0] + M[1] * M[2], n1 = M[0] * M[1] + M[1] * M[3];
      const double n2 = M[2] * M[0] + M[3] * M[2], n3 = M[2] * M[1] + M[3] * M[3];
      M[0] = n0, M[1] = n1, M[2] = n2, M[3] = n3;
    }
  }
  // the cascade as ONE system of NS = 2 nsec states (iir_scan.hip casc_filtfilt_pad): its A and C by stepping the
  // cascade from unit states with zero input, the steady state w = the per-section states above, A^(L 2^s) and
  // the rows C A^k of the chunk fix-up
  const int NS = 2 * nsec, L = p.casc_L;
  const size_t casc_off = tab.size();
  tab.resize(casc_off + 48 + 64 * 12 + 8 * (size_t)L, 0.0);
  double* ct = tab.data() + casc_off;
  std::vector<double> A((size_t)NS * NS), C(NS);
  auto step = [&](const double* z, double x, double* zo) {
    double u = x;
    for (int j = 0; j < nsec; ++j) {
      const double* t = tab.data() + (size_t)j * p.stride();
      const double y = t[0] * u + z[2 * j];
      zo[2 * j] = t[1] * u - t[3] * y + z[2 * j + 1];
      zo[2 * j + 1] = t[2] * u - t[4] * y;
      u = y;
    }
    return u;
  };
  for (int i = 0; i < NS; ++i) {
    std::vector<double> z(NS, 0.0), zo(NS, 0.0);
    z[i] = 1.0;
    C[i] = step(z.data(), 0.0, zo.data());
    for (int r = 0; r < NS; ++r) A[(size_t)r * NS + i] = zo[r];
  }
  for (int j = 0; j < nsec; ++j) {
    const double* t = tab.data() + (size_t)j * p.stride();
    for (int q = 0; q < 5; ++q) ct[5 * j + q] = t[q];
    ct[40 + 2 * j] = t[8];
    ct[40 + 2 * j + 1] = t[9];
  }
  auto mul = [&](const std::vector<double>& X, const std::vector<double>& Y) {
    std::vector<double> Z((size_t)NS * NS, 0.0);
    for (int r = 0; r < NS; ++r)
      for (int q = 0; q < NS; ++q)
        for (int k = 0; k < NS; ++k) Z[(size_t)r * NS + q] += X[(size_t)r * NS + k] * Y[(size_t)k * NS + q];
    return Z;
  };
  std::vector<double> M((size_t)NS * NS, 0.0);
  for (int i = 0; i < NS; ++i) M[(size_t)i * NS + i] = 1.0;
  std::vector<double> row(C);  // C A^k
  for (int k = 0; k < L; ++k) {
    for (int i = 0; i < NS; ++i) ct[48 + 64 * 12 + 8 * k + i] = row[i];
    std::vector<double> nr(NS, 0.0);
    for (int q = 0; q < NS; ++q)
      for (int i = 0; i < NS; ++i) nr[q] += row[i] * A[(size_t)i * NS + q];
    row = nr;
    M = mul(A, M);  // A^(k + 1)
  }
  for (int sidx = 0; sidx < 12; ++sidx) {  // pow[s] = A^(L 2^s), NS x NS in an 8 x 8 block
    for (int r = 0; r < NS; ++r)
      for (int q = 0; q < NS; ++q) ct[48 + 64 * sidx + 8 * r + q] = M[(size_t)r * NS + q];
    M = mul(M, M);
  }
  RVCX_HIP(hipSetDevice(c.device));
  c.hp_sos_buf.~DevBuf();
  new (&c.hp_sos_buf) DevBuf();
  const size_t bytes = tab.size() * sizeof(double);
  if (hipMalloc(&c.hp_sos_buf.p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    throw Error(RVCX_E_OOM, "highpass: device allocation failed");
  }
  c.hp_sos_buf.bytes = bytes;
  RVCX_HIP(hipMemcpy(c.hp_sos_buf.p, tab.data(), bytes, hipMemcpyHostToDevice));
  p.dev = static_cast<const double*>(c.hp_sos_buf.p);
  p.casc = p.dev + casc_off;
  c.hp_sos = p;
}

void highpass_pad(Ctx& c, const double* audio, int64_t n, int64_t t_pad, double* pad64, float* pad32, hipStream_t s) {
  if (c.hp_order == 0) throw Error(RVCX_E_STATE, "pipeline: high-pass filter not configured");
  if (c.hp_sos.nsec > 0) {
    double* ws = c.buf<double>("pl.sosws", filtfilt_sos_ws_doubles(n, c.hp_order, c.hp_sos.L), s);
    check(filtfilt_sos_pad(c.hp_sos, c.hp_order, audio, n, t_pad, ws, pad64, pad32, s), "filtfilt_sos");
    return;
  }
  double* ws = c.buf<double>("pl.iirws", filtfilt_ws_doubles(n, c.hp_order), s);
  check(filtfilt_pad(audio, n, c.hp_b.data(), c.hp_a.data(), c.hp_zi.data(), nullptr, c.hp_order, t_pad, ws, pad64,
                     pad32, s),
        "filtfilt_pad");
}

int hubert_version_for(const Ctx& c) { return c.scfg.emb_dim == 256 ? 1 : 2; }

int64_t vc_forward(Ctx& c, const float* audio, int64_t n, const int32_t* pitch, const float* pitchf,
                   int64_t pitch_len, int sid, float protect, double index_rate, const float* eps_z,
                   const float* eps_src, uint64_t seed, float* out, int64_t cap, hipStream_t s,
                   const float* feats_pre, int64_t L_pre) {
  if (sid < 0 || sid >= c.scfg.n_spk) throw Error(RVCX_E_INVALID, "sid out of range");
  const int E = c.scfg.emb_dim;
  const float* feats = feats_pre;
  int64_t L = L_pre;
  if (!feats) {
    const int64_t cap_rows = n / 320 + 8;  // HuBERT frames for n samples (upper bound n/320)
    float* fb = c.buf<float>("vc.feats", (size_t)cap_rows * E, s);
    L = hubert_forward(c, audio, n, hubert_version_for(c), fb, cap_rows, s);
    feats = fb;
  }
  const int T = (int)std::min<int64_t>(n / 160, 2 * L);
  if (T <= 0) throw Error(RVCX_E_SHAPE, "voice_conversion: input shorter than one frame");
  if (c.scfg.f0 && (!pitch || !pitchf)) throw Error(RVCX_E_INVALID, "voice_conversion: pitch-guided model needs pitch");
  if (!c.scfg.f0) pitch = nullptr, pitchf = nullptr;  // pitch_guidance False: no protect, no pitch (pipeline.py:324-365)
  if (pitch && T > pitch_len) throw Error(RVCX_E_SHAPE, "voice_conversion: pitch track shorter than the features");
  const int upp = c.scfg.upp();
  if ((int64_t)T * upp > cap)
    throw Error(RVCX_E_CAPACITY, "voice_conversion: output needs " + std::to_string((int64_t)T * upp) + " samples");
  // speaker-embedding retrieval on the raw features (pipeline.py:338-342); feats0 stays raw for protect
  const float* fx = feats;
  if (index_rate > 0 && c.ivf) {
    float* fr = c.buf<float>("vc.feats_idx", (size_t)L * E, s);
    index_retrieve(c, feats, L, E, index_rate, fr, s);
    fx = fr;
  }
  float* phone = c.buf<float>("vc.phone", (size_t)T * E, s);
  check(upsample2_protect(fx, feats, (int)L, E, phone, T, protect < 0.5f ? pitchf : nullptr, protect, s),
        "upsample");
  int32_t* lens = c.buf<int32_t>("vc.len", 4, s);
  set_i32_once(c, "vc.len.T", lens, T, s);
  set_i32_once(c, "vc.len.sid", lens + 1, sid, s);
  {
    ScopedFullLengths full(c);
    synth_forward(c, 1, T, phone, lens, pitch, pitchf, lens + 1, eps_z, eps_src, seed, out, nullptr, nullptr, s);
  }
  return (int64_t)T * upp;
}

// key offset of proposed_pitch (pipeline.py:250-277): median of the voiced-interpolated track
int proposed_key(const std::vector<double>& f0, double threshold) {
  std::vector<int64_t> valid;
  for (size_t i = 0; i < f0.size(); ++i)
    if (f0[i] > 0) valid.push_back((int64_t)i);
  if (valid.size() < 2) return 0;
  // np.interp(arange(F), valid, f0[valid]): clamps outside [valid[0], valid[-1]]
  std::vector<double> v(f0.size());
  size_t k = 0;
  for (size_t i = 0; i < f0.size(); ++i) {
    const int64_t x = (int64_t)i;
    if (x <= valid.front()) {
      v[i] = f0[valid.front()];
    } else if (x >= valid.back()) {
      v[i] = f0[valid.back()];
    } else {
      while (valid[k + 1] < x) ++k;
      const double x0 = (double)valid[k], x1 = (double)valid[k + 1];
      const double y0 = f0[valid[k]], y1 = f0[valid[k + 1]];
      v[i] = (x == valid[k + 1]) ? y1 : y0 + (y1 - y0) * ((double)x - x0) / (x1 - x0);
    }
  }
  std::sort(v.begin(), v.end());
  const size_t m = v.size();
  const double med = (m & 1) ? v[m / 2] : 0.5 * (v[m / 2 - 1] + v[m / 2]);
  if (!(med > 0)) return 0;
  const double key = std::nearbyint(12.0 * std::log2(threshold / med));  // np.round: half to even
  return (int)std::max(-12.0, std::min(12.0, key));
}

int64_t pipeline_forward_ex(Ctx& c, const double* audio, int64_t n, const rvcx_pipeline_opts& o,
                            const float* eps_z, const float* eps_src, uint64_t seed, float* out, int64_t cap,
                            double* f0_out, hipStream_t s) {
  if (c.hp_order == 0) throw Error(RVCX_E_STATE, "pipeline: high-pass filter not configured");
  if (o.t_pad < 0 || o.t_pad_tgt < 0 || o.t_pad >= n) throw Error(RVCX_E_INVALID, "pipeline: bad t_pad");
  if (o.f0_method < 0 || o.f0_method > 2)
    throw Error(RVCX_E_INVALID, "pipeline: f0_method must be 0 (rmvpe), 1 (crepe, MLX) or 2 (crepe, rvc/)");
  if (o.f0_method >= 1 && c.scfg.f0 && !c.ready[RVCX_MODEL_CREPE])
    throw Error(RVCX_E_STATE, "pipeline: f0_method crepe but no CREPE weights finalized");
  if (o.index_rate > 0 && !c.ivf) throw Error(RVCX_E_STATE, "pipeline: index_rate > 0 but no feature index loaded");
  if (o.index_rate > 0 && c.ivf->view.d != c.scfg.emb_dim)
    throw Error(RVCX_E_SHAPE, "pipeline: feature index dimension does not match the model's feature width");
  if (o.version != 0 && o.version != hubert_version_for(c))
    throw Error(RVCX_E_INVALID, "pipeline: version does not match the synthesizer's embedding width");
  const int64_t W = 160;  // Pipeline.window
  const int64_t m = n + 2 * o.t_pad;
  // 1. zero-phase high-pass, reflect pad t_pad (pipeline.py:439, :459); fp64 copy kept for the split
  //    search and the RMS envelope, fp32 copy feeds the models (torch.from_numpy(...).float()).
  float* pad32 = c.buf<float>("pl.pad32", (size_t)m, s);
  double* pad64 = c.buf<double>("pl.pad64", (size_t)m, s);
  highpass_pad(c, audio, n, o.t_pad, pad64, pad32, s);
  const double* filtered = pad64 + o.t_pad;
  // 2. split points for inputs longer than t_max (pipeline.py:440-452)
  std::vector<int64_t> opt_ts;
  if (o.t_max > 0 && n + W > o.t_max && o.t_center > 0) {
    if (o.t_query <= 0 || o.t_query > o.t_center) throw Error(RVCX_E_INVALID, "pipeline: bad t_query/t_center");
    const int nts = n > o.t_center ? (int)((n - 1 - o.t_center) / o.t_center + 1) : 0;
    double* sum = c.buf<double>("pl.winsum", (size_t)n, s);
    long long* dts = c.buf<long long>("pl.ts", (size_t)std::max(1, nts), s);
    check(split_points(filtered, n, (int)W, o.t_center, o.t_query, sum, dts, nts, s), "split_points");
    opt_ts.resize(nts);
    if (nts > 0 && c.sizing_plan) {
      // rvcx_workspace_bytes: the plan whose longest chunk is the longest any audio can give (each split point lies
      // in [k t_center - t_query, k t_center + t_query]): a middle chunk from the lowest split to the highest next one
      // (or, with one split, the first chunk up to its highest split); the rest centred
      for (int k = 0; k < nts; ++k) opt_ts[k] = (int64_t)(k + 1) * o.t_center;
      if (nts == 1) opt_ts[0] += o.t_query;
      else opt_ts[0] -= o.t_query, opt_ts[1] += o.t_query;
      for (auto& t : opt_ts) t = std::max<int64_t>(0, std::min<int64_t>(t, n - 1));
    } else if (nts > 0) {
      RVCX_HIP(hipMemcpyAsync(opt_ts.data(), dts, sizeof(long long) * nts, hipMemcpyDeviceToHost, s));
      RVCX_HIP(hipStreamSynchronize(s));
      c.check_device_status();
    }
  }
  // 3. chunk plan (pipeline.py:486-512): [a0, a1) samples and [f_lo, f_hi) pitch frames per chunk
  struct Chunk {
    int64_t a0, a1, f_lo, f_hi;
  };
  std::vector<Chunk> chunks;
  {
    const int64_t t_pad2 = 2 * o.t_pad;
    int64_t st = 0, t = 0;
    bool have_t = false;
    for (int64_t t_raw : opt_ts) {
      t = t_raw / W * W;
      chunks.push_back({st, std::min(m, t + t_pad2 + W), st / W, (t + t_pad2) / W});
      st = t;
      have_t = true;
    }
    chunks.push_back(have_t ? Chunk{t, m, t / W, m / W} : Chunk{0, m, 0, m / W});
  }
  // 4. HuBERT of every chunk on the aux stream, beside RMVPE on the caller's stream (they only share
  //    the padded input); the chunk loop waits for it before the upsample. Kernel timing (rvcx_profile)
  //    and RVCX_NO_OVERLAP=1 keep it on the caller's stream so per-kernel durations are not shared.
  const int E = c.scfg.emb_dim;
  std::vector<float*> cfeats(chunks.size());
  std::vector<int64_t> cL(chunks.size());
  //    The encoder's last layers are issued only when RMVPE reaches its BiGRU (which holds 4 CUs for ~2 ms):
  //    the U-Net then shares the GPU with less of HuBERT and the rest of HuBERT fills the BiGRU's idle CUs.
  hipStream_t ax = fork_aux(c, s);
  static const int gate_layer = [] {
    const char* e = rvcx_knob("RVCX_HUBERT_GATE");  // first layer issued beside the BiGRU (12: none)
    // A/B on MI355X (BiGRU launched first), round 2: 2 21.84 ms, 3 21.87, 4 21.96, 1 22.03, 0 22.12, 6 22.30; round 4 (same
    // box, 4 runs each, profiles/r04q_ab_hubert_gate.txt): 0 13.39 ms, 1 13.45, 2 13.53 -- with the fp16-split U-Net
    // and HuBERT the whole encoder fits beside the BiGRU, and the U-Net then shares the GPU with the front alone
    const int v = e ? std::atoi(e) : 0;
    return v < 0 ? 0 : (v > HUBERT_LAYERS ? HUBERT_LAYERS : v);
  }();
  // without pitch guidance there is no RMVPE (pipeline.py:461-472 skipped): HuBERT runs in one piece
  const bool guided = c.scfg.f0;
  const int split = (ax != s && guided) ? gate_layer : HUBERT_LAYERS;
  std::vector<HubertRun> hruns(chunks.size());
  // chunks are processed longest first: every later chunk fits the shared work buffers the first one grew, so a
  // call regrows nothing past its first chunk (a caller-sized arena, rvcx_workspace_bytes, holds any split plan);
  // the per-chunk noise offsets, seeds and output positions keep the reference's order (computed up front below)
  std::vector<size_t> order(chunks.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) {
    return chunks[x].a1 - chunks[x].a0 > chunks[y].a1 - chunks[y].a0;
  });
  // HuBERT's feature encoder (and the layers before the gate) on the aux stream beside the U-Net. Measured and removed:
  // issuing it from a later U-Net level on (neutral) and on a CU-masked stream of 64 / 128 CUs (+3.6 ms)
  {
    struct FrontScope {  // the throttle ends with the front end's issue, also when an exception ends it
      Ctx& c;
      ~FrontScope() { c.aux_front = false; }
    } front_scope{c};
    c.aux_front = ax != s;
    for (size_t i : order) {
      const int64_t len = chunks[i].a1 - chunks[i].a0;
      const int64_t cap_rows = len / 320 + 8;
      cfeats[i] = c.buf<float>("pl.hb" + std::to_string(i), (size_t)cap_rows * E, ax);
      hruns[i] = hubert_front(c, pad32 + chunks[i].a0, len, len, 1, hubert_version_for(c), cfeats[i], cap_rows, ax);
      if (chunks.size() == 1) {
        hubert_layers(c, hruns[i], 0, split, ax);
      } else {  // several chunks share the HuBERT workspace: each runs to completion before the next
        hubert_layers(c, hruns[i], 0, HUBERT_LAYERS, ax);
        cL[i] = hubert_tail(c, hruns[i], ax);
      }
    }
  }
  // the caller records c.ev_gate on `main` where the rest may start (gate_here), then calls this
  auto gate_here = [&](hipStream_t main) {
    if (ax != main && c.ev_gate) RVCX_HIP(hipEventRecord(c.ev_gate, main));
  };
  auto hubert_rest = [&](hipStream_t main) {
    if (chunks.size() != 1) return;
    if (split < HUBERT_LAYERS && ax != main) RVCX_HIP(hipStreamWaitEvent(ax, c.ev_gate, 0));
    hubert_layers(c, hruns[0], split, HUBERT_LAYERS, ax);
    cL[0] = hubert_tail(c, hruns[0], ax);
  };
  struct HookScope {
    Ctx& c;
    ~HookScope() { c.before_gru = nullptr; }
  } hook_scope{c};
  c.before_gru = hubert_rest;
  // 5. f0 over the whole padded input (pipeline.py:462-472) + get_f0 adjustments (:248-291)
  const int64_t F = 1 + m / W;
  int32_t* pitch = nullptr;
  float* pitchf = nullptr;
  if (guided) {
  double* f0 = c.buf<double>("pl.f0", (size_t)F, s);
  if (o.f0_method >= 1) {
    // CREPE (PitchExtractor.extract, rvc_mlx/lib/mlx/pitch_extractors.py:155-156, with PipelineMLX's f0_min 50 /
    // f0_max 1100 and CREPE.get_f0's threshold 0.1; f0_method 2: rvc/'s CREPE.get_f0, pipeline.py:223-234, viterbi
    // decode without its dither): no BiGRU, so HuBERT's remaining layers go out first and overlap the CREPE convs on
    // the aux stream
    if (c.before_gru) {
      auto rest = std::move(c.before_gru);
      c.before_gru = nullptr;
      gate_here(s);
      rest(s);
    }
    float* f0f = c.buf<float>("pl.f0f", (size_t)F, s);
    crepe_forward(c, pad32, m, 50.0, 1100.0, 0.1f, f0f, f0, nullptr, nullptr, s, o.f0_method == 2 ? 1 : 0);
  } else {
    rmvpe_forward(c, pad32, m, o.rmvpe_threshold > 0 ? o.rmvpe_threshold : 0.03f, f0, F, nullptr, s);
  }
  if (c.before_gru) {  // RMVPE did not reach a BiGRU launch (cannot happen for valid input): issue it now
    auto rest = std::move(c.before_gru);
    c.before_gru = nullptr;
    gate_here(s);
    rest(s);
  }
  double shift_semitones = o.pitch;
  if (o.f0_autotune) {
    check(f0_autotune(f0, (int)F, o.f0_autotune_strength, o.mlx_semantics ? 1 : 0, s), "f0_autotune");
    if (!o.mlx_semantics) shift_semitones = 0.0;  // rvc/: autotune replaces the shift (pipeline.py:248-279)
  } else if (o.proposed_pitch) {
    std::vector<double> h(F);
    RVCX_HIP(hipMemcpyAsync(h.data(), f0, sizeof(double) * F, hipMemcpyDeviceToHost, s));
    RVCX_HIP(hipStreamSynchronize(s));
    c.check_device_status();
    shift_semitones = o.pitch + proposed_key(h, o.proposed_pitch_threshold);
  }
  pitch = c.buf<int32_t>("pl.pitch", (size_t)F, s);
  pitchf = c.buf<float>("pl.pitchf", (size_t)F, s);
  check(f0_post(f0, (int)F, std::pow(2.0, shift_semitones / 12.0), pitch, pitchf, f0_out, s), "f0_post");
  } else {
    auto rest = std::move(c.before_gru);
    c.before_gru = nullptr;
    gate_here(s);
    rest(s);
    if (f0_out) RVCX_HIP(hipMemsetAsync(f0_out, 0, sizeof(double) * (size_t)F, s));
  }
  join_aux(c, s, ax);
  // 6. voice conversion per chunk (pipeline.py:486-512), outputs trimmed t_pad_tgt per side
  const int upp = c.scfg.upp();
  const int I = c.scfg.I;
  // per chunk, in the reference's order: frames T = min(len / 160, 2 L) (vc_forward), noise offsets, seed, output
  // position
  const size_t nch = chunks.size();
  std::vector<int64_t> ez_off(nch), es_off(nch), pos(nch);
  std::vector<uint64_t> cseed(nch);
  int64_t written = 0;
  {
    int64_t ez = 0, es = 0;
    uint64_t sd = seed;
    for (size_t i = 0; i < nch; ++i) {
      ez_off[i] = ez;
      es_off[i] = es;
      cseed[i] = sd;
      pos[i] = written;
      if (nch > 1) {
        const int64_t T = std::min<int64_t>((chunks[i].a1 - chunks[i].a0) / W, 2 * cL[i]);
        ez += (int64_t)I * T;
        es += c.scfg.src_noise_total(1, T);  // this chunk's decoder draws (include/rvcx.h layouts)
        const int64_t keep = T * upp - 2 * o.t_pad_tgt;
        if (keep <= 0) throw Error(RVCX_E_SHAPE, "pipeline: chunk too short for the padding");
        written += keep;
      }
      sd += 0x9E3779B97F4A7C15ull;
    }
    if (written > cap)
      throw Error(RVCX_E_CAPACITY, "pipeline: output needs more than " + std::to_string(cap) + " samples");
  }
  const bool fuse_trim = nch == 1 && o.volume_envelope == 1.0;
  const float* trimmed = out;
  for (size_t i : order) {
    const Chunk& ch = chunks[i];
    const int64_t len = ch.a1 - ch.a0;
    const int64_t cap_vc = (len / W) * upp;
    float* vc = c.buf<float>("pl.vc", (size_t)std::max<int64_t>(cap_vc, 1), s);
    // pitch[:, f_lo:f_hi], then [:p_len] inside voice_conversion with p_len = min(len/160, 2L)
    const int64_t nvc = vc_forward(c, pad32 + ch.a0, len, pitch ? pitch + ch.f_lo : nullptr,
                                   pitchf ? pitchf + ch.f_lo : nullptr, ch.f_hi - ch.f_lo, o.sid,
                                   o.protect, o.index_rate, eps_z ? eps_z + ez_off[i] : nullptr,
                                   eps_src ? eps_src + es_off[i] : nullptr, cseed[i], vc, cap_vc, s, cfeats[i], cL[i]);
    const int64_t keep = nvc - 2 * o.t_pad_tgt;
    if (keep <= 0) throw Error(RVCX_E_SHAPE, "pipeline: chunk too short for the padding");
    if (nch == 1) {
      if (keep > cap)
        throw Error(RVCX_E_CAPACITY, "pipeline: output needs more than " + std::to_string(cap) + " samples");
      written = keep;
    }
    if (fuse_trim)
      trimmed = vc + o.t_pad_tgt;  // one chunk, no envelope: the peak normalisation reads it in place
    else
      RVCX_HIP(hipMemcpyAsync(out + pos[i], vc + o.t_pad_tgt, (size_t)keep * sizeof(float), hipMemcpyDeviceToDevice,
                              s));
  }
  // 7. volume envelope (pipeline.py:545-549) and peak normalisation (:550-552)
  if (o.volume_envelope != 1.0) {
    const int n1 = rms_frame_count(n, 16000), n2 = rms_frame_count(written, c.scfg.sr);
    float* rws = c.buf<float>("pl.rms", (size_t)(n1 + n2), s);
    check(change_rms(filtered, n, 16000, out, written, c.scfg.sr, (float)o.volume_envelope, rws, s), "change_rms");
  }
  float* mx = c.buf<float>("pl.max", peak_normalize_ws_floats(1), s);
  check(peak_normalize(trimmed, out, written, mx, s), "peak_normalize");
  return written;
}

// Batched offline conversion (config C4): B equal-length utterances, each no longer than t_max (one chunk
// each, pipeline.py:486-512 with opt_ts empty), through one batched RMVPE, one batched HuBERT and one
// batched Synthesizer.infer. Per utterance the result is Pipeline.pipeline's; the batch only widens
// every GEMM (B x rows). audio row b at audio + b*lda (fp64); out row b at out + b*ldo, n_out samples each.
int64_t pipeline_forward_batch(Ctx& c, const double* audio, int64_t n, int64_t lda, int B, const rvcx_pipeline_opts& o,
                               const int32_t* sids, const float* eps_z, const float* eps_src, uint64_t seed,
                               float* out, int64_t ldo, double* f0_out, float* hidden_out, hipStream_t s) {
  if (B < 1) throw Error(RVCX_E_INVALID, "pipeline_batch: B < 1");
  if (c.hp_order == 0) throw Error(RVCX_E_STATE, "pipeline: high-pass filter not configured");
  if (o.t_pad < 0 || o.t_pad_tgt < 0 || o.t_pad >= n) throw Error(RVCX_E_INVALID, "pipeline: bad t_pad");
  if (o.f0_method < 0 || o.f0_method > 2)
    throw Error(RVCX_E_INVALID, "pipeline: f0_method must be 0 (rmvpe), 1 (crepe, MLX) or 2 (crepe, rvc/)");
  if (o.f0_method >= 1 && c.scfg.f0 && !c.ready[RVCX_MODEL_CREPE])
    throw Error(RVCX_E_STATE, "pipeline: f0_method crepe but no CREPE weights finalized");
  if (o.t_max > 0 && n + 160 > o.t_max)
    throw Error(RVCX_E_INVALID, "pipeline_batch: utterances longer than t_max take the single-utterance path");
  if (o.index_rate > 0 && !c.ivf) throw Error(RVCX_E_STATE, "pipeline: index_rate > 0 but no feature index loaded");
  if (o.version != 0 && o.version != hubert_version_for(c))
    throw Error(RVCX_E_INVALID, "pipeline: version does not match the synthesizer's embedding width");
  for (int b = 0; b < B; ++b)
    if (sids[b] < 0 || sids[b] >= c.scfg.n_spk) throw Error(RVCX_E_INVALID, "pipeline_batch: sid out of range");
  const int64_t W = 160;
  const int64_t m = n + 2 * o.t_pad;
  const int64_t ldm = (m + 7) & ~int64_t(7);
  const int E = c.scfg.emb_dim, upp = c.scfg.upp();
  // 1. zero-phase high-pass + reflect pad per utterance (pipeline.py:439, :459)
  float* pad32 = c.buf<float>("pb.pad32", (size_t)B * ldm, s);
  double* pad64 = c.buf<double>("pb.pad64", (size_t)B * m, s);
  for (int b = 0; b < B; ++b)
    highpass_pad(c, audio + (size_t)b * lda, n, o.t_pad, pad64 + (size_t)b * m, pad32 + (size_t)b * ldm, s);
  // 2. f0 (batched RMVPE) + get_f0 adjustments per utterance (pipeline.py:462-472, :248-291)
  const int64_t F = 1 + m / W, T = m / W;
  double* f0 = c.buf<double>("pb.f0", (size_t)B * F, s);
  const int64_t L = hubert_frames(m);
  float* feats = c.buf<float>("pb.feats", (size_t)B * L * E, s);
  hipStream_t ax = fork_aux(c, s);  // batched HuBERT beside batched RMVPE
  hubert_forward_b(c, pad32, m, ldm, B, hubert_version_for(c), feats, L, ax);
  const bool guided = c.scfg.f0;  // no RMVPE, pitch or protect without pitch guidance (pipeline.py:324-365)
  int32_t* pitch = nullptr;
  float* pitchf = nullptr;
  if (guided) {
  if (o.f0_method >= 1) {  // CREPE per utterance (frames of all rows would not batch any better: B x F frames)
    float* f0f = c.buf<float>("pb.f0f", (size_t)F, s);
    for (int b = 0; b < B; ++b)
      crepe_forward(c, pad32 + (size_t)b * ldm, m, 50.0, 1100.0, 0.1f, f0f, f0 + (size_t)b * F, nullptr, nullptr, s,
                    o.f0_method == 2 ? 1 : 0);
  } else {
    rmvpe_forward_b(c, pad32, m, ldm, B, o.rmvpe_threshold > 0 ? o.rmvpe_threshold : 0.03f, f0, F, hidden_out, s);
  }
  std::vector<double> shift(B, o.pitch);
  if (o.f0_autotune) {
    check(f0_autotune(f0, (int)(B * F), o.f0_autotune_strength, o.mlx_semantics ? 1 : 0, s), "f0_autotune");
    if (!o.mlx_semantics) std::fill(shift.begin(), shift.end(), 0.0);
  } else if (o.proposed_pitch) {
    std::vector<double> h((size_t)B * F);
    RVCX_HIP(hipMemcpyAsync(h.data(), f0, sizeof(double) * h.size(), hipMemcpyDeviceToHost, s));
    RVCX_HIP(hipStreamSynchronize(s));
    c.check_device_status();
    for (int b = 0; b < B; ++b) {
      std::vector<double> one(h.begin() + (size_t)b * F, h.begin() + (size_t)(b + 1) * F);
      shift[b] = o.pitch + proposed_key(one, o.proposed_pitch_threshold);
    }
  }
  pitch = c.buf<int32_t>("pb.pitch", (size_t)B * F, s);
  pitchf = c.buf<float>("pb.pitchf", (size_t)B * F, s);
  for (int b = 0; b < B; ++b)
    check(f0_post(f0 + (size_t)b * F, (int)F, std::pow(2.0, shift[b] / 12.0), pitch + (size_t)b * F,
                  pitchf + (size_t)b * F, f0_out ? f0_out + (size_t)b * F : nullptr, s),
          "f0_post");
  } else if (f0_out) {
    RVCX_HIP(hipMemsetAsync(f0_out, 0, sizeof(double) * (size_t)B * F, s));
  }
  // 3. batched HuBERT, retrieval, x2 upsample + protect (pipeline.py:327-362)
  join_aux(c, s, ax);
  const int64_t Tv = std::min<int64_t>(T, 2 * L);
  if (Tv <= 0) throw Error(RVCX_E_SHAPE, "pipeline_batch: input shorter than one frame");
  const float* fx = feats;
  if (o.index_rate > 0) {
    if (c.ivf->view.d != E) throw Error(RVCX_E_SHAPE, "pipeline: feature index dimension mismatch");
    float* fr = c.buf<float>("pb.feats_idx", (size_t)B * L * E, s);
    index_retrieve(c, feats, B * L, E, o.index_rate, fr, s);  // row-wise: the B sequences stack
    fx = fr;
  }
  float* phone = c.buf<float>("pb.phone", (size_t)B * Tv * E, s);
  int32_t* pc = nullptr;
  float* pf = nullptr;
  if (guided) {
    pc = c.buf<int32_t>("pb.pc", (size_t)B * Tv, s);
    pf = c.buf<float>("pb.pf", (size_t)B * Tv, s);
    RVCX_HIP(hipMemcpy2DAsync(pc, Tv * sizeof(int32_t), pitch, F * sizeof(int32_t), Tv * sizeof(int32_t), B,
                              hipMemcpyDeviceToDevice, s));
    RVCX_HIP(hipMemcpy2DAsync(pf, Tv * sizeof(float), pitchf, F * sizeof(float), Tv * sizeof(float), B,
                              hipMemcpyDeviceToDevice, s));
  }
  for (int b = 0; b < B; ++b)
    check(upsample2_protect(fx + (size_t)b * L * E, feats + (size_t)b * L * E, (int)L, E, phone + (size_t)b * Tv * E,
                            (int)Tv, (guided && o.protect < 0.5f) ? pf + (size_t)b * Tv : nullptr, o.protect, s),
          "upsample");
  // 4. one batched Synthesizer.infer (pipeline.py:365-372)
  int32_t* meta = c.buf<int32_t>("pb.meta", 2 * (size_t)B, s);
  std::vector<int32_t> hm(2 * (size_t)B);
  for (int b = 0; b < B; ++b) {
    hm[b] = (int32_t)Tv;
    hm[B + b] = sids[b];
  }
  RVCX_HIP(hipMemcpyAsync(meta, hm.data(), sizeof(int32_t) * hm.size(), hipMemcpyHostToDevice, s));
  const int64_t nvc = Tv * upp;
  float* vc = c.buf<float>("pb.vc", (size_t)B * nvc, s);
  {
    ScopedFullLengths full(c);  // every row Tv long (hm above)
    synth_forward(c, B, (int)Tv, phone, meta, pc, pf, meta + B, eps_z, eps_src, seed, vc, nullptr, nullptr, s);
  }
  // 5. trim, volume envelope, peak normalisation per utterance (pipeline.py:545-552)
  const int64_t keep = nvc - 2 * o.t_pad_tgt;
  if (keep <= 0) throw Error(RVCX_E_SHAPE, "pipeline_batch: utterance too short for the padding");
  if (keep > ldo) throw Error(RVCX_E_CAPACITY, "pipeline_batch: output rows need " + std::to_string(keep));
  float* mx = c.buf<float>("pb.max", peak_normalize_ws_floats(B), s);
  if (o.volume_envelope == 1.0) {  // trim + normalise in one pass over all rows
    check(peak_normalize(vc + o.t_pad_tgt, out, keep, mx, s, B, nvc, ldo), "peak_normalize");
    return keep;
  }
  RVCX_HIP(hipMemcpy2DAsync(out, ldo * sizeof(float), vc + o.t_pad_tgt, nvc * sizeof(float), keep * sizeof(float), B,
                            hipMemcpyDeviceToDevice, s));
  for (int b = 0; b < B; ++b) {
    const int n1 = rms_frame_count(n, 16000), n2 = rms_frame_count(keep, c.scfg.sr);
    float* rws = c.buf<float>("pl.rms", (size_t)(n1 + n2), s);
    check(change_rms(pad64 + (size_t)b * m + o.t_pad, n, 16000, out + (size_t)b * ldo, keep, c.scfg.sr,
                     (float)o.volume_envelope, rws, s),
          "change_rms");
  }
  check(peak_normalize(out, out, keep, mx, s, B, ldo, ldo), "peak_normalize");
  return keep;
}

rvcx_pipeline_opts default_pipeline_opts() {
  rvcx_pipeline_opts o;
  std::memset(&o, 0, sizeof(o));
  o.version = 0;
  o.protect = 0.33f;
  o.rmvpe_threshold = 0.03f;
  o.t_pad = 16000;
  o.t_pad_tgt = 48000;
  o.t_query = 16000 * 6;
  o.t_center = 16000 * 38;
  o.t_max = 16000 * 41;
  o.f0_autotune_strength = 1.0;
  o.proposed_pitch_threshold = 155.0;
  o.volume_envelope = 1.0;
  return o;
}

}  // namespace rvcx
