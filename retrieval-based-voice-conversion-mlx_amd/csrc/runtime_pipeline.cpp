// Whole-utterance pipeline on device (Pipeline.pipeline, rvc/infer/pipeline.py:390-558, single-chunk
// case audio_pad <= t_max; rvc_mlx/infer/pipeline_mlx.py:263-373): filtfilt -> reflect pad -> RMVPE ->
// f0 post -> HuBERT -> x2 upsample + protect -> Synthesizer.infer -> trim -> peak normalise.
#include <cmath>
#include <cstring>

#include "runtime.h"

namespace rvcx {

void set_highpass(Ctx& c, const double* b, const double* a, const double* zi, int order) {
  if (order < 1 || order > IIR_MAXO) throw Error(RVCX_E_INVALID, "highpass order out of range");
  c.hp_order = order;
  c.hp_b.assign(b, b + order + 1);
  c.hp_a.assign(a, a + order + 1);
  c.hp_zi.assign(zi, zi + order);
  const double a0 = a[0];
  for (auto& v : c.hp_b) v /= a0;
  for (auto& v : c.hp_a) v /= a0;
  // state transition of DF2T with zero input: z'_i = z_{i+1} - a_{i+1} z_0 ; F^L for chunk length 256
  std::vector<double> F(IIR_MAXO * IIR_MAXO, 0.0), P(IIR_MAXO * IIR_MAXO, 0.0), T(IIR_MAXO * IIR_MAXO);
  for (int i = 0; i < order; ++i) {
    F[i * IIR_MAXO + 0] = -c.hp_a[i + 1];
    if (i + 1 < order) F[i * IIR_MAXO + i + 1] += 1.0;
  }
  for (int i = 0; i < order; ++i) P[i * IIR_MAXO + i] = 1.0;
  for (int step = 0; step < 256; ++step) {
    std::fill(T.begin(), T.end(), 0.0);
    for (int i = 0; i < order; ++i)
      for (int k = 0; k < order; ++k) {
        double acc = 0.0;
        for (int j = 0; j < order; ++j) acc += F[i * IIR_MAXO + j] * P[j * IIR_MAXO + k];
        T[i * IIR_MAXO + k] = acc;
      }
    P = T;
  }
  c.hp_FL = P;
}

int64_t pipeline_forward(Ctx& c, const double* audio, int64_t n, int sid, double semitones, float protect,
                         int64_t t_pad, int64_t t_pad_tgt, const float* eps_z, const float* eps_src, uint64_t seed,
                         float* out, int64_t cap, double* f0_out, hipStream_t s) {
  if (c.hp_order == 0) throw Error(RVCX_E_STATE, "pipeline: high-pass filter not configured");
  const int64_t m = n + 2 * t_pad;
  float* pad32 = c.buf<float>("pl.pad32", (size_t)m, s);
  double* ws = c.buf<double>("pl.iirws", filtfilt_ws_doubles(n, c.hp_order), s);
  check(filtfilt_pad(audio, n, c.hp_b.data(), c.hp_a.data(), c.hp_zi.data(), c.hp_FL.data(), c.hp_order, t_pad, ws,
                     nullptr, pad32, s),
        "filtfilt_pad");
  const int64_t F = 1 + m / 160;
  const int64_t p_len = m / 160;
  double* f0 = c.buf<double>("pl.f0", (size_t)F, s);
  rmvpe_forward(c, pad32, m, 0.03f, f0, F, nullptr, s);
  int32_t* pitch = c.buf<int32_t>("pl.pitch", (size_t)p_len, s);
  float* pitchf = c.buf<float>("pl.pitchf", (size_t)p_len, s);
  check(f0_post(f0, (int)p_len, std::pow(2.0, semitones / 12.0), pitch, pitchf, f0_out, s), "f0_post");
  // HuBERT -> upsample/protect -> synth
  const int E = c.scfg.emb_dim;
  const int64_t cap_rows = m / 320 + 8;
  float* feats = c.buf<float>("vc.feats", (size_t)cap_rows * E, s);
  const int64_t L = hubert_forward(c, pad32, m, 2, feats, cap_rows, s);
  const int T = (int)std::min<int64_t>(p_len, 2 * L);
  const int upp = c.scfg.upp();
  const int64_t nvc = (int64_t)T * upp;
  const int64_t nout = nvc - 2 * t_pad_tgt;
  if (nout <= 0) throw Error(RVCX_E_SHAPE, "pipeline: input too short for the padding");
  if (nout > cap) throw Error(RVCX_E_CAPACITY, "pipeline: output needs " + std::to_string(nout) + " samples");
  float* phone = c.buf<float>("vc.phone", (size_t)T * E, s);
  check(upsample2_protect(feats, (int)L, E, phone, T, protect < 0.5f ? pitchf : nullptr, protect, s), "upsample");
  int32_t* lens = c.buf<int32_t>("vc.len", 4, s);
  set_i32(lens, T, s);
  set_i32(lens + 1, sid, s);
  float* vc = c.buf<float>("pl.vc", (size_t)nvc, s);
  synth_forward(c, 1, T, phone, lens, pitch, pitchf, lens + 1, eps_z, eps_src, seed, vc, nullptr, nullptr, s);
  RVCX_HIP(hipMemcpyAsync(out, vc + t_pad_tgt, (size_t)nout * sizeof(float), hipMemcpyDeviceToDevice, s));
  unsigned* mx = c.buf<unsigned>("pl.max", 4, s);
  check(peak_normalize(out, nout, mx, s), "peak_normalize");
  return nout;
}

}  // namespace rvcx
