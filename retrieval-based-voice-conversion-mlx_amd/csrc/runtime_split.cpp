// split_audio (rvc/lib/tools/split_audio.py:5-27, used by rvc/infer/infer.py:282-316): librosa.effects.split
// of the 16 kHz input into non-silent intervals. The frame RMS runs on device (k_rms_frames_f64); the interval
// edges over the few hundred frames are host control logic, as in librosa (effects.py split /
// _signal_to_frame_nonsilent): db = 10 log10(max(1e-10, rms^2)) - 10 log10(max(1e-10, max rms^2)) > -top_db,
// edges where that flips, frames -> samples (x hop), clipped to n.
#include <cmath>

#include "runtime.h"

namespace rvcx {

int64_t split_intervals(Ctx& c, const double* audio, int64_t n, int sr, double silence_thresh_db, int min_silence_ms,
                        int64_t* iv, int64_t cap, hipStream_t s) {
  const int frame = (int)((double)min_silence_ms / 1000.0 * sr);  // int(min_silence_len / 1000 * sr)
  const int hop = frame / 2;
  if (frame < 2 || hop < 1 || n <= 0) throw Error(RVCX_E_INVALID, "split_audio: frame length below 2 samples");
  const int64_t nf = 1 + (n + 2 * (frame / 2) - frame) / hop;
  double* d = c.buf<double>("split.rms", (size_t)nf, s);
  check(rms_frames_f64(audio, n, frame, hop, d, (int)nf, s), "rms_frames_f64");
  std::vector<double> rms((size_t)nf);
  RVCX_HIP(hipMemcpyAsync(rms.data(), d, sizeof(double) * nf, hipMemcpyDeviceToHost, s));
  RVCX_HIP(hipStreamSynchronize(s));
  std::vector<double> mse((size_t)nf);
  double ref = 0.0;
  for (int64_t i = 0; i < nf; ++i) {
    mse[i] = rms[i] * rms[i];
    ref = std::max(ref, mse[i]);
  }
  const double top_db = -silence_thresh_db;
  const double ref_db = 10.0 * std::log10(std::max(1e-10, ref));
  std::vector<char> on((size_t)nf);
  for (int64_t i = 0; i < nf; ++i) on[i] = (10.0 * std::log10(std::max(1e-10, mse[i])) - ref_db) > -top_db;
  std::vector<int64_t> edges;
  if (on[0]) edges.push_back(0);
  for (int64_t i = 0; i + 1 < nf; ++i)
    if (on[i] != on[i + 1]) edges.push_back(i + 1);
  if (on[nf - 1]) edges.push_back(nf);
  const int64_t cnt = (int64_t)edges.size() / 2;
  if (cnt > cap) throw Error(RVCX_E_CAPACITY, "split_audio: more intervals than the output holds");
  for (int64_t i = 0; i < cnt; ++i) {
    iv[2 * i] = std::min<int64_t>(edges[2 * i] * hop, n);
    iv[2 * i + 1] = std::min<int64_t>(edges[2 * i + 1] * hop, n);
  }
  return cnt;
}

}  // namespace rvcx
