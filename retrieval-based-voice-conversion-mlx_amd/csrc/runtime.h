// rvcx runtime internals: context, weight store, workspace.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/rvcx.h"
#include "rvcx_kernels.h"

namespace rvcx {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define RVCX_HIP(expr)                                                                                 \
  do {                                                                                                 \
    hipError_t e_ = (expr);                                                                            \
    if (e_ != hipSuccess)                                                                              \
      throw ::rvcx::Error(RVCX_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_) + " at " +     \
                                          __FILE__ + ":" + std::to_string(__LINE__));                  \
  } while (0)

struct HostTensor {
  std::vector<float> v;
  std::vector<int64_t> shape;
  size_t numel() const { return v.size(); }
};

// Device buffer (owned).
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  bool borrowed = false;  // carved from the caller's workspace arena (rvcx_set_workspace): not freed here
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p && !borrowed) (void)hipFree(p);
  }
};

struct SynthCfg {
  int I = 192, H = 192, F = 768, n_heads = 2, n_layers = 6, ksize = 3;
  std::vector<int> rb_k{3, 7, 11};
  std::vector<std::vector<int>> rb_d{{1, 3, 5}, {1, 3, 5}, {1, 3, 5}};
  std::vector<int> ups{12, 10, 2, 2};
  int C0 = 512;
  std::vector<int> up_k{24, 20, 4, 4};
  int n_spk = 109, gin = 256, sr = 48000, emb_dim = 768;
  int window = 10, flow_k = 5, flow_layers = 3, flow_n = 4;
  bool f0 = true;   // pitch-guided (NSF decoders) or not (HiFiGANGenerator): synthesizers.py:84-139
  int vocoder = 0;  // 0 HiFi-GAN (NSF), 1 MRF HiFi-GAN, 2 RefineGAN (synthesizers.py:86-118)
  int upp() const {
    int u = 1;
    for (int x : ups) u *= x;
    return u;
  }
  // harmonics of the decoder's source: NSF 1 (harmonic_num 0), MRF 9 (synthesizers.py:95), RefineGAN 1
  int src_harmonics() const { return vocoder == 1 ? 9 : 1; }
  // floats of injected source noise per batch row of T frames (the decoder's randn_like / rand draws):
  // NSF [T*upp]; MRF / RefineGAN [T*upp][H] noise, the B x H initial phases of all rows follow the B rows
  long long src_noise_row(long long T) const { return f0 ? T * upp() * src_harmonics() : 0; }
  long long src_noise_tail() const { return (f0 && vocoder != 0) ? src_harmonics() : 0; }
  // every injected decoder draw of a B x T call (RefineGAN adds its AdaIN noise: runtime_refinegan.cpp)
  long long src_noise_total(int B, long long T) const;
};

// ConvTranspose1d lowered to a polyphase conv: input row for output q, tap t is q + t - pad.
struct UpsLayer {
  int cin = 0, cout = 0, u = 0, k = 0, taps = 0, pad = 0;
  float* w = nullptr;     // [taps][u*cout][cin]
  float* b = nullptr;     // [u*cout]
};

// FAISS IndexIVFFlat resident in HBM (index_ivf.cpp; layout in ivf.hip)
struct IvfIndex {
  IvfView view;
  DevBuf cent, vecs, off, ids, slot_of_id;
};

struct Ctx {
  int device = 0;
  std::string err;
  SynthCfg scfg;
  bool synth_cfg_set = false;
  std::map<std::string, HostTensor> host[4];  // synth, hubert, rmvpe, crepe
  std::map<std::string, std::unique_ptr<DevBuf>> dev;  // packed weights
  bool ready[4] = {false, false, false, false};
  std::vector<UpsLayer> ups;
  // pipeline high-pass (rvc/infer/pipeline.py:22-27), normalised so a[0] = 1
  int hp_order = 0;
  std::vector<double> hp_b, hp_a, hp_zi;
  // the same filter as second-order sections (rvcx_set_highpass_sos): chunk-parallel scan (iir_scan.hip)
  SosPlan hp_sos;
  DevBuf hp_sos_buf;
  // workspace pool
  std::map<std::string, std::unique_ptr<DevBuf>> ws;
  uint64_t call_counter = 0;
  // kernel timing (rvcx_profile): event pairs around every conv-GEMM launch, on its stream
  bool prof = false;
  int conv_math = 0;  // ConvArgs::math of every conv launch (rvcx_set_conv_math): 0 default, 1 fp32 MFMA, 2 split
  // the arithmetic a launch without ConvArgs::math gets: rvcx_set_conv_math, else RVCX_CONV_MATH
  int conv_math_default() const {
    ConvArgs a;
    a.math = conv_math;
    return conv_math_of(a);
  }
  static constexpr double PEAK_SPLIT = 2500.0 / 6.0, PEAK_F16X2 = 2500.0 / 3.0, PEAK_F16 = 2500.0;
  struct ProfRec {
    hipEvent_t a, b;
    double flops;
    int two_d, M, N, C_in, taps, batch, ksplit;  // shape, for RVCX_PROF_DUMP
    double bytes;  // algorithmic HBM bytes: operands read once, result written once (RVCX_PROF_DUMP)
    double peak_tf;  // the MFMA ceiling of the launch's arithmetic, algorithmic fp32 TFLOP/s
    int kind = CK_OTHER;  // the kernel family that ran (ConvKind)
  };
  std::vector<ProfRec> prof_recs;
  std::vector<hipEvent_t> prof_pool;
  std::unique_ptr<IvfIndex> ivf;  // speaker-embedding index (optional)
  // pre-split weight images of the weight-streamed conv kernel, per (weight, layout); an entry is dropped when its
  // weight tensor is re-packed (alloc_weight), so finalizing one model keeps the other models' images
  std::map<std::tuple<const void*, int, long long, int, int, int, int>, std::unique_ptr<DevBuf>> wsplit_cache;
  const void* wsplit_for(const ConvArgs& a, hipStream_t s);
  // pre-split images of the fused ResBlock pair kernel (resblock_fused.hip), per weight tensor
  std::map<std::pair<const void*, int>, std::unique_ptr<DevBuf>> rb_wsplit_cache;
  const void* rb_wsplit_for(const float* w, int C, int k, int wfmt, hipStream_t s);
  // set by the internal callers of synth_forward whose every row has the full length T (the pipeline, its batched form,
  // the streaming hop): the TextEncoder's attention then runs without the all-ones key mask (ScopedFullLengths)
  bool synth_full_lengths = false;
  // set while HuBERT's feature encoder is being issued (runtime_pipeline.cpp issue_front): the launches RVCX_AUX_LDS
  // throttles
  bool aux_front = false;
  // second stream for work independent of the caller's stream (HuBERT beside RMVPE), created lazily
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_gate = nullptr;
  hipStream_t aux_stream();
  // issued by RMVPE's E2E right before the BiGRU launch (host callback, cleared when taken)
  std::function<void(hipStream_t)> before_gru;
  // device-side fault flags in pinned host-mapped memory (bit 0: a BiGRU partner hand-off timed out).
  // Kernels store into it; the host reads it after a synchronisation: every compute entry point checks
  // it on entry (faults of earlier, completed calls), the pipeline at its own sync points, and
  // rvcx_device_status after synchronising the caller's stream.
  // buffers whose zero parts survive from call to call (the BiGRU hand-off tags, the NSF source's pad columns): zeroed
  // only when the buffer or its layout changes, not by a fill launch every call
  std::map<std::string, std::pair<const void*, long long>> zero_marks;
  // small device scalars written from the host (the synthesizer's length / speaker id): the launch is skipped when the
  // named buffer already holds the value (C2 writes the same two every call)
  std::map<std::string, std::pair<const void*, int32_t>> i32_marks;
  // returns true when it zeroed
  bool zero_once(const std::string& name, void* p, size_t bytes, long long layout, hipStream_t s) {
    auto& m = zero_marks[name];
    if (m.first == p && m.second == layout) return false;
    RVCX_HIP(hipMemsetAsync(p, 0, bytes, s));
    m = {p, layout};
    return true;
  }
  // the BiGRU hand-off tag counter of each zeroed xchg slice (gru_bidir), reset whenever the buffer is re-zeroed
  std::map<const void*, unsigned> gru_tags;
  unsigned* status_host = nullptr;
  unsigned* status_dev = nullptr;
  unsigned* device_status();
  void check_device_status();  // throws Error(RVCX_E_HIP, ...) and clears the flags when any is set
  ~Ctx();

  float* W(const std::string& name) const;
  // address ranges of the packed weights (alloc_weight): a contraction whose B operand lies in one is static
  std::map<uintptr_t, uintptr_t> wranges;
  bool is_weight(const void* p) const;
  // forget the split images cached for weights in [lo, hi) (a tensor replaced or an address reused)
  void drop_splits(uintptr_t lo, uintptr_t hi);
  float* alloc_weight(const std::string& name, const std::vector<float>& data);
  template <class T>
  T* buf(const std::string& name, size_t count, hipStream_t s);
  // caller-owned workspace arena (rvcx_set_workspace): the named pool is carved from it (256-B aligned, bump order)
  // instead of hipMalloc; a buffer that has to grow takes a new region; past the end a call fails with RVCX_E_OOM
  char* arena = nullptr;
  size_t arena_bytes = 0, arena_used = 0;
  size_t carved = 0;  // bytes the pool has taken since the last release (every region, regrown ones included)
  bool sizing_plan = false;  // rvcx_workspace_bytes: long inputs take the worst-case chunk plan (runtime_pipeline.cpp)
  // Call-to-call ordering: every compute entry point starts with begin_call(), which records an event on
  // each stream the previous call took pool buffers on; the first pool buffer a call takes on a stream makes that
  // stream wait for the previous call's events on OTHER streams. A call on stream B therefore never overwrites a
  // region (arena mode: the same offsets under other names; pool mode: the same named buffers) that a call still
  // running on stream A uses; calls on one stream stay ordered by the stream itself (no wait is issued).
  std::vector<hipStream_t> call_streams;                              // streams the current call took buffers on
  std::vector<std::pair<hipStream_t, hipEvent_t>> prev_call_events;  // the previous call's, recorded at begin_call
  std::map<hipStream_t, hipEvent_t> call_ev;                           // one reusable event per stream
  void begin_call() {
    prev_call_events.clear();
    for (hipStream_t st : call_streams) {
      hipEvent_t& e = call_ev[st];
      if (!e) RVCX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      RVCX_HIP(hipEventRecord(e, st));
      prev_call_events.emplace_back(st, e);
    }
    call_streams.clear();
    arena_rewind();
  }
  void touch_stream(hipStream_t s) {
    for (hipStream_t st : call_streams)
      if (st == s) return;
    call_streams.push_back(s);
    for (const auto& pe : prev_call_events)
      if (pe.first != s) RVCX_HIP(hipStreamWaitEvent(s, pe.second, 0));
  }
  // Arena mode: every API call carves its regions from offset 0 again (begin_call, before any work), so a call never
  // inherits the regions earlier calls regrew; reuse is ordered by the caller's stream and, across streams, by
  // begin_call's events. The marks describing buffer contents go with the regions (a caller that wrote into its arena
  // between calls cannot leave a stale zeroed buffer or memoised scalar behind).
  void arena_rewind() {
    if (!arena) return;
    ws.clear();
    zero_marks.clear();
    i32_marks.clear();
    gru_tags.clear();
    arena_used = 0;
    carved = 0;
  }
  // synchronise the device and drop the named pool, with the marks that describe its contents (zeroed buffers,
  // memoised scalars, BiGRU tag counters)
  void release_pool() {
    RVCX_HIP(hipDeviceSynchronize());
    ws.clear();
    zero_marks.clear();
    i32_marks.clear();
    gru_tags.clear();
    arena_used = 0;
    carved = 0;
  }
  size_t pool_bytes() const {
    size_t t = 0;
    for (const auto& kv : ws) t += kv.second ? kv.second->bytes : 0;
    return t;
  }
};

template <class T>
T* Ctx::buf(const std::string& name, size_t count, hipStream_t s) {
  size_t bytes = count * sizeof(T);
  if (bytes == 0) bytes = 16;
  bytes = (bytes + 255) & ~size_t(255);
  touch_stream(s);
  auto& slot = ws[name];
  if (!slot || slot->bytes < bytes) {
    if (slot && slot->p) RVCX_HIP(hipStreamSynchronize(s));
    slot.reset(new DevBuf());
    if (arena) {
      const size_t off = (arena_used + 255) & ~size_t(255);
      if (off + bytes > arena_bytes) {
        ws.erase(name);
        throw Error(RVCX_E_OOM, "workspace arena exhausted: " + name + " needs " + std::to_string(bytes) + " B at offset " +
                                    std::to_string(off) + " of " + std::to_string(arena_bytes));
      }
      slot->p = arena + off;
      slot->borrowed = true;
      arena_used = off + bytes;
    } else if (hipMalloc(&slot->p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      ws.erase(name);
      throw Error(RVCX_E_OOM, "workspace allocation failed: " + name + " (" + std::to_string(bytes) + " B)");
    }
    slot->bytes = bytes;
    carved += bytes;
  }
  return static_cast<T*>(slot->p);
}

// model forward passes (runtime_*.cpp)
void finalize_synth(Ctx& c);
void finalize_refinegan(Ctx& c);
long long refinegan_noise_floats(const SynthCfg& g, int B, long long T);
void refinegan_forward(Ctx& c, int B, int T, const float* z_btc, const float* mask, const float* f0, const float* g,
                       const float* eps_src, uint64_t seed, float* out, hipStream_t s);
void finalize_hubert(Ctx& c);
void finalize_rmvpe(Ctx& c);
void finalize_crepe(Ctx& c);
// librosa.effects.split of split_audio.process_audio (rvc/lib/tools/split_audio.py:5-27): intervals [cnt][2]
int64_t split_intervals(Ctx& c, const double* audio, int64_t n, int sr, double silence_thresh_db, int min_silence_ms,
                        int64_t* iv, int64_t cap, hipStream_t s);
// CREPE.get_f0 (rvc_mlx/lib/mlx/crepe.py:282-325) on audio [n] fp32: returns F = 1 + n/160
int64_t crepe_forward(Ctx& c, const float* audio, int64_t n, double f0_min, double f0_max, float thr, float* f0,
                      double* f0d, float* per, float* probs_out, hipStream_t s, int sem = 0,
                      const float* dither = nullptr);
int64_t hubert_forward(Ctx& c, const float* audio, int64_t n, int version, float* feats, int64_t cap,
                       hipStream_t s);
// HuBERT in three parts, so a caller can issue the encoder's last layers later on another stream:
// front end (feature convs, projection, positional conv, encoder LN), layers [l0, l1), tail (v1 projection)
constexpr int HUBERT_LAYERS = 12;
struct HubertRun {
  int B = 0, L = 0, version = 0;
  float* feats = nullptr;
};
HubertRun hubert_front(Ctx& c, const float* audio, int64_t n, int64_t lda, int B, int version, float* feats,
                       int64_t cap, hipStream_t s);
void hubert_layers(Ctx& c, const HubertRun& run, int l0, int l1, hipStream_t s);
int64_t hubert_tail(Ctx& c, const HubertRun& run, hipStream_t s);
int64_t rmvpe_forward(Ctx& c, const float* audio, int64_t n, float thred, double* f0, int64_t cap, float* hidden,
                      hipStream_t s);
// batched over B equal-length inputs (rows of stride lda); outputs back to back per sequence
int64_t hubert_forward_b(Ctx& c, const float* audio, int64_t n, int64_t lda, int B, int version, float* feats,
                         int64_t cap, hipStream_t s);
int64_t rmvpe_forward_b(Ctx& c, const float* audio, int64_t n, int64_t lda, int B, float thred, double* f0,
                        int64_t cap, float* hidden, hipStream_t s);
void synth_forward(Ctx& c, int B, int T, const float* phone, const int32_t* lengths, const int32_t* pitch,
                   const float* pitchf, const int32_t* sid, const float* eps_z, const float* eps_src, uint64_t seed,
                   float* out, float* zp_out, float* z_out, hipStream_t s, int gen_lowp = 0, int head = 0,
                   float* mp_out = nullptr, float* logsp_out = nullptr);
// head: Synthesizer.infer's rate (synthesizers.py:230-234) as the first kept frame -- the flow and the decoder run on
// T - head frames (out [B][(T - head) upp], zp_out / z_out [B][T - head][I]); mp_out / logsp_out [B][T][I]
// gen_lowp: the generator's weight-streamed convs and fused ResBlock pairs on fp16 operands (one MFMA product per
// step): the realtime hop's opt-in (rvcx_rt_opts::gen_precision), never set by an offline entry point
// noise_pre: the NSF source and the noise convs of the multi-tap stages were computed ahead by dec_noise_prepare (same
// B, T, f0, eps_src, seed), on a stream this one has joined since; the ConvTransposes add them as their residual
void dec_forward(Ctx& c, int B, int T, const float* z_btc, const float* mask, const float* f0, const float* g,
                 const float* eps_src, uint64_t seed, float* out, hipStream_t s, int gen_lowp = 0,
                 bool noise_pre = false);
// the NSF harmonic source (SineGen) and every multi-tap noise conv (hifigan_nsf.py:196-199) into their own buffers:
// the synthesizer issues it on the aux stream beside the TextEncoder and flow, which leave most of the GPU idle.
// Returns false (nothing issued) for configurations without the NSF noise branch.
bool dec_noise_prepare(Ctx& c, int B, int T, const float* f0, const float* eps_src, uint64_t seed, hipStream_t s);

void set_highpass(Ctx& c, const double* b, const double* a, const double* zi, int order);
void set_highpass_sos(Ctx& c, const double* sos, int nsec);
// filtfilt + reflect pad of one utterance with whichever high-pass form is configured
void highpass_pad(Ctx& c, const double* audio, int64_t n, int64_t t_pad, double* pad64, float* pad32, hipStream_t s);
int hubert_version_for(const Ctx& c);
// feats_pre (optional): HuBERT rows of this chunk computed ahead (e.g. on the aux stream), L_pre rows
int64_t vc_forward(Ctx& c, const float* audio, int64_t n, const int32_t* pitch, const float* pitchf,
                   int64_t pitch_len, int sid, float protect, double index_rate, const float* eps_z,
                   const float* eps_src, uint64_t seed, float* out, int64_t cap, hipStream_t s,
                   const float* feats_pre = nullptr, int64_t L_pre = 0);
// streaming (runtime_stream.cpp)
struct RtState;
RtState* rt_create(Ctx& c, const rvcx_rt_desc& d);
void rt_destroy(RtState* s);
void rt_geometry(const RtState& s, int64_t* g);
void rt_reset(Ctx& c, RtState& s, hipStream_t st);
void rt_process(Ctx& c, RtState& s, const float* in48, const int32_t* sids, const rvcx_rt_opts& o,
                const float* eps_z, const float* eps_src, uint64_t seed, float* out48, float* vol_out, int* offs_out,
                hipStream_t st);
// index (index_ivf.cpp)
struct ParsedIvf {  // a validated faiss IndexIVFFlat image on the host (lists in list order)
  int d = 0, nprobe = 1;
  long long nlist = 0, ntotal = 0;
  std::vector<float> cent, vecs;
  std::vector<long long> off, ids;
  std::vector<int> slot;  // id -> slot
};
ParsedIvf parse_ivf(const uint8_t* bytes, int64_t nbytes);  // host only; throws Error(RVCX_E_INVALID)
void index_load(Ctx& c, const uint8_t* bytes, int64_t nbytes);
void index_search(Ctx& c, const float* x, int64_t n, int k, float* dist, int64_t* ids, hipStream_t s);
void index_retrieve(Ctx& c, const float* feats, int64_t L, int d, double index_rate, float* out, hipStream_t s);
void index_reconstruct_n(Ctx& c, int64_t i0, int64_t ni, float* out, hipStream_t s);
int64_t pipeline_forward_ex(Ctx& c, const double* audio, int64_t n, const rvcx_pipeline_opts& o,
                            const float* eps_z, const float* eps_src, uint64_t seed, float* out, int64_t cap,
                            double* f0_out, hipStream_t s);
int64_t pipeline_forward_batch(Ctx& c, const double* audio, int64_t n, int64_t lda, int B, const rvcx_pipeline_opts& o,
                               const int32_t* sids, const float* eps_z, const float* eps_src, uint64_t seed,
                               float* out, int64_t ldo, double* f0_out, float* hidden_out, hipStream_t s);
rvcx_pipeline_opts default_pipeline_opts();
int proposed_key(const std::vector<double>& f0, double threshold);
int64_t hubert_frames(int64_t n);  // HuBERT output rows for n samples (0 when too short)
void set_i32(int32_t* p, int32_t v, hipStream_t s);
void set_i32_once(Ctx& c, const std::string& name, int32_t* p, int32_t v, hipStream_t s);
// Overlap of independent stages: fork_aux returns the aux stream, ordered after everything queued on s so
// far (or s itself when overlap is off: kernel timing on, or RVCX_NO_OVERLAP=1); join_aux makes s wait for
// everything queued on the aux stream so far.
hipStream_t fork_aux(Ctx& c, hipStream_t s);
// whether launch_conv would run this 1-D contraction on the weight-streamed fp16 kernel without split-K (the kernels
// whose epilogue takes the fused NSF noise conv, ConvArgs::nz_*)
bool conv_routes_wsb16(Ctx& c, const ConvArgs& a);
// marks a synth_forward call whose rows all have the full length T (Ctx::synth_full_lengths) for its lifetime
struct ScopedFullLengths {
  Ctx& c;
  explicit ScopedFullLengths(Ctx& cc) : c(cc) { c.synth_full_lengths = true; }
  ~ScopedFullLengths() { c.synth_full_lengths = false; }
};
void join_aux(Ctx& c, hipStream_t s, hipStream_t ax);
// launch one implicit-GEMM conv (1-D or 2-D) with optional event timing; flops = algorithmic FLOPs
void launch_conv(Ctx& c, const ConvArgs& a_in, bool two_d, hipStream_t s, double flops = -1.0);
// one fused ResBlock pair (resblock_fused.hip) with optional event timing (counted with the conv family)
void launch_rb_pair(Ctx& c, const RbPairArgs& a, hipStream_t s);
inline void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error(RVCX_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace rvcx
