// extern "C" boundary (include/rvcx.h). Every entry point converts C++ exceptions into an
// rvcx_status and stores the message for rvcx_last_error.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unistd.h>
#include <vector>

#include "runtime.h"

extern char** environ;

using namespace rvcx;

namespace rvcx {
// read at every knob read (not cached): most knobs are read once into a static at their first use, the BiGRU's
// fault-injection hook (RVCX_GRU_SPIN_LIMIT) per call, so a test can set and clear it with the opt-in
static bool experimental_on() {
  const char* e = std::getenv("RVCX_EXPERIMENTAL");
  return e && std::atoi(e) == 1;
}
const char* rvcx_knob(const char* name) { return experimental_on() ? std::getenv(name) : nullptr; }
}  // namespace rvcx

struct rvcx_ctx : public Ctx {};
struct rvcx_rt {
  RtState* s = nullptr;
};

namespace {

template <class F>
int guard(rvcx_ctx* c, F&& f) {
  if (!c) return RVCX_E_INVALID;
  try {
    c->err.clear();
    f();
    return RVCX_OK;
  } catch (const Error& e) {
    c->err = e.what();
    return e.code;
  } catch (const std::exception& e) {
    c->err = e.what();
    return RVCX_E_INVALID;
  }
}

// every compute entry point: select the device and report device-side faults of earlier, completed calls
void set_device(rvcx_ctx* c) {
  RVCX_HIP(hipSetDevice(c->device));
  c->check_device_status();
  c->begin_call();
}

}  // namespace

namespace rvcx {
hipStream_t Ctx::aux_stream() {
  if (!aux) {
    RVCX_HIP(hipSetDevice(device));
    // (the aux stream at the device's least priority measured neutral: 18.22 vs 18.19 ms, round 3)
    RVCX_HIP(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
    RVCX_HIP(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
    RVCX_HIP(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
    RVCX_HIP(hipEventCreateWithFlags(&ev_gate, hipEventDisableTiming));
  }
  return aux;
}

unsigned* Ctx::device_status() {
  if (!status_host) {
    RVCX_HIP(hipSetDevice(device));
    void* h = nullptr;
    RVCX_HIP(hipHostMalloc(&h, 64, hipHostMallocMapped));
    std::memset(h, 0, 64);
    status_host = static_cast<unsigned*>(h);
    void* d = nullptr;
    RVCX_HIP(hipHostGetDevicePointer(&d, h, 0));
    status_dev = static_cast<unsigned*>(d);
  }
  return status_dev;
}

void Ctx::check_device_status() {
  if (!status_host) return;
  const unsigned v = __atomic_load_n(status_host, __ATOMIC_ACQUIRE);
  if (v == 0) return;
  __atomic_store_n(status_host, 0u, __ATOMIC_RELEASE);
  std::string what;
  if (v & 1u) what += "gru: partner hand-off timed out (the RMVPE BiGRU's workgroups were not co-resident); ";
  throw Error(RVCX_E_HIP, what + "the outputs of the call that raised this flag are invalid");
}

Ctx::~Ctx() {
  if (status_host) (void)hipHostFree(status_host);
  for (auto& kv : call_ev)
    if (kv.second) (void)hipEventDestroy(kv.second);
  if (aux) {
    (void)hipStreamSynchronize(aux);
    (void)hipEventDestroy(ev_fork);
    (void)hipEventDestroy(ev_join);
    (void)hipEventDestroy(ev_gate);
    (void)hipStreamDestroy(aux);
  }
}

hipStream_t fork_aux(Ctx& c, hipStream_t s) {
  static const bool no_overlap = [] {
    const char* e = rvcx_knob("RVCX_NO_OVERLAP");
    return e && std::atoi(e) != 0;
  }();
  if (c.prof || no_overlap) return s;
  hipStream_t ax = c.aux_stream();
  RVCX_HIP(hipEventRecord(c.ev_fork, s));
  RVCX_HIP(hipStreamWaitEvent(ax, c.ev_fork, 0));
  return ax;
}

void join_aux(Ctx& c, hipStream_t s, hipStream_t ax) {
  if (ax == s) return;
  RVCX_HIP(hipEventRecord(c.ev_join, ax));
  RVCX_HIP(hipStreamWaitEvent(s, c.ev_join, 0));
}

// the weight tensor's pre-split image (built once on first use; the stream then synchronises so a later use on
// another stream never races the build)
const void* Ctx::wsplit_for(const ConvArgs& a, hipStream_t s) {
  const auto key = std::make_tuple(static_cast<const void*>(a.w), a.ldw, a.w_ts, a.N, a.C_in, a.taps, a.wsplit_fmt);
  auto& slot = wsplit_cache[key];
  if (!slot) {
    std::unique_ptr<DevBuf> b(new DevBuf());
    const size_t bytes = (size_t)conv_wsplit_bytes(a);
    if (hipMalloc(&b->p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      throw Error(RVCX_E_OOM, "split-weight allocation failed");
    }
    b->bytes = bytes;
    check(conv_wsplit_build(a, b->p, s), "conv_wsplit_build");
    RVCX_HIP(hipStreamSynchronize(s));
    slot = std::move(b);
  }
  return slot->p;
}

const void* Ctx::rb_wsplit_for(const float* w, int C, int k, int wfmt, hipStream_t s) {
  auto& slot = rb_wsplit_cache[{static_cast<const void*>(w), wfmt}];
  if (!slot) {
    std::unique_ptr<DevBuf> b(new DevBuf());
    const size_t bytes = (size_t)rb_wsplit_bytes(C, k, wfmt);
    if (hipMalloc(&b->p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      throw Error(RVCX_E_OOM, "split-weight allocation failed");
    }
    b->bytes = bytes;
    check(rb_wsplit_build(w, C, k, b->p, s, wfmt), "rb_wsplit_build");
    RVCX_HIP(hipStreamSynchronize(s));
    slot = std::move(b);
  }
  return slot->p;
}

void launch_rb_pair(Ctx& c, const RbPairArgs& a, hipStream_t s) {
  constexpr int cfg = 0;
  if (!c.prof) {
    check(rb_pair(a, cfg, s), "rb_pair");
    return;
  }
  hipEvent_t ev[2];
  for (auto& e : ev) {
    if (!c.prof_pool.empty()) {
      e = c.prof_pool.back();
      c.prof_pool.pop_back();
    } else {
      RVCX_HIP(hipEventCreate(&e));
    }
  }
  // algorithmic work: the two convs over the valid rows
  const double flops = 2.0 * 2.0 * a.B * (double)a.T * a.C * a.C * a.k;
  // x read, y written (+ read when accumulating), both weight tensors
  const double bytes = 4.0 * ((double)a.B * a.T * a.C * (2 + (a.acc_mode != ACC_STORE ? 1 : 0)) + 2.0 * a.k * a.C * a.C);
  Ctx::ProfRec r{ev[0], ev[1], flops, 0, a.T, a.C, a.C, -a.k, a.B, 1, bytes,
                 a.wfmt == RB_WF16 ? (a.lowp ? Ctx::PEAK_F16 : Ctx::PEAK_F16X2) : Ctx::PEAK_SPLIT};
  r.kind = CK_RBPAIR;
  RVCX_HIP(hipEventRecord(r.a, s));
  check(rb_pair(a, cfg, s), "rb_pair");
  RVCX_HIP(hipEventRecord(r.b, s));
  c.prof_recs.push_back(r);
}

bool conv_routes_wsb16(Ctx& c, const ConvArgs& a_in) {
  ConvArgs b = a_in;
  if (c.conv_math > 0 && b.math == 0) b.math = c.conv_math;
  if (!(b.w_static || c.is_weight(b.w)) || b.force_cfg >= 0) return false;
  if (!(conv_math_of(b) == 3 || b.lowp)) return false;  // the fp16 image (launch_conv below)
  if (conv_wsb_route(b, false) != 1) return false;
  b.wsb = 1;
  return conv_plan_splitk(b, false) == 0 && conv_wsb_pick(b) >= 23;
}

void launch_conv(Ctx& c, const ConvArgs& a_in, bool two_d, hipStream_t s, double flops) {
  ConvArgs a = a_in;
  if (c.conv_math > 0 && a.math == 0) a.math = c.conv_math;
  // weight-streamed kernel: forced (numerics tests / benchmarks: force_cfg >= 20 on a w_static weight) or routed by
  // the policy for a packed (static) weight; decided before the split-K plan, whose geometry depends on it
  const bool stat = a.w_static || c.is_weight(a.w);
  a.wsb = !stat ? 0
          : (a.force_cfg >= 30 && a.force_cfg < 40 ? 2
             : (a.force_cfg >= 20 && !two_d) ? 1 : (a.force_cfg < 0 ? conv_wsb_route(a, two_d) : 0));
  if (a.force_cfg == 40 && !two_d && stat) a.wsb = 1;  // the weight-stationary kernel (conv_wst.hip), forced
  const long long need = conv_plan_splitk(a, two_d);
  // the few-channel 3x3 convs' fp16-split form reads a pre-split image (conv2d_small.hip)
  if (two_d && !a.wsb && stat && !a.wsplit && conv_math_of(a) == 3 && conv2d_small_fits(a)) {
    a.wsplit_fmt = WSPLIT_S2D;
    a.wsplit = c.wsplit_for(a, s);
  }
  if (a.wsb) {
    // the weight-streamed kernel's fp16 image: the two-plane fp16 arithmetic (math 3) or the reduced-precision mode
    if (!a.wsplit)
      a.wsplit_fmt = ((a.wsb == 1 && a.lowp) || conv_math_of(a) == 3) ? WSPLIT_H16 : WSPLIT_BF16;
    if (!a.wsplit) a.wsplit = c.wsplit_for(a, s);  // a caller-built image (rvcx_conv1d) is used as given
    a.wsplit_npad = conv_wsplit_npad(a.N);
  }
  // split-K slabs are per stream: the aux stream's convs run concurrently with the caller's
  // HuBERT's feature-encoder contractions (issued on the aux stream beside the U-Net, with ~1.5 ms of slack before the
  // BiGRU) take 64 KB more LDS per workgroup: one or two of them per CU at most, so the U-Net's latency-bound chain
  // finds free workgroup slots instead of waiting out ~50 us feature-conv workgroups. Same-box A/B (ms/step): r05ac
  // none 13.53 / 13.47, 64 KB 13.28 / 13.35, 88 KB 13.25 / 13.27, 40 KB 13.39 / 13.51; r05ae none 13.53 / 13.54 /
  // 13.48 / 13.51, 64 KB 13.39 / 13.16 / 13.37 / 13.33, 88 KB 13.48 / 13.29. Throttling HuBERT's transformer too
  // (r05aa) costs +0.3-0.5 ms: it runs beside the BiGRU with little slack. RVCX_AUX_LDS=KB overrides (0: off)
  static const int aux_lds = [] {
    const char* e = rvcx_knob("RVCX_AUX_LDS");
    return e ? std::max(0, std::atoi(e)) : 64;
  }();
  if (aux_lds > 0 && c.aux_front) a.lds_pad = aux_lds * 1024;
  if (need > 0) {
    a.ws = c.buf<float>(c.aux && s == c.aux ? "conv.splitk.aux" : "conv.splitk", (size_t)need, s);
  }
  if (flops < 0) {
    const double M = two_d ? (double)a.T_out * a.W_out : (double)a.T_out;
    flops = 2.0 * M * a.N * (double)a.C_in * a.taps * a.batch * a.batch_inner;
  }
  if (!c.prof) {
    check(two_d ? conv2d(a, s) : conv1d(a, s), two_d ? "conv2d" : "conv1d");
    return;
  }
  auto get_ev = [&]() {
    hipEvent_t e;
    if (!c.prof_pool.empty()) {
      e = c.prof_pool.back();
      c.prof_pool.pop_back();
    } else {
      RVCX_HIP(hipEventCreate(&e));
    }
    return e;
  };
  // input rows read once, weights once, output written once (+ read again for a residual / accumulate)
  const double in_rows = two_d ? (double)a.T_in * a.W_in : (double)a.T_in;
  const double out_el = (two_d ? (double)a.T_out * a.W_out : (double)a.T_out) * a.N * a.batch * a.batch_inner;
  const double alg_bytes = 4.0 * (in_rows * a.C_in * a.batch * a.batch_inner + (double)a.taps * a.N * a.C_in +
                                  out_el * (1 + (a.res && a.res_mode != RES_NONE ? 1 : 0) +
                                            (a.acc_mode != ACC_STORE ? 1 : 0)));
  // the launch's arithmetic ceiling (the rest of the family is priced at the bf16 split's, a lower bound for the few
  // launches on the fp32-input MFMA)
  const double peak = (a.wsb && a.wsplit_fmt == WSPLIT_H16) ? ((a.lowp && a.wsb == 1) ? Ctx::PEAK_F16 : Ctx::PEAK_F16X2)
                      : (a.wsplit && a.wsplit_fmt == WSPLIT_S2D) ? Ctx::PEAK_F16X2
                                                                  : Ctx::PEAK_SPLIT;
  Ctx::ProfRec r{get_ev(), get_ev(), flops, two_d ? 1 : 0, two_d ? a.T_out * a.W_out : a.T_out, a.N, a.C_in,
                 a.taps, a.batch * a.batch_inner, a.ksplit, alg_bytes, peak};
  RVCX_HIP(hipEventRecord(r.a, s));
  check(two_d ? conv2d(a, s) : conv1d(a, s), two_d ? "conv2d" : "conv1d");
  r.kind = conv_last_kind();
  RVCX_HIP(hipEventRecord(r.b, s));
  c.prof_recs.push_back(r);
}

__global__ void k_set_i32(int32_t* p, int32_t v) { p[0] = v; }
void set_i32(int32_t* p, int32_t v, hipStream_t s) {
  hipLaunchKernelGGL(k_set_i32, dim3(1), dim3(1), 0, s, p, v);
  check(hipGetLastError(), "set_i32");
}
void set_i32_once(Ctx& c, const std::string& name, int32_t* p, int32_t v, hipStream_t s) {
  auto it = c.i32_marks.find(name);
  if (it != c.i32_marks.end() && it->second.first == p && it->second.second == v) return;
  set_i32(p, v, s);
  c.i32_marks[name] = {p, v};
}
}  // namespace rvcx

extern "C" {

int rvcx_create(rvcx_ctx** out, int device) {
  if (!out) return RVCX_E_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return RVCX_E_HIP;
  auto* c = new rvcx_ctx();
  c->device = device;
  *out = c;
  return RVCX_OK;
}

int rvcx_destroy(rvcx_ctx* ctx) {
  if (!ctx) return RVCX_E_INVALID;
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();
  delete ctx;
  return RVCX_OK;
}

const char* rvcx_last_error(const rvcx_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int rvcx_set_synth_config(rvcx_ctx* ctx, const rvcx_synth_desc* d) {
  return guard(ctx, [&] {
    if (!d) throw Error(RVCX_E_INVALID, "null desc");
    SynthCfg g;
    g.I = d->inter_channels;
    g.H = d->hidden_channels;
    g.F = d->filter_channels;
    g.n_heads = d->n_heads;
    g.n_layers = d->n_layers;
    g.ksize = d->kernel_size;
    if (d->n_resblocks < 1 || d->n_resblocks > 4 || d->n_dilations < 1 || d->n_dilations > 4)
      throw Error(RVCX_E_INVALID, "resblock config out of range");
    g.rb_k.assign(d->resblock_kernel_sizes, d->resblock_kernel_sizes + d->n_resblocks);
    g.rb_d.clear();
    for (int j = 0; j < d->n_resblocks; ++j)
      g.rb_d.emplace_back(d->resblock_dilation_sizes[j], d->resblock_dilation_sizes[j] + d->n_dilations);
    if (d->n_upsample < 1 || d->n_upsample > 8) throw Error(RVCX_E_INVALID, "n_upsample out of range");
    g.ups.assign(d->upsample_rates, d->upsample_rates + d->n_upsample);
    g.up_k.assign(d->upsample_kernel_sizes, d->upsample_kernel_sizes + d->n_upsample);
    g.C0 = d->upsample_initial_channel;
    g.n_spk = d->spk_embed_dim;
    g.gin = d->gin_channels;
    g.sr = d->sr;
    g.emb_dim = d->text_enc_hidden_dim;
    g.f0 = d->no_f0 == 0;
    g.vocoder = d->vocoder;
    if (g.vocoder < 0 || g.vocoder > 2) throw Error(RVCX_E_INVALID, "unsupported vocoder id");
    if (!g.f0 && g.vocoder != 0)
      throw Error(RVCX_E_INVALID, "models without pitch guidance use the HiFi-GAN decoder only (synthesizers.py:119-139)");
    if (g.H % g.n_heads || g.I % 2 || g.C0 % (1 << g.ups.size()))
      throw Error(RVCX_E_INVALID, "inconsistent synthesizer dimensions");
    ctx->scfg = g;
    ctx->synth_cfg_set = true;
    ctx->ready[0] = false;
  });
}

int rvcx_upload(rvcx_ctx* ctx, int model, const char* name, const float* host, const int64_t* shape, int ndim) {
  return guard(ctx, [&] {
    if (model < 0 || model > 3 || !name || !host || (ndim > 0 && !shape) || ndim < 0 || ndim > 8)
      throw Error(RVCX_E_INVALID, "rvcx_upload: bad arguments");
    HostTensor t;
    size_t n = 1;
    for (int i = 0; i < ndim; ++i) {
      if (shape[i] < 0) throw Error(RVCX_E_INVALID, "negative dim");
      t.shape.push_back(shape[i]);
      n *= (size_t)shape[i];
    }
    t.v.assign(host, host + n);
    ctx->host[model][name] = std::move(t);
    ctx->ready[model] = false;
  });
}

int rvcx_finalize(rvcx_ctx* ctx, int model) {
  return guard(ctx, [&] {
    set_device(ctx);
    if (model == RVCX_MODEL_SYNTH) {
      finalize_synth(*ctx);
    } else if (model == RVCX_MODEL_HUBERT) {
      finalize_hubert(*ctx);
    } else if (model == RVCX_MODEL_RMVPE) {
      finalize_rmvpe(*ctx);
    } else if (model == RVCX_MODEL_CREPE) {
      finalize_crepe(*ctx);
    } else {
      throw Error(RVCX_E_INVALID, "unknown model");
    }
    RVCX_HIP(hipDeviceSynchronize());
    ctx->ready[model] = true;
  });
}

int rvcx_synth_upp(const rvcx_ctx* ctx) { return ctx ? ctx->scfg.upp() : 0; }

int rvcx_hubert(rvcx_ctx* ctx, const float* d_audio, int64_t n, int version, float* d_feats, int64_t cap_rows,
                int64_t* rows_out, void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[1]) throw Error(RVCX_E_STATE, "hubert weights not finalized");
    if (!d_audio || !d_feats || n <= 0) throw Error(RVCX_E_INVALID, "rvcx_hubert: bad arguments");
    set_device(ctx);
    const int64_t L = hubert_forward(*ctx, d_audio, n, version == 1 ? 1 : 2, d_feats, cap_rows,
                                     static_cast<hipStream_t>(stream));
    if (rows_out) *rows_out = L;
  });
}

int rvcx_rmvpe(rvcx_ctx* ctx, const float* d_audio, int64_t n, float thred, double* d_f0, int64_t cap_frames,
               int64_t* frames_out, float* d_hidden, void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[2]) throw Error(RVCX_E_STATE, "rmvpe weights not finalized");
    if (!d_audio || !d_f0 || n <= 0) throw Error(RVCX_E_INVALID, "rvcx_rmvpe: bad arguments");
    set_device(ctx);
    const int64_t F = rmvpe_forward(*ctx, d_audio, n, thred, d_f0, cap_frames, d_hidden,
                                    static_cast<hipStream_t>(stream));
    if (frames_out) *frames_out = F;
  });
}

int rvcx_crepe(rvcx_ctx* ctx, const float* d_audio, int64_t n, float f0_min, float f0_max, float threshold,
               float* d_f0, float* d_periodicity, float* d_probs, int64_t cap_frames, int64_t* frames_out,
               void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[RVCX_MODEL_CREPE]) throw Error(RVCX_E_STATE, "crepe weights not finalized");
    if (!d_audio || !d_f0 || n <= 0) throw Error(RVCX_E_INVALID, "rvcx_crepe: bad arguments");
    if (cap_frames < 1 + n / 160) throw Error(RVCX_E_SHAPE, "rvcx_crepe: output capacity below 1 + n/160 frames");
    set_device(ctx);
    const int64_t F = crepe_forward(*ctx, d_audio, n, f0_min, f0_max, threshold, d_f0, nullptr, d_periodicity,
                                    d_probs, static_cast<hipStream_t>(stream));
    if (frames_out) *frames_out = F;
  });
}

int rvcx_crepe_ex(rvcx_ctx* ctx, const float* d_audio, int64_t n, float f0_min, float f0_max, float threshold,
                  int semantics, const float* d_dither, float* d_f0, float* d_periodicity, float* d_probs,
                  int64_t cap_frames, int64_t* frames_out, void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[RVCX_MODEL_CREPE]) throw Error(RVCX_E_STATE, "crepe weights not finalized");
    if (!d_audio || !d_f0 || n <= 0 || semantics < 0 || semantics > 1 || (d_dither && semantics != 1))
      throw Error(RVCX_E_INVALID, "rvcx_crepe_ex: bad arguments");
    if (cap_frames < 1 + n / 160) throw Error(RVCX_E_SHAPE, "rvcx_crepe_ex: output capacity below 1 + n/160 frames");
    set_device(ctx);
    const int64_t F = crepe_forward(*ctx, d_audio, n, f0_min, f0_max, threshold, d_f0, nullptr, d_periodicity, d_probs,
                                    static_cast<hipStream_t>(stream), semantics, d_dither);
    if (frames_out) *frames_out = F;
  });
}

int rvcx_crepe_decode(rvcx_ctx* ctx, const float* d_probs, int64_t F, float f0_min, float f0_max, float threshold,
                      int semantics, const float* d_dither, float* d_f0, float* d_periodicity, void* stream) {
  return guard(ctx, [&] {
    if (!d_probs || !d_f0 || F <= 0 || F > INT32_MAX / 360 || semantics < 0 || semantics > 1 ||
        (d_dither && semantics != 1) || !(f0_min > 0.f) || !(f0_max >= f0_min))
      throw Error(RVCX_E_INVALID, "rvcx_crepe_decode: bad arguments");
    set_device(ctx);
    const hipStream_t s = static_cast<hipStream_t>(stream);
    float* f0r = ctx->buf<float>("cr.f0raw", (size_t)F, s);
    float* pr = ctx->buf<float>("cr.perraw", (size_t)F, s);
    const double off = 1997.3794084376191;
    if (semantics == 1) {
      const int minidx = (int)std::min(360.0, std::max(0.0, std::floor((1200.0 * std::log2(f0_min / 10.0) - off) / 20.0)));
      const int maxidx = (int)std::min(360.0, std::max(0.0, std::ceil((1200.0 * std::log2(f0_max / 10.0) - off) / 20.0)));
      if (minidx >= maxidx) throw Error(RVCX_E_INVALID, "rvcx_crepe_decode: [f0_min, f0_max] covers no pitch bin");
      float* lp = ctx->buf<float>("cr.lp", (size_t)F * 360, s);
      int* ptr = ctx->buf<int>("cr.ptr", (size_t)F * 360, s);
      int* bins = ctx->buf<int>("cr.bins", (size_t)F, s);
      check(crepe_decode_viterbi(d_probs, (int)F, minidx, maxidx, d_dither, threshold, lp, ptr, bins, f0r, pr, d_f0,
                                 nullptr, d_periodicity, s), "crepe_decode_viterbi");
    } else {
      check(crepe_decode(d_probs, (int)F, 1200.0 * std::log2(f0_min / 10.0), 1200.0 * std::log2(f0_max / 10.0),
                         threshold, f0r, pr, d_f0, nullptr, d_periodicity, s), "crepe_decode");
    }
  });
}

int rvcx_split_audio(rvcx_ctx* ctx, const double* d_audio, int64_t n, int sr, double silence_thresh_db,
                     int min_silence_len_ms, int64_t* intervals, int64_t cap, int64_t* count, void* stream) {
  return guard(ctx, [&] {
    if (!d_audio || !intervals || n <= 0 || sr <= 0 || cap < 0 || !count)
      throw Error(RVCX_E_INVALID, "rvcx_split_audio: bad arguments");
    set_device(ctx);
    *count = split_intervals(*ctx, d_audio, n, sr, silence_thresh_db, min_silence_len_ms, intervals, cap,
                             static_cast<hipStream_t>(stream));
  });
}

int rvcx_hubert_batch(rvcx_ctx* ctx, const float* d_audio, int64_t n, int64_t lda, int B, int version, float* d_feats,
                      int64_t cap_rows, int64_t* rows_out, void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[1]) throw Error(RVCX_E_STATE, "hubert weights not finalized");
    if (!d_audio || !d_feats || n <= 0 || B < 1 || lda < n) throw Error(RVCX_E_INVALID, "rvcx_hubert_batch: bad arguments");
    set_device(ctx);
    const int64_t L = hubert_forward_b(*ctx, d_audio, n, lda, B, version == 1 ? 1 : 2, d_feats, cap_rows,
                                       static_cast<hipStream_t>(stream));
    if (rows_out) *rows_out = L;
  });
}

int rvcx_rmvpe_batch(rvcx_ctx* ctx, const float* d_audio, int64_t n, int64_t lda, int B, float thred, double* d_f0,
                     int64_t cap_frames, int64_t* frames_out, float* d_hidden, void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[2]) throw Error(RVCX_E_STATE, "rmvpe weights not finalized");
    if (!d_audio || !d_f0 || n <= 0 || B < 1 || lda < n) throw Error(RVCX_E_INVALID, "rvcx_rmvpe_batch: bad arguments");
    set_device(ctx);
    const int64_t F = rmvpe_forward_b(*ctx, d_audio, n, lda, B, thred, d_f0, cap_frames, d_hidden,
                                      static_cast<hipStream_t>(stream));
    if (frames_out) *frames_out = F;
  });
}

int rvcx_rmvpe_decode(rvcx_ctx* ctx, const float* d_hidden, int64_t F, float thred, double* d_f0, void* stream) {
  return guard(ctx, [&] {
    if (!d_hidden || !d_f0 || F < 0) throw Error(RVCX_E_INVALID, "rvcx_rmvpe_decode: bad arguments");
    if (F == 0) return;
    set_device(ctx);
    check(rmvpe_decode(d_hidden, (int)F, 360, thred, d_f0, static_cast<hipStream_t>(stream)), "rmvpe_decode");
  });
}

int rvcx_f0_post(rvcx_ctx* ctx, const double* d_f0, int64_t F, double semitones, int32_t* d_coarse, float* d_pitchf,
                 double* d_f0_shifted, void* stream) {
  return guard(ctx, [&] {
    if (!d_f0 || !d_coarse || !d_pitchf || F < 0) throw Error(RVCX_E_INVALID, "rvcx_f0_post: bad arguments");
    set_device(ctx);
    check(f0_post(d_f0, (int)F, std::pow(2.0, semitones / 12.0), d_coarse, d_pitchf, d_f0_shifted,
                  static_cast<hipStream_t>(stream)),
          "f0_post");
  });
}

int rvcx_f0_autotune(rvcx_ctx* ctx, double* d_f0, int64_t F, double strength, int skip_unvoiced, void* stream) {
  return guard(ctx, [&] {
    if (!d_f0 || F < 0) throw Error(RVCX_E_INVALID, "rvcx_f0_autotune: bad arguments");
    if (F == 0) return;
    set_device(ctx);
    check(f0_autotune(d_f0, (int)F, strength, skip_unvoiced, static_cast<hipStream_t>(stream)), "f0_autotune");
  });
}

int rvcx_synth_infer(rvcx_ctx* ctx, int B, int T, const float* d_phone, const int32_t* d_lengths,
                     const int32_t* d_pitch, const float* d_pitchf, const int32_t* d_sid, const float* d_eps_z,
                     const float* d_eps_src, uint64_t seed, float* d_out, float* d_zp, float* d_z, void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[0]) throw Error(RVCX_E_STATE, "synthesizer weights not finalized");
    if (B <= 0 || T <= 0 || !d_phone || !d_lengths || !d_sid || !d_out)
      throw Error(RVCX_E_INVALID, "rvcx_synth_infer: bad arguments");
    if (ctx->scfg.f0 && (!d_pitch || !d_pitchf))
      throw Error(RVCX_E_INVALID, "rvcx_synth_infer: a pitch-guided model needs pitch and pitchf");
    if (!ctx->scfg.f0) d_pitch = nullptr, d_pitchf = nullptr;  // Synthesizer.infer ignores them (:233-239)
    set_device(ctx);
    synth_forward(*ctx, B, T, d_phone, d_lengths, d_pitch, d_pitchf, d_sid, d_eps_z, d_eps_src, seed, d_out, d_zp,
                  d_z, static_cast<hipStream_t>(stream));
  });
}

int rvcx_synth_infer_ex(rvcx_ctx* ctx, int B, int T, const float* d_phone, const int32_t* d_lengths,
                        const int32_t* d_pitch, const float* d_pitchf, const int32_t* d_sid, double rate,
                        const float* d_eps_z, const float* d_eps_src, uint64_t seed, float* d_out, float* d_zp,
                        float* d_z, float* d_m_p, float* d_logs_p, int* t_out, void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[0]) throw Error(RVCX_E_STATE, "synthesizer weights not finalized");
    if (B <= 0 || T <= 0 || !d_phone || !d_lengths || !d_sid || !d_out)
      throw Error(RVCX_E_INVALID, "rvcx_synth_infer_ex: bad arguments");
    if (ctx->scfg.f0 && (!d_pitch || !d_pitchf))
      throw Error(RVCX_E_INVALID, "rvcx_synth_infer_ex: a pitch-guided model needs pitch and pitchf");
    if (!ctx->scfg.f0) d_pitch = nullptr, d_pitchf = nullptr;
    // head = int(z_p.shape[2] * (1.0 - rate)) (synthesizers.py:231), then Python's slice [head:]: a negative head
    // (rate > 1) keeps the last -head frames (all T when -head >= T); rate < 0: no rate (None)
    int head = 0;
    if (rate >= 0.0) {
      const double h = (double)T * (1.0 - rate);
      if (std::isnan(h)) throw Error(RVCX_E_INVALID, "rvcx_synth_infer_ex: rate is not a number");
      const double ht = std::trunc(h);  // int(): toward zero
      head = ht >= 0.0 ? (int)std::min(ht, (double)T) : (int)std::max(0.0, (double)T + ht);
      if (head >= T) throw Error(RVCX_E_SHAPE, "rvcx_synth_infer_ex: rate keeps no frame (the reference's slice is empty)");
    }
    set_device(ctx);
    synth_forward(*ctx, B, T, d_phone, d_lengths, d_pitch, d_pitchf, d_sid, d_eps_z, d_eps_src, seed, d_out, d_zp,
                  d_z, static_cast<hipStream_t>(stream), 0, head, d_m_p, d_logs_p);
    if (t_out) *t_out = T - head;
  });
}

int rvcx_dec_only(rvcx_ctx* ctx, int B, int T, const float* d_z, const float* d_f0, const int32_t* d_sid,
                  const float* d_eps_src, uint64_t seed, float* d_out, void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[0]) throw Error(RVCX_E_STATE, "synthesizer weights not finalized");
    if (B <= 0 || T <= 0 || !d_z || !d_sid || !d_out || (ctx->scfg.f0 && !d_f0))
      throw Error(RVCX_E_INVALID, "rvcx_dec_only: bad arguments");
    set_device(ctx);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int I = ctx->scfg.I;
    float* zt = ctx->buf<float>("dec_only.z", (size_t)B * T * I, s);
    check(transpose_bct_btc(d_z, zt, B, I, T, s), "transpose");
    float* g = ctx->buf<float>("dec_only.g", (size_t)B * ctx->scfg.gin, s);
    check(gather_rows(ctx->W("emb_g"), ctx->scfg.gin, d_sid, g, B, ctx->scfg.gin, s), "emb_g");
    dec_forward(*ctx, B, T, zt, nullptr, d_f0, g, d_eps_src, seed, d_out, s);
  });
}

int rvcx_voice_conversion(rvcx_ctx* ctx, const float* d_audio, int64_t n, const int32_t* d_pitch,
                          const float* d_pitchf, int sid, float protect, double index_rate, const float* d_eps_z,
                          const float* d_eps_src, uint64_t seed, float* d_out, int64_t cap, int64_t* n_out,
                          void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[0] || !ctx->ready[1]) throw Error(RVCX_E_STATE, "synthesizer/hubert not finalized");
    if (!d_audio || !d_out || n <= 0 || (ctx->scfg.f0 && (!d_pitch || !d_pitchf)))
      throw Error(RVCX_E_INVALID, "bad arguments");
    set_device(ctx);
    if (index_rate > 0 && !ctx->ivf) throw Error(RVCX_E_STATE, "index_rate > 0 but no feature index loaded");
    const int64_t no = vc_forward(*ctx, d_audio, n, d_pitch, d_pitchf, n / 160, sid, protect, index_rate, d_eps_z,
                                  d_eps_src, seed, d_out, cap, static_cast<hipStream_t>(stream));
    if (n_out) *n_out = no;
  });
}

int rvcx_set_highpass(rvcx_ctx* ctx, const double* b, const double* a, const double* zi, int order) {
  return guard(ctx, [&] {
    if (!b || !a || !zi) throw Error(RVCX_E_INVALID, "null coefficients");
    set_highpass(*ctx, b, a, zi, order);
  });
}

int rvcx_set_highpass_sos(rvcx_ctx* ctx, const double* sos, int nsec) {
  return guard(ctx, [&] {
    if (!sos) throw Error(RVCX_E_INVALID, "null sections");
    if (ctx->hp_order == 0) throw Error(RVCX_E_STATE, "set the (b, a) form first (rvcx_set_highpass)");
    set_device(ctx);
    set_highpass_sos(*ctx, sos, nsec);
  });
}

int rvcx_highpass_pad(rvcx_ctx* ctx, const double* d_audio, int64_t n, int64_t t_pad, double* d_pad64, float* d_pad32,
                      void* stream) {
  return guard(ctx, [&] {
    if (!d_audio || !d_pad32 || n <= 0 || t_pad < 0) throw Error(RVCX_E_INVALID, "rvcx_highpass_pad: bad arguments");
    set_device(ctx);
    highpass_pad(*ctx, d_audio, n, t_pad, d_pad64, d_pad32, static_cast<hipStream_t>(stream));
  });
}

int rvcx_pipeline(rvcx_ctx* ctx, const double* d_audio, int64_t n, int sid, double semitones, float protect,
                  int64_t t_pad, int64_t t_pad_tgt, const float* d_eps_z, const float* d_eps_src, uint64_t seed,
                  float* d_out, int64_t cap, int64_t* n_out, double* d_f0, void* stream) {
  rvcx_pipeline_opts o = default_pipeline_opts();
  o.sid = sid;
  o.pitch = semitones;
  o.protect = protect;
  o.t_pad = t_pad;
  o.t_pad_tgt = t_pad_tgt;
  o.t_max = 0;  // single chunk
  return rvcx_pipeline_ex(ctx, d_audio, n, &o, d_eps_z, d_eps_src, seed, d_out, cap, n_out, d_f0, stream);
}

int rvcx_pipeline_default_opts(rvcx_pipeline_opts* opts) {
  if (!opts) return RVCX_E_INVALID;
  *opts = default_pipeline_opts();
  return RVCX_OK;
}

int rvcx_pipeline_ex(rvcx_ctx* ctx, const double* d_audio, int64_t n, const rvcx_pipeline_opts* opts,
                     const float* d_eps_z, const float* d_eps_src, uint64_t seed, float* d_out, int64_t cap,
                     int64_t* n_out, double* d_f0, void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[0] || !ctx->ready[1] || !ctx->ready[2]) throw Error(RVCX_E_STATE, "models not finalized");
    if (!d_audio || !d_out || !opts || n <= 0) throw Error(RVCX_E_INVALID, "bad arguments");
    set_device(ctx);
    const int64_t no = pipeline_forward_ex(*ctx, d_audio, n, *opts, d_eps_z, d_eps_src, seed, d_out, cap, d_f0,
                                           static_cast<hipStream_t>(stream));
    if (n_out) *n_out = no;
  });
}

int rvcx_set_workspace(rvcx_ctx* ctx, void* d_base, int64_t bytes) {
  return guard(ctx, [&] {
    if ((d_base && bytes <= 0) || (!d_base && bytes != 0) || (reinterpret_cast<uintptr_t>(d_base) & 255))
      throw Error(RVCX_E_INVALID, "rvcx_set_workspace: a 256-B aligned base with bytes > 0, or NULL and 0");
    set_device(ctx);
    ctx->release_pool();
    ctx->arena = static_cast<char*>(d_base);
    ctx->arena_bytes = d_base ? (size_t)bytes : 0;
  });
}

int rvcx_workspace_info(const rvcx_ctx* ctx, int64_t* held, int64_t* arena_bytes, int64_t* arena_used) {
  if (!ctx) return RVCX_E_INVALID;
  if (held) *held = (int64_t)ctx->pool_bytes();
  if (arena_bytes) *arena_bytes = (int64_t)ctx->arena_bytes;
  if (arena_used) *arena_used = (int64_t)ctx->arena_used;
  return RVCX_OK;
}

int rvcx_workspace_bytes(rvcx_ctx* ctx, int B, int64_t n, const rvcx_pipeline_opts* opts, int64_t* bytes,
                         void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[0] || !ctx->ready[1] || !ctx->ready[2]) throw Error(RVCX_E_STATE, "models not finalized");
    if (!opts || !bytes || n <= 0 || B < 1) throw Error(RVCX_E_INVALID, "rvcx_workspace_bytes: bad arguments");
    set_device(ctx);
    const hipStream_t s = static_cast<hipStream_t>(stream);
    // the call itself on zero audio, from an empty internally allocated pool; the pool is released again after, and
    // a caller arena stays attached (its regions are carved anew by the next call)
    char* const arena = ctx->arena;
    const size_t arena_bytes = ctx->arena_bytes;
    ctx->release_pool();
    ctx->arena = nullptr;
    ctx->arena_bytes = 0;
    struct PlanScope {
      Ctx& c;
      ~PlanScope() { c.sizing_plan = false; }
    } plan_scope{*ctx};
    ctx->sizing_plan = true;
    DevBuf audio, out;
    const int64_t m = n + 2 * opts->t_pad;
    const int64_t cap = (m / 160 + (opts->t_center > 0 ? n / opts->t_center : 0) + 2) * ctx->scfg.upp();
    int64_t need = 0;
    try {
      RVCX_HIP(hipMalloc(&audio.p, sizeof(double) * (size_t)(B * n)));
      RVCX_HIP(hipMalloc(&out.p, sizeof(float) * (size_t)(B * cap)));
      RVCX_HIP(hipMemsetAsync(audio.p, 0, sizeof(double) * (size_t)(B * n), s));
      if (B == 1) {
        pipeline_forward_ex(*ctx, static_cast<const double*>(audio.p), n, *opts, nullptr, nullptr, 0,
                            static_cast<float*>(out.p), cap, nullptr, s);
      } else {
        std::vector<int32_t> sids((size_t)B, opts->sid);
        pipeline_forward_batch(*ctx, static_cast<const double*>(audio.p), n, n, B, *opts, sids.data(), nullptr, nullptr, 0,
                               static_cast<float*>(out.p), cap, nullptr, nullptr, s);
      }
      RVCX_HIP(hipStreamSynchronize(s));
      need = (int64_t)ctx->carved;
      // the per-chunk HuBERT feature buffers (pl.hb<i>) sum to the same total over any split plan up to one row and
      // the 256-B rounding per chunk
      if (B == 1 && opts->t_max > 0 && n + 160 > opts->t_max && opts->t_center > 0) {
        const int64_t nts = n > opts->t_center ? (n - 1 - opts->t_center) / opts->t_center + 1 : 0;
        need += (nts + 1) * ((int64_t)ctx->scfg.emb_dim * 4 + 512);
      }
    } catch (...) {
      ctx->release_pool();
      ctx->arena = arena;
      ctx->arena_bytes = arena_bytes;
      throw;
    }
    ctx->release_pool();
    ctx->arena = arena;
    ctx->arena_bytes = arena_bytes;
    *bytes = need;
  });
}

int rvcx_device_status(rvcx_ctx* ctx, void* stream) {
  return guard(ctx, [&] {
    RVCX_HIP(hipSetDevice(ctx->device));
    RVCX_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    if (ctx->aux) RVCX_HIP(hipStreamSynchronize(ctx->aux));
    ctx->check_device_status();
  });
}

int rvcx_index_parse(const void* bytes, int64_t nbytes, int64_t* d, int64_t* ntotal, int64_t* nlist,
                     int64_t* nprobe, char* err, int64_t err_cap) {
  try {
    if (!bytes || nbytes <= 0) throw Error(RVCX_E_INVALID, "index_parse: empty buffer");
    const ParsedIvf P = parse_ivf(static_cast<const uint8_t*>(bytes), nbytes);
    if (d) *d = P.d;
    if (ntotal) *ntotal = P.ntotal;
    if (nlist) *nlist = P.nlist;
    if (nprobe) *nprobe = P.nprobe;
    if (err && err_cap > 0) err[0] = 0;
    return RVCX_OK;
  } catch (const Error& e) {
    if (err && err_cap > 0) std::snprintf(err, (size_t)err_cap, "%s", e.what());
    return e.code;
  } catch (const std::exception& e) {
    if (err && err_cap > 0) std::snprintf(err, (size_t)err_cap, "%s", e.what());
    return RVCX_E_INVALID;
  }
}

int rvcx_set_conv_math(rvcx_ctx* ctx, int mode) {
  return guard(ctx, [&] {
    if (mode < 0 || mode > 3) throw Error(RVCX_E_INVALID, "conv math mode must be 0, 1, 2 or 3");
    ctx->conv_math = mode;
  });
}

int rvcx_config_info(const rvcx_ctx* ctx, char* buf, int64_t cap, int64_t* len) {
  // JSON: the effective contraction arithmetic, the developer-knob opt-in and every RVCX_* variable of the process
  // environment with whether it is honoured (ctx may be NULL: the process-wide part only, no device needed)
  std::string j = "{\"arch\": \"gfx950\"";
  if (ctx) j += ", \"conv_math_ctx\": " + std::to_string(ctx->conv_math);
  const char* cm = rvcx_knob("RVCX_CONV_MATH");
  j += ", \"conv_math_default\": \"" + std::string(cm ? cm : "h16") + "\"";
  j += ", \"experimental\": " + std::string(experimental_on() ? "true" : "false");
  if (ctx) j += ", \"arena_bytes\": " + std::to_string(ctx->arena_bytes);
  j += ", \"env\": {";
  bool first = true;
  for (char** e = environ; e && *e; ++e) {
    if (std::strncmp(*e, "RVCX_", 5) != 0) continue;
    const char* eq = std::strchr(*e, '=');
    if (!eq) continue;
    std::string k(*e, eq - *e), v(eq + 1);
    std::string ve;
    for (char ch : v)
      if (ch != '"' && ch != '\\' && (unsigned char)ch >= 32) ve += ch;
    const bool honoured = k == "RVCX_EXPERIMENTAL" || k == "RVCX_PROF_DUMP" || k == "RVCX_LIB" || experimental_on();
    j += std::string(first ? "" : ", ") + "\"" + k + "\": {\"value\": \"" + ve + "\", \"honoured\": " +
         (honoured ? "true" : "false") + "}";
    first = false;
  }
  j += "}}";
  if (len) *len = (int64_t)j.size();
  if (buf && cap > 0) {
    const size_t n = std::min<size_t>(j.size(), (size_t)cap - 1);
    std::memcpy(buf, j.data(), n);
    buf[n] = 0;
  }
  return (int64_t)j.size() < cap || !buf ? RVCX_OK : RVCX_E_CAPACITY;
}

int rvcx_set_generator_precision(rvcx_ctx* ctx, int) {
  return guard(ctx, [&] {
    throw Error(RVCX_E_INVALID,
                "rvcx_set_generator_precision was removed: set rvcx_rt_opts.gen_precision per streaming hop instead");
  });
}

int rvcx_conv1d(rvcx_ctx* ctx, const float* d_x, int64_t T, int C_in, const float* d_w, const float* d_bias, int N,
                int taps, int dilation, int pad, int stride, int math, float* d_y, int64_t T_out, void* stream) {
  return guard(ctx, [&] {
    set_device(ctx);
    ctx->check_device_status();
    if (!d_x || !d_w || !d_y || T <= 0 || C_in <= 0 || N <= 0 || taps <= 0 || dilation <= 0 || stride <= 0 ||
        pad < 0 || T_out <= 0 || math < 0 || math > 7)
      throw Error(RVCX_E_INVALID, "rvcx_conv1d: bad argument");
    if ((T_out - 1) * stride + (int64_t)(taps - 1) * dilation + 1 > T + 2 * (int64_t)pad)
      throw Error(RVCX_E_SHAPE, "rvcx_conv1d: T_out exceeds the padded input");
    if (T > INT32_MAX || T_out > INT32_MAX || (int64_t)taps * N * C_in > INT32_MAX)
      throw Error(RVCX_E_SHAPE, "rvcx_conv1d: size out of range");
    ConvArgs a;
    a.x = d_x; a.ldx = C_in; a.T_in = (int)T; a.C_in = C_in;
    a.w = d_w; a.ldw = C_in; a.w_ts = (long long)N * C_in; a.taps = taps; a.dil = dilation; a.pad = pad;
    a.stride = stride;
    a.y = d_y; a.ldy = N; a.T_out = (int)T_out; a.N = N; a.bias = d_bias;
    a.math = math >= 5 ? 3 : (math >= 3 ? 2 : math);
    if (math == 7) a.wsplit_fmt = WSPLIT_H16;  // the two-plane fp16 arithmetic on the gather-streamed kernel
    if (math == 5 || math == 6) {  // the two-plane fp16 arithmetic / its hi plane alone on the weight-streamed kernel
      a.wsplit_fmt = WSPLIT_H16;
      a.lowp = math == 6;
    }
    if (math == 3 || math == 5 || math == 6) {  // the weight-streamed split kernel (conv_wsb.hip) whatever the size policy would pick
      if (!conv_wsb_eligible(a)) throw Error(RVCX_E_SHAPE, "rvcx_conv1d: shape not eligible for the weight-streamed kernel");
      a.w_static = 1;
      a.force_cfg = conv_wsb_pick(a);  // the tile the pipeline's policy picks for this shape
      a.no_splitk = 1;
      // a fresh split image every call, never the address-keyed cache: the caller may reuse d_w (or torch's
      // allocator may hand the address back) with new weights of the same shape
      void* img = ctx->buf<char>("conv.test.wsplit", (size_t)conv_wsplit_bytes(a), static_cast<hipStream_t>(stream));
      check(conv_wsplit_build(a, img, static_cast<hipStream_t>(stream)), "conv_wsplit_build");
      a.wsplit = img;
    }
    if (math == 4 || math == 7) {  // the gather-streamed split kernel (conv_gs.hip), split-K by the size policy
      if (!conv_gs_eligible(a, false)) throw Error(RVCX_E_SHAPE, "rvcx_conv1d: shape not eligible for the gather-streamed kernel");
      a.w_static = 1;
      a.force_cfg = 30;
      void* img = ctx->buf<char>("conv.test.wsplit", (size_t)conv_wsplit_bytes(a), static_cast<hipStream_t>(stream));
      check(conv_wsplit_build(a, img, static_cast<hipStream_t>(stream)), "conv_wsplit_build");
      a.wsplit = img;
    }
    launch_conv(*ctx, a, false, static_cast<hipStream_t>(stream), -1.0);
  });
}

int rvcx_conv1d_gen(rvcx_ctx* ctx, const float* d_x, int64_t T, int C_in, const float* d_w, const float* d_bias,
                    int N, int taps, int dilation, int pad, int pre_act, float pre_slope, int act, float slope,
                    const float* d_res, int acc_mode, float acc_div, int kernel, float* d_y, void* stream) {
  return guard(ctx, [&] {
    set_device(ctx);
    ctx->check_device_status();
    if (!d_x || !d_w || !d_y || T <= 0 || C_in <= 0 || N <= 0 || taps <= 0 || dilation <= 0 || pad < 0 || act < 0 ||
        act > 1 || pre_act < 0 || pre_act > 1 || acc_mode < 0 || acc_mode > 2 || kernel < 0 || kernel > 2 || (d_res && d_res == d_x))
      throw Error(RVCX_E_INVALID, "rvcx_conv1d_gen: bad argument");
    const int64_t T_out = T + 2 * (int64_t)pad - (int64_t)(taps - 1) * dilation;
    if (T_out <= 0 || T > INT32_MAX || (int64_t)taps * N * C_in > INT32_MAX)
      throw Error(RVCX_E_SHAPE, "rvcx_conv1d_gen: size out of range");
    ConvArgs a;
    a.x = d_x; a.ldx = C_in; a.T_in = (int)T; a.C_in = C_in;
    a.w = d_w; a.ldw = C_in; a.w_ts = (long long)N * C_in; a.taps = taps; a.dil = dilation; a.pad = pad;
    a.y = d_y; a.ldy = N; a.T_out = (int)T_out; a.N = N; a.bias = d_bias;
    a.pre_act = pre_act ? ACT_LRELU : ACT_NONE;
    a.pre_slope = pre_slope;
    a.act = act ? ACT_LRELU : ACT_NONE;
    a.slope = slope;
    if (d_res) {
      a.res = d_res;
      a.ldr = N;
      a.res_mode = RES_ADD_POST;
    }
    a.acc_mode = acc_mode == 0 ? ACC_STORE : (acc_mode == 1 ? ACC_ADD : ACC_ADD_DIV);
    a.acc_div = acc_div;
    a.math = 3;
    a.wsplit_fmt = WSPLIT_H16;
    a.w_static = 1;
    a.no_splitk = 1;
    if (!conv_wsb_eligible(a)) throw Error(RVCX_E_SHAPE, "rvcx_conv1d_gen: shape not eligible for the weight-streamed kernel");
    // 0: the size policy's route, 1: the weight-streamed tile the policy would pick, 2: the weight-stationary kernel
    a.force_cfg = kernel == 1 ? conv_wsb_pick(a) : (kernel == 2 ? 40 : -1);
    // a fresh image every call (rvcx_conv1d's reason)
    a.wsplit_npad = conv_wsplit_npad(a.N);
    void* img = ctx->buf<char>("conv.test.wsplit", (size_t)conv_wsplit_bytes(a), static_cast<hipStream_t>(stream));
    check(conv_wsplit_build(a, img, static_cast<hipStream_t>(stream)), "conv_wsplit_build");
    a.wsplit = img;
    ConvArgs b = a;
    b.wsb = 1;
    if (kernel == 2 && !conv_wst_fits(b, false))
      throw Error(RVCX_E_SHAPE, "rvcx_conv1d_gen: shape not eligible for the weight-stationary kernel");
    launch_conv(*ctx, a, false, static_cast<hipStream_t>(stream), -1.0);
  });
}

int rvcx_conv2d3x3(rvcx_ctx* ctx, const float* d_x, int H, int W, int C_in, const float* d_w, const float* d_bias,
                   int N, int act, int math, float* d_y, void* stream) {
  return guard(ctx, [&] {
    set_device(ctx);
    ctx->check_device_status();
    if (!d_x || !d_w || !d_y || H <= 0 || W <= 0 || C_in <= 0 || N <= 0 || act < 0 || act > 1 || math < 0 || math > 2)
      throw Error(RVCX_E_INVALID, "rvcx_conv2d3x3: bad argument");
    if ((int64_t)H * W * (C_in > N ? C_in : N) > INT32_MAX) throw Error(RVCX_E_SHAPE, "rvcx_conv2d3x3: size out of range");
    ConvArgs a;
    a.x = d_x; a.ldx = C_in; a.T_in = H; a.W_in = W; a.C_in = C_in;
    a.w = d_w; a.ldw = C_in; a.w_ts = (long long)N * C_in; a.taps = 9; a.KH = 3; a.KW = 3; a.padh = 1; a.padw = 1;
    a.y = d_y; a.ldy = N; a.T_out = H; a.W_out = W; a.N = N; a.bias = d_bias;
    a.act = act ? ACT_RELU : ACT_NONE;
    a.math = math == 1 ? 1 : (math >= 2 ? 3 : 0);
    if (a.math == 0 && ctx->conv_math > 0) a.math = ctx->conv_math;
    if (math == 2) {
      // the windowed gather-streamed kernel of the U-Net's deep levels in the two-plane fp16 split (64 x 64 tiles, K
      // split over workgroups by the size policy); a fresh image every call
      a.wsb = 2;
      a.wsplit_fmt = WSPLIT_H16;
      if (!conv_gsw_eligible(a)) throw Error(RVCX_E_SHAPE, "rvcx_conv2d3x3: shape not eligible for the windowed kernel");
      a.w_static = 1;
      a.force_cfg = 30;
      void* img = ctx->buf<char>("conv.test.wsplit", (size_t)conv_wsplit_bytes(a), static_cast<hipStream_t>(stream));
      check(conv_wsplit_build(a, img, static_cast<hipStream_t>(stream)), "conv_wsplit_build");
      a.wsplit = img;
      a.wsplit_npad = conv_wsplit_npad(a.N);
    } else if (conv_math_of(a) == 3 && conv2d_small_fits(a)) {
      // a fresh image every call, never the address-keyed cache (the caller may reuse d_w with new weights)
      a.wsplit_fmt = WSPLIT_S2D;
      void* img = ctx->buf<char>("conv.test.s2d", (size_t)small2d_wsplit_bytes(a), static_cast<hipStream_t>(stream));
      check(small2d_wsplit_build(a, img, static_cast<hipStream_t>(stream)), "small2d_wsplit_build");
      a.wsplit = img;
    }
    launch_conv(*ctx, a, true, static_cast<hipStream_t>(stream), -1.0);
  });
}

int rvcx_convtranspose2d_s2(rvcx_ctx* ctx, const float* d_x, int H, int W, int C_in, const float* d_w,
                            const float* d_bias, int N, int act, int math, float* d_y, void* stream) {
  return guard(ctx, [&] {
    set_device(ctx);
    ctx->check_device_status();
    if (!d_x || !d_w || !d_y || H <= 0 || W <= 0 || C_in <= 0 || N <= 0 || act < 0 || act > 1 || math < 0 || math > 1)
      throw Error(RVCX_E_INVALID, "rvcx_convtranspose2d_s2: bad argument");
    if ((int64_t)4 * H * W * (C_in > 4 * N ? C_in : 4 * N) > INT32_MAX)
      throw Error(RVCX_E_SHAPE, "rvcx_convtranspose2d_s2: size out of range");
    hipStream_t s = static_cast<hipStream_t>(stream);
    // the phase-conv weights (and its bias per virtual column) in test buffers, rebuilt every call
    float* wp = ctx->buf<float>("conv.test.upw", (size_t)16 * N * C_in, s);
    check(upconv_phase_pack(d_w, C_in, N, wp, s), "upconv_phase_pack");
    float* bp = nullptr;
    if (d_bias) {
      bp = ctx->buf<float>("conv.test.upb", (size_t)4 * N, s);
      for (int p = 0; p < 4; ++p)
        RVCX_HIP(hipMemcpyAsync(bp + (size_t)p * N, d_bias, sizeof(float) * N, hipMemcpyDeviceToDevice, s));
    }
    ConvArgs a;  // runtime_fe.cpp's decoder up-conv
    a.x = d_x; a.ldx = C_in; a.T_in = H; a.W_in = W; a.C_in = C_in;
    a.w = wp; a.ldw = C_in; a.w_ts = (long long)4 * N * C_in; a.taps = 4; a.KH = 2; a.KW = 2;
    a.y = d_y; a.ldy = N; a.T_out = H; a.W_out = W; a.N = 4 * N;
    a.out_map = OUT_UPSAMPLE2D;
    a.out_cv = N;
    a.bias = bp;
    a.act = act ? ACT_RELU : ACT_NONE;
    a.math = math == 1 ? 1 : 0;
    if (a.math == 0 && ctx->conv_math > 0) a.math = ctx->conv_math;
    if (math == 0 && conv_math_of(a) >= 2) {
      // the gather-streamed kernel the pipeline's policy routes the up-convs to, with a fresh image every call
      a.wsb = 2;
      a.wsplit_fmt = conv_math_of(a) == 3 ? WSPLIT_H16 : WSPLIT_BF16;
      if (!conv_gs_eligible(a, true)) throw Error(RVCX_E_SHAPE, "rvcx_convtranspose2d_s2: shape not eligible");
      a.w_static = 1;
      a.force_cfg = 30;
      void* img = ctx->buf<char>("conv.test.wsplit", (size_t)conv_wsplit_bytes(a), s);
      check(conv_wsplit_build(a, img, s), "conv_wsplit_build");
      a.wsplit = img;
      a.wsplit_npad = conv_wsplit_npad(a.N);
    }
    launch_conv(*ctx, a, true, s, -1.0);
  });
}

int rvcx_flash_attention(rvcx_ctx* ctx, const float* d_qkv, int B, int T, int n_heads, int dk, float qscale,
                         const float* d_rel_k, const float* d_rel_v, int window, const float* d_mask, float* d_out,
                         void* stream) {
  return guard(ctx, [&] {
    set_device(ctx);
    ctx->check_device_status();
    if (!d_qkv || !d_out || B <= 0 || T <= 0 || n_heads <= 0 || (dk != 64 && dk != 96) || window < 0 ||
        (d_rel_k != nullptr) != (d_rel_v != nullptr))
      throw Error(RVCX_E_INVALID, "rvcx_flash_attention: bad argument");
    if ((long long)B * T * 3 * n_heads * dk > INT32_MAX) throw Error(RVCX_E_SHAPE, "rvcx_flash_attention: too large");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int nsplit = flash_attn_splits(B, n_heads, T);
    float* po = ctx->buf<float>("att.test.o", (size_t)flash_attn_ws_floats(B, n_heads, T, dk, nsplit), s);
    float* pml = ctx->buf<float>("att.test.ml", (size_t)nsplit * B * n_heads * T * 2, s);
    check(flash_attn(d_qkv, 3 * n_heads * dk, B, T, n_heads, dk, qscale, d_rel_k, d_rel_v, window, d_mask, po, pml,
                     nsplit, d_out, n_heads * dk, s),
          "flash_attn");
  });
}

int rvcx_resblock_pair(rvcx_ctx* ctx, const float* d_x, int B, int64_t T, int C, const float* d_w1, const float* d_b1,
                       const float* d_w2, const float* d_b2, int k, int dilation, int acc_mode, float acc_div, int cfg,
                       float* d_y, void* stream) {
  return guard(ctx, [&] {
    set_device(ctx);
    ctx->check_device_status();
    if (!d_x || !d_y || !d_w1 || !d_w2 || !d_b1 || !d_b2 || B <= 0 || T <= 0 || acc_mode < 0 || acc_mode > 2 ||
        d_x == d_y || cfg < 0)
      throw Error(RVCX_E_INVALID, "rvcx_resblock_pair: bad argument");
    if (!rb_pair_fits(C, k, dilation) || T > INT32_MAX / C)
      throw Error(RVCX_E_SHAPE, "rvcx_resblock_pair: shape not supported by the fused kernel");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int fmt = (cfg >> 4) & 3;
    if (fmt > 2) throw Error(RVCX_E_INVALID, "rvcx_resblock_pair: arithmetic (cfg bits 4-5) must be 0, 1 or 2");
    cfg &= 15;
    const int wfmt = fmt ? RB_WF16 : RB_WBF16;
    // fresh split images every call (test entry: the weight pointers may be reused by the caller)
    void* w1s = ctx->buf<char>("rb.test.w1s", (size_t)rb_wsplit_bytes(C, k, wfmt), s);
    void* w2s = ctx->buf<char>("rb.test.w2s", (size_t)rb_wsplit_bytes(C, k, wfmt), s);
    check(rb_wsplit_build(d_w1, C, k, w1s, s, wfmt), "rb_wsplit_build");
    check(rb_wsplit_build(d_w2, C, k, w2s, s, wfmt), "rb_wsplit_build");
    RbPairArgs a;
    a.wfmt = wfmt;
    a.lowp = fmt == 2;
    a.x = d_x;
    a.x_bs = T * C;
    a.w1s = w1s;
    a.b1 = d_b1;
    a.w2s = w2s;
    a.b2 = d_b2;
    a.C = C;
    a.k = k;
    a.d = dilation;
    a.T = (int)T;
    a.B = B;
    a.y = d_y;
    a.y_bs = T * C;
    a.acc_mode = acc_mode;
    a.acc_div = acc_div;
    check(rb_pair(a, cfg, s), "rb_pair");
  });
}

int rvcx_profile(rvcx_ctx* ctx, int enable) {
  return guard(ctx, [&] { ctx->prof = enable != 0; });
}

int rvcx_profile_read(rvcx_ctx* ctx, double* total_ms, double* total_flops, int64_t* launches) {
  return rvcx_profile_read_ex(ctx, total_ms, total_flops, launches, nullptr);
}

int rvcx_profile_read_ex(rvcx_ctx* ctx, double* total_ms, double* total_flops, int64_t* launches, double* ceiling_ms) {
  return rvcx_profile_read_kinds(ctx, total_ms, total_flops, launches, ceiling_ms, 0, nullptr, nullptr, nullptr,
                                 nullptr, nullptr);
}

const char* rvcx_profile_kind_name(int kind) { return (kind >= 0 && kind < CK_COUNT) ? conv_kind_name(kind) : nullptr; }

int rvcx_profile_read_kinds(rvcx_ctx* ctx, double* total_ms, double* total_flops, int64_t* launches, double* ceiling_ms,
                            int nk, double* k_ms, double* k_flops, double* k_ceiling_ms, double* k_bytes,
                            int64_t* k_launches) {
  return guard(ctx, [&] {
    if (nk < 0 || (nk > 0 && (!k_ms || !k_flops || !k_ceiling_ms || !k_bytes || !k_launches)))
      throw Error(RVCX_E_INVALID, "profile_read_kinds: nk > 0 needs all five per-kind arrays");
    set_device(ctx);
    for (int k = 0; k < nk; ++k) k_ms[k] = k_flops[k] = k_ceiling_ms[k] = k_bytes[k] = 0.0, k_launches[k] = 0;
    double ms = 0.0, fl = 0.0, cms = 0.0;
    const char* dump = std::getenv("RVCX_PROF_DUMP");  // append one CSV line per conv launch
    FILE* fd = dump ? std::fopen(dump, "a") : nullptr;
    for (auto& r : ctx->prof_recs) {
      RVCX_HIP(hipEventSynchronize(r.b));
      float t = 0.f;
      RVCX_HIP(hipEventElapsedTime(&t, r.a, r.b));
      if (fd)
        std::fprintf(fd, "%d,%d,%d,%d,%d,%d,%d,%.6f,%.0f,%.0f,%.1f\n", r.two_d, r.M, r.N, r.C_in, r.taps, r.batch, r.ksplit,
                     t, r.flops, r.bytes, r.peak_tf);
      ms += t;
      fl += r.flops;
      cms += r.flops / (r.peak_tf * 1e9);
      if (r.kind >= 0 && r.kind < nk) {
        k_ms[r.kind] += t;
        k_flops[r.kind] += r.flops;
        k_ceiling_ms[r.kind] += r.flops / (r.peak_tf * 1e9);
        k_bytes[r.kind] += r.bytes;
        k_launches[r.kind] += 1;
      }
      ctx->prof_pool.push_back(r.a);
      ctx->prof_pool.push_back(r.b);
    }
    if (fd) std::fclose(fd);
    if (total_ms) *total_ms = ms;
    if (total_flops) *total_flops = fl;
    if (launches) *launches = (int64_t)ctx->prof_recs.size();
    if (ceiling_ms) *ceiling_ms = cms;
    ctx->prof_recs.clear();
  });
}

}  // extern "C"

// ------------------------------------------------------------------ feature index (FAISS IVFFlat)
int rvcx_index_load(rvcx_ctx* ctx, const void* bytes, int64_t nbytes) {
  return guard(ctx, [&] {
    if (!bytes || nbytes <= 0) throw Error(RVCX_E_INVALID, "index_load: empty buffer");
    set_device(ctx);
    index_load(*ctx, static_cast<const uint8_t*>(bytes), nbytes);
  });
}

int rvcx_index_unload(rvcx_ctx* ctx) {
  return guard(ctx, [&] {
    set_device(ctx);
    RVCX_HIP(hipDeviceSynchronize());
    ctx->ivf.reset();
  });
}

int rvcx_index_info(const rvcx_ctx* ctx, int64_t* d, int64_t* ntotal, int64_t* nlist, int64_t* nprobe) {
  if (!ctx) return RVCX_E_INVALID;
  if (!ctx->ivf) return RVCX_E_STATE;
  const IvfView& v = ctx->ivf->view;
  if (d) *d = v.d;
  if (ntotal) *ntotal = v.ntotal;
  if (nlist) *nlist = v.nlist;
  if (nprobe) *nprobe = v.nprobe;
  return RVCX_OK;
}

int rvcx_index_set_nprobe(rvcx_ctx* ctx, int64_t nprobe) {
  return guard(ctx, [&] {
    if (!ctx->ivf) throw Error(RVCX_E_STATE, "no feature index loaded");
    if (nprobe < 1) throw Error(RVCX_E_INVALID, "nprobe must be >= 1");
    ctx->ivf->view.nprobe = (int)std::min<int64_t>(nprobe, ctx->ivf->view.nlist);
  });
}

int rvcx_index_search(rvcx_ctx* ctx, const float* d_x, int64_t n, int k, float* d_dist, int64_t* d_ids,
                      void* stream) {
  return guard(ctx, [&] {
    if ((!d_x && n > 0) || !d_dist || !d_ids || n < 0) throw Error(RVCX_E_INVALID, "index_search: bad arguments");
    set_device(ctx);
    index_search(*ctx, d_x, n, k, d_dist, d_ids, static_cast<hipStream_t>(stream));
  });
}

int rvcx_index_reconstruct_n(rvcx_ctx* ctx, int64_t i0, int64_t ni, float* d_out, void* stream) {
  return guard(ctx, [&] {
    if (!d_out && ni > 0) throw Error(RVCX_E_INVALID, "reconstruct_n: null output");
    set_device(ctx);
    index_reconstruct_n(*ctx, i0, ni, d_out, static_cast<hipStream_t>(stream));
  });
}

int rvcx_index_retrieve(rvcx_ctx* ctx, const float* d_feats, int64_t L, int d, double index_rate, float* d_out,
                        void* stream) {
  return guard(ctx, [&] {
    if ((!d_feats || !d_out) && L > 0) throw Error(RVCX_E_INVALID, "index_retrieve: bad arguments");
    set_device(ctx);
    index_retrieve(*ctx, d_feats, L, d, index_rate, d_out, static_cast<hipStream_t>(stream));
  });
}

// ------------------------------------------------------------------ streaming (C5)
int rvcx_rt_default_desc(rvcx_rt_desc* d) {
  if (!d) return RVCX_E_INVALID;
  d->n_streams = 1;
  d->read_chunk_size = 192;  // rvc/realtime/callbacks.py:16-18
  d->cross_fade_overlap_size = 0.1;
  d->extra_convert_size = 0.5;
  d->silent_threshold = -90.0;
  return RVCX_OK;
}

int rvcx_rt_default_opts(rvcx_rt_opts* o) {
  if (!o) return RVCX_E_INVALID;
  std::memset(o, 0, sizeof(*o));
  o->index_rate = 0.0;
  o->protect = 0.5f;
  o->volume_envelope = 1.0;
  o->f0_autotune_strength = 1.0;
  o->proposed_pitch_threshold = 155.0;
  return RVCX_OK;
}

int rvcx_rt_create(rvcx_ctx* ctx, const rvcx_rt_desc* desc, rvcx_rt** out) {
  return guard(ctx, [&] {
    if (!desc || !out) throw Error(RVCX_E_INVALID, "rt_create: null argument");
    set_device(ctx);
    auto* h = new rvcx_rt();
    try {
      h->s = rt_create(*ctx, *desc);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int rvcx_rt_destroy(rvcx_ctx* ctx, rvcx_rt* rt) {
  return guard(ctx, [&] {
    if (!rt) return;
    set_device(ctx);
    RVCX_HIP(hipDeviceSynchronize());
    rt_destroy(rt->s);
    delete rt;
  });
}

int rvcx_rt_geometry(const rvcx_rt* rt, int64_t* g) {
  if (!rt || !rt->s || !g) return RVCX_E_INVALID;
  rt_geometry(*rt->s, g);
  return RVCX_OK;
}

int rvcx_rt_reset(rvcx_ctx* ctx, rvcx_rt* rt, void* stream) {
  return guard(ctx, [&] {
    if (!rt || !rt->s) throw Error(RVCX_E_INVALID, "rt_reset: null stream group");
    set_device(ctx);
    rt_reset(*ctx, *rt->s, static_cast<hipStream_t>(stream));
  });
}

int rvcx_rt_process(rvcx_ctx* ctx, rvcx_rt* rt, const float* d_in, const int32_t* sids, const rvcx_rt_opts* opts,
                    const float* d_eps_z, const float* d_eps_src, uint64_t seed, float* d_out, float* d_vol,
                    int32_t* d_offs, void* stream) {
  return guard(ctx, [&] {
    if (!rt || !rt->s || !d_in || !sids || !opts || !d_out) throw Error(RVCX_E_INVALID, "rt_process: null argument");
    set_device(ctx);
    rt_process(*ctx, *rt->s, d_in, sids, *opts, d_eps_z, d_eps_src, seed, d_out, d_vol, d_offs,
               static_cast<hipStream_t>(stream));
  });
}

// ------------------------------------------------------------------ batched offline conversion (C4)
int rvcx_pipeline_batch(rvcx_ctx* ctx, const double* d_audio, int64_t n, int64_t lda, int B,
                        const rvcx_pipeline_opts* opts, const int32_t* sids, const float* d_eps_z,
                        const float* d_eps_src, uint64_t seed, float* d_out, int64_t ldo, int64_t* n_out,
                        double* d_f0, float* d_hidden, void* stream) {
  return guard(ctx, [&] {
    if (!ctx->ready[0] || !ctx->ready[1] || !ctx->ready[2]) throw Error(RVCX_E_STATE, "models not finalized");
    if (!d_audio || !opts || !sids || !d_out || n <= 0 || B < 1 || lda < n)
      throw Error(RVCX_E_INVALID, "rvcx_pipeline_batch: bad arguments");
    set_device(ctx);
    if (d_hidden && (opts->f0_method != 0 || !ctx->scfg.f0))
      throw Error(RVCX_E_INVALID, "rvcx_pipeline_batch: d_hidden needs the RMVPE f0 method and a pitch-guided model");
    const int64_t no = pipeline_forward_batch(*ctx, d_audio, n, lda, B, *opts, sids, d_eps_z, d_eps_src, seed, d_out,
                                              ldo, d_f0, d_hidden, static_cast<hipStream_t>(stream));
    if (n_out) *n_out = no;
  });
}
