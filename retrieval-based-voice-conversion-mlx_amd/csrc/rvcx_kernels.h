// rvcx kernel launchers (internal; the public C-ABI is include/rvcx.h).
//
// Tensor convention on device: frame-major ("time-major") rows, channels
// contiguous: a [T][C] matrix with row stride ld (floats). 2-D images (RMVPE
// U-Net) are NHWC: pixel-major rows (h*W + w), channels contiguous.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace rvcx {

// Process-wide developer knobs (RVCX_* environment variables: A/B switches, tile / split-K policy overrides, the
// contraction arithmetic): honoured ONLY when RVCX_EXPERIMENTAL=1 is set, so a stray variable in a user's shell cannot
// change a result or a kernel path. Returns getenv(name), or nullptr without the opt-in. rvcx_config_info reports
// the opt-in and every RVCX_* variable present (honoured or ignored). Defined in capi.cpp.
const char* rvcx_knob(const char* name);

enum Act : int {
  ACT_NONE = 0,
  ACT_LRELU = 1,    // leaky relu with slope
  ACT_RELU = 2,
  ACT_GELU = 3,     // exact erf GELU (HF "gelu", torch F.gelu default)
  ACT_TANH = 4,
  ACT_SIGMOID = 5,
  ACT_LOGCLAMP = 6, // log(max(v, slope))  (RMVPE mel: log(clamp(.,1e-5)))
};

enum ResMode : int {
  RES_NONE = 0,
  RES_ADD_PRE = 1,   // v = (acc + bias) + R, then alpha, act
  RES_ADD_POST = 2,  // v = act(alpha*(acc + bias)) + R
  RES_RSUB_POST = 3, // v = R - act(alpha*(acc + bias))
};

enum AccMode : int {
  ACC_STORE = 0,   // y = v
  ACC_ADD = 1,     // y = y + v
  ACC_ADD_DIV = 2, // y = (y + v) / acc_div
};

enum OutMap : int {
  OUT_ROWS = 0,       // y[b][m][n]
  OUT_UPSAMPLE2D = 1, // 2-D ConvTranspose phase scatter: n = (ph*2+pw)*Cv + co -> pixel (2h+ph, 2w+pw)
};

// Implicit-GEMM convolution:  y[b][m][n] = epi( sum_tap sum_c pre(X[b][row(m,tap)][c]) * W[tap][n][c] )
// WSPLIT_S2D: the few-channel 3x3 convs' fp16 image (conv2d_small.hip k_s2d_wsplit: fragment-major, no column padding)
enum WsplitFmt : int { WSPLIT_BF16 = 0, WSPLIT_H16 = 1, WSPLIT_S2D = 2 };

struct ConvArgs {
  // A operand (activations)
  const float* x = nullptr;
  long long x_bs = 0;   // batch stride (floats)
  int ldx = 0;          // row stride
  int T_in = 0;         // valid input rows (1-D) ; for 2-D: H_in
  int W_in = 0;         // 2-D: input width
  int C_in = 0;         // contraction channels per tap
  int pre_act = ACT_NONE;
  float pre_slope = 0.f;
  const float* pre_mask = nullptr;  // [b][row] multiplier applied to input rows (1-D only)
  long long pre_mask_bs = 0;
  // B operand (weights): NK: w + tap*w_ts + n*ldw + c ; KN: w + tap*w_ts + c*ldw + n
  const float* w = nullptr;
  long long w_bs = 0;
  long long w_ts = 0;
  int ldw = 0;
  int b_kn = 0;
  // geometry
  int taps = 1;
  int stride = 1, dil = 1, pad = 0;     // 1-D
  int KH = 1, KW = 1, padh = 0, padw = 0; // 2-D (taps = KH*KW; tap = kh*KW + kw)
  // output
  float* y = nullptr;
  long long y_bs = 0;
  int ldy = 0;
  int T_out = 0;   // output rows (1-D) ; 2-D: H_out (tile grid), W_out
  int W_out = 0;
  int N = 0;
  int out_map = OUT_ROWS;
  int out_cv = 0;  // OUT_UPSAMPLE2D: real output channels
  // epilogue
  const float* bias = nullptr;
  long long bias_bs = 0;
  float alpha = 1.f;
  int act = ACT_NONE;
  float slope = 0.f;
  const float* res = nullptr;
  long long res_bs = 0;
  int ldr = 0;
  int res_mode = RES_NONE;
  const float* mask = nullptr;  // [b][m] output-row multiplier (applied last, after acc_mode)
  long long mask_bs = 0;
  int acc_mode = ACC_STORE;
  float acc_div = 1.f;
  // WaveNet gate (commons.py:88-103) in the split-K combine: N = 2 gate_h columns; y[m][c] (c < gate_h) =
  // tanh(v[c] + g[c]) * sigmoid(v[c + gate_h] + g[c + gate_h]), v = acc + bias, g = gate_g + b * gate_g_bs. Forces a
  // split (ksplit >= 2); no other epilogue field may be set.
  int gate_h = 0;
  const float* gate_g = nullptr;
  long long gate_g_bs = 0;
  // post-norm LayerNorm in the split-K combine (a Transformer block's residual + norm, attentions.py:221-231 with
  // norm_layers_2, modeling_hubert.py final_layer_norm): y[m] = LN(res[m] + v[m]) * ln_g + ln_b over the N columns, v the
  // epilogue value (bias, alpha, act, mask) with res_mode RES_NONE (res / ldr / res_bs name the LN's residual input).
  // Forces a split (ksplit >= 2); 1-D, batch_inner 1, N <= 1024. Equals the two passes to fp32 rounding of the row sums.
  const float* ln_g = nullptr;
  const float* ln_b = nullptr;
  float ln_eps = 1e-5f;
  // grid z = batch * batch_inner; pointer offset = zo * *_bs + zi * *_bs2 (mask: zo only)
  int batch = 1;
  int batch_inner = 1;
  long long x_bs2 = 0, w_bs2 = 0, y_bs2 = 0, res_bs2 = 0, bias_bs2 = 0;
  // tuning / benchmarking: force a tile configuration and the software pipeline on/off
  int force_cfg = -1;
  int pipe = 0;
  int astage = 0;  // A-tile staging batch: 0 = default (1), 1 = serial, 4 = 4 loads in flight
  int math = 0;    // contraction arithmetic: 0 = default (RVCX_CONV_MATH), 1 = native fp32 MFMA, 2 = fp32 via 3 bf16 planes
  // split-K: set by conv_plan_splitk; ws holds ksplit partial [rows][N] tiles per batch entry
  // weight-streamed split kernel (conv_wsb.hip): w pre-split into bf16 planes, set by the runtime for static weights
  int w_static = 0;             // the B operand is a constant weight tensor (callers set it; enables the cache)
  const void* wsplit = nullptr;  // ((chunk * taps + tap) * wsplit_npad + n) rows of [hi|mid|lo] x 32 bf16
  int wsplit_npad = 0;
  int wsb = 0;  // set by the runtime (conv_wsb_route on a static weight): 1 weight-streamed kernel, 2 gather-streamed
  int wsplit_fmt = 0;  // WSPLIT_BF16: three bf16 planes (every streamed kernel); WSPLIT_H16: two fp16 planes + scale tail
                       // (conv_wsb16_kernel only: the two-plane fp16 arithmetic and the reduced-precision mode)
  int ksplit = 1;
  int no_splitk = 0;
  // opt-in reduced precision (the generator's weight-streamed convs of a realtime hop, rvcx_rt_opts::gen_precision):
  // fp16 operands (the WSPLIT_H16 image's hi plane), one MFMA product per step. Never set on the parity path.
  int lowp = 0;
  long long ws_rows = 0;
  float* ws = nullptr;
  // + the NSF noise conv of this output (hifigan_nsf.py:196-199: x = ups(x) + noise_convs(har)), fused into the
  // epilogue of the polyphase ConvTranspose (1-D, unsplit, store_tile16 kernels, plain bias epilogue; one tap,
  // nz_kk = 1, the only length the dispatcher admits): output row m,
  // column n = p * nz_C + c (phase p of nz_u) gets nz_b[c] + sum_q w(q, c) har[(m nz_u + p) nz_stride + q], q < nz_kk,
  // with w(q, c) = nz_w[((q / nz_stride) nz_C + c) nz_stride + q % nz_stride] (k_noise_add's layout and fma order)
  const float* nz_har = nullptr;
  long long nz_bs = 0;
  int nz_stride = 0, nz_kk = 0, nz_u = 1, nz_C = 0;
  const float* nz_w = nullptr;
  const float* nz_b = nullptr;
  // extra dynamic LDS per workgroup (bytes): fewer of this launch's workgroups fit a CU beside the critical stream's
  // (an occupancy throttle for off-critical-path work; the gather-streamed and LDS-staged kernels honour it)
  int lds_pad = 0;
};

hipError_t conv1d(const ConvArgs& a, hipStream_t s);
// the kernel family the last conv1d / conv2d on this host thread launched (kernel-timing records, rvcx_profile)
enum ConvKind : int { CK_WSB16 = 0, CK_WSB, CK_GS, CK_GSW, CK_RBPAIR, CK_SMALL2D, CK_EMU, CK_GEMM, CK_TINY, CK_WST,
                      CK_OTHER, CK_COUNT };
int conv_last_kind();
const char* conv_kind_name(int k);
// the contraction arithmetic a launch gets: ConvArgs::math, else RVCX_CONV_MATH (1 fp32 MFMA, 2 bf16 split, 3 fp16 split)
int conv_math_of(const ConvArgs& a);
hipError_t conv2d(const ConvArgs& a, hipStream_t s);
// 3x3/pad-1 2-D convs with C_in, N in {16, 32} on 16x16x4 MFMA fragments (conv2d_small.hip); conv2d routes
// the shapes conv2d_small_fits accepts there
bool conv2d_small_fits(const ConvArgs& a);
hipError_t conv2d_small(const ConvArgs& a, hipStream_t s);
// their WSPLIT_S2D image (the fp16-split form reads it; built by conv_wsplit_build for that format)
long long small2d_wsplit_bytes(const ConvArgs& a);
hipError_t small2d_wsplit_build(const ConvArgs& a, void* out, hipStream_t s);
// choose split-K for small output grids; returns the workspace floats needed (0 = no split)
long long conv_plan_splitk(ConvArgs& a, bool two_d);

// ---------------------------------------------------------------- misc kernels
hipError_t fill(float* p, float v, long long n, hipStream_t s);
hipError_t transpose_bct_btc(const float* x, float* y, int B, int C, int T, hipStream_t s); // [B][C][T] -> [B][T][C]
hipError_t transpose_btc_bct(const float* x, float* y, int B, int T, int C, int ldx, hipStream_t s);
hipError_t channel_flip(const float* x, float* y, int rows, int C, hipStream_t s);
hipError_t gather_rows(const float* table, int ld_table, const int32_t* idx, float* y, int rows, int C,
                       hipStream_t s);
hipError_t seq_mask(const int32_t* lengths, float* mask, int B, int T, hipStream_t s);
// ConvTranspose2d 3x3 / stride 2 / pad 1 / output pad 1 weights w [C][co][3][3] -> the 2x2-tap phase conv's
// [4][4 co][C] (virtual column (ph 2 + pw) co + o; ConvArgs::out_map OUT_UPSAMPLE2D scatters the phases)
hipError_t upconv_phase_pack(const float* w, int C, int co, float* out, hipStream_t s);
hipError_t layernorm_rows(const float* x, const float* r, float* y, const float* gamma, const float* beta,
                          int rows, int D, float eps, const float* mask, hipStream_t s);
hipError_t gate_tanh_sigmoid(const float* xin, int ldx, const float* g, long long g_bs, float* acts, int B,
                             int T, int H, hipStream_t s);
// y[b][t][c] += nb[c] + sum_{q < taps*stride} wf[(q / stride) * C + c][q % stride] * har[b*har_bs + t*stride + q]
// (the NSF noise conv, hifigan_nsf.py:196-199, in its framed form); C % 4 == 0, taps*stride <= 16
// weight-streamed split conv (conv_wsb.hip): eligibility (1-D, stride 1, C_in % 32 == 0, halo <= 64 rows, no
// split-K), the pre-split weight image and its launch; conv_wsb_wants = eligible + split arithmetic + a grid
// large enough to fill the chip (conv_gemm.hip policy)
bool conv_wsb_eligible(const ConvArgs& a, bool two_d = false);
bool conv_wsb_wants(const ConvArgs& a);
// route a contraction with a static weight to the weight-streamed kernel (the big 1-D grids, conv_wsb_wants) or the
// gather-streamed one (the rest with 32-channel chunks and >= 64 outputs)
// 0: not routed (conv_emu / conv_gemm), 1: conv_wsb.hip, 2: conv_gs.hip
int conv_wsb_route(const ConvArgs& a, bool two_d);
bool conv_wsb_tile(int cfg, int& BM, int& BN);  // cfg 23, 24, 25, 27 -> tile
int conv_wsb_pick(const ConvArgs& a);  // the weight-streamed tile cfg the size policy picks for a
// gather-streamed split conv (conv_gs.hip) for the short contractions: pre-split weights (the conv_wsb image) in a
// register ring, A gathered per (chunk, tap) step; 1-D (any stride / dilation) and 2-D (stride 1, OUT_ROWS), C_in % 32
// == 0, split-K capable. cfg 30 -> its 64 x 64 tile
bool conv_gs_eligible(const ConvArgs& a, bool two_d);
bool conv_gsw_eligible(const ConvArgs& a);  // the windowed 2-D form (split-K slices of whole 32-channel chunks)
bool conv_gs_tile(int cfg, int& BM, int& BN);
hipError_t conv_gs_launch(const ConvArgs& a, int cfg, int ntn_enable, hipStream_t s, bool two_d, int ksplit);
int conv_wsplit_npad(int N);
long long conv_wsplit_bytes(const ConvArgs& a);
hipError_t conv_wsplit_build(const ConvArgs& a, void* out, hipStream_t s);
hipError_t conv_wsb_launch(const ConvArgs& a, int cfg, int ntn_enable, hipStream_t s, bool two_d = false,
                           int ksplit = 1);
// weight-stationary form of the fp16-split conv (conv_wst.hip) for the short 64 / 128-channel convs (k = 3 ResBlock
// convs, ConvTranspose phases): 1-D, C_in = N in {64, 128}, 2-3 taps, halo <= 16, no or leaky-ReLU pre-activation,
// the WSPLIT_H16 image, bias / leaky-ReLU / RES_ADD_POST / acc modes / the fused noise conv; bit-identical to
// conv_wsb16_kernel. The dispatcher takes it ahead of the weight-streamed tiles
bool conv_wst_fits(const ConvArgs& a, bool two_d);
hipError_t conv_wst_launch(const ConvArgs& a, hipStream_t s);
// fused ResBlock dilation pair (resblock_fused.hip): y (acc_mode) <- conv2(lrelu(conv1_d(lrelu(x)) + b1)) + b2 + x,
// x / y [B][T][C] (x != y), C in {32, 64}, odd k, (k - 1) / 2 * d <= 30; w1s / w2s are rb_wsplit_build images
// of [k][C][C] fp32 weights
struct RbPairArgs {
  const float* x = nullptr;
  long long x_bs = 0;
  const void* w1s = nullptr;
  const float* b1 = nullptr;
  const void* w2s = nullptr;
  const float* b2 = nullptr;
  int C = 0, k = 0, d = 1, T = 0, B = 1;
  float* y = nullptr;
  long long y_bs = 0;
  int acc_mode = ACC_STORE;
  float acc_div = 1.f;
  int wfmt = 0;   // RB_WBF16: w1s / w2s are three-plane bf16 images (the exact split); RB_WF16: two-plane fp16 images
  int lowp = 0;   // opt-in reduced precision (rvcx_rt_opts::gen_precision): the fp16 images' hi planes alone
};
enum RbWfmt : int { RB_WBF16 = 0, RB_WF16 = 1 };
bool rb_pair_fits(int C, int k, int d);
long long rb_wsplit_bytes(int C, int k, int wfmt = RB_WBF16);
hipError_t rb_wsplit_build(const float* w, int C, int k, void* out, hipStream_t s, int wfmt = RB_WBF16);
hipError_t rb_pair(const RbPairArgs& a, int cfg, hipStream_t s);
// fused attention (flash_attn.hip): qkv [B][T][ldq] (q | k | v, heads of dk inside each), optional relative
// window (rel_k / rel_v [2w+1][dk]) and key/query mask [B][T]; partials part_o [nsplit][B*nh][T][dk], part_ml
// [nsplit][B*nh][T][2]; out [B][T][ldo] at column h*dk
int flash_attn_splits(int B, int nh, int T);
// floats the caller allocates for part_o: the split partials and the fp16 form's K / V fragment images
long long flash_attn_ws_floats(int B, int nh, int T, int dk, int nsplit);
hipError_t flash_attn(const float* qkv, int ldq, int B, int T, int nh, int dk, float qscale, const float* rel_k,
                      const float* rel_v, int window, const float* mask, float* part_o, float* part_ml, int nsplit,
                      float* out, int ldo, hipStream_t s);
// CREPE (crepe.hip): frames [nf][ld] (254 zeros | 1024 normalised samples | 254 zeros) of frames f_first..;
// relu -> BatchNorm (bn = mean | 1/sqrt(var+eps) | gamma | beta, C each) -> max over row pairs [rows_in][C] ->
// [rows_in/2][C]; decode + 3-tap filters: probs [F][360] -> f0 (fp32), f0d (fp64, optional), per (optional)
hipError_t crepe_frames(const float* audio, long long n, long long f_first, int nf, float* out, int ld, hipStream_t s,
                        int torch_sem = 0);
hipError_t crepe_relu_bn_pool(const float* x, long long rows_in, int C, const float* bn, float* y, hipStream_t s);
hipError_t crepe_decode(const float* probs, int F, double lo_cents, double hi_cents, float thr, float* f0_raw,
                        float* per_raw, float* f0, double* f0d, float* per, hipStream_t s);
// torchcrepe's viterbi decode + rvc/'s filters (bins [minidx, maxidx) allowed; dither [F] cents or NULL): workspace
// lp [F][360] fp32, ptr [F][360] int32, bins [F] int32. Every run of `seg` frames is decoded as its own sequence
// (torchcrepe.predict's batches, CREPE_RVC_BATCH at rvc/'s batch_size); the filters run over all F frames.
constexpr int CREPE_RVC_BATCH = 512;  // rvc/lib/predictors/f0.py:38
hipError_t crepe_decode_viterbi(const float* probs, int F, int minidx, int maxidx, const float* dither, float thr,
                                float* lp, int* ptr, int* bins, float* f0_raw, float* per_raw, float* f0, double* f0d,
                                float* per, hipStream_t s, int seg = CREPE_RVC_BATCH);
// (store: y = the noise conv itself, not accumulated)
hipError_t noise_conv_add(const float* har, long long har_bs, int stride, int taps, const float* wf, const float* nb,
                          float* y, int B, int T, int C, hipStream_t s, bool store = false);
hipError_t upsample2_protect(const float* feats, const float* feats0, int L, int D, float* out, int T, const float* pitchf,
                             float protect,
                             hipStream_t s);
hipError_t sine_source(const float* f0, int B, int L, int upp, float sr, const float* eps, uint64_t seed,
                       float lin_w, float lin_b, double* cum_ws, float* har, long long har_ld, hipStream_t s);
hipError_t conv_post_tanh(const float* x, int B, int T, int C, const float* w, int K, float slope, float* y,
                          hipStream_t s, float bias = 0.f);
// per-sample harmonic source of the MRF HiFi-GAN / RefineGAN decoders (source_harm.hip): f0 [B][L] -> har row b
// at har + b*har_ld, N = L*upp samples; eps [B][N][H] and ini [B][H] injected or drawn (Philox(seed))
size_t harm_source_ws_doubles(int B, int L, int upp, int H);
// RefineGAN (refinegan.hip): depthwise kaiser-sinc downsampling by `orig` (new_freq 1), linear x rate upsampling of
// lrelu(x) concatenated with a skip, AdaIN (mode 0 store, 1 add, 2 add then / div)
hipError_t resample_dw(const float* x, int B, int T_in, int C, const float* ker, int K, int orig, int width, float* y,
                       int T_out, hipStream_t s);
hipError_t lerp_up_cat(const float* x, int B, int T, int C, int ldx, int rate, float slope, const float* skip, int Cd,
                       float* y, int ldy, hipStream_t s);
hipError_t adain(const float* x, int B, int T, int C, const float* w, const float* eps, uint64_t seed, float slope,
                 float* y, int mode, float div, hipStream_t s);
hipError_t harm_source(const float* f0, int B, int L, int upp, float sr, int H, int linear_up, const float* eps,
                       const float* ini, uint64_t seed, const float* lin_w, float lin_b, double* ws, float* har,
                       long long har_ld, hipStream_t st);
hipError_t randn(float* y, long long n, uint64_t seed, uint64_t offset, hipStream_t s);
hipError_t zp_sample(const float* stats, int B, int T, int I, const float* eps, uint64_t seed, const float* mask,
                     float* zp, hipStream_t s);
// ws: groupnorm_ws_doubles(C, B) doubles; x = B sequences of T rows back to back
constexpr int GN_CHUNKS = 256;
inline size_t groupnorm_ws_doubles(int C, int B = 1) { return (size_t)B * (GN_CHUNKS * C * 2 + C); }
hipError_t groupnorm_time_gelu(float* x, int T, int C, const float* gamma, const float* beta, float eps,
                               double* ws, hipStream_t s, int B = 1);
// HuBERT conv_layers.0 fused: y[b][t][c] = GELU(GroupNorm_c(sum_k w10[c][k] x[b ldx + 5t + k])), T rows, C % 64 == 0,
// C <= 1024, y 16-byte aligned; ws as above (aux_kernels.hip)
hipError_t hubert_conv0_gn_gelu(const float* x, long long ldx, const float* w10, int T, int C, const float* gamma,
                                const float* beta, float eps, double* ws, float* y, hipStream_t s, int B = 1);
hipError_t act_inplace(float* x, long long n, int act, float slope, hipStream_t s);
hipError_t reflect_pad_1d(const float* x, int n, int pad_l, int pad_r, float* y, hipStream_t s, int B = 1,
                          long long ldx = 0, long long ldy = 0);
hipError_t reflect_pad_rows(const float* x, int rows, int C, int pad_r, float* y, hipStream_t s, int B = 1);
hipError_t stft_magnitude(const float* spec, int F, int nbins, float* mag, int ldm, hipStream_t s);
hipError_t affine_inplace(float* x, long long n, float a, float b, hipStream_t s);
hipError_t avgpool2(const float* x, int H, int W, int C, int ldx, float* y, hipStream_t s);
hipError_t nhwc_to_hcw(const float* x, int H, int W, int C, float* y, hipStream_t s);
// B independent sequences (gi [B][T][1536], out [B][T][512], xchg gru_xchg_words(B) words); next_tag: the
// hand-off tag counter of this xchg buffer, owned by the caller (0 = buffer state unknown: zeroed first)
hipError_t gru_bidir(const float* gi, const float* whh_f, const float* bhh_f, const float* whh_b,
                     const float* bhh_b, int T, float* out, unsigned long long* xchg, unsigned* status,
                     unsigned* next_tag, hipStream_t s, int B = 1);
inline size_t gru_xchg_words(int B) { return (size_t)B * 4 * 2 * 128; }
// B sequences: sal rows of sequence b start at b*Fs (Fs = F when 0), f0 [B][F]
hipError_t rmvpe_decode(const float* sal, int F, int ncls, float thred, double* f0, hipStream_t s, int B = 1,
                        int Fs = 0);
hipError_t f0_post(const double* f0, int F, double shift, int32_t* coarse, float* pitchf, double* f0_out,
                   hipStream_t s);

// pipeline DSP
constexpr int IIR_MAXO = 8;
hipError_t filtfilt_pad(const double* x, long long n, const double* b, const double* a, const double* zi,
                        const double* FL, int order, long long t_pad, double* ws, double* pad64, float* pad32,
                        hipStream_t s);
size_t filtfilt_ws_doubles(long long n, int order);
// dst row b = src row b / (max|src row b| / 0.99) when that exceeds 1, else a copy (src == dst: in place)
hipError_t peak_normalize(const float* src, float* dst, long long n, float* ws, hipStream_t s, int B = 1,
                          long long lds = 0, long long ldd = 0);
size_t peak_normalize_ws_floats(int B);
// Pipeline.get_f0 / Pipeline.pipeline host DSP moved on device (aux_kernels.hip)
hipError_t f0_autotune(double* f0, int F, double strength, int skip_unvoiced, hipStream_t s);
hipError_t split_points(const double* x, long long n, int window, long long t_center, long long t_query,
                        double* sum_ws, long long* ts, int nts, hipStream_t s);
int rms_frame_count(long long n, int sr);
// fp64 frame RMS (librosa.feature.rms, center=True, constant pad): nframes = 1 + (n + 2*(frame/2) - frame)/hop
hipError_t rms_frames_f64(const double* x, long long n, int frame, int hop, double* rms, int nframes, hipStream_t s);
hipError_t change_rms(const double* src, long long n_src, int sr_src, float* y, long long n_y, int sr_y, float rate,
                      float* ws, hipStream_t s);

// FAISS IndexIVFFlat on device (ivf.hip): search + the retrieval blend of pipeline.py:378-388
struct IvfView {
  int d = 0, nprobe = 1;
  long long nlist = 0, ntotal = 0;
  const float* cent = nullptr;       // [nlist][d]
  const float* vecs = nullptr;       // [ntotal][d], list order
  const long long* off = nullptr;    // [nlist + 1]
  const long long* ids = nullptr;    // [ntotal], list order
  const int* slot_of_id = nullptr;   // [ntotal]
};
constexpr int IVF_MAX_K = 16;
size_t ivf_ws_floats(long long n, long long nlist, int nprobe);
// dist_out/ids_out [n][k] (optional); out [n][d] = retrieval blend (optional)
hipError_t ivf_search(const IvfView& v, const float* x, long long n, int k, float* dist_out, long long* ids_out,
                      float rate, float one_minus_rate, float* out, float* ws, hipStream_t s);

// streaming (stream.hip): B streams of one geometry per launch
hipError_t rt_resample(const float* x, long long ldx, int n_in, const float* ker, int K, int width, int orig, int nw,
                       float* y, long long ldy, int n_out, const float* pre, int B, hipStream_t s);
hipError_t rt_ingest(const float* in16, int n16, const float* abuf_old, float* abuf_new, int na, const float* cbuf_old,
                     float* cbuf_new, int nc, double sensitivity, float* vol, float* volsq, int* gate, int B,
                     hipStream_t s);
hipError_t rt_pitch(const double* f0, int F, const double* factor, const int* pold, int* pnew, const float* fold,
                    float* fnew, int nbuf, int B, hipStream_t s);
hipError_t rt_up2(const float* feats, const float* feats0, int L, int D, float* phone, int T, const float* pitchf_buf,
                  int nbuf, float pscale, float protect, int use_protect, int* pitch_out, const int* pitch_buf,
                  float* pitchf_out, int B, hipStream_t s);
hipError_t rt_clip(float* x, long long ld, int n, int B, hipStream_t s);
hipError_t rt_sola(const float* audio, long long lda, const float* volsq, const int* gate, float* sola_buf, int cf,
                   int search, const float* fade_in, float* out, int block, int* offs, int B, hipStream_t s);
hipError_t change_rms_f32src(const float* src, long long n_src, int sr_src, float* y, long long n_y, int sr_y,
                             float rate, float* ws, hipStream_t s);

// second-order-section filtfilt (iir_scan.hip): per-section tables in one device buffer
struct SosPlan {
  int nsec = 0, L = 256;
  const double* dev = nullptr;  // nsec x stride doubles: coef[0..4] @0, w[2] @8, pow[11][4] @16, CA[L][2] @64
  const double* casc = nullptr;  // the cascade as one system (iir_scan.hip casc_filtfilt_pad), chunks of casc_L
  int casc_L = 128;
  int stride() const { return 64 + 2 * L; }
  const double* coef(int j) const { return dev + (size_t)j * stride(); }
  const double* w(int j) const { return coef(j) + 8; }
  const double* pow(int j) const { return coef(j) + 16; }
  const double* ca(int j) const { return coef(j) + 64; }
};
// filtfilt over the odd-extended input ext [ne] as two passes of the whole cascade (p.casc), trimmed and reflect-padded
hipError_t casc_filtfilt_pad(const SosPlan& p, const double* ext, long long ne, int padlen, long long n,
                             long long t_pad, double* ws, double* pad64, float* pad32, hipStream_t s);
size_t casc_ws_doubles(long long ne, int L);
// filtfilt (odd padding 3*(order+1)) through the SOS plan + reflect pad t_pad (pipeline.py:439, :459)
hipError_t filtfilt_sos_pad(const SosPlan& p, int order, const double* x, long long n, long long t_pad, double* ws,
                            double* pad64, float* pad32, hipStream_t s);
size_t filtfilt_sos_ws_doubles(long long n, int order, int L);

}  // namespace rvcx
