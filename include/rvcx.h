/*
 * rvcx — MI355X-native RVC v2 inference engine: public C ABI.
 *
 * Plain pointers and sizes only. All d_* pointers are device (HBM) pointers owned by the
 * caller (e.g. torch tensors' data_ptr()); every compute call is asynchronous on the given
 * hipStream_t (passed as void*; NULL = the null stream). The context owns the uploaded
 * weights, the workspace and the RNG state; one context = one device, one host thread at a
 * time. Every function returns an rvcx_status (0 = ok, < 0 = error); the message of the
 * last error is rvcx_last_error(ctx). Nothing prints and continues.
 *
 * The reference (Acelogic/Retrieval-based-Voice-Conversion-MLX) has no native code on this
 * path; each entry point below replaces a Python-level interface of the reference, cited
 * file:line (paths relative to the reference root).
 */
#ifndef RVCX_H_
#define RVCX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rvcx_ctx rvcx_ctx;

typedef enum {
  RVCX_OK = 0,
  RVCX_E_INVALID = -1, /* bad argument (null pointer, negative size, unknown name) */
  RVCX_E_SHAPE = -2,   /* tensor shape / length does not match the model */
  RVCX_E_HIP = -3,     /* HIP runtime error or kernel launch failure */
  RVCX_E_OOM = -4,     /* device allocation failed */
  RVCX_E_STATE = -5,   /* model not finalized / weights missing */
  RVCX_E_CAPACITY = -6 /* caller's output buffer too small */
} rvcx_status;

typedef enum { RVCX_MODEL_SYNTH = 0, RVCX_MODEL_HUBERT = 1, RVCX_MODEL_RMVPE = 2, RVCX_MODEL_CREPE = 3 } rvcx_model;

/* Synthesizer hyper-parameters = the 18-element ``cpt["config"]`` list of an RVC .pth
 * (rvc/train/process/extract_model.py:62-81) plus text_enc_hidden_dim (768 for v2). */
typedef struct {
  int inter_channels, hidden_channels, filter_channels, n_heads, n_layers, kernel_size;
  int n_resblocks;                  /* len(resblock_kernel_sizes) (3) */
  int resblock_kernel_sizes[4];
  int resblock_dilation_sizes[4][4];
  int n_dilations;                  /* len of each dilation list (3) */
  int n_upsample;                   /* len(upsample_rates) (4) */
  int upsample_rates[8];
  int upsample_initial_channel;
  int upsample_kernel_sizes[8];
  int spk_embed_dim, gin_channels, sr, text_enc_hidden_dim;
  int no_f0;   /* 1: model without pitch guidance (cpt["f0"] == 0): TextEncoder without emb_pitch and the plain
                  HiFiGANGenerator (synthesizers.py:84, :122-139, :233-239; generators/hifigan.py:9-104) */
  int vocoder; /* decoder of a pitch-guided model (cpt["vocoder"], infer.py:478): 0 "HiFi-GAN" (NSF),
                  1 "MRF HiFi-GAN", 2 "RefineGAN" (synthesizers.py:86-118) */
} rvcx_synth_desc;

/* Create a context on HIP device `device`. */
int rvcx_create(rvcx_ctx** out, int device);
int rvcx_destroy(rvcx_ctx* ctx);
const char* rvcx_last_error(const rvcx_ctx* ctx);

/* Model structure (replaces Synthesizer(*cpt["config"]) in rvc/infer/infer.py:467-488 and
 * the hard-coded defaults of rvc_mlx/infer/infer_mlx.py:130-244). */
int rvcx_set_synth_config(rvcx_ctx* ctx, const rvcx_synth_desc* desc);

/* Weight ingestion: one fp32 host tensor in the REFERENCE layout under its REFERENCE
 * state-dict name (weight-norm already fused to ``.weight``; BatchNorm as its 4 tensors).
 * Replaces load_state_dict in rvc/infer/infer.py:480-486 (synth), HubertModel
 * from_pretrained in rvc/lib/utils.py:125-153 (hubert), RMVPE0Predictor.__init__
 * torch.load in rvc/lib/predictors/RMVPE.py:429-434 (rmvpe). */
int rvcx_upload(rvcx_ctx* ctx, int model, const char* name, const float* host, const int64_t* shape, int ndim);
/* Validate names/shapes, fold BatchNorm, repack to kernel layouts, copy to HBM. */
int rvcx_finalize(rvcx_ctx* ctx, int model);

/* HuBERT/ContentVec: hubert_model(audio[1,N])["last_hidden_state"] -> [L][768] (v2) or final_proj
 * [L][256] (v1). Replaces transformers HubertModel.forward as called at rvc/infer/pipeline.py:331-334
 * and rvc_mlx/lib/mlx/hubert.py:174-201 (pipeline_mlx.py:172-173). */
int rvcx_hubert(rvcx_ctx* ctx, const float* d_audio, int64_t n, int version, float* d_feats, int64_t cap_rows,
                int64_t* rows_out, void* stream);

/* RMVPE: RMVPE0Predictor.infer_from_audio(audio, thred) -> f0 (fp64, [F], F = 1 + n/160).
 * Replaces rvc/lib/predictors/RMVPE.py:497-513 and rvc_mlx/lib/mlx/rmvpe.py:408-412.
 * d_hidden (optional, [F][360] fp32) receives the salience (mel2hidden output). */
int rvcx_rmvpe(rvcx_ctx* ctx, const float* d_audio, int64_t n, float thred, double* d_f0, int64_t cap_frames,
               int64_t* frames_out, float* d_hidden, void* stream);

/* Batched forms over B equal-length inputs (rows of stride lda floats; HuBERT needs lda % 5 == 0 when B > 1):
 * feats [B][L][D] and f0 [B][F] (d_hidden [B][F][360]) back to back. Used by the streaming path (B streams
 * per hop) and the batched offline mode; each sequence's result equals the unbatched call's. */
int rvcx_hubert_batch(rvcx_ctx* ctx, const float* d_audio, int64_t n, int64_t lda, int B, int version, float* d_feats,
                      int64_t cap_rows, int64_t* rows_out, void* stream);
int rvcx_rmvpe_batch(rvcx_ctx* ctx, const float* d_audio, int64_t n, int64_t lda, int B, float thred, double* d_f0,
                     int64_t cap_frames, int64_t* frames_out, float* d_hidden, void* stream);

/* CREPE (f0 methods "crepe" / "crepe-tiny"): CREPE.get_f0(audio, f0_min, f0_max, threshold) of
 * rvc_mlx/lib/mlx/crepe.py:282-325 (the torchcrepe network of rvc/lib/predictors/f0.py:25-57; MLX dispatch
 * rvc_mlx/lib/mlx/pitch_extractors.py:155-156). Weights: RVCX_MODEL_CREPE under torchcrepe's names (conv1..6 +
 * _BN, classifier), full or tiny by conv1's filter count. d_audio [n] fp32 @16 kHz (n > 512) -> d_f0 [F] fp32,
 * F = 1 + n/160; d_periodicity ([F], filtered) and d_probs ([F][360], the sigmoid outputs) are optional. */
int rvcx_crepe(rvcx_ctx* ctx, const float* d_audio, int64_t n, float f0_min, float f0_max, float threshold,
               float* d_f0, float* d_periodicity, float* d_probs, int64_t cap_frames, int64_t* frames_out,
               void* stream);

/* rvcx_crepe with a choice of semantics: 0 = as rvcx_crepe (the MLX port's CREPE.get_f0); 1 = rvc/'s CREPE.get_f0
 * (rvc/lib/predictors/f0.py:31-55): torchcrepe.predict's framing (zero padding of 512, unbiased std), its default
 * viterbi decoder (torchcrepe.decode.viterbi: the sigmoid outputs outside [f0_min, f0_max] masked, softmax over the
 * bins, librosa.sequence.viterbi with the +-11-bin triangular transition matrix), periodicity = the output at the
 * decoded bin, then torchcrepe.filter.median(periodicity, 3), filter.mean(f0, 3) and f0 = 0 where the periodicity <
 * threshold. torchcrepe dithers the decoded cents with scipy.stats.triang noise on [-20, 20] cents: d_dither [F]
 * (optional, semantics 1 only) supplies it, NULL decodes without. torchcrepe / librosa are not importable here: the
 * restatement follows their published source (parity unpinned; tests/test_gpu_crepe.py checks it against
 * oracle/crepe.py's numpy restatement). Any n > 0. In rvcx_pipeline_opts: f0_method 2 (no dither). */
int rvcx_crepe_ex(rvcx_ctx* ctx, const float* d_audio, int64_t n, float f0_min, float f0_max, float threshold,
                  int semantics, const float* d_dither, float* d_f0, float* d_periodicity, float* d_probs,
                  int64_t cap_frames, int64_t* frames_out, void* stream);
/* The decode alone (the tail of rvcx_crepe_ex after the network: CREPE._decode + filters for semantics 0,
 * torchcrepe's viterbi + rvc/'s filters for 1) on caller-given probabilities d_probs [F][360]. */
int rvcx_crepe_decode(rvcx_ctx* ctx, const float* d_probs, int64_t F, float f0_min, float f0_max, float threshold,
                      int semantics, const float* d_dither, float* d_f0, float* d_periodicity, void* stream);

/* split_audio.process_audio (rvc/lib/tools/split_audio.py:5-27; rvc/infer/infer.py:282-284): the non-silent
 * intervals librosa.effects.split(audio, top_db=-silence_thresh_db, frame_length=int(min_silence_len_ms/1000*sr),
 * hop_length=frame_length//2) returns. d_audio [n] fp64 on device; intervals (HOST [cap][2] int64, start/end
 * samples) receives *count of them; the call synchronises the stream (the edges are host logic over the frame
 * RMS computed on device). RVCX_E_CAPACITY when more than cap intervals. */
int rvcx_split_audio(rvcx_ctx* ctx, const double* d_audio, int64_t n, int sr, double silence_thresh_db,
                     int min_silence_len_ms, int64_t* intervals, int64_t cap, int64_t* count, void* stream);

/* RMVPE0Predictor.decode (rvc/lib/predictors/RMVPE.py:515-540; rvc_mlx/lib/mlx/rmvpe.py:357-406):
 * salience [F][360] fp32 -> f0 [F] fp64 (argmax, +-4-bin weighted cents, threshold, 10 * 2^(c/1200), 10 -> 0). */
int rvcx_rmvpe_decode(rvcx_ctx* ctx, const float* d_hidden, int64_t F, float thred, double* d_f0, void* stream);

/* f0 post-processing of Pipeline.get_f0 (rvc/infer/pipeline.py:278-291): f0 *= 2^(semitones/12),
 * mel quantisation to coarse 1..255. Writes coarse (int32), pitchf (fp32) and shifted f0 (fp64, optional). */
int rvcx_f0_post(rvcx_ctx* ctx, const double* d_f0, int64_t F, double semitones, int32_t* d_coarse, float* d_pitchf,
                 double* d_f0_shifted, void* stream);

/* Autotune.autotune_f0 in place (rvc/infer/pipeline.py:151-162; rvc_mlx/infer/pipeline_mlx.py:72-80):
 * f0 += (nearest note - f0) * strength. skip_unvoiced = 1 leaves f0 <= 0 frames untouched (MLX). */
int rvcx_f0_autotune(rvcx_ctx* ctx, double* d_f0, int64_t F, double strength, int skip_unvoiced, void* stream);

/* Synthesizer.infer (rvc/lib/algorithm/synthesizers.py:206-243; rvc_mlx/lib/mlx/synthesizers.py:193-235).
 * For a model without pitch guidance (no_f0) d_pitch / d_pitchf may be NULL and are ignored (:233-239); the
 * same holds for d_f0 of rvcx_dec_only and d_pitch / d_pitchf of rvcx_voice_conversion.
 * phone [B][T][E], lengths [B], pitch [B][T], pitchf [B][T], sid [B] -> out [B][T*upp].
 * Source noise layout by decoder: HiFi-GAN (NSF) [B][T*upp] (randn_like, generators/hifigan.py:223); MRF HiFi-GAN
 * [B][T*upp][9] (randn_like(sine_waves), hifigan_mrf.py:222) followed by the [B][9] initial phases (torch.rand,
 * :174-178, element 0 of each row unused); RefineGAN [B][T*upp] (randn_like, refinegan.py:233) then [B][1]
 * (torch.rand, :203) then, per upsampling stage and ParallelResBlock branch j = 0..2, the AdaIN draws (in, out)
 * [B][C_stage][T_stage] each (refinegan.py:90); no source for models without pitch guidance.
 * d_eps_z ([B][I][T], reference layout of randn_like(m_p)) and d_eps_src ([B][T*upp], randn_like at
 * generators/hifigan.py:223) are optional injected noise; when NULL the noise is drawn from the
 * context's Philox stream keyed by `seed`. d_zp / d_z (optional, [B][T][I]) receive z_p and z. */
int rvcx_synth_infer(rvcx_ctx* ctx, int B, int T, const float* d_phone, const int32_t* d_lengths,
                     const int32_t* d_pitch, const float* d_pitchf, const int32_t* d_sid, const float* d_eps_z,
                     const float* d_eps_src, uint64_t seed, float* d_out, float* d_zp, float* d_z, void* stream);
/* Synthesizer.infer with its remaining arguments and full return value (synthesizers.py:206-243): rate (the partial
 * re-synthesis of :230-234; < 0 = None) keeps z_p, x_mask and nsff0 [:, head:] before the flow with the reference's
 * head = int(T (1 - rate)) and Python's slice semantics: a negative head (rate > 1) keeps the last -head frames (all T
 * when -head >= T); a rate that keeps no frame (rate 0) is RVCX_E_SHAPE. d_out holds [B][T' upp] and d_zp / d_z
 * [B][T'][I] with T' the kept frames; *t_out = T'.
 * d_m_p / d_logs_p (optional) [B][T][I] receive the TextEncoder's m_p / logs_p (the rest of the tuple :243). Noise as
 * rvcx_synth_infer (d_eps_z over all T frames, d_eps_src over the T - head synthesized ones). */
int rvcx_synth_infer_ex(rvcx_ctx* ctx, int B, int T, const float* d_phone, const int32_t* d_lengths,
                        const int32_t* d_pitch, const float* d_pitchf, const int32_t* d_sid, double rate,
                        const float* d_eps_z, const float* d_eps_src, uint64_t seed, float* d_out, float* d_zp,
                        float* d_z, float* d_m_p, float* d_logs_p, int* t_out, void* stream);

/* HiFiGAN-NSF generator alone (config C3): dec(z, f0, g=emb_g(sid)) with z in reference layout
 * [B][I][T] (rvc/lib/algorithm/generators/hifigan_nsf.py:173-212). out [B][T*upp]. */
int rvcx_dec_only(rvcx_ctx* ctx, int B, int T, const float* d_z, const float* d_f0, const int32_t* d_sid,
                  const float* d_eps_src, uint64_t seed, float* d_out, void* stream);

/* Pipeline.voice_conversion on one padded chunk (rvc/infer/pipeline.py:293-376;
 * rvc_mlx/infer/pipeline_mlx.py:166-261): HuBERT -> [speaker-embedding retrieval from the loaded
 * feature index when index_rate > 0] -> x2 nearest upsample -> protect blend -> Synthesizer.infer,
 * all on device. d_audio [n] @16 kHz (already filtered and padded); d_pitch/d_pitchf [>= n/160].
 * Output out [p_len*upp], p_len = min(n/160, 2L). */
int rvcx_voice_conversion(rvcx_ctx* ctx, const float* d_audio, int64_t n, const int32_t* d_pitch,
                          const float* d_pitchf, int sid, float protect, double index_rate, const float* d_eps_z,
                          const float* d_eps_src, uint64_t seed, float* d_out, int64_t cap, int64_t* n_out,
                          void* stream);

/* Pipeline high-pass (rvc/infer/pipeline.py:22-27: signal.butter(5, 48, 'high', fs=16000)) as
 * transfer-function coefficients b[order+1], a[order+1] and lfilter_zi(b, a) zi[order]; used by
 * rvcx_pipeline's zero-phase filtfilt (padtype 'odd', padlen 3*(order+1)). */
int rvcx_set_highpass(rvcx_ctx* ctx, const double* b, const double* a, const double* zi, int order);

/* The same high-pass as second-order sections sos[nsec][6] = (b0 b1 b2 a0 a1 a2) per section (scipy
 * butter(5, 48, 'high', fs=16000, output='sos'): exact zpk sections). When set, filtfilt runs as a
 * chunk-parallel scan over the sections (stable: each section's 2x2 state matrix is well conditioned, unlike
 * the order-5 companion form). Call after rvcx_set_highpass (which sets the padding length). */
int rvcx_set_highpass_sos(rvcx_ctx* ctx, const double* sos, int nsec);
/* signal.filtfilt(bh, ah, audio) then np.pad(..., (t_pad, t_pad), 'reflect') (pipeline.py:439, :459):
 * d_audio [n] fp64 -> d_pad64 (optional) / d_pad32 [n + 2 t_pad]. */
int rvcx_highpass_pad(rvcx_ctx* ctx, const double* d_audio, int64_t n, int64_t t_pad, double* d_pad64, float* d_pad32,
                      void* stream);

/* Options of Pipeline.pipeline (rvc/infer/pipeline.py:390-408; rvc_mlx/infer/pipeline_mlx.py:263) that
 * reach the device path. Fill with rvcx_pipeline_default_opts, then override. Times are in samples. */
typedef struct {
  int sid;                          /* speaker id (emb_g row) */
  int version;                      /* 0 = from the synthesizer (768-d -> v2, 256-d -> v1), or 1 / 2 */
  double pitch;                     /* semitones, f0 *= 2^(pitch/12) (pipeline.py:278-279) */
  float protect;                    /* consonant protection, active when < 0.5 (pipeline.py:350-362) */
  float rmvpe_threshold;            /* decode threshold (0.03, pipeline.py:237) */
  int64_t t_pad, t_pad_tgt;         /* x_pad * 16000 and x_pad * tgt_sr (pipeline.py:176-177) */
  int64_t t_query, t_center, t_max; /* x_query/x_center/x_max * 16000: long-input split search (:440-452);
                                       t_max = 0 disables splitting */
  int f0_autotune;                  /* Autotune.autotune_f0 (pipeline.py:151-162, :248-249) */
  double f0_autotune_strength;
  int proposed_pitch;               /* key offset from the median f0 (pipeline.py:250-277) */
  double proposed_pitch_threshold;
  double volume_envelope;           /* AudioProcessor.change_rms rate; 1 = off (pipeline.py:545-549) */
  int mlx_semantics;                /* 1: f0 adjustments as rvc_mlx PipelineMLX.get_f0 (pipeline_mlx.py:135-164):
                                       autotune skips f0 <= 0 and the pitch shift is applied after it */
  double index_rate;                /* speaker-embedding retrieval blend (pipeline.py:338-342, :378-388); 0 = off;
                                       > 0 needs rvcx_index_load */
  int f0_method;                    /* 0 = RMVPE (default), 1 = CREPE with the loaded RVCX_MODEL_CREPE weights
                                       (PitchExtractor.extract, pitch_extractors.py:155-156; f0_min 50, f0_max
                                       1100, threshold 0.1), 2 = CREPE as rvc/ runs it (pipeline.py:223-234;
                                       rvcx_crepe_ex semantics 1, without the dither) */
} rvcx_pipeline_opts;

/* Defaults of the rvc/ Config (x_pad 1, x_query 6, x_center 38, x_max 41; rvc/configs/config.py) at
 * 48 kHz, protect 0.33, volume_envelope 1. */
int rvcx_pipeline_default_opts(rvcx_pipeline_opts* opts);

/* Pipeline.pipeline, all on device (rvc/infer/pipeline.py:390-558 with pitch_guidance and
 * index_rate 0; rvc_mlx/infer/pipeline_mlx.py:263-373): filtfilt(audio) -> reflect pad t_pad -> RMVPE
 * -> get_f0 adjustments -> [split at the quietest points near every t_center when the input exceeds
 * t_max] -> voice_conversion per chunk -> trim t_pad_tgt per side -> concatenate -> change_rms ->
 * peak-normalise. d_audio [n] fp64 @16 kHz; out fp32 @tgt_sr, n_out samples (cap >=
 * ((n + 2 t_pad)/160 + n/t_center + 2) * upp is always enough). d_eps_z / d_eps_src (optional)
 * hold the injected noise of all chunks back to back ([192][T_i] then [T_i * upp] per chunk);
 * d_f0 (optional) receives the adjusted f0 [1 + (n + 2 t_pad)/160]. The host synchronises the
 * stream once to read the split points (long inputs only) and once for proposed_pitch. */
int rvcx_pipeline_ex(rvcx_ctx* ctx, const double* d_audio, int64_t n, const rvcx_pipeline_opts* opts,
                     const float* d_eps_z, const float* d_eps_src, uint64_t seed, float* d_out, int64_t cap,
                     int64_t* n_out, double* d_f0, void* stream);

/* Batched offline conversion (config C4): B equal-length utterances (each n + 160 <= t_max, i.e. one chunk),
 * d_audio row b at d_audio + b*lda (fp64 @16 kHz), sids host [B]. Every stage runs once for the whole batch
 * (batched RMVPE, HuBERT and Synthesizer.infer); row b of d_out (stride ldo) receives Pipeline.pipeline's
 * output for utterance b, n_out samples. Noise when injected: d_eps_z [B][inter][T], d_eps_src [B][T*upp].
 * Optional outputs: d_f0 [B][F] the adjusted f0 of each row (as rvcx_pipeline_ex's d_f0), d_hidden [B][F][360] the
 * RMVPE salience each row's f0 was decoded from (RMVPE f0 method only), F = 1 + (n + 2 t_pad)/160. */
int rvcx_pipeline_batch(rvcx_ctx* ctx, const double* d_audio, int64_t n, int64_t lda, int B,
                        const rvcx_pipeline_opts* opts, const int32_t* sids, const float* d_eps_z,
                        const float* d_eps_src, uint64_t seed, float* d_out, int64_t ldo, int64_t* n_out,
                        double* d_f0, float* d_hidden, void* stream);

/* Single-chunk shorthand of rvcx_pipeline_ex (t_max = 0, defaults otherwise). */
int rvcx_pipeline(rvcx_ctx* ctx, const double* d_audio, int64_t n, int sid, double semitones, float protect,
                  int64_t t_pad, int64_t t_pad_tgt, const float* d_eps_z, const float* d_eps_src, uint64_t seed,
                  float* d_out, int64_t cap, int64_t* n_out, double* d_f0, void* stream);

/* Device workspace (SURVEY.md 8(b) "Ownership"; replaces nothing in the reference, whose MLX / torch allocators own
 * all scratch). Every intermediate of a call (activations, split-K slabs, filter state, attention partials ...) lives
 * in the context's named pool, allocated on first use and kept across calls; the weights and their pre-split images
 * are not part of it.
 * rvcx_workspace_bytes: the pool a pipeline call of B utterances of n samples under opts takes (B = 1 as
 *   rvcx_pipeline_ex, B > 1 as rvcx_pipeline_batch). It runs that call once on zero audio on `stream` from an empty
 *   pool (loaded models required; outputs discarded) and reports every region the pool took, regrown ones included,
 *   so an arena of that size holds the call; the pool is released again before it returns. Inputs above t_max are
 *   sized on the worst-case split plan (the longest chunk any audio can give: the pipeline processes its chunks
 *   longest first, so the work buffers grow only inside the first chunk), so the size holds for any audio of n samples.
 * rvcx_set_workspace: hand the context a caller-owned device arena (e.g. a torch uint8 tensor's data_ptr(), 256-B
 *   aligned), valid until replaced or the context is destroyed: the pool is then carved from it and never allocated,
 *   and a call that would need more fails with RVCX_E_OOM. NULL, 0 returns to internal allocation. The current pool
 *   is released first (the device is synchronised). While attached the arena belongs to the library: every compute
 *   call carves its regions from offset 0 again (a sized arena then holds any sequence of calls each of which it
 *   holds alone), and nothing is assumed to survive between calls, so a caller's writes into the arena between calls
 *   cannot change results -- but they must be stream-ordered after the previous call's work.
 * rvcx_workspace_info: bytes the pool holds now, the arena size and the arena bytes carved so far (any may be NULL). */
int rvcx_workspace_bytes(rvcx_ctx* ctx, int B, int64_t n, const rvcx_pipeline_opts* opts, int64_t* bytes,
                         void* stream);
int rvcx_set_workspace(rvcx_ctx* ctx, void* d_base, int64_t bytes);
int rvcx_workspace_info(const rvcx_ctx* ctx, int64_t* held, int64_t* arena_bytes, int64_t* arena_used);

/* Kernel timing for roofline reporting: when enabled, every implicit-GEMM conv launch (the MFMA
 * kernel family that carries ~all FLOPs) is bracketed by hipEvents recorded on its own stream.
 * rvcx_profile_read synchronises those events and returns the summed kernel time (ms), the
 * summed ALGORITHMIC FLOPs of those launches and the launch count, then clears the record. */
int rvcx_profile(rvcx_ctx* ctx, int enable);

/* Synchronise `stream` (and the context's internal side stream) and report device-side faults raised by
 * kernels of earlier calls: RVCX_E_HIP when, e.g., the RMVPE BiGRU's cross-workgroup hand-off timed out (its
 * outputs are then invalid). The flags are cleared once reported. Every compute entry point also reports
 * flags of already-completed calls on entry, and the pipeline checks them at its own synchronisation points.
 * (Replaces nothing in the reference, whose computations cannot fail this way; it never prints and continues.) */
int rvcx_device_status(rvcx_ctx* ctx, void* stream);
int rvcx_profile_read(rvcx_ctx* ctx, double* total_ms, double* total_flops, int64_t* launches);
/* As rvcx_profile_read, plus the launches' time at their arithmetic's MFMA ceiling (ms): sum of flops / ceiling,
 * with the ceiling 2500 / 6 TF for the exact bf16 split, 2500 / 3 for the two-plane fp16 split and 2500 for the fp16
 * reduced-precision mode (the dense bf16 / fp16 MFMA peak over the MFMA products per fp32 product). */
int rvcx_profile_read_ex(rvcx_ctx* ctx, double* total_ms, double* total_flops, int64_t* launches, double* ceiling_ms);
/* As rvcx_profile_read_ex, plus the same sums per kernel family (the kernel each launch actually ran, after routing):
 * arrays of nk entries indexed by family id (0 .. RVCX_PROF_KINDS - 1; names from rvcx_profile_kind_name), each
 * with the summed event time (ms), algorithmic FLOPs, time at the arithmetic's ceiling (ms), algorithmic HBM bytes
 * (operands read once, result written once) and launch count. A family's time includes its split-K combine. */
#define RVCX_PROF_KINDS 10
int rvcx_profile_read_kinds(rvcx_ctx* ctx, double* total_ms, double* total_flops, int64_t* launches, double* ceiling_ms,
                            int nk, double* k_ms, double* k_flops, double* k_ceiling_ms, double* k_bytes,
                            int64_t* k_launches);
const char* rvcx_profile_kind_name(int kind);

/* ---------------------------------------------------------------- feature index (FAISS IndexIVFFlat)
 * The bytes of a faiss .index file (IndexIVFFlat over IndexFlatL2, METRIC_L2, ArrayInvertedLists;
 * faiss 1.7.4 write_index layout). Replaces faiss.read_index + index.reconstruct_n(0, ntotal) at
 * rvc/infer/pipeline.py:430-434 (rvc_mlx/infer/pipeline_mlx.py:267-278). The lists, centroids and ids
 * are kept in HBM; nprobe comes from the file. ids must be a permutation of 0..ntotal-1 (RVC indexes). */
int rvcx_index_load(rvcx_ctx* ctx, const void* bytes, int64_t nbytes);
int rvcx_index_unload(rvcx_ctx* ctx);
/* Validate a faiss .index image on the host only (no context, no device): the same parser rvcx_index_load runs.
 * Fills d/ntotal/nlist/nprobe (each optional); on failure writes the message to err (err_cap bytes). Every size
 * in the file is untrusted: counts are checked against the bytes left and list sizes against ntotal. */
int rvcx_index_parse(const void* bytes, int64_t nbytes, int64_t* d, int64_t* ntotal, int64_t* nlist, int64_t* nprobe,
                     char* err, int64_t err_cap);
/* RVCX_E_STATE when no index is loaded. */
int rvcx_index_info(const rvcx_ctx* ctx, int64_t* d, int64_t* ntotal, int64_t* nlist, int64_t* nprobe);
/* faiss.extract_index_ivf(index).nprobe = nprobe (clamped to nlist). */
int rvcx_index_set_nprobe(rvcx_ctx* ctx, int64_t nprobe);
/* index.search(x, k) (IndexIVF::search, L2; used at pipeline.py:380 with k = 8): d_x [n][d] fp32 ->
 * d_dist [n][k] fp32 squared L2, d_ids [n][k] int64, ordered by (distance, id), (+inf, -1) padding. k <= 16. */
int rvcx_index_search(rvcx_ctx* ctx, const float* d_x, int64_t n, int k, float* d_dist, int64_t* d_ids,
                      void* stream);
/* index.reconstruct_n(i0, ni) -> d_out [ni][d] (big_npy rows, pipeline.py:434). */
int rvcx_index_reconstruct_n(rvcx_ctx* ctx, int64_t i0, int64_t ni, float* d_out, void* stream);
/* Pipeline._retrieve_speaker_embeddings (pipeline.py:378-388): d_feats [L][d] -> d_out [L][d] =
 * index_rate * sum_j w_j big_npy[ix_j] + (1 - index_rate) * feats, w = (1/dist)^2 normalised, k = 8,
 * with numpy/torch float32 rounding. */
int rvcx_index_retrieve(rvcx_ctx* ctx, const float* d_feats, int64_t L, int d, double index_rate, float* d_out,
                        void* stream);

/* ---------------------------------------------------------------- streaming (config C5)
 * A group of n_streams concurrent realtime streams of one buffer geometry, converted together per hop.
 * Replaces VoiceChanger / Realtime / Realtime_Pipeline of rvc/realtime/core.py:329-484 and
 * rvc/realtime/pipeline.py:99-334 (the MLX port of this path, rvc_mlx/realtime, is not functional).
 * Geometry follows VoiceChanger.__init__ + Realtime.realloc (core.py:165-216, :351-374): block =
 * read_chunk_size * 128 samples @48 kHz; convert buffer = block + sola (10 ms) + extra + crossfade
 * @16 kHz rounded up to 10 ms; skip_head = extra / 10 ms; return_length = frames - skip_head. */
typedef struct rvcx_rt rvcx_rt;

typedef struct {
  int n_streams;                  /* B streams per hop batch */
  int read_chunk_size;            /* block = read_chunk_size * 128 samples @48 kHz (callbacks.py default 192) */
  double cross_fade_overlap_size; /* seconds (default 0.1) */
  double extra_convert_size;      /* seconds (default 0.5) */
  double silent_threshold;        /* dB; hops with RMS below 10^(dB/20) output silence (core.py:58-59, :268-289) */
} rvcx_rt_desc;

typedef struct {                  /* per-hop options of VoiceChanger.on_request (core.py:453-484) */
  double f0_up_key;
  double index_rate;              /* > 0 needs rvcx_index_load; retrieval from skip_head // 2 */
  float protect;                  /* active when < 0.5 */
  double volume_envelope;         /* 1 = off */
  int f0_autotune;
  double f0_autotune_strength;
  int proposed_pitch;             /* one host sync per hop */
  double proposed_pitch_threshold;
  int gen_precision;              /* 0 (default) fp32-accurate everywhere; 1 = this hop's GENERATOR (HiFi-GAN-NSF
                                   * decoder: its weight-streamed convs and 32-channel fused ResBlock pairs) on fp16
                                   * operands with fp32 accumulation, one MFMA product per step: BASELINE C5's fp16
                                   * streaming. RMVPE, HuBERT, the TextEncoder and the flow stay fp32-accurate, and no
                                   * other entry point is affected (the setting travels with the hop, not the ctx). */
} rvcx_rt_opts;

int rvcx_rt_default_desc(rvcx_rt_desc* desc);
int rvcx_rt_default_opts(rvcx_rt_opts* opts);
/* Needs the synthesizer, HuBERT and RMVPE finalized. State lives in HBM, zero-initialised. */
int rvcx_rt_create(rvcx_ctx* ctx, const rvcx_rt_desc* desc, rvcx_rt** out);
int rvcx_rt_destroy(rvcx_ctx* ctx, rvcx_rt* rt);
/* geometry[12] = {n_streams, block48, block16, convert16, frames (p_len), skip_head, return_length,
 *                 crossfade48, sola_search48, extra48, resampled_block16, silence_front} */
int rvcx_rt_geometry(const rvcx_rt* rt, int64_t* geometry);
int rvcx_rt_reset(rvcx_ctx* ctx, rvcx_rt* rt, void* stream);
/* One hop for every stream: d_in [B][block48] fp32 @48 kHz -> d_out [B][block48] fp32 @48 kHz
 * (VoiceChanger.process_audio). sids: host [B]. d_vol (optional, device [B]) receives each stream's
 * input RMS (the `vol` of on_request); d_offs (optional, device int [B]) the SOLA offsets. Noise: d_eps_z
 * [B][inter][frames] and d_eps_src [B][frames * upp] when injected, else Philox(seed). */
int rvcx_rt_process(rvcx_ctx* ctx, rvcx_rt* rt, const float* d_in, const int32_t* sids, const rvcx_rt_opts* opts,
                    const float* d_eps_z, const float* d_eps_src, uint64_t seed, float* d_out, float* d_vol,
                    int32_t* d_offs, void* stream);

/* Contraction arithmetic of every convolution / linear / attention matmul of this context (replaces nothing in
 * the reference; torch's fp32 CPU conv is what every mode reproduces): 0 = default (3), 1 = fp32-input MFMA
 * (v_mfma_f32_32x32x2_f32, an exact fp32 fma chain at 157 TF), 2 = fp32 through an exact 3-way bf16 split of both
 * operands with the six significant plane products on bf16 MFMA (error below fp32's own rounding, 2.67x the
 * MFMA rate), 3 = as 2, except that the generator's weight-streamed convs and fused ResBlock pairs split both
 * operands into two fp16 planes (x = h + 2^-11 l, 11 significand bits each) with three plane products into two
 * fp32 accumulators (csrc/split_bf16.h; error against fp64 measured at or below the fp32-input MFMA's, 5.3x the
 * fp32 MFMA rate). Env RVCX_CONV_MATH=f32 | split | h16 sets the process default when RVCX_EXPERIMENTAL=1. */
int rvcx_set_conv_math(rvcx_ctx* ctx, int mode);

/* The effective configuration as a NUL-terminated JSON object (cap bytes; *len, optional, gets its length): the
 * context's contraction arithmetic, whether developer knobs are enabled, and every RVCX_* environment variable of the
 * process with whether it is honoured. The RVCX_* tuning / A-B switches (tile and split-K policy, kernel-path and
 * arithmetic overrides such as RVCX_CONV_MATH) are read only when RVCX_EXPERIMENTAL=1: without it they are ignored and
 * listed here as not honoured. RVCX_E_CAPACITY when cap is too small (the string is truncated). ctx may be NULL (the
 * process-wide fields only; no device is touched). */
int rvcx_config_info(const rvcx_ctx* ctx, char* buf, int64_t cap, int64_t* len);

/* Removed in round 4 (deprecated shim, kept so existing callers link): the reduced-precision generator is now a
 * per-hop setting, rvcx_rt_opts.gen_precision. Always returns RVCX_E_INVALID with a message saying so. */
int rvcx_set_generator_precision(rvcx_ctx* ctx, int precision);

/* One Conv1d forward, time-major: d_x [T][C_in], d_w [taps][N][C_in] (torch weight [N][C_in][taps] permuted),
 * d_bias [N] (optional), d_y [T_out][N]; y[t] = bias + sum_k W[k] x[t*stride - pad + k*dilation] (zero outside).
 * The kernel family behind every contraction of the path, exposed for numerics tests; replaces
 * torch.nn.Conv1d.forward as used throughout rvc/lib/algorithm (e.g. residuals.py:34-80). math as above, plus
 * 3 = the split arithmetic on the weight-streamed kernel (weights pre-split in HBM; 1-D stride-1 convs with
 * C_in % 32 == 0 and (taps - 1) * dilation <= 64, else RVCX_E_SHAPE), 4 = the split arithmetic on the gather-streamed
 * kernel (weights pre-split in HBM, A gathered per step, split-K by the size policy; C_in % 32 == 0), 5 = the
 * two-plane fp16 split on the weight-streamed kernel (rvcx_set_conv_math mode 3's generator arithmetic), 6 = its fp16
 * hi planes alone (the realtime reduced-precision mode); 5 and 6 take the shapes 3 does; 7 = the two-plane fp16 split
 * on the gather-streamed kernel (the shapes 4 takes). */
int rvcx_conv1d(rvcx_ctx* ctx, const float* d_x, int64_t T, int C_in, const float* d_w, const float* d_bias, int N,
                int taps, int dilation, int pad, int stride, int math, float* d_y, int64_t T_out, void* stream);

/* The generator's fused conv form, time-major (rvcx_conv1d's layouts, stride 1, T_out = T + 2 pad - (taps - 1)
 * dilation): y = acc(act(conv(pre(x)) + bias) + res), pre = leaky ReLU(pre_slope) when pre_act = 1 (else identity),
 * act = leaky ReLU(slope) when act = 1, res
 * optional ([T_out][N]), acc_mode 0 store, 1 y + v, 2 (y + v) / acc_div -- one ResBlock conv (residuals.py:71-80:
 * convs1 with act, convs2 with the residual and the ResBlock mean on the last pair) or one ConvTranspose phase group
 * (hifigan_nsf.py:184-199) in the two-plane fp16 split. kernel 0 = the size policy's route, 1 = the weight-streamed
 * kernel (conv_wsb.hip, the tile the policy picks), 2 = the weight-stationary kernel (conv_wst.hip: C_in = N in {64,
 * 128}, 2-3 taps, (taps - 1) dilation <= 16, else RVCX_E_SHAPE). Exposed for numerics tests; C_in % 32 == 0. */
int rvcx_conv1d_gen(rvcx_ctx* ctx, const float* d_x, int64_t T, int C_in, const float* d_w, const float* d_bias,
                    int N, int taps, int dilation, int pad, int pre_act, float pre_slope, int act, float slope,
                    const float* d_res, int acc_mode, float acc_div, int kernel, float* d_y, void* stream);

/* One 3x3 / pad-1 Conv2d forward, NHWC: d_x [H][W][C_in], d_w [9][N][C_in] (torch weight [N][C_in][3][3] permuted to
 * (kh * 3 + kw, N, C_in)), d_bias [N] (optional), d_y [H][W][N]; act 0 none, 1 ReLU. The RMVPE U-Net's conv
 * (RMVPE.py:13-57 ConvBlockRes, torch.nn.Conv2d(kernel 3, padding 1)), exposed for the numerics tests of its
 * few-channel kernels (C_in, N in {16, 32}: csrc/conv2d_small.hip) and deep levels: math 0 = the context's arithmetic
 * (the two-plane fp16 split by default), 1 = exact fp32 (v_mfma_f32_16x16x4_f32), 2 = the deep levels' windowed
 * gather-streamed kernel in the fp16 split (images at most 32 wide, C_in % 32 == 0, else RVCX_E_SHAPE). Other shapes
 * take the general 2-D path. */
int rvcx_conv2d3x3(rvcx_ctx* ctx, const float* d_x, int H, int W, int C_in, const float* d_w, const float* d_bias,
                   int N, int act, int math, float* d_y, void* stream);

/* One ConvTranspose2d(C_in, N, kernel 3, stride 2, padding 1, output_padding 1) forward, NHWC: d_x [H][W][C_in],
 * d_w [C_in][N][3][3] (the torch layout as stored), d_bias [N] (optional), d_y [2H][2W][N]; act 0 none, 1 ReLU. The
 * RMVPE U-Net decoder's up-conv (RMVPE.py ResDecoderBlock conv1, torch.nn.ConvTranspose2d), run as the pipeline runs
 * it: a 2x2-tap phase conv with 4 N virtual output columns whose epilogue scatters the phases. math 0 = the context's
 * arithmetic (the two-plane fp16 split on the gather-streamed kernel where it applies), 1 = exact fp32. Exposed for the
 * numerics tests. */
int rvcx_convtranspose2d_s2(rvcx_ctx* ctx, const float* d_x, int H, int W, int C_in, const float* d_w,
                            const float* d_bias, int N, int act, int math, float* d_y, void* stream);

/* Multi-head attention core on the fused kernel (csrc/flash_attn.hip), time-major: d_qkv [B][T][3 H] (q | k | v, head
 * h at columns h dk .. of each, H = n_heads dk), d_out [B][T][H]: per head softmax(qscale q k^T + band) v + band(p)
 * rel_v, where, with d_rel_k / d_rel_v [2 window + 1][dk] (both or neither), band adds qscale q . rel_k[j - i + window]
 * to the logit of key j of query i for |j - i| <= window and band(p) is the probabilities of those keys
 * (MultiHeadAttention.attention with window_size, rvc/lib/algorithm/attentions.py:79-185), and d_mask [B][T]
 * (optional) fills the logits of masked query-key pairs with -1e4 (:106-107). Without the relative tables it is
 * HuBERT's attention (modeling_hubert.py HubertAttention: softmax((q dk^-0.5) k^T) v). dk 64 or 96, window <= 15.
 * Exposed for the numerics tests. */
int rvcx_flash_attention(rvcx_ctx* ctx, const float* d_qkv, int B, int T, int n_heads, int dk, float qscale,
                         const float* d_rel_k, const float* d_rel_v, int window, const float* d_mask, float* d_out,
                         void* stream);

/* One ResBlock dilation pair as one fused kernel (csrc/resblock_fused.hip), time-major: d_x, d_y [B][T][C] (distinct
 * buffers), d_w1 / d_w2 [k][C][C] (torch weight [C][C][k] permuted), d_b1 / d_b2 [C]:
 *     out = conv2(lrelu(conv1_d(lrelu(x), 0.1) + b1, 0.1)) + b2 + x     (zero padding; conv2 dilation 1)
 *     acc_mode 0: y = out; 1: y = y + out; 2: y = (y + out) / acc_div
 * Replaces one iteration of ResBlock.forward (rvc/lib/algorithm/residuals.py:71-80) and MRFLayer.forward
 * (generators/hifigan_mrf.py:45-50), plus the ResBlock mean of HiFiGANNSFGenerator.forward (hifigan_nsf.py:190-207)
 * on the last pair. C in {32, 64}, odd k, (k - 1) / 2 * dilation <= 30, else RVCX_E_SHAPE. cfg bits 0-3: 0 the
 * default kernels (the k = 3, 32-channel fp16 pairs on the weight-resident form), 1 the streamed-weight kernel for
 * every shape (comparisons; bit-identical results); bits 4-5 the arithmetic: 0 the exact 3-plane bf16 split, 1 the two-plane
 * fp16 split, 2 fp16 hi planes alone (the realtime reduced-precision mode). Exposed for numerics tests and A/B timing. */
int rvcx_resblock_pair(rvcx_ctx* ctx, const float* d_x, int B, int64_t T, int C, const float* d_w1, const float* d_b1,
                       const float* d_w2, const float* d_b2, int k, int dilation, int acc_mode, float acc_div, int cfg,
                       float* d_y, void* stream);

/* Upsampling factor of the loaded synthesizer (prod(upsample_rates); net_g.dec.upp). */
int rvcx_synth_upp(const rvcx_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* RVCX_H_ */
