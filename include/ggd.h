/*
 * ggd.h -- C ABI of the MI355X-native gesture-diffusion sampler (libggd.so).
 *
 * The reference is pure Python; its drop-in boundary for the hot path is the
 * model protocol and the sampler/generator API:
 *
 *   eps = model(x_t (N,C,L) f32, t (N,) i64, wav=...)        models/model.py:12-15
 *   diffusion.p_sample_loop / ddim_sample_loop(...)           models/modules/gaussian_diffusion.py:331-529
 *   Generator.generate_sample(shape, wavs, noise, inpaint..)  models/generator.py:218-296
 *
 * Each entry point below names the reference interface it replaces.  Plain
 * pointers and sizes only.  Device pointers are HIP device addresses owned by
 * the caller (e.g. the PyTorch caching allocator); `stream` is a hipStream_t
 * (0 = legacy default stream).  The context owns weights, workspaces and
 * captured hipGraphs; nothing is allocated inside the step loop.  Its work runs
 * on a private non-blocking stream created at the device's highest priority
 * and is ordered against the caller's `stream` with events in both directions.
 * Another stream may therefore run beside it, e.g. a speech encoder for the
 * next batch.
 *
 * Error convention: every call returns 0 (GGD_OK) or a negative ggd_status;
 * ggd_last_error(ctx) returns a message for the last failure on ctx.  The
 * Python host layer maps these to the reference's exception types
 * (ValueError for unsupported options, AssertionError for shape checks,
 * RuntimeError for HIP failures) -- SURVEY.md section 8b "Error conventions".
 *
 * Threading: one ctx per (process, device); a ctx is not thread-safe.
 */
#ifndef GGD_H
#define GGD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ggd_ctx ggd_ctx;

enum ggd_status {
  GGD_OK = 0,
  GGD_IGNORED = 1,          /* ggd_load_weight: name belongs to the speech encoder */
  GGD_ERR_ARG = -1,         /* bad argument / shape (Python: AssertionError / ValueError) */
  GGD_ERR_UNSUPPORTED = -2, /* option not supported (Python: ValueError) */
  GGD_ERR_HIP = -3,         /* HIP runtime failure (Python: RuntimeError) */
  GGD_ERR_STATE = -4,       /* call out of order, e.g. sample before weights */
  GGD_ERR_NAME = -5         /* unknown or mis-shaped state_dict entry */
};

/* models/model_creation.py:133-161 -- Model.type */
enum ggd_model_type { GGD_MODEL_S2G_V2 = 0, GGD_MODEL_DEFAULT = 1, GGD_MODEL_INPAINT = 2 };
/* models/model_creation.py:72-93 -- Decoder.type */
enum ggd_decoder_type { GGD_DEC_ONEWAY = 0, GGD_DEC_TWOWAY = 1 };
/* compute dtype of the decoder GEMM operands (accumulation is always f32).
 * GGD_FP8W: bf16 activations; the Linears evaluated inside every denoise step (emb_x, the
 * attention / FFN projections of every layer, out_layers.1) are stored as OCP fp8 e4m3fn with
 * one f32 scale per output channel (amax / 448), dequantized exactly into the bf16 MFMA tiles
 * and scaled in the GEMM epilogue -- BASELINE.json configs[3] (long clip, fp8 weights).  The
 * step-invariant projections (memory K/V, blend, step MLP) stay bf16.  Generic kernels and the
 * long-clip loop; the loop runs its FFN and LayerNorm-projection GEMMs on block-scaled fp8 MFMA
 * (e4m3 activations with one e8m0 scale per 32 values) unless GGD_ROUTE_FP8_MFMA = 1. */
enum ggd_dtype { GGD_F32 = 0, GGD_BF16 = 1, GGD_FP8W = 2 };
/* models/generator.py:34-45 -- sample_alg */
enum ggd_alg { GGD_DDPM = 0, GGD_DDIM = 1 };

typedef struct ggd_desc {
  int32_t model_type;    /* ggd_model_type */
  int32_t decoder_type;  /* ggd_decoder_type */
  int32_t d_model;       /* Model.d_model (256 beat, 512 tedexp) */
  int32_t heads;         /* Decoder.heads */
  int32_t n_layers;      /* Decoder.n_layers */
  int32_t d_pose;        /* C: pose channels (123 beat) */
  int32_t seq_len;       /* L: pose window frames (40 beat) */
  int32_t speech_len;    /* Ts: speech memory tokens (31 beat); memory = 1 + Ts */
  int32_t max_batch;     /* largest N any call will use (workspaces sized once) */
  int32_t dtype;         /* ggd_dtype */
  int32_t diffusion_steps; /* Diffusion.diffusion_steps: range of original t */
} ggd_desc;

/* Create a context on `device` (hip device ordinal).
 * Replaces: create_model(...) model construction, models/model_creation.py:51-161. */
int ggd_create(int device, const ggd_desc* desc, ggd_ctx** out);

/* Destroy a context and every resource it owns. */
int ggd_destroy(ggd_ctx* ctx);

/* Message describing the last failure on ctx (never NULL). */
const char* ggd_last_error(const ggd_ctx* ctx);

/* Stage one host f32 tensor keyed by its reference state_dict name, e.g.
 * "pose_decoder.layers.0.self_attn.query.0.linear.weight".  Names under
 * "speech_encoder." return GGD_IGNORED.
 * Replaces: model.load_state_dict(chkpt["model_state_dict"]), main.py:113-115. */
int ggd_load_weight(ggd_ctx* ctx, const char* name, const float* host_data, int64_t numel);

/* Check that every decoder weight is present, upload them in the compute
 * dtype and precompute the step-token tables for all original t. */
int ggd_finalize_weights(ggd_ctx* ctx);

/* Install a diffusion schedule: the respaced betas (fp64, length T) and the
 * respaced->original timestep map.  Coefficient tables are derived in fp64 and
 * rounded to f32 exactly as _extract_into_tensor does.
 * Replaces: GaussianSpacedDiffusion.__init__, respace.py:80-93 +
 *           GaussianDiffusion.__init__, gaussian_diffusion.py:87-143. */
int ggd_set_schedule(ggd_ctx* ctx, const double* betas, int32_t T, const int64_t* timestep_map);

/* Install the step-invariant speech memory of N clips: device f32
 * (N, Ts, dz) with dz = 3*d_model (s2g_v2: the left-zero-padded concat of
 * z_low|z_mid|z_high; the blend layer runs here) or dz = d_model (default:
 * tokens already concatenated on time).  Computes emb_mem + PE and the
 * cross-attention K/V projections once per clip.
 * Replaces: Speech2GestureModelV2.myforward memory assembly, models/model.py:93-112
 * (there recomputed on every denoise step). */
int ggd_set_memory(ggd_ctx* ctx, const float* speech_tokens, int32_t n, int32_t ts, int32_t dz,
                   void* stream);

/* Inpaint conditioning of a GGD_MODEL_INPAINT context: poses device f32 (N, L, C), masks device f32
 * (N, L) (1 = seed frame).  Computes proj([pose*mask, mask]) = Linear(C+1 -> d) SiLU Linear(d -> d)
 * SiLU Linear(d -> C) once; every following ggd_denoise / ggd_sample adds it to x_t before the
 * decoder.  poses == NULL clears it (the model then sees x_t alone, i.e. an all-zero projection
 * input is NOT assumed).  Step-invariant, like the speech memory.
 * Replaces: Speech2GestureModelInpaint.myforward, models/model.py:152-166 (there recomputed on every
 * denoise step). */
int ggd_set_inpaint(ggd_ctx* ctx, const float* poses, const float* masks, int32_t n, void* stream);

/* Model protocol: eps = model(x_t, t).  x_t, eps: device f32 (N, C, L);
 * t: device int32 (N,) ORIGINAL timesteps; N = the batch given to ggd_set_memory.
 * Replaces: Speech2GestureModelBase.forward, models/model.py:12-15. */
int ggd_denoise(ggd_ctx* ctx, const float* x_t, const int32_t* t, float* eps, int32_t n, void* stream);

/* One reverse-diffusion update without the model call, for a caller-supplied
 * denoise_fn: given eps and the (possibly replaced) x0 of respaced step i,
 * writes x_{i-1}.  If x0 == NULL it is predicted from eps.  All (N,C,L) f32.
 * Replaces: p_sample :300-329 / ddim_sample :443-484 after p_mean_variance. */
int ggd_posterior_step(ggd_ctx* ctx, int32_t alg, float eta, int32_t i, const float* x,
                       const float* eps, const float* x0, const float* noise, float* x_out,
                       float* x0_out, int32_t n, void* stream);

typedef struct ggd_sample_args {
  int32_t alg;            /* ggd_alg */
  float eta;              /* DDIM eta (0 in the reference) */
  int32_t n;              /* clips in this call (<= max_batch) */
  const float* x_T;       /* device (N,C,L) initial noise; NULL = draw from the counter stream */
  const float* noise;     /* device (T',N,C,L) per-step noise in loop order; NULL = counter stream */
  uint64_t seed;          /* counter-stream key */
  int64_t clip_offset;    /* global id of clip 0 (rank sharding keeps streams GPU-count invariant) */
  const float* inpaint_poses; /* device (N,L,C) or NULL  -- generator.py:249-281 */
  const float* inpaint_masks; /* device (N,L) or NULL */
  const float* trans;     /* device (L,) ramp or NULL (= trans_factor None -> 0) */
  float* out;             /* device (N,C,L): final sample */
  float* extras;          /* device (6,N,C,L) or NULL: last step's mean, variance, log_variance,
                             eps, pred_x_start, raw_x_start (gaussian_diffusion.py:278-285) */
  int32_t n_steps;        /* run only the first n_steps iterations (<=0: all T') */
  int32_t use_graph;      /* 1: replay a captured hipGraph per step */
  int32_t sync;           /* 0 (default): return once the work is issued; a persistent loop's status
                             words are checked by a later call (ggd_sample, ggd_sync), and a failure is
                             returned by that call.  1: block until the loop has finished, check it,
                             and re-run a loop whose workgroups were never co-resident on a route
                             that needs no co-residency (per-phase launches / one workgroup per clip).
                             The clip-group loop is always blocking where the one-workgroup-per-clip
                             loop cannot stand behind it as a device-gated fallback: f32, and bf16
                             clips of 49..64 frames */
} ggd_sample_args;

/* Full reverse loop, i = T'-1 ... 0, one fused model+update per step.
 * Replaces: GaussianDiffusion.p_sample_loop / ddim_sample_loop
 * (gaussian_diffusion.py:331-529) as driven by Generator.generate_sample
 * (generator.py:283-294). */
int ggd_sample(ggd_ctx* ctx, const ggd_sample_args* args, void* stream);

/* Wait for the ctx stream and every deferred status check of earlier non-blocking ggd_sample
 * calls; returns the error of a failed one (GGD_ERR_HIP) or GGD_OK -- the point at which the
 * reference's asynchronous CUDA errors would surface (reading the result). */
int ggd_sync(ggd_ctx* ctx);

/* Timing of the dominant kernel over the last profiled ggd_sample: average microseconds of one
 * launch of `which` (0 = the dominant kernel: fused path kb_kernel, timed by its own per-workgroup
 * stamps on the device realtime clock while the step graph replays; generic path the FFN-up GEMM,
 * timed by hipEvent pairs on the ctx stream), and the number of launches averaged.  Sampling
 * with ggd_set_profiling(ctx, 1) records; this call synchronises the ctx stream and reduces. */
int ggd_set_profiling(ggd_ctx* ctx, int32_t on);
int ggd_kernel_time(ggd_ctx* ctx, int32_t which, double* avg_us, int64_t* launches);
/* What the last profiled ggd_sample timed: 0 = kb_kernel launches of the per-phase path,
 * 1 = the persistent loop (mk_kernel: one launch for all denoise steps), 2 = the generic path's
 * FFN-up GEMM (LayerNorm prologue + Linear d -> 4d + ReLU^2, hipEvent pairs per launch), 3 = the
 * one-workgroup-per-clip loop (psk_kernel: one launch for all steps; chosen for large batches), 4 = the
 * clip-pair loop (psk_kernel with two workgroups per clip: one launch per <= 128 clips). */
int ggd_profile_kind(ggd_ctx* ctx);

/* Route selection of ggd_sample (not part of the reference surface: the reference has one
 * path).  Every route computes the same model; the knobs exist for A/B measurements and for
 * the tests that compare routes.  Defaults (all 0) pick the fastest measured route per shape. */
enum {
  GGD_ROUTE_PER_CLIP = 0,            /* 0 auto, 1 never, 2 always: the per-clip persistent loops
                                        (one workgroup or a clip pair per clip, ggd_persist.hip) */
  GGD_ROUTE_PAIR = 1,                /* per-clip loops: 0 auto, 1 never, 2 always two workgroups per clip */
  GGD_ROUTE_PAIR_WRITE_THROUGH = 2,  /* 1: clip-pair hand-offs written through on any placement */
  GGD_ROUTE_PHASE_LAUNCHES = 3,      /* 1: per-phase launches instead of the clip-group loop (ggd_rows.hip
                                        bf16, ggd_mega.hip f32) */
  GGD_ROUTE_PLACEMENT = 4,           /* clip-group loop: 0 XCD-local, 1 part p on XCD p, 2 group per XCD */
  GGD_ROUTE_GEMM_LAUNCHES = 5,       /* generic one-way route: 1 = one launch per GEMM instead of the
                                        row-block chains (ggd_chain.hip) */
  GGD_ROUTE_ATTN_QSPLIT = 6,         /* 1: clips of >= 96 frames on the query-split attention kernel
                                        instead of the whole-clip kernel (ggd_attn.hip) */
  GGD_ROUTE_LONG_LOOP = 7,           /* 1: never the long-clip persistent loop (ggd_long.hip): every
                                        step on launches (chains + whole-clip attention) */
  GGD_ROUTE_SIMULATE_UNRESIDENT = 8, /* test hook, 1: the clip-group and clip-pair loops report status 2
                                        ("workgroups never all resident") without running, so the
                                        device-gated one-workgroup-per-clip fallback runs the clips;
                                        2: only the odd parts report 2, the others wait in their first
                                        barrier and must drain without hiding that 2 */
  GGD_ROUTE_FP8_MFMA = 9             /* GGD_FP8W long-clip loop: 0 the FFN and LayerNorm-projection GEMMs
                                        on block-scaled fp8 MFMA (e4m3 activations, one e8m0 scale per
                                        32 values), 1 the e4m3 weights widened into bf16 MFMAs (the
                                        launch route's arithmetic, bit-equal to it) */
};
int ggd_set_route(ggd_ctx* ctx, int32_t knob, int32_t value);
enum {
  GGD_INFO_PER_CLIP_AVAILABLE = 0,   /* 1 when the per-clip loops support this shape / dtype */
  GGD_INFO_LOOP_CAPACITY = 1,        /* clips per launch of the clip-group loop (0: unavailable) */
  GGD_INFO_PAIR_LAUNCHES = 2,        /* last ggd_sample: clip-pair launches (0: another route) */
  GGD_INFO_XL_LAUNCHES = 3,          /* last ggd_sample: XCD-local clip-group launches */
  GGD_INFO_WT_RERUNS = 4,            /* last ggd_sample: clip-group launches re-run write-through */
  GGD_INFO_CHAIN_AVAILABLE = 5,      /* 1 when the generic one-way route runs as row-block chains */
  GGD_INFO_LONG_LAUNCHES = 6,        /* last ggd_sample: long-clip loop launches (0: another route) */
  GGD_INFO_CLIP_ATTN_LAUNCHES = 7,   /* running count of whole-clip attention launches (generic routes) */
  GGD_INFO_GATED_FALLBACKS = 8       /* last settled ggd_sample: chunks (clip-group loop) or batches
                                        (clip pairs) the device-gated fallback loop ran instead */,
  GGD_INFO_ROWS_LOOP = 9,            /* 1 when the last clip-group loop issued was the row-block loop
                                        (bf16; f32 contexts run the head / chunk loop) */
  GGD_INFO_BARRIER_TIMEOUTS = 10     /* running count of persistent-loop launches (clip-group chunks, clip-pair
                                        batches, long-clip chunks) whose status word carried a barrier
                                        timeout: such a launch is reported as an error, never covered by
                                        a device-gated fallback */
};
int ggd_route_info(ggd_ctx* ctx, int32_t what, double* out);

/* ggd_diag (microbenchmarks, phase stamps, calibration kernels) is exported by the separate
 * diagnostics library libggd_diag.so only (built from the same sources with -DGGD_DIAG plus
 * ggd_diag.hip; scripts/ load it with GGD_DIAG=1), never by the product libggd.so.  It launches
 * one kernel configuration `iters`
 * times back to back on the ctx stream and return the average microseconds per launch
 * (hipEvents).  what = 0: GEMM, p = {pro, epi, M, N, K, force_mt, no_xcd_remap};
 * what = 1: attention, p = {cross, n[, no_qsplit]}; what = 2: one full denoise step (eager launches),
 * p = {n}; what = 3: the same step as one hipGraph replay, p = {n}; what = 4: one fused kernel,
 * p = {0 KA | 1 KB | 2 KC | 3 KD | 4 KE, n}; what = 5: calibration micro-kernels, p = {mode, arg,
 * blocks, buffer MiB} with mode 0 empty launch, 1 dependent-load chase (arg loads), 2 shader clock
 * (returns GHz instead of microseconds), 3 / 4 bulk 64 KiB / 16 KiB load per block, 6 clip-group
 * hand-off inside one launch (arg = rounds | variant << 20; avg_us[1..3] = errors, misplaced,
 * timeouts; scripts/handoff_bench.py); what = 6: as
 * 4 with in-kernel phase stamps (avg_us[0..7] = phase ends in us); what = 7: p = {0} forces the
 * one-workgroup-per-clip loop (psk_kernel), {1} never uses it, {2} automatic (the default: used when
 * the clip-group loop would need >= 3 chunks); returns 1 in *avg_us when psk_kernel is available; what = 8: persistent-kernel phase stamps of
 * iteration 0, p = {1} arm, {2} read (avg_us[0..7]), {0} disarm; what = 9: p = {1} routes
 * ggd_sample through the per-phase launches instead of the persistent loop (ggd_mega.hip), {0}
 * back (returns the loop's clip capacity in *avg_us); what = 10 / 11: clip-group loop barrier / phase
 * stamps; what = 12 / 14: as GGD_ROUTE_PLACEMENT / GGD_ROUTE_PAIR (p[1]: write-through);
 * what = 13 / 15: as ggd_route_info; what = 16: long-clip loop barrier stamps ({1} arm, {2} read:
 * avg_us[j] = us from the loop start to barrier j of clip group 0, {0} off). */
#ifdef GGD_DIAG
int ggd_diag(ggd_ctx* ctx, int32_t what, const int32_t* p, int32_t np, int32_t iters, double* avg_us);
#endif

/* ------------------------------------------------------------------------------------
 * Speech encoder: HA2GSpeechEncoder (models/modules/ha2g/speech_encoder.py:9-61 ->
 * ha2g/model/hierarchy_net.py:10-19 -> ResNetSE34V2.py:118-188 / ResNetBlocks.py:7-96),
 * run once per clip.  Its own context: the reference module is constructed inside
 * Speech2GestureModelV2.__init__ (models/model.py:79-80) and called at model.py:95-96.
 * -------------------------------------------------------------------------------------- */
typedef struct ggd_enc ggd_enc;

/* Encoder for wav windows of `wav_len` samples (16 kHz), batches up to max_batch, tokens
 * projected to d_model.  dtype GGD_BF16: convolutions on bf16 MFMA (f32 accumulate, f32
 * front end / norms / heads); GGD_F32: every product in f32.
 * Replaces: HA2GSpeechEncoder.__init__, speech_encoder.py:9-34. */
int ggd_enc_create(int device, int32_t d_model, int32_t wav_len, int32_t max_batch, int32_t dtype, ggd_enc** out);
int ggd_enc_destroy(ggd_enc* enc);
const char* ggd_enc_last_error(const ggd_enc* enc);

/* Stage one "speech_encoder.*" state_dict tensor (other names return GGD_IGNORED).
 * Replaces: the encoder part of model.load_state_dict, main.py:113-115. */
int ggd_enc_load_weight(ggd_enc* enc, const char* name, const float* host_data, int64_t numel);

/* Check every encoder tensor, fold the eval-mode BatchNorms, pack the convolution filters and
 * upload them; size the workspaces. */
int ggd_enc_finalize(ggd_enc* enc);

/* Token counts of z_low / z_mid / z_high for this wav length (31 / 30 / 30 at 32,000). */
int ggd_enc_lengths(const ggd_enc* enc, int32_t* t_low, int32_t* t_mid, int32_t* t_high);

/* wav: device f32 (N, wav_len) -> z_low (N, t_low, d), z_mid (N, t_mid, d), z_high (N, t_high, d),
 * device f32, caller-owned.  Enqueued on `stream`.
 * Replaces: HA2GSpeechEncoder.forward, speech_encoder.py:37-61. */
int ggd_enc_run(ggd_enc* enc, const float* wav, int32_t n, float* z_low, float* z_mid, float* z_high,
                void* stream);

/* The same encoder run, its tokens written straight into the decoder's speech memory (the input of
 * ggd_set_memory) instead of three tensors.  layout GGD_MEM_BLEND (s2g_v2): mem (N, Ts, 3 d) with
 * Ts = max(T_low, T_mid, T_high), level l in columns [l d, l d + d), left-zero-padded to Ts -- the
 * F.pad + th.cat of models/model.py:97-104.  GGD_MEM_CONCAT (default / inpaint): mem
 * (N, T_low + T_mid + T_high, d), the levels concatenated on time (models/model.py:55-68). */
enum { GGD_MEM_BLEND = 0, GGD_MEM_CONCAT = 1 };
int ggd_enc_run_memory(ggd_enc* enc, const float* wav, int32_t n, int32_t layout, float* mem, void* stream);

/* The encoder's front end only: wav (N, wav_len) -> the InstanceNorm'd mel image img (N, 128, F)
 * f32 (pre-emphasis, STFT power, mel, +1e-6, InstanceNorm1d: speech_encoder.py:18-34,53-58), the
 * parameter-free input of the SE-ResNet that the training path differentiates through. */
int ggd_enc_frontend(ggd_enc* enc, const float* wav, int32_t n, float* img, void* stream);

/* Verification entry (not part of the reference surface): ONE Linear on block-scaled fp8 MFMA exactly
 * as the long-clip loop's fp8-MFMA stages run it (GGD_ROUTE_FP8_MFMA = 0) -- a (M, K) device f32 rows
 * quantised to e4m3 with one e8m0 scale per 32 consecutive values (2^(E - 7) for the block max
 * 1.f 2^E), w_e4m3 (N, K) device e4m3fn codes with per-output-channel scales wscale (N), then
 * out (M, N) = (a_q . w^T) * wscale + bias.  K % 256 == 0, K <= 1024, N % 64 == 0; blocking.  The
 * tests pin the stages' arithmetic against a numpy restatement of the same quantisation. */
int ggd_mx_linear(int32_t M, int32_t N, int32_t K, const float* a, const uint8_t* w_e4m3, const float* wscale,
                  const float* bias, float* out, void* stream);
/* Verification entry (not part of the reference surface): the long-clip loop's LayerNorm into the
 * block-scaled fp8 A image of its MX stages (the same device function), on one block of 32 rows:
 * rows (32, 256) device f32, gamma / beta (256) -> codes (32, 256) e4m3 bytes and scales (32, 8) e8m0
 * bytes, one per 32 consecutive columns (2^(E - 7) for the block max 1.f 2^E).  Blocking. */
int ggd_mx_layernorm(const float* rows, const float* gamma, const float* beta, uint8_t* codes, uint8_t* scales,
                     void* stream);
/* Verification entry (not part of the reference surface): the long-clip loop's FFN-up stage on
 * block-scaled fp8 MFMA (the same device functions: the transposed MFMA chunk and the ReLU^2 epilogue
 * that quantises the hidden rows), on one block of 32 rows: a_codes (32, 256) e4m3 bytes with
 * a_scales (32, 8) e8m0 bytes (one per 32 consecutive k), w_e4m3 (1024, 256) e4m3fn codes with
 * per-output-channel wscale (1024) and bias (1024), all device memory -> h_codes (32, 1024) e4m3
 * bytes of relu(a . w^T * wscale + bias)^2 / scale and h_scales (32, 32) e8m0 bytes, one per 32
 * consecutive hidden columns (2^(E - 7) for the block max 1.f 2^E).  Blocking.
 * Reference: models/modules/transformer.py:8-16 (SquaredReLU), :151-154 (FFN). */
int ggd_mx_ffn_up(const uint8_t* a_codes, const uint8_t* a_scales, const uint8_t* w_e4m3, const float* wscale,
                  const float* bias, uint8_t* h_codes, uint8_t* h_scales, void* stream);

/* Library version string. */
const char* ggd_version(void);

#ifdef __cplusplus
}
#endif

#endif /* GGD_H */
