// ggd_kernels.h -- device-side types and launch entry points of libggd (gfx950 only).
//
// Data layout in HBM (token-major, one clip's frames contiguous):
//   x state   f32 [N][L][C]            pose channels innermost (C = d_pose)
//   h         f32 [N*L][d]             residual stream
//   qkv       T   [N*L][3d]            Q|K|V pre-conv projections (T = bf16 or f32)
//   q/o       T   [N*L][d]
//   ffn       T   [N*L][4d]
//   eps       f32 [N*L][Cpad]
//   kv_mem    f32 [layer][N*Ts][2d]    step-invariant cross-attn K|V pre-conv (memory rows 1..Ts)
//   kv_step   f32 [layer][T_orig][2d]  memory row 0 (the diffusion-step token) for every original t
// Weights: T [Npad][Kpad] (torch Linear layout, rows = output features), zero padded.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ggd {

typedef uint16_t bf16_t;  // storage type of bf16 values

enum Pro { PRO_T = 0, PRO_LN = 1, PRO_F32 = 2 };
enum Epi {
  EPI_T = 0,      // out T   = acc + b
  EPI_RELU2 = 1,  // out T   = relu(acc + b)^2               (transformer.py:8-16)
  EPI_F32 = 2,    // out f32 = acc + b  (columns >= n_valid skipped)
  EPI_SILU = 3,   // out f32 = silu(acc + b)                 (nn.py:43)
  EPI_RESID = 4,  // h  f32 += acc + b                       (nn.py:162,167,172)
  EPI_PE = 5      // out f32 = acc + b + PE[(m % pe_period) + pe_offset]  (transformer.py:176-180)
};

struct GemmArgs {
  int M, N, K;           // K = padded reduction length (multiple of 128)
  int k_valid;           // PRO_F32: columns of A actually present (rest read as 0)
  const void* A; int lda;
  const void* W;         // T [Npad][K]
  const float* bias;     // [Npad]
  const float* ln_g; const float* ln_b;  // PRO_LN
  void* out; int ldo; int n_valid;
  const float* pe; int pe_period; int pe_offset;  // EPI_PE, pe table [max_len][N]
  int* step_counter;     // if non-null, block 0 thread 0 increments it (one step begins)
  int no_xcd_remap;      // diagnostics: 1 = plain blockIdx tile order
  int force_mt;          // diagnostics: 0 = automatic tile height, else 32 or 64
  // row maps (0 = identity): logical row m of A / of out is physical row
  // (m / len) * stride + off + m % len -- a segment of every clip's rows in a joint layout
  int a_len, a_stride, a_off;
  int o_len, o_stride, o_off;
  // fp8 weights (GGD_FP8W): non-null = W is OCP e4m3fn bytes [Npad][K] and out column n is
  // scaled by wscale[n] before the bias (per-output-channel dequantization)
  const float* wscale;
  // PRO_F32: A + a_add elementwise (same layout) -- the inpaint model's x + proj([pose*mask, mask])
  const float* a_add;
};

__host__ __device__ __forceinline__ size_t map_row(int m, int len, int stride, int off) {
  return len ? (size_t)(m / len) * stride + off + (m % len) : (size_t)m;
}

// Per-iteration diffusion coefficients, f32, computed on the host from fp64
// tables in the reference's operation order (gaussian_diffusion.py:234-329,443-484).
struct StepRec {
  float sra;      // sqrt_recip_alphas_cumprod[i]
  float srm1;     // sqrt_recipm1_alphas_cumprod[i]
  float c1, c2;   // posterior_mean_coef1/2[i]
  float var;      // posterior_variance[i]
  float logvar;   // posterior_log_variance_clipped[i]
  float sigma;    // DDPM: exp(0.5*logvar) ; DDIM: eta*sqrt((1-abp)/(1-ab))*sqrt(1-ab/abp)
  float sqrt_abp; // DDIM: sqrt(alphas_cumprod_prev[i])
  float c_eps;    // DDIM: sqrt(1 - abp - sigma^2)
  int i;          // respaced index (nonzero mask)
  int t_orig;     // timestep_map[i] (model input)
  // the call's counter-noise key (the same in every record): kept in the table rather than in
  // kernel arguments so one captured step graph serves every seed / shard offset
  uint32_t seed_lo, seed_hi, clip_offset;
};

struct AttnArgs {
  int cross;               // 0: self-attention over qkv, 1: cross-attention to memory
  const void* q; int ldq;  // T rows [N*Lq][ldq]
  const void* k; const void* v; int ldkv;  // self: T rows [N*Lk][ldkv]
  const float* kv_mem;     // cross: f32 [N*(Lk-1)][2d]
  const float* kv_step;    // cross: f32 [T_orig][2d]
  const int* t_clip;       // cross: per-clip original t, or null -> steps[*step_counter].t_orig
  const StepRec* steps; const int* step_counter;
  const float* cw_q; const float* cb_q;   // [dk][3], [dk]
  const float* cw_k; const float* cb_k;
  const float* cw_v; const float* cb_v;
  void* out; int ldo;      // T rows [N*Lq][ldo]
  int Lq, Lk, dk, heads, d;
  float scale;
  int seq_stride, seq_off;  // self mode: clip b's rows start at b * seq_stride + seq_off (0: b * Lq)
  int no_qsplit;            // diagnostics: 1 = one workgroup per (head, clip) (attn_kernel)
  const float* zero;        // >= 256 zero bytes in global memory (the conv's padding rows)
  int no_clip;              // 1: long clips on the query-split kernel instead of attn_clip_kernel
};

// Fused diffusion update on the internal layout (one denoise step's epilogue).
struct UpdArgs {
  int n, C, L, ld_eps, alg;
  const float* eps;        // f32 [N*L][ld_eps]
  float* x;                // f32 state [N][L][C], updated in place
  const StepRec* steps; const int* step_counter; int fixed_k;  // fixed_k >= 0 overrides the counter
  const float* noise;      // (T',N,C,L) per-step noise or null -> counter stream
  uint64_t seed; int64_t clip_offset;
  const float* inp_pose;   // [N][L][C] or null
  const float* inp_mask;   // [N][L]
  const float* trans;      // [L]
  float* extras;           // (6,N,C,L) or null
};

// Per-step posterior update on reference-layout (N,C,L) tensors (caller-supplied x0).
struct PostArgs {
  int n, C, L, alg;
  StepRec rec;
  const float* x; const float* eps; const float* x0;  // x0 may be null -> predicted from eps
  const float* noise;      // (N,C,L)
  float* x_out; float* x0_out;
};

// Fused per-clip decoder (ggd_fused.hip): fragment-packed weights of one layer.
constexpr int KVC_ELEMS = 2 * 64 * 32;  // per (clip, head): cross-attn K [64 keys][32] + V^T [32][64 keys]

struct FusedLayer {
  const void *qkv, *o_sa, *q_ca, *o_ca, *ff1, *ff2;  // T fragments [tile][k step][64 lanes][16 B]
  const float *qkv_b, *o_sa_b, *q_ca_b, *o_ca_b, *ff1_b, *ff2_b;
  const float *ln1_g, *ln1_b, *ln2_g, *ln2_b, *ln3_g, *ln3_b;
  const float *sa_qw, *sa_qb, *sa_kw, *sa_kb, *sa_vw, *sa_vb;
  const float *ca_qw, *ca_qb, *ca_kw, *ca_kb, *ca_vw, *ca_vb;
  const float *kv_mem, *kv_step;
  const void* kvc;   // [max_batch][heads][KVC_ELEMS] T: step-invariant convolved cross-attn K | V^T images
};

struct FusedArgs {
  FusedLayer w;
  int L, Ts;
  float* h;          // residual rows read (f32 [N*L][256])
  float* h_out;      // KB / KC: updated residual rows written (ping-pong buffer); KD updates h in place
  void *o_sa, *o_ca, *hid;
  float* ffp;        // KC -> KD: FFN-down partial sums [N][8 chunks][L][256], as T (bf16 / f32)
  const int* t_clip; const StepRec* steps; int* step_counter; int bump_counter;
  float scale;
  // KA of layer 0 with x_emb set: h = emb_x(x) + PE is computed in the kernel (x_emb = state
  // (N, L, C), packed emb_x weights, PE table) and written to h_out for KB's residual
  const float* x_emb; const void* w_emb; const float* b_emb; const float* pe; int C;
  unsigned long long* stamps;  // diagnostics: block (0,0) writes s_memtime at phase boundaries
  // profiling: KB's per-workgroup start / end on the device realtime clock, slot
  // (*step_counter * span_stride + span_layer) holds [2][workgroups] stamps (host reduces min / max)
  unsigned long long* span; int span_stride, span_layer;
};

// KE: grid (8 channel blocks, clips); block p owns pose channels [16p, 16p + 16)
struct FinalArgs {
  int n, L, C, alg;
  float* h; const float *ln_g, *ln_b;
  const void* w_out; const float* b_out;   // packed out_layers.1 (8 tiles, K 256)
  const void* w_emb; const float* b_emb;   // packed emb_x (16 tiles, K 128)
  const float* pe;
  float* x;                // state (N, L, C)
  float* eps_out;          // model-protocol mode: (N, C, L)
  const StepRec* steps; int* step_counter;
  const float* noise; uint64_t seed; int64_t clip_offset;
  const float *inp_pose, *inp_mask, *trans;
  float* extras;
  int extras_k;            // extras are written at iteration extras_k only (< 0: at every iteration)
  int do_out, do_update;
  unsigned long long* stamps;  // diagnostics
  // the persistent loop's KE rows phase also runs the last layer's FFN-down reduction for its rows
  const void* ffp;             // FFN-down partials [N][8 chunks][L][d] (the loop's dtype)
  const float* ff2_b;          // the last layer's FFN-down bias
};

// Persistent per-clip sampler (ggd_persist.hip): one workgroup per clip runs iterations
// k0 .. k0 + n_steps - 1 of the reverse loop with the clip's state in LDS / registers.
struct PersistArgs {
  const FusedLayer* layers;    // device array [n_layers]
  int n_layers, n, L, Ts, C, alg;
  const float *ln_g, *ln_b;
  const void* w_out; const float* b_out;   // packed out_layers.1 (8 tiles, K 256)
  const void* w_emb; const float* b_emb;   // packed emb_x (16 tiles, K 128)
  const float* pe;
  float* x;                    // state (N, L, C): x_T in, final sample out
  const StepRec* steps; int k0, n_steps;
  const float* noise; uint64_t seed; int64_t clip_offset;
  const float *inp_pose, *inp_mask, *trans;
  float* extras;               // (6, N, C, L) of the last iteration, or null
  float scale;
  unsigned long long* stamps;  // diagnostics: workgroup 0 stamps phase boundaries of iteration 0
  // clip pairs (launch_persist_pair): two workgroups per clip, each half the heads and FFN chunks
  unsigned* ctl;               // PAIR_CTL_WORDS control words, zeroed before every launch
  int* status;                 // 0 ok, 1 a pair barrier timed out, 2 workgroups not co-resident
  unsigned char* xbuf;         // hand-off slots [pairs][2 parts][2 epochs][PAIR_SLOT_BYTES]
  int clip0;                   // first clip of this launch (batches above the capacity run as chunks)
  int force_coh;               // diagnostics: take the write-through placement even when XCD-local fits
  // device-gated fallback (one workgroup per clip, clips clip0 ..): non-null -> the launch runs only
  // if the loop it stands in for reported status 2 (its workgroups were never all resident).
  // gate_xl = 0: *gate is that loop's status word; 1: gate[0] is an XCD-local clip-group launch's word
  // and gate[MEGA_MAX_CHUNKS] its gated write-through re-run's (used when gate[0] == 3)
  const int* gate;
  int gate_xl;
  int sim_unresident;          // test hook (GGD_ROUTE_SIMULATE_UNRESIDENT): 1 the clip-pair loop reports 2, runs nothing; 2 part 1 reports 2
};
constexpr int PAIR_MAX = 128;                              // clip pairs per launch (ctl words)
constexpr int PAIR_CTL_WORDS = 256 + PAIR_MAX * 32;        // tickets / arrival, one flag line per pair
constexpr size_t PAIR_SLOT_BYTES = 48 * 256 * 4;           // f32 [48 rows][256] FFN-down partial

// Persistent reverse loop (ggd_mega.hip): ONE launch of 8 workgroups per clip runs iterations
// k0 .. k0 + n_steps - 1; the phases of ggd_phases.h meet at clip-group barriers instead of
// kernel boundaries.  Workgroups pick their (clip, part) from their XCD, so a clip's group
// shares one L2; data between phases is written through / read past L1 (CP_COH).
struct MegaArgs {
  const FusedArgs* fa;   // device [n_layers][4]: KA, KB, KC, KD args
  const FinalArgs* fe;   // device: KE args (do_out, do_update)
  int n_layers, k0, n_steps;
  unsigned* ctl;         // control words (MEGA_CTL_WORDS), zeroed before every launch
  int* status;           // 0 ok, 1 clip-group barrier timed out, 2 workgroups not co-resident,
                         // 3 (XCD-local launch) a clip group could not be placed on one XCD: nothing ran
  unsigned long long* stamps;  // diagnostics: clip 0 / part 0 stamps s_memtime around every barrier
                               // of the first MEGA_STAMP_STEPS iterations ([phase][2]: done, passed)
  int clip0;             // first clip of this launch (batches above the capacity run as chunks)
  int placement;         // 0: a clip's 8 workgroups share one XCD; 1: workgroup part p of every clip on XCD p
  const int* gate;       // non-null: the launch runs only if *gate == 3 (the XCD-local launch of the same
                         // chunk could not place its clip groups) -- the write-through re-run, decided on
                         // the device so the host never waits for the first launch's status
  int sim_unresident;    // test hook (GGD_ROUTE_SIMULATE_UNRESIDENT): 1 report status 2 and run nothing; 2 odd parts do
};
// A persistent loop's barrier that timed out ORs this bit into the loop's status word beside its
// code 1: codes of other workgroups (2 not resident, 3 not placeable) are merged by atomicMax and
// cannot hide it, and a word carrying it never equals 2 / 3, so no device-gated fallback runs in
// its place -- the host reports the timeout (ggd_api.hip settle) instead of a fallback's success.
constexpr int STATUS_TIMEOUT = 1 << 16;
constexpr int MEGA_STAMP_STEPS = 2;
constexpr int MEGA_MAX_CHUNKS = 16;  // status words: one per launch of up to mega_capacity() clips
// PersistArgs::gate: open when the stood-in loop reported status 2 (nothing of it may be trusted)
__device__ __forceinline__ bool gate_open(const int* g, int xl) {
  if (!g) return true;
  const int s0 = g[0];
  return xl ? (s0 == 2 || (s0 == 3 && g[MEGA_MAX_CHUNKS] == 2)) : s0 == 2;
}
constexpr int MEGA_CTL_WORDS = 256 + 32 * 16 + 32 * 32;  // tickets/arrival, group counters, group flag lines

// Row-block chains of the one-way decoder (ggd_chain.hip): one launch runs, on 32-row blocks of
// the residual stream, R (h += A W_r^T + b), F (h += FFN(LN_f(h))) and P (out = LN_p(h) W_p^T + b)
// as enabled (w non-null).  Weights are fragment-packed copies made by launch_chain_pack.
struct ChainLin {
  const void* w;          // fragment-packed (bf16, or e4m3 bytes when scale is set)
  const float* b;         // [npad]
  const float* scale;     // fp8: per-output-channel dequantization scale [npad]
  int npad, kpad;
};
struct ChainArgs {
  int M;                  // rows (clips x frames)
  float* h;               // residual stream f32 [M][256], updated in place by R / F
  const bf16_t* a_in;     // R operand: bf16 rows [M][256] (the attention output)
  ChainLin r;
  const float *f_g, *f_b; ChainLin f1, f2;   // F: LayerNorm, [1024][256], [256][1024]
  const float *p_g, *p_b; ChainLin p;        // P: LayerNorm, [npad][256]
  void* out; int ldo;     // P output rows: bf16, or f32 when out_f32 (columns >= n_valid skipped)
  int out_f32, n_valid;
};

// Long-clip persistent loop (ggd_long.hip): 8 workgroups per clip run every step; per layer the
// chain-route weights (fragment-packed ChainLin) and the attention conv taps / memory K|V.
struct LongLayer {
  ChainLin qkv, o_sa, q_ca, o_ca, ff1, ff2;
  const float *ln1_g, *ln1_b, *ln2_g, *ln2_b, *ln3_g, *ln3_b;
  const float *sa_qw, *sa_qb, *sa_kw, *sa_kb, *sa_vw, *sa_vb;
  const float *ca_qw, *ca_qb, *ca_kw, *ca_kb, *ca_vw, *ca_vb;
  const float *kv_mem, *kv_step;   // this layer's memory K|V rows [N * Ts][2d], step-token rows [T_orig][2d]
  const bf16_t* kvc;               // convolved memory keys 2.. as [N][heads][K [Lk_pad][32] | V^T [32][Lk_pad]]
};
// one GEMM stage of a long-loop chain phase: weights, the LayerNorm in front, hand-off output rows
struct ChainStage {
  ChainLin w;
  const float *ln_g, *ln_b;
  void* out;
  int ldo;
};
constexpr int LONG_STAGES_PER_LAYER = 8;   // chain A: 2 stages, chain B: 4 (+ emb, QKV at the last layer)
struct LongArgs {
  const LongLayer* layers;   // device [n_layers]
  const ChainStage* stages;  // device [2 + 8 n_layers]: loop start (emb_x, QKV), then per layer A, B
  int n_layers;
  int n, L, Ts, C, alg;      // n: clips of the whole sampling call (noise indexing)
  int k0, n_steps, clip0;    // iterations k0 .. k0 + n_steps - 1 of clips clip0 .. clip0 + G - 1
  ChainLin emb, out;         // emb_x (K = C padded to 256), out_layers.1 (N = C padded to 128)
  const float *out_g, *out_b, *pe;
  float* x;                  // state (N, L, C): x_T in, the sample out
  const float* h;            // h = emb_x(x_T) + PE of the first iteration (layer 0's QKV rows in qkv)
  void *qkv, *att, *q;       // hand-off rows (bf16)
  const StepRec* steps;
  const float* noise;        // (T', N, C, L) injected noise, or null: the counter stream
  float* extras;             // (6, N, C, L) of iteration k0 + n_steps - 1, or null
  float scale;
  unsigned* ctl;             // LONG_CTL_WORDS, zeroed by launch_long_loop
  int* status;               // 0 ok, 1 barrier timeout, 2 not resident, 3 not placeable (nothing ran)
  unsigned long long* stamps;  // diagnostics: clip group 0 part 0 stamps the realtime clock at the loop
                               // start [0] and after each of the first LONG_STAMPS - 1 barriers
};
constexpr int LONG_CTL_WORDS = 256 + 32 * 32;
constexpr int LONG_STAMPS = 64;

// launchers (return hipError_t of the launch)
bool long_loop_supported(int dtype, int d_model, int heads, int L, int Ts, int C, int out_npad);
int long_loop_capacity();   // clips per launch
// w8: 0 bf16 weights, 1 e4m3 weights widened into bf16 MFMAs, 2 e4m3 weights AND activations on
// block-scaled fp8 MFMA in the FFN / LayerNorm-projection stages (a.stages' F1 / F2 / P / P2 weights
// then hold launch_chain_pack(2, ...) copies)
hipError_t launch_long_loop(int w8, const LongArgs& a, int G, hipStream_t s);
// step-invariant convolved memory K / V^T of one layer for the long loop (keys 0, 1 and >= 1 + Ts zero)
hipError_t launch_long_kv_cache(const float* kv_mem, const float* kw, const float* kb, const float* vw, const float* vb,
                                int n, int Ts, int heads, bf16_t* out, hipStream_t s);
size_t long_kv_cache_bytes(int n, int Ts, int heads);
hipError_t launch_chain(int w8, const ChainArgs& a, hipStream_t s);
// w8: 0 bf16, 1 e4m3 (bf16-widened chain order), 2 e4m3 in the block-scaled fp8 MFMA's B order
hipError_t launch_chain_pack(int w8, const void* src, void* dst, int npad, int kpad, hipStream_t s);
size_t chain_pack_bytes(int w8, int npad, int kpad);
bool chain_p_supported(int npad);   // P stage widths with a kernel instance
hipError_t launch_fused(int which, int dtype, const FusedArgs& a, int n, hipStream_t s);  // 0 KA, 1 KB, 2 KC, 3 KD
hipError_t launch_final(int dtype, const FinalArgs& a, hipStream_t s);
// step-invariant convolved cross-attention K | V^T images of one layer (ggd_set_memory; fused paths)
hipError_t launch_ca_kv_conv(int dtype, const float* kv_mem, const float* kw, const float* kb, const float* vw,
                             const float* vb, int n, int Ts, void* out, hipStream_t s);
bool fused_supported(int dtype, int d_model, int heads, int L, int Ts, int C);
hipError_t launch_persist(const PersistArgs& a, hipStream_t s);
// clips [a.clip0, a.clip0 + clips) of a batch of a.n, one workgroup per clip (the gated fallback)
hipError_t launch_persist_range(const PersistArgs& a, int clips, hipStream_t s);
// clip pairs: clips [a.clip0, a.clip0 + pairs) with two co-resident workgroups each (pairs <=
// persist_pair_capacity()); a.ctl must hold PAIR_CTL_WORDS words (zeroed here)
hipError_t launch_persist_pair(const PersistArgs& a, int pairs, hipStream_t s);
int persist_pair_capacity();
bool persist_supported(int dtype, int d_model, int heads, int L, int Ts, int C);
// xl: the XCD-local variant (CP_XL, grid padded to whole XCDs; placement 0 only)
hipError_t launch_mega(int dtype, int L, const MegaArgs& a, int n, bool xl, hipStream_t s);
int mega_capacity(int dtype, int L);   // clips one launch can hold (all workgroups co-resident)
// the same loop with the decoder split by row blocks where its work is row-local (ggd_rows.hip, bf16;
// Ts = memory tokens): one launch of 8 workgroups per clip, MegaArgs as launch_mega
bool rows_supported(int dtype, int L, int Ts);
hipError_t launch_rows(int dtype, int L, int Ts, const MegaArgs& a, int n, bool xl, hipStream_t s);
hipError_t launch_mb(int mode, void* buf, size_t buf_bytes, int arg, int blocks, hipStream_t s);  // ggd_diag.hip
hipError_t launch_gemm(int dtype, int pro, int epi, const GemmArgs& a, hipStream_t s);
hipError_t launch_attention(int dtype, const AttnArgs& a, int n, hipStream_t s);
// whole-clip attention (ggd_attn.hip): bf16, d_k 32, 96 <= Lq <= 192, self (no row map) or memory
bool attention_clip_supported(int dtype, const AttnArgs& a);
hipError_t launch_attention_clip(const AttnArgs& a, int n, hipStream_t s);
hipError_t launch_update(const UpdArgs& a, hipStream_t s);
hipError_t launch_inpaint_input(float* out, const float* pose, const float* mask, int M, int C, hipStream_t s);
hipError_t launch_posterior(const PostArgs& a, hipStream_t s);
hipError_t launch_step_embed(float* out, int T, int d, hipStream_t s);
hipError_t launch_init_state(float* x, const float* x_T_ncl, uint64_t seed, int64_t clip_offset,
                             int n, int C, int L, hipStream_t s);
// the same for clips [clip0, clip0 + n) of the batch, run only if the gate (PersistArgs::gate) is open:
// a loop that did not run re-initialises the clips it stood for before its fallback runs them
hipError_t launch_init_state_gated(float* x, const float* x_T_ncl, uint64_t seed, int64_t clip_offset, int clip0,
                                   int n, int C, int L, const int* gate, int gate_xl, hipStream_t s);
hipError_t launch_nlc_to_ncl(float* dst, const float* src, int n, int C, int L, int ld_src,
                             hipStream_t s);
hipError_t launch_set_int(int* p, int v, hipStream_t s);
// LayerNorm (eps 1e-5) of f32 rows (row map len/stride/off) -> T rows [M][d], d <= 1024
hipError_t launch_layernorm(int dtype, const float* in, int len, int stride, int off, const float* g, const float* b,
                            void* out, int M, int d, hipStream_t s);
// two-way decoder memory rows of every clip in the joint layout [n][L + 1 + Ts][d]:
// row L = step token of the clip's t (tab[t] already holds emb_mem + PE[L]), rows L+1.. = base
hipError_t launch_mem_assemble(float* h, const float* base, const float* tab, const int* t_clip, const StepRec* steps,
                               const int* step_counter, int n, int L, int Ts, int d, hipStream_t s);

}  // namespace ggd
