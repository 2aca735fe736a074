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
};

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
  int pad;
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

// launchers (return hipError_t of the launch)
hipError_t launch_gemm(int dtype, int pro, int epi, const GemmArgs& a, hipStream_t s);
hipError_t launch_attention(int dtype, const AttnArgs& a, int n, hipStream_t s);
hipError_t launch_update(const UpdArgs& a, hipStream_t s);
hipError_t launch_posterior(const PostArgs& a, hipStream_t s);
hipError_t launch_step_embed(float* out, int T, int d, hipStream_t s);
hipError_t launch_init_state(float* x, const float* x_T_ncl, uint64_t seed, int64_t clip_offset,
                             int n, int C, int L, hipStream_t s);
hipError_t launch_nlc_to_ncl(float* dst, const float* src, int n, int C, int L, int ld_src,
                             hipStream_t s);
hipError_t launch_set_int(int* p, int v, hipStream_t s);

}  // namespace ggd
