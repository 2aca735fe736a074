// ggd_fused.hip -- the fused per-clip decoder kernels (d_model 256, 8 heads, L <= 64).
//
// One denoise step of the one-way decoder (models/nn.py:154-228) is 4 launches per layer
// plus one epilogue launch, instead of one launch per op:
//
//   KA (head, clip)   LN1 + QKV projection of the head + 3-tap conv + self-attention
//   KB (head, clip)   SA out-proj + residual (+ h write) + LN2 + cross-attn query of the
//                     head + conv + cross-attention to the cached speech memory
//   KC (chunk, clip)  CA out-proj + residual (+ h write) + LN3 + FFN-up chunk + ReLU^2
//   KD                FFN-down + residual: the generic LDS-tiled GEMM (gemm_kernel)
//   KE (clip)         LN_out + output projection + DDPM/DDIM update (+ the next step's
//                     emb_x + PE), or eps for the model protocol
//
// Every workgroup owns one clip's rows, so the depthwise conv, the attention and every
// LayerNorm see whole sequences / whole rows in LDS.  The small out-projections are
// recomputed by each head workgroup of a clip (x8 redundant MFMA work, ~10 % of the step)
// instead of paying a launch boundary and an HBM round trip for them.  Weights are packed
// on the host in MFMA B-fragment order -- [n tile][k step][lane][16 bytes] -- so a wave
// streams its fragments straight into registers with fully coalesced 1 KiB loads, issued
// before the activations they multiply have arrived.
#include <algorithm>

#include "ggd_common.h"

namespace ggd {

constexpr int FD = 256, FDK = 32, FRT = 4;  // d_model, d_k, max row tiles (L <= 64)

template <typename T> struct Frag {
  static constexpr int KF = 64 / sizeof(T);   // k covered by one fragment: 32 (bf16) / 16 (f32)
  static constexpr int PT = 16 / sizeof(T);   // 16-byte LDS row pad
};

__device__ __forceinline__ size_t al16(size_t v) { return (v + 15) & ~(size_t)15; }

// diagnostics: phase stamps of workgroup (0, 0), written only when the stamp buffer is set
#define STAMP(i)                                                                                \
  do {                                                                                          \
    if (a.stamps && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)                     \
      a.stamps[i] = __builtin_amdgcn_s_memtime();                                               \
  } while (0)

// one B fragment: packed weights as uint4 [tile][k step][64 lanes]
__device__ __forceinline__ uint4 wfrag(const uint4* W, int nt, int kf, int KT, int lane) {
  return W[((size_t)nt * KT + kf) * 64 + lane];
}

// acc += A[rt*16 .. +16)[k step kf] x fragment wb   (A row-major in LDS, stride SA)
template <typename T>
__device__ __forceinline__ void mma_aw(f32x4& acc, const T* A, int SA, int rt, int kf, uint4 wb, int lane) {
  const int r16 = lane & 15, g = lane >> 4;
  if constexpr (sizeof(T) == 2) {
    const bf16x8 av = *(const bf16x8*)(A + (rt * 16 + r16) * SA + kf * 32 + g * 8);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, __builtin_bit_cast(bf16x8, wb), acc, 0, 0, 0);
  } else {
    const f32x4 av = *(const f32x4*)(A + (rt * 16 + r16) * SA + kf * 16 + g * 4);
    const f32x4 bv = __builtin_bit_cast(f32x4, wb);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], acc, 0, 0, 0);
  }
}

// acc[rt][j] = A[RT row tiles] x W tiles tiles[j] (j < NJ, skipped if !on[j]); K = KT k steps.
// bf16: all of the wave's fragments are loaded up front (<= 32 x 16 B per lane); f32 streams.
template <typename T, int NJ, int KT>
__device__ __forceinline__ void gemm_aw(f32x4 (&acc)[FRT][NJ], const T* A, int SA, int RT, const uint4* W,
                                        const int (&tiles)[NJ], const bool (&on)[NJ], int lane) {
#pragma unroll
  for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (sizeof(T) == 2 && NJ * KT <= 32) {
    uint4 wb[NJ][KT];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int kf = 0; kf < KT; ++kf) wb[j][kf] = on[j] ? wfrag(W, tiles[j], kf, KT, lane) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int kf = 0; kf < KT; ++kf)
#pragma unroll
      for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          if (rt < RT && on[j]) mma_aw<T>(acc[rt][j], A, SA, rt, kf, wb[j][kf], lane);
  } else {
#pragma unroll 2
    for (int kf = 0; kf < KT; ++kf) {
      uint4 wb[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) wb[j] = on[j] ? wfrag(W, tiles[j], kf, KT, lane) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          if (rt < RT && on[j]) mma_aw<T>(acc[rt][j], A, SA, rt, kf, wb[j], lane);
    }
  }
}

// LayerNorm (eps 1e-5, two-pass) of L rows of width 256 at src (stride ss, f32, global or LDS)
// into dst (T, stride sd); rows L .. Lp-1 are zeroed.  4 lanes per row: the same summation
// order as the generic GEMM's LN prologue.
template <typename T>
__device__ __forceinline__ void ln_rows(const float* src, int ss, int L, int Lp, const float* g, const float* bta,
                                        T* dst, int sd) {
  const int tid = threadIdx.x, r = tid >> 2, j = tid & 3;
  if (r >= Lp) return;
  const bool ok = r < L;
  float4 v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    v[i] = ok ? *(const float4*)(src + (size_t)r * ss + (j + 4 * i) * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  const float mu = s / (float)FD;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float d0 = v[i].x - mu, d1 = v[i].y - mu, d2 = v[i].z - mu, d3 = v[i].w - mu;
    q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
  }
  q += __shfl_xor(q, 1);
  q += __shfl_xor(q, 2);
  const float rs = 1.0f / sqrtf(q / (float)FD + 1e-5f);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int k = (j + 4 * i) * 4;
    const float4 gg = *(const float4*)(g + k);
    const float4 bb = *(const float4*)(bta + k);
    T* o = dst + (size_t)r * sd + k;
    o[0] = from_f32<T>(ok ? (v[i].x - mu) * rs * gg.x + bb.x : 0.f);
    o[1] = from_f32<T>(ok ? (v[i].y - mu) * rs * gg.y + bb.y : 0.f);
    o[2] = from_f32<T>(ok ? (v[i].z - mu) * rs * gg.z + bb.z : 0.f);
    o[3] = from_f32<T>(ok ? (v[i].w - mu) * rs * gg.w + bb.w : 0.f);
  }
}

// copy `rows` rows of `bytes_per_row` (multiple of 16) from global to LDS (stride in bytes);
// rows rows .. rows_pad-1 are zero filled
__device__ __forceinline__ void copy_rows(void* dst, size_t dst_stride, const void* src, size_t src_stride, int rows,
                                          int rows_pad, int bytes_per_row) {
  const int vpr = bytes_per_row / 16;
  for (int v = threadIdx.x; v < rows_pad * vpr; v += NTHREADS) {
    const int r = v / vpr, c = v % vpr;
    const uint4 val = r < rows ? *(const uint4*)((const char*)src + (size_t)r * src_stride + c * 16)
                               : make_uint4(0, 0, 0, 0);
    *(uint4*)((char*)dst + (size_t)r * dst_stride + c * 16) = val;
  }
}

// 3-tap conv along the sequence of column block [col0, col0 + 32) of Y (f32, stride sy, rows
// 0..L-1, zero outside) into an operand image (rows or transposed).
template <typename T, bool TRANS>
__device__ __forceinline__ void conv_from(T* dst, int S, const float* Y, int sy, int col0, int L, const float* w,
                                          const float* b) {
  for (int idx = threadIdx.x; idx < L * FDK; idx += NTHREADS) {
    const int i = idx / FDK, c = idx % FDK;
    const float p0 = i > 0 ? Y[(i - 1) * sy + col0 + c] : 0.f;
    const float p1 = Y[i * sy + col0 + c];
    const float p2 = i + 1 < L ? Y[(i + 1) * sy + col0 + c] : 0.f;
    const float v = b[c] + w[c * 3 + 0] * p0 + w[c * 3 + 1] * p1 + w[c * 3 + 2] * p2;
    if (TRANS)
      dst[c * S + i] = from_f32<T>(v);
    else
      dst[i * S + c] = from_f32<T>(v);
  }
}

// ------------------------------------------------------------------------------------------
// LDS plans
// ------------------------------------------------------------------------------------------
template <typename T>
__host__ __device__ inline size_t ka_lds(int L, size_t* off_y, size_t* off_att, AttGeom* G) {
  const int Lp = (L + 15) & ~15;
  const size_t x = sizeof(T) * (size_t)Lp * (FD + Frag<T>::PT);
  const size_t y = sizeof(float) * (size_t)Lp * (96 + 4);
  *G = att_geom<T>(L, L, FDK);
  *off_y = (x + 15) & ~(size_t)15;
  *off_att = (*off_y + y + 15) & ~(size_t)15;
  return *off_att + G->off_raw;  // the attention raw staging area is not used here
}

template <typename T>
__host__ __device__ inline size_t kb_lds(int L, int Lk, size_t* off_h, size_t* off_y, size_t* off_att, AttGeom* G) {
  const int Lp = (L + 15) & ~15;
  const size_t x = sizeof(T) * (size_t)Lp * (FD + Frag<T>::PT);
  const size_t hs = sizeof(float) * (size_t)Lp * (FD + 4);
  const size_t y = sizeof(float) * (size_t)Lp * (FDK + 4);
  *G = att_geom<T>(L, Lk, FDK);
  *off_h = (x + 15) & ~(size_t)15;
  *off_y = (*off_h + hs + 15) & ~(size_t)15;
  *off_att = (*off_y + y + 15) & ~(size_t)15;
  return *off_att + G->off_raw + sizeof(float) * 2 * (size_t)(Lk + 2) * FDK;  // raw memory K and V
}

template <typename T>
__host__ __device__ inline size_t kc_lds(int L, size_t* off_h) {
  const int Lp = (L + 15) & ~15;
  const size_t x = sizeof(T) * (size_t)Lp * (FD + Frag<T>::PT);
  *off_h = (x + 15) & ~(size_t)15;
  return *off_h + sizeof(float) * (size_t)Lp * (FD + 4);
}

template <typename T>
__host__ __device__ inline size_t ke_lds(int L, size_t* off_e, size_t* off_xs, size_t* off_xb) {
  const int Lp = (L + 15) & ~15;
  const size_t x = sizeof(T) * (size_t)Lp * (FD + Frag<T>::PT);
  const size_t e = sizeof(float) * (size_t)Lp * (128 + 4);
  *off_e = (x + 15) & ~(size_t)15;
  *off_xs = (*off_e + e + 15) & ~(size_t)15;
  *off_xb = (*off_xs + e + 15) & ~(size_t)15;
  return *off_xb + sizeof(T) * (size_t)Lp * (128 + Frag<T>::PT);
}

// ------------------------------------------------------------------------------------------
// KA: LN1 + QKV(head) + conv + self-attention          grid (heads, clips)
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(NTHREADS) ka_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int PT = Frag<T>::PT, KT = FD / Frag<T>::KF, SX = FD + PT, SY = 96 + 4;
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = a.L, Lp = (L + 15) & ~15, RT = Lp / 16;
  size_t off_y, off_att;
  AttGeom G;
  ka_lds<T>(L, &off_y, &off_att, &G);
  T* Xn = (T*)smem;
  float* Y = (float*)(smem + off_y);
  unsigned char* att = smem + off_att;
  T *Qm = (T*)(att + G.off_q), *Km = (T*)(att + G.off_k), *Vt = (T*)(att + G.off_v), *Pw = (T*)(att + G.off_p);
  const FusedLayer& w = a.w;

  STAMP(0);
  if (a.bump_counter && h == 0 && b == 0 && tid == 0) atomicAdd(a.step_counter, 1);
  for (int i = tid; i < (int)(G.off_p / 16); i += NTHREADS) ((uint4*)att)[i] = make_uint4(0, 0, 0, 0);

  ln_rows<T>(a.h + (size_t)b * L * FD, FD, L, Lp, w.ln1_g, w.ln1_b, Xn, SX);
  __syncthreads();
  STAMP(1);
  // QKV of head h: packed as 6 tiles [q0 q1 k0 k1 v0 v1]; wave w owns tiles w and w + 4
  const uint4* W = (const uint4*)w.qkv + (size_t)h * 6 * KT * 64;
  const int tiles[2] = {wave, wave + 4};
  const bool on[2] = {true, wave + 4 < 6};
  f32x4 acc[FRT][2];
  gemm_aw<T, 2, KT>(acc, Xn, SX, RT, W, tiles, on, lane);
  const int c16 = lane & 15, g4 = lane >> 4;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (!on[j]) continue;
    const int col = tiles[j] * 16 + c16;
    const float bias = w.qkv_b[h * 96 + col];
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt)
      if (rt < RT)
#pragma unroll
        for (int r = 0; r < 4; ++r) Y[(rt * 16 + 4 * g4 + r) * SY + col] = acc[rt][j][r] + bias;
  }
  __syncthreads();
  STAMP(2);
  conv_from<T, false>(Qm, G.SQ, Y, SY, 0, L, w.sa_qw, w.sa_qb);
  conv_from<T, false>(Km, G.SQ, Y, SY, 32, L, w.sa_kw, w.sa_kb);
  conv_from<T, true>(Vt, G.SV, Y, SY, 64, L, w.sa_vw, w.sa_vb);
  __syncthreads();
  STAMP(3);
  attn_core<T>(Qm, Km, Vt, Pw, G, L, L, FDK, a.scale, (T*)a.o_sa + (size_t)b * L * FD + h * FDK, FD);
  if (a.stamps) {
    __syncthreads();
    STAMP(4);
  }
}

// out-proj of a full d x d block + residual, in place in Hs (f32, stride FD + 4):
// Hs[i][n] += A[i] . W[n] + bias[n] for i < L.  Wave w owns the 64 columns [64w, 64w + 64).
template <typename T>
__device__ __forceinline__ void outproj_residual(float* Hs, const T* A, int L, int RT, const void* Wp,
                                                 const float* bias, int lane, int wave) {
  constexpr int KT = FD / Frag<T>::KF, SX = FD + Frag<T>::PT, SH = FD + 4;
  const int tiles[4] = {4 * wave, 4 * wave + 1, 4 * wave + 2, 4 * wave + 3};
  const bool on[4] = {true, true, true, true};
  f32x4 acc[FRT][4];
  gemm_aw<T, 4, KT>(acc, A, SX, RT, (const uint4*)Wp, tiles, on, lane);
  const int c16 = lane & 15, g4 = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = tiles[j] * 16 + c16;
    const float bb = bias[col];
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt)
      if (rt < RT)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = rt * 16 + 4 * g4 + r;
          if (i < L) Hs[i * SH + col] = Hs[i * SH + col] + (acc[rt][j][r] + bb);
        }
  }
}

// ------------------------------------------------------------------------------------------
// KB: SA out-proj + residual + LN2 + cross-attn Q(head) + conv + cross-attention  (heads, clips)
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(NTHREADS) kb_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int PT = Frag<T>::PT, KT = FD / Frag<T>::KF, SX = FD + PT, SH = FD + 4, SY = FDK + 4;
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = a.L, Lp = (L + 15) & ~15, RT = Lp / 16, Lk = 1 + a.Ts;
  size_t off_h, off_y, off_att;
  AttGeom G;
  kb_lds<T>(L, Lk, &off_h, &off_y, &off_att, &G);
  T* Ax = (T*)smem;                   // O_sa image, then LN2(h) image
  float* Hs = (float*)(smem + off_h);
  float* Yq = (float*)(smem + off_y);
  unsigned char* att = smem + off_att;
  T *Qm = (T*)(att + G.off_q), *Km = (T*)(att + G.off_k), *Vt = (T*)(att + G.off_v), *Pw = (T*)(att + G.off_p);
  float* raw = (float*)(att + G.off_raw);
  const FusedLayer& w = a.w;

  STAMP(0);
  for (int i = tid; i < (int)(G.off_p / 16); i += NTHREADS) ((uint4*)att)[i] = make_uint4(0, 0, 0, 0);
  const size_t row0 = (size_t)b * L;
  copy_rows(Ax, sizeof(T) * SX, (const T*)a.o_sa + row0 * FD, sizeof(T) * FD, L, Lp, sizeof(T) * FD);
  copy_rows(Hs, sizeof(float) * SH, a.h + row0 * FD, sizeof(float) * FD, L, Lp, sizeof(float) * FD);
  __syncthreads();
  STAMP(1);
  outproj_residual<T>(Hs, Ax, L, RT, w.o_sa, w.o_sa_b, lane, wave);
  __syncthreads();
  STAMP(2);
  if (h == 0) copy_rows(a.h_out + row0 * FD, sizeof(float) * FD, Hs, sizeof(float) * SH, L, L, sizeof(float) * FD);
  ln_rows<T>(Hs, SH, L, Lp, w.ln2_g, w.ln2_b, Ax, SX);
  // memory K / V of head h (independent of the above): row 0 = step token of this clip's t
  const int t = a.t_clip ? a.t_clip[b] : a.steps[*a.step_counter].t_orig;
  const float* r0 = w.kv_step + (size_t)t * 2 * FD;
  __syncthreads();
  STAMP(3);
  // cross-attn query of head h: tiles 2h, 2h+1 of the natural packing (waves 0, 1)
  {
    const int tiles[1] = {2 * h + (wave & 1)};
    const bool on[1] = {wave < 2};
    f32x4 acc[FRT][1];
    gemm_aw<T, 1, KT>(acc, Ax, SX, RT, (const uint4*)w.q_ca, tiles, on, lane);
    if (wave < 2) {
      const int c16 = lane & 15, g4 = lane >> 4, col = (wave & 1) * 16 + c16;
      const float bias = w.q_ca_b[h * FDK + col];
#pragma unroll
      for (int rt = 0; rt < FRT; ++rt)
        if (rt < RT)
#pragma unroll
          for (int r = 0; r < 4; ++r) Yq[(rt * 16 + 4 * g4 + r) * SY + col] = acc[rt][0][r] + bias;
    } else {
      // waves 2, 3: memory K / V through the conv into the operand images
      for (int half = 0; half < 2; ++half) {
        const int col = half * FD + h * FDK;
        for (int v = tid - 128; v < (Lk + 2) * FDK; v += 128) {
          const int r = v / FDK, c = v % FDK;  // haloed row r = memory row r - 1
          float val = 0.f;
          if (r == 1) val = r0[col + c];
          else if (r >= 2 && r <= Lk) val = w.kv_mem[((size_t)b * a.Ts + (r - 2)) * 2 * FD + col + c];
          raw[half * (Lk + 2) * FDK + v] = val;
        }
      }
    }
  }
  __syncthreads();
  STAMP(4);
  conv_from<T, false>(Qm, G.SQ, Yq, SY, 0, L, w.ca_qw, w.ca_qb);
  {
    const float* rk = raw;
    const float* rv = raw + (Lk + 2) * FDK;
    for (int idx = tid; idx < Lk * FDK; idx += NTHREADS) {
      const int i = idx / FDK, c = idx % FDK;
      const float* pk = rk + i * FDK + c;
      const float* pv = rv + i * FDK + c;
      Km[i * G.SQ + c] = from_f32<T>(w.ca_kb[c] + w.ca_kw[c * 3] * pk[0] + w.ca_kw[c * 3 + 1] * pk[FDK] +
                                     w.ca_kw[c * 3 + 2] * pk[2 * FDK]);
      Vt[c * G.SV + i] = from_f32<T>(w.ca_vb[c] + w.ca_vw[c * 3] * pv[0] + w.ca_vw[c * 3 + 1] * pv[FDK] +
                                     w.ca_vw[c * 3 + 2] * pv[2 * FDK]);
    }
  }
  __syncthreads();
  STAMP(5);
  attn_core<T>(Qm, Km, Vt, Pw, G, L, Lk, FDK, a.scale, (T*)a.o_ca + row0 * FD + h * FDK, FD);
  if (a.stamps) {
    __syncthreads();
    STAMP(6);
  }
}

// ------------------------------------------------------------------------------------------
// KC: CA out-proj + residual + LN3 + FFN-up chunk (128 hidden) + ReLU^2   grid (8 chunks, clips)
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(NTHREADS) kc_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int PT = Frag<T>::PT, KT = FD / Frag<T>::KF, SX = FD + PT, SH = FD + 4;
  const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = a.L, Lp = (L + 15) & ~15, RT = Lp / 16;
  size_t off_h;
  kc_lds<T>(L, &off_h);
  T* Ax = (T*)smem;
  float* Hs = (float*)(smem + off_h);
  const FusedLayer& w = a.w;
  STAMP(0);
  const size_t row0 = (size_t)b * L;
  copy_rows(Ax, sizeof(T) * SX, (const T*)a.o_ca + row0 * FD, sizeof(T) * FD, L, Lp, sizeof(T) * FD);
  copy_rows(Hs, sizeof(float) * SH, a.h + row0 * FD, sizeof(float) * FD, L, Lp, sizeof(float) * FD);
  __syncthreads();
  STAMP(1);
  outproj_residual<T>(Hs, Ax, L, RT, w.o_ca, w.o_ca_b, lane, wave);
  __syncthreads();
  STAMP(2);
  if (c == 0) copy_rows(a.h_out + row0 * FD, sizeof(float) * FD, Hs, sizeof(float) * SH, L, L, sizeof(float) * FD);
  ln_rows<T>(Hs, SH, L, Lp, w.ln3_g, w.ln3_b, Ax, SX);
  __syncthreads();
  STAMP(3);
  const int tiles[2] = {8 * c + 2 * wave, 8 * c + 2 * wave + 1};
  const bool on[2] = {true, true};
  f32x4 acc[FRT][2];
  gemm_aw<T, 2, KT>(acc, Ax, SX, RT, (const uint4*)w.ff1, tiles, on, lane);
  const int c16 = lane & 15, g4 = lane >> 4;
  T* out = (T*)a.hid + row0 * (4 * FD);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = tiles[j] * 16 + c16;
    const float bb = w.ff1_b[col];
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt)
      if (rt < RT)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = rt * 16 + 4 * g4 + r;
          float v = fmaxf(acc[rt][j][r] + bb, 0.f);
          if (i < L) out[(size_t)i * (4 * FD) + col] = from_f32<T>(v * v);
        }
  }
  if (a.stamps) {
    __syncthreads();
    STAMP(4);
  }
}

// ------------------------------------------------------------------------------------------
// KE: LN_out + out-proj (eps) [+ diffusion update] [+ next step's emb_x + PE]   grid (clips)
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(NTHREADS) ke_kernel(FinalArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int PT = Frag<T>::PT, KT = FD / Frag<T>::KF, SX = FD + PT, SE = 128 + 4, SB = 128 + PT;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = a.L, C = a.C, Lp = (L + 15) & ~15, RT = Lp / 16;
  size_t off_e, off_xs, off_xb;
  ke_lds<T>(L, &off_e, &off_xs, &off_xb);
  T* Xn = (T*)smem;
  float* E = (float*)(smem + off_e);
  float* Xs = (float*)(smem + off_xs);
  T* Xb = (T*)(smem + off_xb);
  const size_t row0 = (size_t)b * L;
  const int c16 = lane & 15, g4 = lane >> 4;

  STAMP(0);
  if (a.do_out) {
    ln_rows<T>(a.h + row0 * FD, FD, L, Lp, a.ln_g, a.ln_b, Xn, SX);
    __syncthreads();
    STAMP(1);
    const int tiles[2] = {2 * wave, 2 * wave + 1};
    const bool on[2] = {true, true};
    f32x4 acc[FRT][2];
    gemm_aw<T, 2, KT>(acc, Xn, SX, RT, (const uint4*)a.w_out, tiles, on, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = tiles[j] * 16 + c16;
      const float bb = a.b_out[col];
#pragma unroll
      for (int rt = 0; rt < FRT; ++rt)
        if (rt < RT)
#pragma unroll
          for (int r = 0; r < 4; ++r) E[(rt * 16 + 4 * g4 + r) * SE + col] = acc[rt][j][r] + bb;
    }
    __syncthreads();
    STAMP(2);
  }
  if (a.do_update) {
    const int k = *a.step_counter;
    const StepRec rec = a.steps[k];
    const size_t plane = (size_t)a.n * C * L;
    for (int idx = tid; idx < L * C; idx += NTHREADS) {
      const int l = idx / C, cc = idx % C;
      const size_t gi = (row0 + l) * C + cc;             // internal (N, L, C)
      const size_t ncl = ((size_t)b * C + cc) * L + l;   // reference (N, C, L)
      const float x = a.x[gi], e = E[l * SE + cc];
      float z;
      if (a.noise)
        z = a.noise[(size_t)k * plane + ncl];
      else
        z = philox_normal(a.seed, (uint32_t)(a.clip_offset + b), (uint32_t)rec.i, TAG_STEP, (uint32_t)(cc * L + l));
      const bool inp = a.inp_mask != nullptr;
      const UpdOut o = upd_math(rec, a.alg, x, e, false, 0.f, inp, inp ? a.inp_mask[row0 + l] : 0.f,
                                inp ? a.inp_pose[gi] : 0.f, inp ? a.trans[l] : 0.f, z);
      a.x[gi] = o.xn;
      Xs[l * SE + cc] = o.xn;
      if (a.extras) {
        a.extras[0 * plane + ncl] = o.mean;
        a.extras[1 * plane + ncl] = rec.var;
        a.extras[2 * plane + ncl] = rec.logvar;
        a.extras[3 * plane + ncl] = e;
        a.extras[4 * plane + ncl] = o.x0;
        a.extras[5 * plane + ncl] = o.raw;
      }
    }
  } else if (a.do_out) {
    for (int idx = tid; idx < L * C; idx += NTHREADS) {
      const int l = idx % L, cc = idx / L;
      a.eps_out[((size_t)b * C + cc) * L + l] = E[l * SE + cc];
    }
  }
  if (!a.do_emb) return;
  if (!a.do_update)
    for (int idx = tid; idx < L * C; idx += NTHREADS) Xs[(idx / C) * SE + idx % C] = a.x[row0 * C + idx];
  __syncthreads();
  STAMP(3);
  for (int idx = tid; idx < Lp * 128; idx += NTHREADS) {
    const int l = idx / 128, cc = idx % 128;
    Xb[l * SB + cc] = from_f32<T>(l < L && cc < C ? Xs[l * SE + cc] : 0.f);
  }
  __syncthreads();
  constexpr int KTE = 128 / Frag<T>::KF;
  const int tiles[4] = {4 * wave, 4 * wave + 1, 4 * wave + 2, 4 * wave + 3};
  const bool on[4] = {true, true, true, true};
  f32x4 acc[FRT][4];
  gemm_aw<T, 4, KTE>(acc, Xb, SB, RT, (const uint4*)a.w_emb, tiles, on, lane);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = tiles[j] * 16 + c16;
    const float bb = a.b_emb[col];
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt)
      if (rt < RT)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = rt * 16 + 4 * g4 + r;
          if (i < L) a.h[(row0 + i) * FD + col] = acc[rt][j][r] + bb + a.pe[(size_t)i * FD + col];
        }
  }
  if (a.stamps) {
    __syncthreads();
    STAMP(4);
  }
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
template <typename K>
static void set_lds_attr(K kernel) {
  (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

static bool fused_attrs_done = false;
static void fused_attrs() {
  if (fused_attrs_done) return;
  set_lds_attr(ka_kernel<float>);
  set_lds_attr(ka_kernel<bf16_t>);
  set_lds_attr(kb_kernel<float>);
  set_lds_attr(kb_kernel<bf16_t>);
  set_lds_attr(kc_kernel<float>);
  set_lds_attr(kc_kernel<bf16_t>);
  set_lds_attr(ke_kernel<float>);
  set_lds_attr(ke_kernel<bf16_t>);
  fused_attrs_done = true;
}

size_t fused_lds_max(int dtype, int L, int Ts) {
  size_t a, b, c, e, t1, t2, t3;
  AttGeom G;
  if (dtype == 0) {
    a = ka_lds<float>(L, &t1, &t2, &G);
    b = kb_lds<float>(L, 1 + Ts, &t1, &t2, &t3, &G);
    c = kc_lds<float>(L, &t1);
    e = ke_lds<float>(L, &t1, &t2, &t3);
  } else {
    a = ka_lds<bf16_t>(L, &t1, &t2, &G);
    b = kb_lds<bf16_t>(L, 1 + Ts, &t1, &t2, &t3, &G);
    c = kc_lds<bf16_t>(L, &t1);
    e = ke_lds<bf16_t>(L, &t1, &t2, &t3);
  }
  return std::max(std::max(a, b), std::max(c, e));
}

hipError_t launch_fused(int which, int dtype, const FusedArgs& a, int n, hipStream_t s) {
  fused_attrs();
  size_t t1, t2, t3;
  AttGeom G;
  const dim3 blk(NTHREADS);
  if (which == 0) {
    const size_t lds = dtype == 0 ? ka_lds<float>(a.L, &t1, &t2, &G) : ka_lds<bf16_t>(a.L, &t1, &t2, &G);
    if (dtype == 0) hipLaunchKernelGGL(ka_kernel<float>, dim3(8, n), blk, lds, s, a);
    else hipLaunchKernelGGL(ka_kernel<bf16_t>, dim3(8, n), blk, lds, s, a);
  } else if (which == 1) {
    const size_t lds = dtype == 0 ? kb_lds<float>(a.L, 1 + a.Ts, &t1, &t2, &t3, &G)
                                  : kb_lds<bf16_t>(a.L, 1 + a.Ts, &t1, &t2, &t3, &G);
    if (dtype == 0) hipLaunchKernelGGL(kb_kernel<float>, dim3(8, n), blk, lds, s, a);
    else hipLaunchKernelGGL(kb_kernel<bf16_t>, dim3(8, n), blk, lds, s, a);
  } else {
    const size_t lds = dtype == 0 ? kc_lds<float>(a.L, &t1) : kc_lds<bf16_t>(a.L, &t1);
    if (dtype == 0) hipLaunchKernelGGL(kc_kernel<float>, dim3(8, n), blk, lds, s, a);
    else hipLaunchKernelGGL(kc_kernel<bf16_t>, dim3(8, n), blk, lds, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_final(int dtype, const FinalArgs& a, hipStream_t s) {
  fused_attrs();
  size_t t1, t2, t3;
  const size_t lds = dtype == 0 ? ke_lds<float>(a.L, &t1, &t2, &t3) : ke_lds<bf16_t>(a.L, &t1, &t2, &t3);
  if (dtype == 0) hipLaunchKernelGGL(ke_kernel<float>, dim3(a.n), dim3(NTHREADS), lds, s, a);
  else hipLaunchKernelGGL(ke_kernel<bf16_t>, dim3(a.n), dim3(NTHREADS), lds, s, a);
  return hipGetLastError();
}

}  // namespace ggd
