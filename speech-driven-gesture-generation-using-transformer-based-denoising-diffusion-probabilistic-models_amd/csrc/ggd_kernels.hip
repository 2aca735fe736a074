// ggd_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the gesture-diffusion denoise step.
//
// Kernel inventory:
//   gemm_kernel     LDS-tiled MFMA GEMM, out = epi(pro(A) . W^T + b).  bf16 operands on
//                   v_mfma_f32_16x16x32_bf16, or f32 operands on v_mfma_f32_16x16x4_f32 (exact
//                   f32 parity mode).  Prologues: plain / LayerNorm-on-load / f32 cast;
//                   epilogues: store, ReLU^2, SiLU, residual add, sinusoidal PE add.
//   attn_kernel     one workgroup per (head, clip): the Primer-EZ 3-tap depthwise conv on
//                   Q/K/V fused on load, QK^T, 64-lane wavefront softmax, PV.
//   update_kernel   fused DDPM / DDIM posterior update with inpaint x0-replacement and
//                   counter-based (Philox4x32-10 + Box-Muller) noise.
#include "ggd_kernels.h"

namespace ggd {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int KC = 128;          // K chunk staged in LDS per iteration
constexpr int NT = 64;           // output columns per workgroup
constexpr int NTHREADS = 256;    // 4 waves

__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
__device__ __forceinline__ float bf2f(bf16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t from_f32<bf16_t>(float v) { return f2bf(v); }
template <typename T> __device__ __forceinline__ float to_f32(T v);
template <> __device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f32<bf16_t>(bf16_t v) { return bf2f(v); }

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------------------
// GEMM
// ---------------------------------------------------------------------------
template <typename T> struct Tile;
template <> struct Tile<bf16_t> { static constexpr int PAD = 8; static constexpr int VE = 8; };
template <> struct Tile<float>  { static constexpr int PAD = 4; static constexpr int VE = 4; };

template <typename T, int MT, int PRO>
__device__ __forceinline__ void stage_a(const GemmArgs& a, T* As, int m0, int kc0,
                                        const float* s_mean, const float* s_rstd) {
  constexpr int STR = KC + Tile<T>::PAD;
  const int tid = threadIdx.x;
  if constexpr (PRO == PRO_T) {
    constexpr int VE = Tile<T>::VE;
    constexpr int VPR = KC / VE;
    const T* A = (const T*)a.A;
    for (int v = tid; v < MT * VPR; v += NTHREADS) {
      const int r = v / VPR, cv = v % VPR, m = m0 + r;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (m < a.M) val = *(const uint4*)(A + (size_t)m * a.lda + kc0 + cv * VE);
      *(uint4*)(As + r * STR + cv * VE) = val;
    }
  } else if constexpr (PRO == PRO_LN) {
    constexpr int VPR = KC / 4;
    const float* A = (const float*)a.A;
    for (int v = tid; v < MT * VPR; v += NTHREADS) {
      const int r = v / VPR, cv = v % VPR, m = m0 + r, k = kc0 + cv * 4;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < a.M) {
        x = *(const float4*)(A + (size_t)m * a.lda + k);
        const float mu = s_mean[r], rs = s_rstd[r];
        const float4 g = *(const float4*)(a.ln_g + k);
        const float4 bb = *(const float4*)(a.ln_b + k);
        x.x = (x.x - mu) * rs * g.x + bb.x;
        x.y = (x.y - mu) * rs * g.y + bb.y;
        x.z = (x.z - mu) * rs * g.z + bb.z;
        x.w = (x.w - mu) * rs * g.w + bb.w;
      }
      T* dst = As + r * STR + cv * 4;
      dst[0] = from_f32<T>(x.x); dst[1] = from_f32<T>(x.y);
      dst[2] = from_f32<T>(x.z); dst[3] = from_f32<T>(x.w);
    }
  } else {  // PRO_F32: f32 rows with only k_valid columns, arbitrary lda
    const float* A = (const float*)a.A;
    for (int v = tid; v < MT * KC; v += NTHREADS) {
      const int r = v / KC, c = v % KC, m = m0 + r, k = kc0 + c;
      float x = 0.f;
      if (m < a.M && k < a.k_valid) x = A[(size_t)m * a.lda + k];
      As[r * STR + c] = from_f32<T>(x);
    }
  }
}

template <typename T>
__device__ __forceinline__ void stage_w(const GemmArgs& a, T* Ws, int n0, int kc0) {
  constexpr int STR = KC + Tile<T>::PAD;
  constexpr int VE = Tile<T>::VE;
  constexpr int VPR = KC / VE;
  const T* W = (const T*)a.W;
  for (int v = threadIdx.x; v < NT * VPR; v += NTHREADS) {
    const int r = v / VPR, cv = v % VPR;
    *(uint4*)(Ws + r * STR + cv * VE) = *(const uint4*)(W + (size_t)(n0 + r) * a.K + kc0 + cv * VE);
  }
}

template <typename T, int TM, int TN>
__device__ __forceinline__ void mma_chunk(const T* As, const T* Ws, int arow0, int wcol0, int lane,
                                          f32x4 (&acc)[TM][TN]) {
  constexpr int STR = KC + Tile<T>::PAD;
  const int r16 = lane & 15, g = lane >> 4;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int kk = 0; kk < KC; kk += 32) {
      bf16x8 af[TM], bw[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *(const bf16x8*)(As + (arow0 + i * 16 + r16) * STR + kk + g * 8);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bw[j] = *(const bf16x8*)(Ws + (wcol0 + j * 16 + r16) * STR + kk + g * 8);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bw[j], acc[i][j], 0, 0, 0);
    }
  } else {
    // f32 operands: each lane reads 4 consecutive k; MFMA step s pairs k = 16*kk' + 4*g + s
    // identically for A and W, so every k is used once (k-permuted f32 fma chain).
#pragma unroll 2
    for (int kk = 0; kk < KC; kk += 16) {
      f32x4 af[TM], bw[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *(const f32x4*)(As + (arow0 + i * 16 + r16) * STR + kk + g * 4);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bw[j] = *(const f32x4*)(Ws + (wcol0 + j * 16 + r16) * STR + kk + g * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bw[j][s], acc[i][j], 0, 0, 0);
    }
  }
}

template <typename T, int MT, int PRO, int EPI>
__global__ void __launch_bounds__(NTHREADS) gemm_kernel(GemmArgs a) {
  constexpr int STR = KC + Tile<T>::PAD;
  constexpr int WM = MT / 2, WN = NT / 2;     // 2x2 waves
  constexpr int TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) T As[MT * STR];
  __shared__ __attribute__((aligned(16))) T Ws[NT * STR];
  __shared__ float s_mean[MT], s_rstd[MT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int n0 = blockIdx.x * NT, m0 = blockIdx.y * MT;

  if (a.step_counter && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) atomicAdd(a.step_counter, 1);

  if constexpr (PRO == PRO_LN) {
    // row statistics over the full K (LayerNorm width), two-pass, 4 threads per row whatever the
    // tile height, so a row's LN result does not depend on the batch size (shard invariance)
    constexpr int TPR = 4;
    if (tid < MT * TPR) {
      const int r = tid / TPR, j = tid % TPR, m = m0 + r;
      const float* row = (const float*)a.A + (size_t)m * a.lda;
      float s = 0.f;
      if (m < a.M)
        for (int k = j * 4; k < a.K; k += TPR * 4) {
          const float4 v = *(const float4*)(row + k);
          s += (v.x + v.y) + (v.z + v.w);
        }
      s += __shfl_xor(s, 1);
      s += __shfl_xor(s, 2);
      const float mu = s / (float)a.K;
      float q = 0.f;
      if (m < a.M)
        for (int k = j * 4; k < a.K; k += TPR * 4) {
          const float4 v = *(const float4*)(row + k);
          const float d0 = v.x - mu, d1 = v.y - mu, d2 = v.z - mu, d3 = v.w - mu;
          q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
        }
      q += __shfl_xor(q, 1);
      q += __shfl_xor(q, 2);
      if (j == 0) {
        s_mean[r] = mu;
        s_rstd[r] = 1.0f / sqrtf(q / (float)a.K + 1e-5f);
      }
    }
    __syncthreads();
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int kc0 = 0; kc0 < a.K; kc0 += KC) {
    stage_a<T, MT, PRO>(a, As, m0, kc0, s_mean, s_rstd);
    stage_w<T>(a, Ws, n0, kc0);
    __syncthreads();
    mma_chunk<T, TM, TN>(As, Ws, wr * WM, wc * WN, lane, acc);
    __syncthreads();
  }

  // epilogue: C/D map of 16x16 MFMA: col = lane & 15, row = 4 * (lane >> 4) + r
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wc * WN + j * 16 + c16;
      const float bn = a.bias[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * WM + i * 16 + g * 4 + r;
        if (m >= a.M) continue;
        float v = acc[i][j][r] + bn;
        if constexpr (EPI == EPI_T) {
          ((T*)a.out)[(size_t)m * a.ldo + n] = from_f32<T>(v);
        } else if constexpr (EPI == EPI_RELU2) {
          v = fmaxf(v, 0.f);
          ((T*)a.out)[(size_t)m * a.ldo + n] = from_f32<T>(v * v);
        } else if constexpr (EPI == EPI_F32) {
          if (n < a.n_valid) ((float*)a.out)[(size_t)m * a.ldo + n] = v;
        } else if constexpr (EPI == EPI_SILU) {
          ((float*)a.out)[(size_t)m * a.ldo + n] = v / (1.0f + expf(-v));
        } else if constexpr (EPI == EPI_RESID) {
          float* o = (float*)a.out + (size_t)m * a.ldo + n;
          *o = *o + v;
        } else {  // EPI_PE
          const int pos = (m % a.pe_period) + a.pe_offset;
          ((float*)a.out)[(size_t)m * a.ldo + n] = v + a.pe[(size_t)pos * a.N + n];
        }
      }
    }
}

template <typename T, int MT, int PRO, int EPI>
static hipError_t gemm_go(const GemmArgs& a, hipStream_t s) {
  dim3 grid(a.N / NT, (a.M + MT - 1) / MT);
  hipLaunchKernelGGL((gemm_kernel<T, MT, PRO, EPI>), grid, dim3(NTHREADS), 0, s, a);
  return hipGetLastError();
}

template <typename T, int PRO, int EPI>
static hipError_t gemm_mt(const GemmArgs& a, hipStream_t s) {
  // 64-row tiles when that still gives >= ~200 workgroups, else 32-row tiles.
  const long tiles64 = (long)(a.N / NT) * ((a.M + 63) / 64);
  if (tiles64 >= 200) return gemm_go<T, 64, PRO, EPI>(a, s);
  return gemm_go<T, 32, PRO, EPI>(a, s);
}

template <typename T, int PRO>
static hipError_t gemm_epi(int epi, const GemmArgs& a, hipStream_t s) {
  switch (epi) {
    case EPI_T: return gemm_mt<T, PRO, EPI_T>(a, s);
    case EPI_RELU2: return gemm_mt<T, PRO, EPI_RELU2>(a, s);
    case EPI_F32: return gemm_mt<T, PRO, EPI_F32>(a, s);
    case EPI_SILU: return gemm_mt<T, PRO, EPI_SILU>(a, s);
    case EPI_RESID: return gemm_mt<T, PRO, EPI_RESID>(a, s);
    case EPI_PE: return gemm_mt<T, PRO, EPI_PE>(a, s);
  }
  return hipErrorInvalidValue;
}

template <typename T>
static hipError_t gemm_pro(int pro, int epi, const GemmArgs& a, hipStream_t s) {
  switch (pro) {
    case PRO_T: return gemm_epi<T, PRO_T>(epi, a, s);
    case PRO_LN: return gemm_epi<T, PRO_LN>(epi, a, s);
    case PRO_F32: return gemm_epi<T, PRO_F32>(epi, a, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_gemm(int dtype, int pro, int epi, const GemmArgs& a, hipStream_t s) {
  if (a.N % NT != 0 || a.K % KC != 0 || a.M <= 0) return hipErrorInvalidValue;
  if (dtype == 0) return gemm_pro<float>(pro, epi, a, s);
  return gemm_pro<bf16_t>(pro, epi, a, s);
}

// ---------------------------------------------------------------------------
// attention with fused depthwise sequence conv (transformer.py:28-44, 88-118)
// ---------------------------------------------------------------------------
constexpr int ATT_LMAX = 192;  // keys per query row handled as 3 x 64 lanes

template <typename T>
__device__ __forceinline__ float ld_any(const void* p, size_t idx) {
  return to_f32<T>(((const T*)p)[idx]);
}

template <typename T>
__global__ void __launch_bounds__(NTHREADS) attn_kernel(AttnArgs a) {
  extern __shared__ float sm[];
  const int h = blockIdx.x, b = blockIdx.y;
  const int dk = a.dk, S = dk + 1, Lq = a.Lq, Lk = a.Lk;
  float* Qs = sm;
  float* Ks = Qs + Lq * S;
  float* Vs = Ks + Lk * S;
  const int tid = threadIdx.x;

  int t = 0;
  if (a.cross) t = a.t_clip ? a.t_clip[b] : a.steps[*a.step_counter].t_orig;

  // Q: 3-tap conv over the query sequence, zero padded
  for (int idx = tid; idx < Lq * dk; idx += NTHREADS) {
    const int i = idx / dk, c = idx % dk;
    const size_t col = (size_t)h * dk + c;
    const float r0 = i > 0 ? ld_any<T>(a.q, (size_t)(b * Lq + i - 1) * a.ldq + col) : 0.f;
    const float r1 = ld_any<T>(a.q, (size_t)(b * Lq + i) * a.ldq + col);
    const float r2 = i + 1 < Lq ? ld_any<T>(a.q, (size_t)(b * Lq + i + 1) * a.ldq + col) : 0.f;
    Qs[i * S + c] = a.cb_q[c] + a.cw_q[c * 3 + 0] * r0 + a.cw_q[c * 3 + 1] * r1 + a.cw_q[c * 3 + 2] * r2;
  }
  // K, V
  for (int idx = tid; idx < Lk * dk; idx += NTHREADS) {
    const int j = idx / dk, c = idx % dk;
    float k3[3], v3[3];
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      const int jj = j + o - 1;
      float kv = 0.f, vv = 0.f;
      if (jj >= 0 && jj < Lk) {
        if (!a.cross) {
          const size_t base = (size_t)(b * Lk + jj) * a.ldkv + (size_t)h * dk + c;
          kv = ld_any<T>(a.k, base);
          vv = ld_any<T>(a.v, base);
        } else {
          const float* row = jj == 0 ? a.kv_step + (size_t)t * 2 * a.d
                                     : a.kv_mem + (size_t)(b * (Lk - 1) + jj - 1) * 2 * a.d;
          kv = row[h * dk + c];
          vv = row[a.d + h * dk + c];
        }
      }
      k3[o] = kv;
      v3[o] = vv;
    }
    Ks[j * S + c] = a.cb_k[c] + a.cw_k[c * 3 + 0] * k3[0] + a.cw_k[c * 3 + 1] * k3[1] + a.cw_k[c * 3 + 2] * k3[2];
    Vs[j * S + c] = a.cb_v[c] + a.cw_v[c * 3 + 0] * v3[0] + a.cw_v[c * 3 + 1] * v3[1] + a.cw_v[c * 3 + 2] * v3[2];
  }
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6;
  const int G = 64 / dk;          // lane groups splitting the keys in P.V (2 at dk=32)
  const int c = lane % dk, g = lane / dk;
  for (int i = wave; i < Lq; i += NTHREADS / 64) {
    const float* q = Qs + i * S;
    float s[3];
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int j = lane + 64 * u;
      s[u] = -INFINITY;
      if (j < Lk) {
        const float* kr = Ks + j * S;
        float acc = 0.f;
        for (int cc = 0; cc < dk; ++cc) acc += q[cc] * kr[cc];
        s[u] = acc * a.scale;
        mx = fmaxf(mx, s[u]);
      }
    }
    mx = wave_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int j = lane + 64 * u;
      s[u] = j < Lk ? expf(s[u] - mx) : 0.f;
      sum += s[u];
    }
    sum = wave_sum(sum);
    const float inv = 1.0f / sum;
#pragma unroll
    for (int u = 0; u < 3; ++u) s[u] *= inv;

    float o = 0.f;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      if (64 * u >= Lk) break;
      for (int jj = 0; jj < 64; jj += G) {
        const int src = jj + g;
        const float p = __shfl(s[u], src);
        const int j = 64 * u + src;
        if (j < Lk) o += p * Vs[j * S + c];
      }
    }
    if (G == 2) o += __shfl_xor(o, 32);
    if (g == 0) ((T*)a.out)[(size_t)(b * Lq + i) * a.ldo + (size_t)h * dk + c] = from_f32<T>(o);
  }
}

hipError_t launch_attention(int dtype, const AttnArgs& a, int n, hipStream_t s) {
  if (a.Lq > ATT_LMAX || a.Lk > ATT_LMAX || (a.dk != 32 && a.dk != 64)) return hipErrorInvalidValue;
  const size_t lds = (size_t)(a.Lq + 2 * a.Lk) * (a.dk + 1) * sizeof(float);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)attn_kernel<float>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)attn_kernel<bf16_t>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  dim3 grid(a.heads, n);
  if (dtype == 0)
    hipLaunchKernelGGL(attn_kernel<float>, grid, dim3(NTHREADS), lds, s, a);
  else
    hipLaunchKernelGGL(attn_kernel<bf16_t>, grid, dim3(NTHREADS), lds, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// counter-based Gaussian noise (oracle/philox.py restates this bit for bit up to libm ulps)
// ---------------------------------------------------------------------------
constexpr uint32_t TAG_STEP = 0, TAG_XT = 1;

__device__ __forceinline__ float philox_normal(uint64_t seed, uint32_t clip, uint32_t step, uint32_t tag,
                                               uint32_t e) {
#pragma clang fp contract(off)
  uint32_t c0 = e >> 2, c1 = clip, c2 = step, c3 = tag;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  const int sel = e & 3;
  const uint32_t ua_i = sel < 2 ? c0 : c2, ub_i = sel < 2 ? c1 : c3;
  const float inv = 2.3283064365386963e-10f;
  const float ua = ((float)ua_i + 1.0f) * inv;
  const float ub = (float)ub_i * inv;
  const float r = sqrtf(-2.0f * logf(ua));
  const float th = 6.283185307179586f * ub;
  return (sel & 1) ? r * sinf(th) : r * cosf(th);
}

// ---------------------------------------------------------------------------
// diffusion update (gaussian_diffusion.py:268-275, 287-298, 207-232, 326-328, 465-483;
// inpaint denoise_fn generator.py:272-281).  IEEE ops in the reference's order, no fma
// contraction, so given the same eps and noise it matches the CPU oracle bit for bit.
// ---------------------------------------------------------------------------
struct UpdOut { float x0, raw, mean, xn; };

__device__ __forceinline__ UpdOut upd_math(const StepRec& r, int alg, float x, float e, bool have_x0,
                                           float x0_in, bool inp, float m, float p, float tf, float z) {
#pragma clang fp contract(off)
  UpdOut o;
  float x0 = r.sra * x - r.srm1 * e;
  o.raw = x0;
  if (have_x0) x0 = x0_in;
  if (inp) {
    const float a1 = ((1.0f - tf) * m) * p;
    const float a2 = (tf * m) * x0;
    const float a3 = (1.0f - m) * x0;
    x0 = (a1 + a2) + a3;
  }
  o.x0 = x0;
  o.mean = r.c1 * x0 + r.c2 * x;
  const float nzs = r.i != 0 ? r.sigma : 0.0f;
  if (alg == 0) {
    o.xn = o.mean + nzs * z;
  } else {
    const float e2 = (r.sra * x - x0) / r.srm1;
    const float mp = x0 * r.sqrt_abp + r.c_eps * e2;
    o.xn = mp + nzs * z;
  }
  return o;
}

__global__ void __launch_bounds__(NTHREADS) update_kernel(UpdArgs a) {
  const int total = a.n * a.L * a.C;
  const int idx = blockIdx.x * NTHREADS + threadIdx.x;
  if (idx >= total) return;
  const int c = idx % a.C, bl = idx / a.C, l = bl % a.L, b = bl / a.L;
  const int k = a.fixed_k >= 0 ? a.fixed_k : *a.step_counter;
  const StepRec r = a.steps[k];
  const float x = a.x[idx];
  const float e = a.eps[(size_t)bl * a.ld_eps + c];
  const size_t ncl = ((size_t)b * a.C + c) * a.L + l;
  float z;
  if (a.noise)
    z = a.noise[(size_t)k * a.n * a.C * a.L + ncl];
  else
    z = philox_normal(a.seed, (uint32_t)(a.clip_offset + b), (uint32_t)r.i, TAG_STEP, (uint32_t)(c * a.L + l));
  const bool inp = a.inp_mask != nullptr;
  const float m = inp ? a.inp_mask[bl] : 0.f;
  const float p = inp ? a.inp_pose[idx] : 0.f;
  const float tf = inp ? a.trans[l] : 0.f;
  const UpdOut o = upd_math(r, a.alg, x, e, false, 0.f, inp, m, p, tf, z);
  a.x[idx] = o.xn;
  if (a.extras) {
    const size_t plane = (size_t)a.n * a.C * a.L;
    a.extras[0 * plane + ncl] = o.mean;
    a.extras[1 * plane + ncl] = r.var;
    a.extras[2 * plane + ncl] = r.logvar;
    a.extras[3 * plane + ncl] = e;
    a.extras[4 * plane + ncl] = o.x0;
    a.extras[5 * plane + ncl] = o.raw;
  }
}

hipError_t launch_update(const UpdArgs& a, hipStream_t s) {
  const int total = a.n * a.L * a.C;
  hipLaunchKernelGGL(update_kernel, dim3((total + NTHREADS - 1) / NTHREADS), dim3(NTHREADS), 0, s, a);
  return hipGetLastError();
}

__global__ void __launch_bounds__(NTHREADS) posterior_kernel(PostArgs a) {
  const int total = a.n * a.C * a.L;
  const int idx = blockIdx.x * NTHREADS + threadIdx.x;
  if (idx >= total) return;
  const UpdOut o = upd_math(a.rec, a.alg, a.x[idx], a.eps[idx], a.x0 != nullptr, a.x0 ? a.x0[idx] : 0.f,
                            false, 0.f, 0.f, 0.f, a.noise ? a.noise[idx] : 0.f);
  if (a.x_out) a.x_out[idx] = o.xn;
  if (a.x0_out) a.x0_out[idx] = o.raw;
}

hipError_t launch_posterior(const PostArgs& a, hipStream_t s) {
  const int total = a.n * a.C * a.L;
  hipLaunchKernelGGL(posterior_kernel, dim3((total + NTHREADS - 1) / NTHREADS), dim3(NTHREADS), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
// sinusoidal step embedding [cos | sin] (nn.py:27-35), one row per original t
__global__ void step_embed_kernel(float* out, int T, int d) {
  const int idx = blockIdx.x * NTHREADS + threadIdx.x;
  const int half = d / 2;
  if (idx >= T * d) return;
  const int t = idx / d, k = idx % d;
  float v = 0.f;
  if (k < 2 * half) {
    const int kk = k < half ? k : k - half;
    const float f = expf((-9.210340371976184f * (float)kk) / (float)half);
    const float arg = (float)t * f;
    v = k < half ? cosf(arg) : sinf(arg);
  }
  out[idx] = v;
}

hipError_t launch_step_embed(float* out, int T, int d, hipStream_t s) {
  hipLaunchKernelGGL(step_embed_kernel, dim3((T * d + NTHREADS - 1) / NTHREADS), dim3(NTHREADS), 0, s,
                     out, T, d);
  return hipGetLastError();
}

__global__ void init_state_kernel(float* x, const float* xT, uint64_t seed, int64_t clip_offset, int n,
                                  int C, int L) {
  const int idx = blockIdx.x * NTHREADS + threadIdx.x;
  if (idx >= n * L * C) return;
  const int c = idx % C, bl = idx / C, l = bl % L, b = bl / L;
  x[idx] = xT ? xT[((size_t)b * C + c) * L + l]
              : philox_normal(seed, (uint32_t)(clip_offset + b), 0u, TAG_XT, (uint32_t)(c * L + l));
}

hipError_t launch_init_state(float* x, const float* x_T_ncl, uint64_t seed, int64_t clip_offset, int n,
                             int C, int L, hipStream_t s) {
  hipLaunchKernelGGL(init_state_kernel, dim3((n * L * C + NTHREADS - 1) / NTHREADS), dim3(NTHREADS), 0, s,
                     x, x_T_ncl, seed, clip_offset, n, C, L);
  return hipGetLastError();
}

__global__ void nlc_to_ncl_kernel(float* dst, const float* src, int n, int C, int L, int ld) {
  const int idx = blockIdx.x * NTHREADS + threadIdx.x;
  if (idx >= n * C * L) return;
  const int l = idx % L, bc = idx / L, c = bc % C, b = bc / C;
  dst[idx] = src[((size_t)b * L + l) * ld + c];
}

hipError_t launch_nlc_to_ncl(float* dst, const float* src, int n, int C, int L, int ld_src, hipStream_t s) {
  hipLaunchKernelGGL(nlc_to_ncl_kernel, dim3((n * C * L + NTHREADS - 1) / NTHREADS), dim3(NTHREADS), 0, s,
                     dst, src, n, C, L, ld_src);
  return hipGetLastError();
}

__global__ void set_int_kernel(int* p, int v) { *p = v; }

hipError_t launch_set_int(int* p, int v, hipStream_t s) {
  hipLaunchKernelGGL(set_int_kernel, dim3(1), dim3(1), 0, s, p, v);
  return hipGetLastError();
}

}  // namespace ggd
