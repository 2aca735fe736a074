// ggd_common.h -- device helpers shared by the libggd kernel files (gfx950 only).
#pragma once
#include "ggd_kernels.h"

namespace ggd {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int KC = 256;          // K chunk staged in LDS per iteration
constexpr int NT = 64;           // output columns per workgroup
constexpr int NTHREADS = 256;    // 4 waves

__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
// two floats -> packed bf16 pair (lo in bits 0-15): one v_cvt_pk_bf16_f32, the same rounding as f2bf
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  typedef float f2v __attribute__((ext_vector_type(2)));
  typedef __bf16 h2v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2v{lo, hi}, h2v));
}
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
// counter-based Gaussian noise (oracle/philox.py restates it: Philox bits exact, the
// Box-Muller floats within a few ulp -- hardware log2 / sin / cos against numpy's libm)
// ---------------------------------------------------------------------------
constexpr uint32_t TAG_STEP = 0, TAG_XT = 1;

// the four normals of quad q (elements 4q .. 4q+3) from ONE Philox call:
//   counter (q, clip, step, tag), key (seed_lo, seed_hi) -> u0..u3 -> two Box-Muller pairs
__device__ __forceinline__ void philox_normal4(uint64_t seed, uint32_t clip, uint32_t step, uint32_t tag,
                                               uint32_t q, float (&z)[4]) {
#pragma clang fp contract(off)
  uint32_t c0 = q, c1 = clip, c2 = step, c3 = tag;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  // hardware transcendentals: v_log_f32 is log2, v_sin/cos_f32 take revolutions (the angle
  // 2 pi u is never formed); within a few ulp of the float32 libm form (oracle/philox.py)
  const float inv = 2.3283064365386963e-10f, m2ln2 = -1.3862943611198906f;  // -2 ln 2
  const float ra = __builtin_amdgcn_sqrtf(m2ln2 * __builtin_amdgcn_logf(((float)c0 + 1.0f) * inv));
  const float rb = __builtin_amdgcn_sqrtf(m2ln2 * __builtin_amdgcn_logf(((float)c2 + 1.0f) * inv));
  const float ua = (float)c1 * inv, ub = (float)c3 * inv;
  z[0] = ra * __builtin_amdgcn_cosf(ua);
  z[1] = ra * __builtin_amdgcn_sinf(ua);
  z[2] = rb * __builtin_amdgcn_cosf(ub);
  z[3] = rb * __builtin_amdgcn_sinf(ub);
}

// element e of the stream (the quad e / 4, lane e % 4)
__device__ __forceinline__ float philox_normal(uint64_t seed, uint32_t clip, uint32_t step, uint32_t tag,
                                               uint32_t e) {
  float z[4];
  philox_normal4(seed, clip, step, tag, e >> 2, z);
  const int sel = e & 3;
  return sel == 0 ? z[0] : sel == 1 ? z[1] : sel == 2 ? z[2] : z[3];
}

// ---------------------------------------------------------------------------
// diffusion update (gaussian_diffusion.py:268-275, 287-298, 207-232, 326-328, 465-483;
// inpaint denoise_fn generator.py:272-281).  IEEE ops in the reference's order, no fma
// contraction, so given the same eps and noise it matches the CPU oracle bit for bit.
// ---------------------------------------------------------------------------
struct UpdOut { float x0, raw, mean, xn; };

// ---------------------------------------------------------------------------
// bounded waits of the persistent loops (clip groups, clip pairs, long clips): a wait ends after
// WAIT_TICKS of ELAPSED time on the chip-wide 100 MHz realtime counter, not after an iteration
// count -- the exit cannot depend on what a poll observes or on how long one poll takes (round 4's
// scalar-load poll variant hung: its polls never saw the partner flags).  No legitimate barrier or
// residency wait comes near the bound; a loop that reaches it sets its status word and leaves.
// ---------------------------------------------------------------------------
constexpr unsigned long long WAIT_TICKS = 200000000ull;  // 2 s at 100 MHz
// a wave leaving a barrier wait early.  `expired`: its OWN wait ran out -- code 1 and the
// STATUS_TIMEOUT bit (ggd_kernels.h; the bit dominates any code, so a timed-out launch opens no
// gate and the host reports the timeout).  Otherwise it only saw another workgroup's code (e.g. 2:
// a workgroup whose residency wait expired) and drains with code 1, which keeps that 2 / 3 intact
// so the device-gated fallback still opens.  One atomic either way (a second one cost the long-clip
// loop a register spill: it sits at 256 VGPRs).
__device__ __forceinline__ void status_leave(int* status, bool expired) {
  atomicMax(status, expired ? (1 | STATUS_TIMEOUT) : 1);
}
// 32-bit: the low word of the 100 MHz counter wraps every 43 s, far above WAIT_TICKS; one register
// fewer than the 64-bit value in the persistent loops' poll code (the long loop sits at 256 VGPRs)
__device__ __forceinline__ unsigned wait_t0() { return (unsigned)__builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ bool wait_expired(unsigned t0) {
  return (unsigned)__builtin_amdgcn_s_memrealtime() - t0 > (unsigned)WAIT_TICKS;
}

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


// ---------------------------------------------------------------------------
// attention building blocks (transformer.py:28-44, 88-118)
// ---------------------------------------------------------------------------
constexpr int ATT_LMAX = 192;
constexpr int ATT_DKMAX = 64;
constexpr int ATT_KT = ATT_LMAX / 16;   // max key tiles

template <typename T> struct AttPad { static constexpr int P = 16 / sizeof(T); };  // 16-byte row pad

struct AttGeom {
  int Lqp, Lkp, SQ, SV, SP;
  size_t off_q, off_k, off_v, off_p, off_raw, total;
};

template <typename T>
__host__ __device__ inline AttGeom att_geom(int Lq, int Lk, int dk) {
  // P V runs K = Lkp: 32-key steps on bf16 MFMA, 4-key steps on f32 (16-key padding suffices)
  constexpr int KA = sizeof(T) == 2 ? 32 : 16;
  AttGeom g;
  g.Lqp = (Lq + 15) / 16 * 16;
  g.Lkp = (Lk + KA - 1) / KA * KA;
  g.SQ = dk + AttPad<T>::P;
  g.SV = g.Lkp + AttPad<T>::P;
  g.SP = g.Lkp + AttPad<T>::P;
  g.off_q = 0;
  g.off_k = g.off_q + sizeof(T) * (size_t)g.Lqp * g.SQ;
  g.off_v = g.off_k + sizeof(T) * (size_t)g.Lkp * g.SQ;
  g.off_p = g.off_v + sizeof(T) * (size_t)dk * g.SV;
  // the f32 staging rows (raw) live only before the core starts and P only inside it: they share
  g.off_raw = g.off_p;
  const int lmax = Lq > Lk ? Lq : Lk;
  const size_t p_bytes = sizeof(T) * (size_t)4 * 16 * g.SP, raw_bytes = sizeof(float) * (size_t)(lmax + 2) * dk;
  g.total = g.off_p + (p_bytes > raw_bytes ? p_bytes : raw_bytes);
  return g;
}

template <typename T>
__device__ __forceinline__ void att_stage_rows(float* raw, const void* src, size_t row0, int ld, int col0,
                                               int rows, int dk) {
  // raw[(r + 1) * dk + c] = src[(row0 + r) * ld + col0 + c]; rows -1 and `rows` are zero halos
  constexpr int VE = 16 / sizeof(T);
  const int vpr = dk / VE;
  for (int v = threadIdx.x; v < rows * vpr; v += NTHREADS) {
    const int r = v / vpr, cv = v % vpr;
    const uint4 u = *(const uint4*)((const T*)src + (row0 + r) * ld + col0 + cv * VE);
    float* dst = raw + (r + 1) * dk + cv * VE;
    if constexpr (sizeof(T) == 2) {
      const bf16_t* h = (const bf16_t*)&u;
#pragma unroll
      for (int e = 0; e < 8; ++e) dst[e] = bf2f(h[e]);
    } else {
      *(uint4*)dst = u;
    }
  }
  for (int c = threadIdx.x; c < dk; c += NTHREADS) {
    raw[c] = 0.f;
    raw[(rows + 1) * dk + c] = 0.f;
  }
}

// conv over the haloed raw image; writes T rows (dst[i * S + c]) or transposed (dst[c * S + i])
template <typename T, bool TRANS>
__device__ __forceinline__ void att_conv(T* dst, int S, const float* raw, int rows, int dk, const float* w,
                                         const float* b) {
  for (int idx = threadIdx.x; idx < rows * dk; idx += NTHREADS) {
    const int i = idx / dk, c = idx % dk;
    const float* p = raw + i * dk + c;  // rows i-1, i, i+1 of the haloed image
    const float v = b[c] + w[c * 3 + 0] * p[0] + w[c * 3 + 1] * p[dk] + w[c * 3 + 2] * p[2 * dk];
    if (TRANS)
      dst[c * S + i] = from_f32<T>(v);
    else
      dst[i * S + c] = from_f32<T>(v);
  }
}

// ------------------------------------------------------------------------------------------
// lane-group reductions on DPP (VALU-rate lane moves, no LDS round trip; __shfl_xor lowers to
// ds_bpermute whose ~100-cycle latency is exposed on every step of a dependent reduction)
// ------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E;               // quad_perm [1,0,3,2], [2,3,0,1]
constexpr int DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;    // within 8 / 16 lanes
// reduce over aligned groups of G lanes (G = 2, 4, 8 or 16); every lane of a group gets the result
template <int G>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (G >= 2) v += dpp_mov<DPP_XOR1>(v);
  if constexpr (G >= 4) v += dpp_mov<DPP_XOR2>(v);
  if constexpr (G >= 8) v += dpp_mov<DPP_HALF_MIRROR>(v);
  if constexpr (G >= 16) v += dpp_mov<DPP_MIRROR>(v);
  return v;
}
template <int G>
__device__ __forceinline__ float group_max(float v) {
  if constexpr (G >= 2) v = fmaxf(v, dpp_mov<DPP_XOR1>(v));
  if constexpr (G >= 4) v = fmaxf(v, dpp_mov<DPP_XOR2>(v));
  if constexpr (G >= 8) v = fmaxf(v, dpp_mov<DPP_HALF_MIRROR>(v));
  if constexpr (G >= 16) v = fmaxf(v, dpp_mov<DPP_MIRROR>(v));
  return v;
}

// LayerNorm statistics of rows held by 4 consecutive lanes, N float4 of the row per lane (two-pass:
// mean, then the centred sum of squares), on packed f32 pairs (v_pk_add / v_pk_mul / v_pk_fma_f32,
// half the instructions of the scalar form) with explicit fma so that the contraction cannot
// depend on the call site: shared by gemm_kernel's PRO_LN prologue, the row-block chains and the
// long-clip loop, which must agree bit for bit.  k = the row length.
template <int N>
__device__ __forceinline__ void ln_stats4(const float4 (&v)[N], float k, float& mu, float& rs) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 s2 = f2{0.f, 0.f};
#pragma unroll
  for (int i = 0; i < N; ++i) s2 += f2{v[i].x, v[i].y} + f2{v[i].z, v[i].w};
  float s = s2.x + s2.y;
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  mu = s / k;
  const f2 m2 = f2{mu, mu};
  f2 q2 = f2{0.f, 0.f};
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const f2 a = f2{v[i].x, v[i].y} - m2, b = f2{v[i].z, v[i].w} - m2;
    q2 += __builtin_elementwise_fma(b, b, a * a);
  }
  float q = q2.x + q2.y;
  q += __shfl_xor(q, 1);
  q += __shfl_xor(q, 2);
  rs = 1.0f / sqrtf(q / k + 1e-5f);
}

// acc += X[xr0 + 0..15][0..K) . Y[yr0 + 0..15][0..K)^T   (both row-major with row stride S)
template <typename T>
__device__ __forceinline__ void att_mma(f32x4& acc, const T* X, int xr0, int SX, const T* Y, int yr0, int SY, int K,
                                        int lane) {
  const int r16 = lane & 15, g = lane >> 4;
  if constexpr (sizeof(T) == 2) {
    for (int k0 = 0; k0 < K; k0 += 32) {
      const bf16x8 a = *(const bf16x8*)(X + (xr0 + r16) * SX + k0 + g * 8);
      const bf16x8 b = *(const bf16x8*)(Y + (yr0 + r16) * SY + k0 + g * 8);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
  } else {
    for (int k0 = 0; k0 < K; k0 += 16) {
      const f32x4 a = *(const f32x4*)(X + (xr0 + r16) * SX + k0 + g * 4);
      const f32x4 b = *(const f32x4*)(Y + (yr0 + r16) * SY + k0 + g * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
    }
  }
}


// Q/K/V operand images in LDS -> O.  Each wave owns 16-row query tiles: S = Q K^T on MFMA
// (16 x Lk_pad accumulators in registers), softmax on the accumulator layout (row reductions
// over the 16 lanes sharing a row: xor 1, 2, 4, 8), P to a per-wave LDS tile, O = P V on MFMA.
// out points at row 0, column 0 of this (clip, head) block; rows i < Lq are written.
template <typename T>
__device__ __forceinline__ void attn_core(const T* Qm, const T* Km, const T* Vt, T* Pw, const AttGeom& G, int Lq,
                                          int Lk, int dk, float scale, T* out, int ldo) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, g4 = lane >> 4;
  const int LKT = G.Lkp / 16;
  T* P = Pw + wave * 16 * G.SP;
  for (int rt = wave; rt * 16 < Lq; rt += 4) {
    f32x4 s[ATT_KT];
#pragma unroll
    for (int t = 0; t < ATT_KT; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (t < LKT) att_mma<T>(s[t], Qm, rt * 16, G.SQ, Km, t * 16, G.SQ, dk, lane);
    }
    // softmax over keys for the 4 rows this lane holds (row = 4 * g4 + r)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < ATT_KT; ++t) {
        const bool ok = t < LKT && t * 16 + c16 < Lk;
        const float v = ok ? s[t][r] * scale : -INFINITY;
        s[t][r] = v;
        mx = fmaxf(mx, v);
      }
      mx = group_max<16>(mx);
      float sum = 0.f;
#pragma unroll
      for (int t = 0; t < ATT_KT; ++t) {
        const bool ok = t < LKT && t * 16 + c16 < Lk;
        const float p = ok ? expf(s[t][r] - mx) : 0.f;
        s[t][r] = p;
        sum += p;
      }
      sum = group_sum<16>(sum);
      const float inv = 1.0f / sum;
#pragma unroll
      for (int t = 0; t < ATT_KT; ++t)
        if (t < LKT) P[(4 * g4 + r) * G.SP + t * 16 + c16] = from_f32<T>(s[t][r] * inv);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // O = P V for the dk / 16 column tiles
#pragma unroll
    for (int ct = 0; ct < ATT_DKMAX / 16; ++ct) {
      if (ct * 16 >= dk) break;
      f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
      att_mma<T>(o, P, 0, G.SP, Vt, ct * 16, G.SV, G.Lkp, lane);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = rt * 16 + 4 * g4 + r;
        if (i < Lq) out[(size_t)i * ldo + ct * 16 + c16] = from_f32<T>(o[r]);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace ggd
