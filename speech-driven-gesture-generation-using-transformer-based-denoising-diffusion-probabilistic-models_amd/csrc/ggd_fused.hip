// ggd_fused.hip -- the fused per-clip decoder kernels (d_model 256, 8 heads, L <= 64,
// memory rows 1 + Ts <= 64, d_pose <= 128).
//
// One denoise step of the one-way decoder (models/nn.py:154-228) is 4 launches per layer
// plus one epilogue launch, instead of one launch per op:
//
//   KA (head, clip)   LN1 + QKV projection of the head + 3-tap conv + self-attention
//   KB (head, clip)   SA out-proj + residual (+ h write) + LN2 + cross-attn query of the
//                     head + conv + cross-attention to the cached speech memory
//   KC (chunk, clip)  CA out-proj + residual (+ h write) + LN3 + FFN-up chunk + ReLU^2
//   KD (chunk, clip)  FFN-down of a 32-column chunk + residual, in place
//   KE (clip)         LN_out + output projection + DDPM/DDIM update (+ the next step's
//                     emb_x + PE), or eps for the model protocol
//
// Every workgroup owns one clip's rows, so the depthwise conv, the attention and every
// LayerNorm see whole sequences / whole rows in LDS.  The small out-projections are
// recomputed by each head workgroup of a clip (x8 redundant MFMA work, served from L2)
// instead of paying a launch boundary and an HBM round trip for them.
//
// The kernels are latency-bound (a clip is 40 rows; a step is ~17 dependent launches), so
// they are written for few dependent memory round trips:
//   * every global load is unconditional (row indices clamped into the clip) and issued in
//     one batch at the top of its phase -- a load under a branch gets its own vmcnt(0) wait;
//   * f32 rows of 1 KiB are staged by LDS-DMA (global_load_lds_dwordx4, one row per wave
//     instruction), bf16 operand images through registers;
//   * row tiles are padded to 64 rows at compile time: no runtime branch wraps an MFMA,
//     rows >= L hold don't-care values whose results are never stored;
//   * weights are packed on the host in MFMA B-fragment order -- [n tile][k step][lane][16 B]
//     -- and stream straight into registers with 1 KiB coalesced loads, issued before the
//     activations they multiply have arrived.
#include <algorithm>

#include "ggd_common.h"

namespace ggd {

constexpr int FD = 256, FDK = 32, FR = 64, FRT = 4, FLK = 64;  // d_model, d_k, rows, row tiles, max keys
constexpr int SH = FD + 4;                                     // f32 residual image row stride
typedef __attribute__((address_space(3))) void lds_void;

template <typename T> struct Frag {
  static constexpr int KF = 64 / sizeof(T);   // k covered by one fragment: 32 (bf16) / 16 (f32)
  static constexpr int PT = 16 / sizeof(T);   // 16-byte LDS row pad
  static constexpr int SX = FD + PT;          // operand image row stride (elements)
};

__host__ __device__ constexpr size_t al16(size_t v) { return (v + 15) & ~(size_t)15; }

// diagnostics: phase stamps of workgroup (0, 0), written only when the stamp buffer is set
#define STAMP(i)                                                                                \
  do {                                                                                          \
    if (a.stamps && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)                     \
      a.stamps[i] = __builtin_amdgcn_s_memtime();                                               \
  } while (0)
#define STAMP_END(i)                                                                            \
  do {                                                                                          \
    if (a.stamps) {                                                                             \
      __syncthreads();                                                                          \
      STAMP(i);                                                                                 \
    }                                                                                           \
  } while (0)

// ------------------------------------------------------------------------------------------
// bounded stores: a raw buffer resource over a clip's output rows; the hardware drops stores
// past num_records, so padded rows are written without a branch.  (A store under a divergent
// branch makes the compiler re-wait vmcnt inside every branch, serialising the stores.)
// ------------------------------------------------------------------------------------------
struct OutRows {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ OutRows(void* base, uint32_t bytes)
      : r(__builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)bytes, 0x00020000)) {}
  __device__ __forceinline__ void put4(uint32_t elem, float4 v) const {  // 4 f32 at elem
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
    const u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(u, r, (int)(elem * 4), 0, 0);
  }
  template <typename T> __device__ __forceinline__ void put(uint32_t elem, float v) const {
    if constexpr (sizeof(T) == 2)
      __builtin_amdgcn_raw_buffer_store_b16(f2bf(v), r, (int)(elem * 2), 0, 0);
    else
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)(elem * 4), 0, 0);
  }
};

// ------------------------------------------------------------------------------------------
// staging
// ------------------------------------------------------------------------------------------
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, NOT for
// its outstanding global loads (prefetches for later phases stay in flight) or stores.
// __syncthreads() waits vmcnt(0) as well: use it where LDS-DMA writes must have landed.
__device__ __forceinline__ void bar_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS-DMA copy of `rows` rows of `pieces` x 1 KiB from src (row stride ss bytes) into dst
// (row stride sd bytes): wave w issues the pieces w, w + NW, ...; lane l moves bytes 16l..16l+15.
template <int NT = NTHREADS>
__device__ __forceinline__ void glds_rows(void* dst, size_t sd, const void* src, size_t ss, int rows, int pieces) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int p = wave; p < rows * pieces; p += NT / 64) {
    const int r = p / pieces, q = p - r * pieces;
    __builtin_amdgcn_global_load_lds((const void*)((const char*)src + r * ss + q * 1024 + lane * 16),
                                     (lds_void*)((char*)dst + r * sd + q * 1024), 16, 0, 0);
  }
}

// A [64][SX] operand image of L rows of d_model activations of type T (global rows of FD).
// bf16 rows are 512 B (two rows per LDS-DMA instruction would cross the pad): registers.
template <typename T> struct ImgStage {
  static constexpr int NV = sizeof(T) == 2 ? FR * FD * 2 / 16 / NTHREADS : 1;
  uint4 v[NV];
  __device__ __forceinline__ void load(T* img, const T* src, int L) {
    if constexpr (sizeof(T) == 4) {
      glds_rows(img, sizeof(T) * Frag<T>::SX, src, sizeof(T) * FD, L, 1);
    } else {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int idx = threadIdx.x + i * NTHREADS, r = idx >> 5, c = idx & 31;
        v[i] = *(const uint4*)(src + (size_t)min(r, L - 1) * FD + c * 8);
      }
    }
  }
  // every image row is written (rows >= L hold copies of row L - 1): a conditional store
  // lets the compiler sink the global load into the branch and serialise the round trips
  __device__ __forceinline__ void store(T* img, int L) {
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int idx = threadIdx.x + i * NTHREADS, r = idx >> 5, c = idx & 31;
        *(uint4*)(img + r * Frag<T>::SX + c * 8) = v[i];
      }
    }
  }
};

// ------------------------------------------------------------------------------------------
// MFMA against fragment-packed weights
// ------------------------------------------------------------------------------------------
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

// C[64 rows][NJ tiles] = A[64][K] x W tiles, K = KT fragment steps starting at step k0.
// Fragments are held in registers in groups of G steps: bf16 the whole K (issued by
// load(0) before the caller's activation staging), f32 (parity mode) in groups of 32 / NJ.
template <typename T, int NJ, int KT>
struct WGemm {
  static constexpr int G = sizeof(T) == 2 ? KT : (32 / NJ < KT ? 32 / NJ : KT);
  static_assert(KT % G == 0, "k steps must split into register groups");
  uint4 wb[NJ][G];
  const uint4* W;
  int tiles[NJ];
  int kt_total, k0;
  __device__ __forceinline__ WGemm(const void* Wp, int kt_total_, int k0_) : W((const uint4*)Wp), kt_total(kt_total_), k0(k0_) {}
  __device__ __forceinline__ void load(int g, int lane) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int k = 0; k < G; ++k) wb[j][k] = W[((size_t)tiles[j] * kt_total + k0 + g * G + k) * 64 + lane];
  }
  // group 0 must have been loaded; tiles j >= nj_on are skipped (wave-uniform)
  __device__ __forceinline__ void run(f32x4 (&acc)[FRT][NJ], const T* A, int SA, int lane, int nj_on = NJ) {
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int g = 0; g < KT / G; ++g) {
      if (g > 0) load(g, lane);
#pragma unroll
      for (int k = 0; k < G; ++k)
#pragma unroll
        for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            if (j < nj_on) mma_aw<T>(acc[rt][j], A, SA, rt, g * G + k, wb[j][k], lane);
    }
  }
};

// ------------------------------------------------------------------------------------------
// LayerNorm (eps 1e-5, two-pass) of the f32 rows Hs[0..L) (stride SH) into a T image
// ------------------------------------------------------------------------------------------
// statistics: 4 lanes per row, each summing 16 float4 (the generic GEMM's LN prologue order)
__device__ __forceinline__ void ln_stats(const float* Hs, int L, float2* st) {
  const int tid = threadIdx.x, r = tid >> 2, j = tid & 3;
  if (r >= FR) return;
  const int rr = min(r, L - 1);
  float4 v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = *(const float4*)(Hs + rr * SH + (j + 4 * i) * 4);
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
  if (j == 0) st[r] = make_float2(mu, 1.0f / sqrtf(q / (float)FD + 1e-5f));
}

// normalize: thread t owns columns 4 (t & 63) .. +3 (gamma / beta preloaded), rows t >> 6 + NW i;
// rows >= L are written as zeros.  All LDS reads are issued before the first write (one wave
// per SIMD hides nothing: a read-use-read loop pays the LDS latency per row).
template <typename T, int NT = NTHREADS>
__device__ __forceinline__ void ln_apply(const float* Hs, int L, const float2* st, float4 g, float4 bb, T* img) {
  constexpr int NW = NT / 64, NI = FR / NW;
  const int c4 = (threadIdx.x & 63) * 4, r0 = threadIdx.x >> 6;
  float4 v[NI];
  float2 s[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int rr = min(r0 + NW * i, L - 1);
    v[i] = *(const float4*)(Hs + rr * SH + c4);
    s[i] = st[rr];
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r = r0 + NW * i;
    const bool ok = r < L;
    T* o = img + r * Frag<T>::SX + c4;
    o[0] = from_f32<T>(ok ? (v[i].x - s[i].x) * s[i].y * g.x + bb.x : 0.f);
    o[1] = from_f32<T>(ok ? (v[i].y - s[i].x) * s[i].y * g.y + bb.y : 0.f);
    o[2] = from_f32<T>(ok ? (v[i].z - s[i].x) * s[i].y * g.z + bb.z : 0.f);
    o[3] = from_f32<T>(ok ? (v[i].w - s[i].x) * s[i].y * g.w + bb.w : 0.f);
  }
}

// ------------------------------------------------------------------------------------------
// depthwise 3-tap conv (Primer-EZ, transformer.py:28-44) and attention (transformer.py:88-118)
// ------------------------------------------------------------------------------------------
struct ConvW { float w0, w1, w2, b; };
__device__ __forceinline__ ConvW conv_w(const float* w, const float* b, int c) {
  return ConvW{w[c * 3 + 0], w[c * 3 + 1], w[c * 3 + 2], b[c]};
}

// dst rows (or transposed columns) i < 64 = conv over rows i-1, i, i+1 of the f32 source (row
// stride ss, column c = tid & 31 of the thread; zero outside [0, rows)); rows >= `rows` are
// written as zeros, so padded keys / values are finite
template <typename T, bool TRANS>
__device__ __forceinline__ void conv_rows(T* dst, int S, const float* src, int ss, int rows, ConvW w) {
  const int c = threadIdx.x & 31, i0 = threadIdx.x >> 5;
  float p0[8], p1[8], p2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int i = i0 + 8 * k;
    p0[k] = src[min(max(i - 1, 0), rows - 1) * ss + c];
    p1[k] = src[min(i, rows - 1) * ss + c];
    p2[k] = src[min(i + 1, rows - 1) * ss + c];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int i = i0 + 8 * k;
    const float v = w.b + w.w0 * (i > 0 ? p0[k] : 0.f) + w.w1 * p1[k] + w.w2 * (i + 1 < rows ? p2[k] : 0.f);
    const T o = from_f32<T>(i < rows ? v : 0.f);
    if (TRANS)
      dst[c * S + i] = o;
    else
      dst[i * S + c] = o;
  }
}

template <typename T> struct FAtt {
  static constexpr int P = 16 / sizeof(T);
  static constexpr int SQ = FDK + P;       // Q / K rows
  static constexpr int SV = FLK + P;       // V^T rows (keys along the row)
  static constexpr int SP = FLK + P;       // per-wave P tile rows
  static constexpr size_t OQ = 0;
  static constexpr size_t OK = OQ + sizeof(T) * FR * SQ;
  static constexpr size_t OV = OK + sizeof(T) * FLK * SQ;
  static constexpr size_t OP = OV + sizeof(T) * FDK * SV;
  static constexpr size_t BYTES = OP + sizeof(T) * 4 * 16 * SP;
};

__device__ __forceinline__ void att_mma16(f32x4& acc, const bf16_t* X, int SX, const bf16_t* Y, int SY, int k0, int lane) {
  const int r16 = lane & 15, g = lane >> 4;
  const bf16x8 a = *(const bf16x8*)(X + r16 * SX + k0 + g * 8);
  const bf16x8 b = *(const bf16x8*)(Y + r16 * SY + k0 + g * 8);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
}
__device__ __forceinline__ void att_mma16(f32x4& acc, const float* X, int SX, const float* Y, int SY, int k0, int lane) {
  const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 32; kk += 16) {
    const f32x4 a = *(const f32x4*)(X + r16 * SX + k0 + kk + g * 4);
    const f32x4 b = *(const f32x4*)(Y + r16 * SY + k0 + kk + g * 4);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
  }
}

// O[Lq][32] = softmax(scale Q K^T) V for one head; wave w owns query rows 16w..16w+15.
// LKT = key tiles of 16 (Lk <= 16 LKT, LKT even).  Keys >= Lk are masked by select (their K
// rows may hold anything); V^T columns >= Lk must be finite (zeroed by the caller).
template <typename T, int LKT>
__device__ __forceinline__ void fattn(unsigned char* att, int Lq, int Lk, float scale, T* out, int ldo) {
  using A = FAtt<T>;
  const T* Qm = (const T*)(att + A::OQ);
  const T* Km = (const T*)(att + A::OK);
  const T* Vt = (const T*)(att + A::OV);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c16 = lane & 15, g4 = lane >> 4;
  T* P = (T*)(att + A::OP) + wave * 16 * A::SP;
  const int rt = wave;
  if (rt * 16 >= Lq) return;
  f32x4 s[LKT];
#pragma unroll
  for (int t = 0; t < LKT; ++t) {
    s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    att_mma16(s[t], Qm + rt * 16 * A::SQ, A::SQ, Km + t * 16 * A::SQ, A::SQ, 0, lane);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < LKT; ++t) {
      const float v = t * 16 + c16 < Lk ? s[t][r] * scale : -INFINITY;
      s[t][r] = v;
      mx = fmaxf(mx, v);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 1));
    mx = fmaxf(mx, __shfl_xor(mx, 2));
    mx = fmaxf(mx, __shfl_xor(mx, 4));
    mx = fmaxf(mx, __shfl_xor(mx, 8));
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < LKT; ++t) {
      const float p = t * 16 + c16 < Lk ? expf(s[t][r] - mx) : 0.f;
      s[t][r] = p;
      sum += p;
    }
    sum += __shfl_xor(sum, 1);
    sum += __shfl_xor(sum, 2);
    sum += __shfl_xor(sum, 4);
    sum += __shfl_xor(sum, 8);
    const float inv = 1.0f / sum;
#pragma unroll
    for (int t = 0; t < LKT; ++t) P[(4 * g4 + r) * A::SP + t * 16 + c16] = from_f32<T>(s[t][r] * inv);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const OutRows dst(out, (uint32_t)(sizeof(T) * ((size_t)(Lq - 1) * ldo + FDK)));  // rows >= Lq dropped
#pragma unroll
  for (int ct = 0; ct < FDK / 16; ++ct) {
    f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k0 = 0; k0 < LKT * 16; k0 += 32) att_mma16(o, P, A::SP, Vt + ct * 16 * A::SV, A::SV, k0, lane);
#pragma unroll
    for (int r = 0; r < 4; ++r) dst.put<T>((uint32_t)((rt * 16 + 4 * g4 + r) * ldo + ct * 16 + c16), o[r]);
  }
}

template <typename T>
__device__ __forceinline__ void fattn_any(unsigned char* att, int Lq, int Lk, float scale, T* out, int ldo) {
  if (Lk <= 32)
    fattn<T, 2>(att, Lq, Lk, scale, out, ldo);
  else
    fattn<T, 4>(att, Lq, Lk, scale, out, ldo);
}

// ------------------------------------------------------------------------------------------
// LDS plans (bytes; FR = 64 rows everywhere)
// ------------------------------------------------------------------------------------------
template <typename T> struct Plan {
  static constexpr size_t IMG = al16(sizeof(T) * FR * Frag<T>::SX);
  static constexpr size_t HS = al16(sizeof(float) * FR * SH);
  static constexpr size_t ST = sizeof(float2) * FR;
  static constexpr size_t Y_KA = al16(sizeof(float) * FR * (96 + 4));
  static constexpr size_t YQ = al16(sizeof(float) * FR * (FDK + 4));
  static constexpr size_t RAW = al16(sizeof(float) * 2 * (FLK + 2) * FDK);
  // KA: [Xn][stats][Hs | Y + att]
  static constexpr size_t KA = IMG + ST + std::max(HS, Y_KA + FAtt<T>::BYTES);
  // KB: [Ax][stats][Hs | Yq + raw + att]
  static constexpr size_t KB = IMG + ST + std::max(HS, YQ + RAW + FAtt<T>::BYTES);
  // KC: [Ax][stats][Hs]
  static constexpr size_t KC = IMG + ST + HS;
  // KD: [hid pass image 64 x (KP + PT)] ; the cross-wave reduction reuses it
  static constexpr int KP = sizeof(T) == 2 ? 4 * FD : 2 * FD;
  static constexpr size_t KD = al16(sizeof(T) * FR * (KP + Frag<T>::PT));
  // KE: [Xn / Xb][stats][Hs | E (64 x 132 f32) + Xs (64 x 128 f32)]
  static constexpr size_t E = al16(sizeof(float) * FR * (128 + 4));
  static constexpr size_t XS = al16(sizeof(float) * FR * 128);
  static constexpr size_t KE = IMG + ST + std::max(HS, E + XS);
};
static_assert(Plan<float>::KA <= 160 * 1024 && Plan<float>::KB <= 160 * 1024 && Plan<float>::KE <= 160 * 1024 &&
                  Plan<float>::KD <= 160 * 1024,
              "fused LDS plans must fit 160 KiB");

// ------------------------------------------------------------------------------------------
// KA: LN1 + QKV(head) + conv + self-attention          grid (heads, clips)
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(NTHREADS) ka_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  using PL = Plan<T>;
  constexpr int KT = FD / Frag<T>::KF, SY = 96 + 4;
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = a.L, c16 = lane & 15, g4 = lane >> 4;
  T* Xn = (T*)smem;
  float2* st = (float2*)(smem + PL::IMG);
  unsigned char* un = smem + PL::IMG + PL::ST;
  float* Hs = (float*)un;
  float* Y = (float*)un;
  unsigned char* att = un + PL::Y_KA;
  const FusedLayer& w = a.w;

  STAMP(0);
  if (a.bump_counter && h == 0 && b == 0 && tid == 0) atomicAdd(a.step_counter, 1);
  glds_rows(Hs, sizeof(float) * SH, a.h + (size_t)b * L * FD, sizeof(float) * FD, L, 1);
  // QKV of head h: packed as 6 tiles [q0 q1 k0 k1 v0 v1]; wave w owns tiles w and w + 4 (< 6)
  WGemm<T, 2, KT> gm(w.qkv, KT, 0);
  gm.tiles[0] = h * 6 + wave;
  gm.tiles[1] = h * 6 + min(wave + 4, 5);
  gm.load(0, lane);
  const float bias0 = w.qkv_b[h * 96 + wave * 16 + c16];
  const float bias1 = w.qkv_b[h * 96 + min(wave + 4, 5) * 16 + c16];
  const float4 lg = *(const float4*)(w.ln1_g + (tid & 63) * 4), lb = *(const float4*)(w.ln1_b + (tid & 63) * 4);
  const ConvW cq = conv_w(w.sa_qw, w.sa_qb, tid & 31), ck = conv_w(w.sa_kw, w.sa_kb, tid & 31),
              cv = conv_w(w.sa_vw, w.sa_vb, tid & 31);
  __syncthreads();  // LDS-DMA rows and every operand above have landed
  ln_stats(Hs, L, st);
  bar_lds();
  ln_apply<T>(Hs, L, st, lg, lb, Xn);
  bar_lds();
  STAMP(1);
  // Hs is dead from here: Y and the attention images overlay it
  f32x4 acc[FRT][2];
  gm.run(acc, Xn, Frag<T>::SX, lane, wave + 4 < 6 ? 2 : 1);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j == 1 && wave + 4 >= 6) continue;
    const int col = (j == 0 ? wave : wave + 4) * 16 + c16;
    const float bias = j == 0 ? bias0 : bias1;
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) Y[(rt * 16 + 4 * g4 + r) * SY + col] = acc[rt][j][r] + bias;
  }
  bar_lds();
  STAMP(2);
  using AT = FAtt<T>;
  conv_rows<T, false>((T*)(att + AT::OQ), AT::SQ, Y, SY, L, cq);
  conv_rows<T, false>((T*)(att + AT::OK), AT::SQ, Y + 32, SY, L, ck);
  conv_rows<T, true>((T*)(att + AT::OV), AT::SV, Y + 64, SY, L, cv);
  bar_lds();
  STAMP(3);
  fattn_any<T>(att, L, L, a.scale, (T*)a.o_sa + (size_t)b * L * FD + h * FDK, FD);
  STAMP_END(4);
}

// Hs[i][n] += A[i] . W[n] + bias[n] for all 64 rows; wave w owns columns [64w, 64w + 64)
template <typename T>
__device__ __forceinline__ void outproj_epilogue(float* Hs, const f32x4 (&acc)[FRT][4], const float (&bias)[4], int lane,
                                                 int wave) {
  const int c16 = lane & 15, g4 = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = (4 * wave + j) * 16 + c16;
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float* p = Hs + (rt * 16 + 4 * g4 + r) * SH + col;
        *p = *p + (acc[rt][j][r] + bias[j]);
      }
  }
}

// rows [0, L) of Hs -> global rows: all 64 rows read, then bounded 16-byte stores
__device__ __forceinline__ void store_rows(float* dst, const float* Hs, int L) {
  const OutRows out(dst, (uint32_t)(sizeof(float) * L * FD));
  float4 v[FR * FD / 4 / NTHREADS];
#pragma unroll
  for (int i = 0; i < FR * FD / 4 / NTHREADS; ++i) {
    const int idx = threadIdx.x + i * NTHREADS, r = idx >> 6, c = (idx & 63) * 4;
    v[i] = *(const float4*)(Hs + min(r, L - 1) * SH + c);
  }
#pragma unroll
  for (int i = 0; i < FR * FD / 4 / NTHREADS; ++i) {
    const int idx = threadIdx.x + i * NTHREADS, r = idx >> 6, c = (idx & 63) * 4;
    out.put4((uint32_t)(r * FD + c), v[i]);
  }
}

// ------------------------------------------------------------------------------------------
// KB: SA out-proj + residual + LN2 + cross-attn Q(head) + conv + cross-attention  (heads, clips)
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(NTHREADS) kb_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  using PL = Plan<T>;
  using AT = FAtt<T>;
  constexpr int KT = FD / Frag<T>::KF, SYQ = FDK + 4;
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = a.L, Lk = 1 + a.Ts, c16 = lane & 15, g4 = lane >> 4;
  T* Ax = (T*)smem;                   // O_sa image, then LN2(h) image
  float2* st = (float2*)(smem + PL::IMG);
  unsigned char* un = smem + PL::IMG + PL::ST;
  float* Hs = (float*)un;
  float* Yq = (float*)un;
  float* raw = (float*)(un + PL::YQ);
  unsigned char* att = un + PL::YQ + PL::RAW;
  const FusedLayer& w = a.w;
  const size_t row0 = (size_t)b * L;

  STAMP(0);
  const int t = a.t_clip ? a.t_clip[b] : a.steps[*a.step_counter].t_orig;
  glds_rows(Hs, sizeof(float) * SH, a.h + row0 * FD, sizeof(float) * FD, L, 1);
  ImgStage<T> so;
  so.load(Ax, (const T*)a.o_sa + row0 * FD, L);
  WGemm<T, 4, KT> go(w.o_sa, KT, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j) go.tiles[j] = 4 * wave + j;
  go.load(0, lane);
  float bo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bo[j] = w.o_sa_b[(4 * wave + j) * 16 + c16];
  const float4 lg = *(const float4*)(w.ln2_g + (tid & 63) * 4), lb = *(const float4*)(w.ln2_b + (tid & 63) * 4);
  so.store(Ax, L);
  __syncthreads();  // LDS-DMA rows and every operand above have landed
  STAMP(1);
  // cross-attn query of head h: waves 0, 1 own tiles 2h, 2h + 1 of the natural packing
  WGemm<T, 1, KT> gq(w.q_ca, KT, 0);
  gq.tiles[0] = 2 * h + (wave & 1);
  gq.load(0, lane);
  const float bq = w.q_ca_b[h * FDK + (wave & 1) * 16 + c16];
  const ConvW cq = conv_w(w.ca_qw, w.ca_qb, tid & 31), ck = conv_w(w.ca_kw, w.ca_kb, tid & 31),
              cv = conv_w(w.ca_vw, w.ca_vb, tid & 31);
  // memory K / V of head h (pre-conv): row 0 = the step token of this clip's t, rows 1.. the
  // cached speech rows; item v = (row, half, 16-byte piece) with row clamped into [0, Lk)
  static_assert(2 * FLK * 8 == 4 * NTHREADS, "four 16-byte memory pieces per thread");
  auto kv_load = [&](int i) -> float4 {
    const int v = tid + i * NTHREADS, r = min(v >> 4, Lk - 1), half = (v >> 3) & 1, q = v & 7;
    const float* src = r == 0 ? w.kv_step + (size_t)t * 2 * FD : w.kv_mem + ((size_t)b * a.Ts + (r - 1)) * 2 * FD;
    return *(const float4*)(src + half * FD + h * FDK + q * 4);
  };
  // named registers, not an array: an array live across the LN is demoted to scratch
  const float4 kv0 = kv_load(0), kv1 = kv_load(1), kv2 = kv_load(2), kv3 = kv_load(3);
  {
    f32x4 acc[FRT][4];
    go.run(acc, Ax, Frag<T>::SX, lane);
    outproj_epilogue<T>(Hs, acc, bo, lane, wave);
  }
  bar_lds();
  STAMP(2);
  if (h == 0) store_rows(a.h_out + row0 * FD, Hs, L);
  ln_stats(Hs, L, st);
  bar_lds();
  ln_apply<T>(Hs, L, st, lg, lb, Ax);
  bar_lds();
  STAMP(3);
  // Hs is dead: Yq, raw and the attention images overlay it
  auto kv_store = [&](int i, float4 val) {
    const int v = tid + i * NTHREADS, r = v >> 4, half = (v >> 3) & 1, q = v & 7;
    if (r < Lk) *(float4*)(raw + half * (FLK + 2) * FDK + (r + 1) * FDK + q * 4) = val;
  };
  kv_store(0, kv0);
  kv_store(1, kv1);
  kv_store(2, kv2);
  kv_store(3, kv3);
  if (tid < 2 * 2 * FDK) {  // zero halo rows 0 and Lk + 1 of both halves
    const int half = tid >> 6, e = tid & 63, r = e < FDK ? 0 : Lk + 1;
    raw[half * (FLK + 2) * FDK + r * FDK + (e & 31)] = 0.f;
  }
  {
    f32x4 acc[FRT][1];
    gq.run(acc, Ax, Frag<T>::SX, lane, wave < 2 ? 1 : 0);
    if (wave < 2) {
      const int col = (wave & 1) * 16 + c16;
#pragma unroll
      for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) Yq[(rt * 16 + 4 * g4 + r) * SYQ + col] = acc[rt][0][r] + bq;
    }
  }
  bar_lds();
  STAMP(4);
  conv_rows<T, false>((T*)(att + AT::OQ), AT::SQ, Yq, SYQ, L, cq);
  conv_rows<T, false>((T*)(att + AT::OK), AT::SQ, raw + FDK, FDK, Lk, ck);
  conv_rows<T, true>((T*)(att + AT::OV), AT::SV, raw + (FLK + 2) * FDK + FDK, FDK, Lk, cv);
  bar_lds();
  STAMP(5);
  fattn_any<T>(att, L, Lk, a.scale, (T*)a.o_ca + row0 * FD + h * FDK, FD);
  STAMP_END(6);
}

// ------------------------------------------------------------------------------------------
// KC: CA out-proj + residual + LN3 + FFN-up chunk (128 hidden) + ReLU^2   grid (8 chunks, clips)
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(NTHREADS) kc_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  using PL = Plan<T>;
  constexpr int KT = FD / Frag<T>::KF;
  const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = a.L, c16 = lane & 15, g4 = lane >> 4;
  T* Ax = (T*)smem;
  float2* st = (float2*)(smem + PL::IMG);
  float* Hs = (float*)(smem + PL::IMG + PL::ST);
  const FusedLayer& w = a.w;
  const size_t row0 = (size_t)b * L;

  STAMP(0);
  glds_rows(Hs, sizeof(float) * SH, a.h + row0 * FD, sizeof(float) * FD, L, 1);
  ImgStage<T> so;
  so.load(Ax, (const T*)a.o_ca + row0 * FD, L);
  WGemm<T, 4, KT> go(w.o_ca, KT, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j) go.tiles[j] = 4 * wave + j;
  go.load(0, lane);
  float bo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bo[j] = w.o_ca_b[(4 * wave + j) * 16 + c16];
  const float4 lg = *(const float4*)(w.ln3_g + (tid & 63) * 4), lb = *(const float4*)(w.ln3_b + (tid & 63) * 4);
  so.store(Ax, L);
  __syncthreads();  // LDS-DMA rows and every operand above have landed
  STAMP(1);
  WGemm<T, 2, KT> gf(w.ff1, KT, 0);  // prefetch: in flight across the out-projection
  gf.tiles[0] = 8 * c + 2 * wave;
  gf.tiles[1] = 8 * c + 2 * wave + 1;
  gf.load(0, lane);
  const float bf0 = w.ff1_b[(8 * c + 2 * wave) * 16 + c16], bf1 = w.ff1_b[(8 * c + 2 * wave + 1) * 16 + c16];
  {
    f32x4 acc[FRT][4];
    go.run(acc, Ax, Frag<T>::SX, lane);
    outproj_epilogue<T>(Hs, acc, bo, lane, wave);
  }
  bar_lds();
  STAMP(2);
  if (c == 0) store_rows(a.h_out + row0 * FD, Hs, L);
  ln_stats(Hs, L, st);
  bar_lds();
  ln_apply<T>(Hs, L, st, lg, lb, Ax);
  bar_lds();
  STAMP(3);
  f32x4 acc[FRT][2];
  gf.run(acc, Ax, Frag<T>::SX, lane);
  const OutRows out((T*)a.hid + row0 * (4 * FD), (uint32_t)(sizeof(T) * L * 4 * FD));
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = (8 * c + 2 * wave + j) * 16 + c16;
    const float bb = j == 0 ? bf0 : bf1;
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = fmaxf(acc[rt][j][r] + bb, 0.f);
        out.put<T>((uint32_t)((rt * 16 + 4 * g4 + r) * (4 * FD) + col), v * v);
      }
  }
  STAMP_END(4);
}

// ------------------------------------------------------------------------------------------
// KD: FFN-down (K = 1024) of 32 output columns + residual, in place     grid (8 chunks, clips)
// wave w: column tile (w & 1), K half (w >> 1); the two K halves meet through LDS.
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(NTHREADS) kd_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  using PL = Plan<T>;
  constexpr int KP = PL::KP, NP = 4 * FD / KP, SA = KP + Frag<T>::PT;
  constexpr int KTT = 4 * FD / Frag<T>::KF, KTW = KP / Frag<T>::KF / 2;  // k steps: total, per wave per pass
  const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = a.L, c16 = lane & 15, g4 = lane >> 4, tile = 2 * c + (wave & 1), kh = wave >> 1;
  T* Hd = (T*)smem;
  const FusedLayer& w = a.w;
  const size_t row0 = (size_t)b * L;
  const int col = tile * 16 + c16;

  STAMP(0);
  float res[FRT][4];
#pragma unroll
  for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) res[rt][r] = a.h[(row0 + min(rt * 16 + 4 * g4 + r, L - 1)) * FD + col];
  const float bias = w.ff2_b[col];
  f32x4 acc[FRT][1];
#pragma unroll
  for (int rt = 0; rt < FRT; ++rt) acc[rt][0] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int p = 0; p < NP; ++p) {
    if (p > 0) __syncthreads();  // the previous pass' image is consumed
    glds_rows(Hd, sizeof(T) * SA, (const T*)a.hid + row0 * (4 * FD) + p * KP, sizeof(T) * 4 * FD, L,
              (int)(sizeof(T) * KP / 1024));
    WGemm<T, 1, KTW> gd(w.ff2, KTT, p * (KP / Frag<T>::KF) + kh * KTW);
    gd.tiles[0] = tile;
    gd.load(0, lane);
    __syncthreads();
    if (p == 0) STAMP(1);
    f32x4 part[FRT][1];
    gd.run(part, Hd + kh * KTW * Frag<T>::KF, SA, lane);
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt) acc[rt][0] += part[rt][0];
  }
  bar_lds();
  STAMP(2);
  f32x4* red = (f32x4*)smem;  // [2 tiles][FRT][64 lanes]
  if (kh == 1)
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt) red[((wave & 1) * FRT + rt) * 64 + lane] = acc[rt][0];
  bar_lds();
  if (kh == 0) {
    const OutRows out(a.h + row0 * FD, (uint32_t)(sizeof(float) * L * FD));
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt) {
      const f32x4 o = red[((wave & 1) * FRT + rt) * 64 + lane];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out.put<float>((uint32_t)((rt * 16 + 4 * g4 + r) * FD + col), res[rt][r] + ((acc[rt][0][r] + o[r]) + bias));
    }
  }
  STAMP_END(3);
}

// ------------------------------------------------------------------------------------------
// KE: LN_out + out-proj (eps) [+ diffusion update] [+ next step's emb_x + PE]   grid (clips)
// 512 threads: the update is VALU work (Philox, Box-Muller, the posterior arithmetic) on one
// clip's L x C elements, and two waves per SIMD issue it twice as fast as one.
// ------------------------------------------------------------------------------------------
constexpr int KE_THREADS = 512;

template <typename T>
__global__ void __launch_bounds__(KE_THREADS) ke_kernel(FinalArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  using PL = Plan<T>;
  constexpr int NT = KE_THREADS;
  constexpr int KT = FD / Frag<T>::KF, SE = 128 + 4, SB = 128 + Frag<T>::PT, KTE = 128 / Frag<T>::KF;
  constexpr int NXV = FR * 128 / NT;  // staged state values per thread (max L x C)
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = a.L, C = a.C, c16 = lane & 15, g4 = lane >> 4, LC = L * C;
  T* Xn = (T*)smem;
  T* Xb = (T*)smem;  // the emb operand image reuses the LN image
  float2* st = (float2*)(smem + PL::IMG);
  unsigned char* un = smem + PL::IMG + PL::ST;
  float* Hs = (float*)un;
  float* E = (float*)un;
  float* Xs = (float*)(un + PL::E);
  const size_t row0 = (size_t)b * L;

  STAMP(0);
  // state x of this clip (internal (L, C) order, contiguous) -> registers
  float xv[NXV];
  if (a.do_update || a.do_emb) {
#pragma unroll
    for (int i = 0; i < NXV; ++i) xv[i] = a.x[row0 * C + min(tid + i * NT, LC - 1)];
  }
  int k = 0;
  StepRec rec{};
  if (a.do_update) {
    k = *a.step_counter;
    rec = a.steps[k];
  }
  if (a.do_out) {
    glds_rows<NT>(Hs, sizeof(float) * SH, a.h + row0 * FD, sizeof(float) * FD, L, 1);
    WGemm<T, 1, KT> go(a.w_out, KT, 0);  // wave w: output tile w (d_pose <= 128)
    go.tiles[0] = wave;
    go.load(0, lane);
    const float bo = a.b_out[wave * 16 + c16];
    const float4 lg = *(const float4*)(a.ln_g + (tid & 63) * 4), lb = *(const float4*)(a.ln_b + (tid & 63) * 4);
    __syncthreads();  // LDS-DMA rows and every operand above have landed
    ln_stats(Hs, L, st);
    bar_lds();
    ln_apply<T, NT>(Hs, L, st, lg, lb, Xn);
    bar_lds();
    STAMP(1);
    f32x4 acc[FRT][1];
    go.run(acc, Xn, Frag<T>::SX, lane);
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) E[(rt * 16 + 4 * g4 + r) * SE + wave * 16 + c16] = acc[rt][0][r] + bo;
  }
  if (a.do_update || a.do_emb) {
#pragma unroll
    for (int i = 0; i < NXV; ++i) {
      const int e = tid + i * NT;
      if (e < LC) Xs[e] = xv[i];
    }
  }
  // emb_x + PE of the new state: fragments / PE / bias issued now, in flight across the update
  WGemm<T, 2, KTE> ge(a.w_emb, KTE, 0);
  float pe[2][FRT][4], be[2];
  if (a.do_emb) {
    ge.tiles[0] = 2 * wave;
    ge.tiles[1] = 2 * wave + 1;
    ge.load(0, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = (2 * wave + j) * 16 + c16;
      be[j] = a.b_emb[col];
#pragma unroll
      for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) pe[j][rt][r] = a.pe[(size_t)min(rt * 16 + 4 * g4 + r, L - 1) * FD + col];
    }
  }
  bar_lds();
  STAMP(2);
  if (a.do_update) {
    // element e = cc * L + l of the reference (N, C, L) block; quads of 4 share one Philox call
    const size_t plane = (size_t)a.n * LC;
    const float* nz = a.noise ? a.noise + (size_t)k * plane + (size_t)b * LC : nullptr;
    const bool inp = a.inp_mask != nullptr;
    for (int q = tid; q * 4 < LC; q += NT) {
      float z[4];
      if (nz) {
#pragma unroll
        for (int u = 0; u < 4; ++u) z[u] = nz[min(4 * q + u, LC - 1)];
      } else {
        philox_normal4(a.seed, (uint32_t)(a.clip_offset + b), (uint32_t)rec.i, TAG_STEP, (uint32_t)q, z);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = 4 * q + u;
        if (e >= LC) break;
        const int cc = e / L, l = e - cc * L;
        const int gi = l * C + cc;
        const float x = Xs[gi], ev = E[l * SE + cc];
        const UpdOut o = upd_math(rec, a.alg, x, ev, false, 0.f, inp, inp ? a.inp_mask[row0 + l] : 0.f,
                                  inp ? a.inp_pose[row0 * C + gi] : 0.f, inp ? a.trans[l] : 0.f, z[u]);
        a.x[row0 * C + gi] = o.xn;
        Xs[gi] = o.xn;
        if (a.extras) {
          const size_t ncl = (size_t)b * LC + e;
          a.extras[0 * plane + ncl] = o.mean;
          a.extras[1 * plane + ncl] = rec.var;
          a.extras[2 * plane + ncl] = rec.logvar;
          a.extras[3 * plane + ncl] = ev;
          a.extras[4 * plane + ncl] = o.x0;
          a.extras[5 * plane + ncl] = o.raw;
        }
      }
    }
  } else if (a.do_out) {
    for (int e = tid; e < LC; e += NT) {
      const int cc = e / L, l = e - cc * L;
      a.eps_out[(size_t)b * LC + e] = E[l * SE + cc];
    }
  }
  if (!a.do_emb) {
    STAMP_END(3);
    return;
  }
  bar_lds();
  STAMP(3);
  for (int idx = tid; idx < FR * 128; idx += NT) {
    const int l = idx >> 7, cc = idx & 127;
    Xb[l * SB + cc] = from_f32<T>(l < L && cc < C ? Xs[l * C + cc] : 0.f);
  }
  bar_lds();
  f32x4 acc[FRT][2];
  ge.run(acc, Xb, SB, lane);
  const OutRows out(a.h + row0 * FD, (uint32_t)(sizeof(float) * L * FD));
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = (2 * wave + j) * 16 + c16;
#pragma unroll
    for (int rt = 0; rt < FRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out.put<float>((uint32_t)((rt * 16 + 4 * g4 + r) * FD + col), acc[rt][j][r] + be[j] + pe[j][rt][r]);
  }
  STAMP_END(4);
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
  set_lds_attr(kd_kernel<float>);
  set_lds_attr(kd_kernel<bf16_t>);
  set_lds_attr(ke_kernel<float>);
  set_lds_attr(ke_kernel<bf16_t>);
  fused_attrs_done = true;
}

bool fused_supported(int dtype, int d_model, int heads, int L, int Ts, int C) {
  (void)dtype;
  return d_model == FD && heads == FD / FDK && L >= 1 && L <= FR && Ts >= 1 && 1 + Ts <= FLK && C >= 1 && C <= 128;
}

hipError_t launch_fused(int which, int dtype, const FusedArgs& a, int n, hipStream_t s) {
  fused_attrs();
  const dim3 blk(NTHREADS), grid(8, n);
  const bool f = dtype == 0;
  switch (which) {
    case 0:
      if (f) hipLaunchKernelGGL(ka_kernel<float>, grid, blk, Plan<float>::KA, s, a);
      else hipLaunchKernelGGL(ka_kernel<bf16_t>, grid, blk, Plan<bf16_t>::KA, s, a);
      break;
    case 1:
      if (f) hipLaunchKernelGGL(kb_kernel<float>, grid, blk, Plan<float>::KB, s, a);
      else hipLaunchKernelGGL(kb_kernel<bf16_t>, grid, blk, Plan<bf16_t>::KB, s, a);
      break;
    case 2:
      if (f) hipLaunchKernelGGL(kc_kernel<float>, grid, blk, Plan<float>::KC, s, a);
      else hipLaunchKernelGGL(kc_kernel<bf16_t>, grid, blk, Plan<bf16_t>::KC, s, a);
      break;
    case 3:
      if (f) hipLaunchKernelGGL(kd_kernel<float>, grid, blk, Plan<float>::KD, s, a);
      else hipLaunchKernelGGL(kd_kernel<bf16_t>, grid, blk, Plan<bf16_t>::KD, s, a);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_final(int dtype, const FinalArgs& a, hipStream_t s) {
  fused_attrs();
  if (dtype == 0) hipLaunchKernelGGL(ke_kernel<float>, dim3(a.n), dim3(KE_THREADS), Plan<float>::KE, s, a);
  else hipLaunchKernelGGL(ke_kernel<bf16_t>, dim3(a.n), dim3(KE_THREADS), Plan<bf16_t>::KE, s, a);
  return hipGetLastError();
}

}  // namespace ggd
