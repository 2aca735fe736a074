// ggd_fusedlib.h -- device building blocks of the per-clip kernels (ggd_fused.hip: one launch
// per decoder phase; ggd_persist.hip: one persistent workgroup per clip for the whole loop).
// gfx950 only.  See the header comment of ggd_fused.hip for the latency rules they follow.
#pragma once
#include <algorithm>

#include "ggd_common.h"

namespace ggd {

constexpr int FD = 256, FDK = 32, FR = 64, FRT = 4, FLK = 64;  // d_model, d_k, rows, row tiles, max keys
#ifndef GGD_SCHED_FENCE
#define GGD_SCHED_FENCE 1
#endif
constexpr bool SCHED_FENCE = GGD_SCHED_FENCE != 0;  // A/B switch of the GEMM read/MFMA ordering fence
constexpr int SH = FD + 4;                                     // f32 residual image row stride
typedef __attribute__((address_space(3))) void lds_void;

template <typename T> struct Frag {
  static constexpr int KF = 64 / sizeof(T);   // k covered by one fragment: 32 (bf16) / 16 (f32)
  static constexpr int PT = 16 / sizeof(T);   // 16-byte LDS row pad
  static constexpr int SX = FD + PT;          // operand image row stride (elements)
};

__host__ __device__ constexpr size_t al16(size_t v) { return (v + 15) & ~(size_t)15; }

// Global-memory view of a pointer.  Pointers read out of argument structs in memory (the
// persistent loop's per-phase arguments) are generic, and generic loads are FLAT loads, which
// count against lgkmcnt too: every LDS wait of a phase would then also wait for its in-flight
// weight stream.  The kernels' own arguments are promoted to global by the compiler anyway.
template <typename T> using gptr = const __attribute__((address_space(1))) T*;
template <typename T> __device__ __forceinline__ gptr<T> G(const T* p) { return (gptr<T>)p; }
// 16 bytes (float4) through the global view
__device__ __forceinline__ float4 ld_f4(const float* p) {
  typedef __attribute__((ext_vector_type(4))) float f32v4;
  const f32v4 v = *G((const f32v4*)p);
  return make_float4(v.x, v.y, v.z, v.w);
}


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

// profiling: launch span of a kernel from the device-wide realtime counter (the same clock in
// every XCD).  Each workgroup stores its own start and, after its last stores have drained, its
// end into slot `slot` = [2][workgroups] — plain stores, no atomics (a same-address atomic from
// every workgroup serialises past the L2s and cost ~3 us per launch); ggd_api.hip reduces them
#define SPAN_BEGIN(slot)                                                                        \
  do {                                                                                          \
    if (a.span && threadIdx.x == 0)                                                             \
      a.span[(size_t)(slot) * 2 * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x] = \
          __builtin_amdgcn_s_memrealtime();                                                     \
  } while (0)
#define SPAN_END(slot)                                                                          \
  do {                                                                                          \
    if (a.span) {                                                                               \
      __syncthreads();                                                                          \
      if (threadIdx.x == 0)                                                                     \
        a.span[((size_t)(slot) * 2 + 1) * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x] = \
            __builtin_amdgcn_s_memrealtime();                                                   \
    }                                                                                           \
  } while (0)

// Buffer resource over `bytes` bytes at a wave-uniform base.  The base and the size are passed
// through readfirstlane so the compiler can PROVE the descriptor uniform: otherwise it wraps
// every buffer op in a waterfall loop (readfirstlane x4, compare, s_and_saveexec, op, loop) --
// slow, and ROCm 7.2's register allocator was seen placing a spill store between such a loop
// and the restore of EXEC (psk_kernel: the store ran with no lanes enabled and a live value of
// the pose state was lost).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uni_rsrc(const void* base, uint32_t bytes) {
  const uint64_t v = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// ------------------------------------------------------------------------------------------
// Cache policy of the loads / stores that carry data between decoder phases.  CP_KERNEL (0):
// the phases are separate launches, the kernel boundary makes their data visible.  CP_COH (sc1):
// the phases run inside one persistent launch (ggd_mega.hip) and hand data to the other
// workgroups of their clip group -- stores write through and loads skip the CU's vector L1
// (device-coherent on any placement; with the group on one XCD both stay in its L2).
// ------------------------------------------------------------------------------------------
constexpr int CP_KERNEL = 0, CP_COH = 16;
// CP_XL (persistent loop, every clip group on ONE XCD, checked at launch): the group shares that
// XCD's L2, so hand-off stores stay plain (the line stays in L2, which the readers' sc1 loads hit)
// instead of writing through to the Infinity Cache; loads are still sc1 (past the CU's L1).
constexpr int CP_XL = 17;
__host__ __device__ constexpr int cp_load(int cp) { return cp == CP_XL ? CP_COH : cp; }
__host__ __device__ constexpr int cp_store(int cp) { return cp == CP_XL ? 0 : cp; }

// bounded stores: a raw buffer resource over a clip's output rows; the hardware drops stores
// past num_records, so padded rows are written without a branch.  (A store under a divergent
// branch makes the compiler re-wait vmcnt inside every branch, serialising the stores.)
template <int CP = CP_KERNEL> struct OutRowsP {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ OutRowsP(void* base, uint32_t bytes)
      : r(uni_rsrc(base, bytes)) {}
  __device__ __forceinline__ void put4(uint32_t elem, float4 v) const {  // 4 f32 at elem
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
    const u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(u, r, (int)(elem * 4), 0, cp_store(CP));
  }
  // 4 consecutive values at elem as T: one 8-byte (bf16) or 16-byte (f32) store
  template <typename T> __device__ __forceinline__ void put4v(uint32_t elem, f32x4 v) const {
    if constexpr (sizeof(T) == 2) {
      typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
      const u32x2 u = {pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3])};
      __builtin_amdgcn_raw_buffer_store_b64(u, r, (int)(elem * 2), 0, cp_store(CP));
    } else {
      put4(elem, make_float4(v[0], v[1], v[2], v[3]));
    }
  }
  template <typename T> __device__ __forceinline__ void put(uint32_t elem, float v) const {
    if constexpr (sizeof(T) == 2)
      __builtin_amdgcn_raw_buffer_store_b16(f2bf(v), r, (int)(elem * 2), 0, cp_store(CP));
    else
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)(elem * 4), 0, cp_store(CP));
  }
};
using OutRows = OutRowsP<CP_KERNEL>;

// one f32 / 16 bytes at a uniform base + per-lane element offset, with cache policy CP
template <int CP>
__device__ __forceinline__ float ld_f32(const float* base, uint32_t idx) {
  if constexpr (CP == CP_KERNEL) {
    return G(base)[idx];
  } else {
    const __amdgpu_buffer_rsrc_t r = uni_rsrc(base, 0x7fffffffu);
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)(idx * 4), 0, cp_load(CP)));
  }
}
template <int CP>
__device__ __forceinline__ uint4 ld_16B(const void* base, uint32_t byte_off) {
  if constexpr (CP == CP_KERNEL) {
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
    const u32x4 v = *G((const u32x4*)((const char*)base + byte_off));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    const __amdgpu_buffer_rsrc_t r = uni_rsrc(base, 0x7fffffffu);
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, cp_load(CP));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
}

template <int CP>
__device__ __forceinline__ uint2 ld_8B(const void* base, uint32_t byte_off) {
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
  if constexpr (CP == CP_KERNEL) {
    const u32x2 v = *G((const u32x2*)((const char*)base + byte_off));
    return make_uint2(v.x, v.y);
  } else {
    const __amdgpu_buffer_rsrc_t r = uni_rsrc(base, 0x7fffffffu);
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)byte_off, 0, cp_load(CP));
    return make_uint2(v.x, v.y);
  }
}

// thread index as an opaque value: inside the persistent step loop (ggd_mega.hip) values derived
// from threadIdx.x are loop invariant, and the compiler hoists them out of the loop and keeps
// them live across every phase (spilling); an opaque index keeps them inside their phase
__device__ __forceinline__ int ltid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// ------------------------------------------------------------------------------------------
// staging
// ------------------------------------------------------------------------------------------
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, NOT for
// its outstanding global loads (prefetches for later phases stay in flight) or stores.
// __syncthreads() waits vmcnt(0) as well: use it where LDS-DMA writes must have landed.
__device__ __forceinline__ void bar_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS-DMA copy of `rows` rows of `pieces` x 1 KiB from src (row stride ss bytes) into dst
// (row stride sd bytes): wave w issues the pieces w, w + NW, ...; lane l moves bytes 16l..16l+15.
template <int NT = NTHREADS, int CP = CP_KERNEL>
__device__ __forceinline__ void glds_rows(void* dst, size_t sd, const void* src, size_t ss, int rows, int pieces) {
  const int tid = ltid(), lane = tid & 63, wave = tid >> 6;
  for (int p = wave; p < rows * pieces; p += NT / 64) {
    const int r = p / pieces, q = p - r * pieces;
    __builtin_amdgcn_global_load_lds((const void*)((const char*)src + r * ss + q * 1024 + lane * 16),
                                     (lds_void*)((char*)dst + r * sd + q * 1024), 16, 0, cp_load(CP));
  }
}

// A [64][SX] operand image of L rows of d_model activations of type T (global rows of FD).
// bf16 rows are 512 B (two rows per LDS-DMA instruction would cross the pad): registers.
template <typename T, int NT = NTHREADS, int CP = CP_KERNEL> struct ImgStage {
  static constexpr int NV = sizeof(T) == 2 ? FR * FD * 2 / 16 / NT : 1;
  uint4 v[NV];
  __device__ __forceinline__ void load(T* img, const T* src, int L) {
    if constexpr (sizeof(T) == 4) {
      glds_rows<NT, CP>(img, sizeof(T) * Frag<T>::SX, src, sizeof(T) * FD, L, 1);
    } else {
      const int tid = ltid();
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int idx = tid + i * NT, r = idx >> 5, c = idx & 31;
        v[i] = ld_16B<CP>(src, (uint32_t)(sizeof(T) * ((size_t)min(r, L - 1) * FD + c * 8)));
      }
    }
  }
  // every image row is written (rows >= L hold copies of row L - 1): a conditional store
  // lets the compiler sink the global load into the branch and serialise the round trips
  __device__ __forceinline__ void store(T* img, int L) {
    if constexpr (sizeof(T) == 2) {
      const int tid = ltid();
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int idx = tid + i * NT, r = idx >> 5, c = idx & 31;
        *(uint4*)(img + r * Frag<T>::SX + c * 8) = v[i];
      }
    }
  }
};

// ------------------------------------------------------------------------------------------
// MFMA against fragment-packed weights
// ------------------------------------------------------------------------------------------
// acc += A[rt*16 .. +16)[k step kf] x fragment wb   (A row-major in LDS, stride SA)
// TR: the product is computed transposed, C^T = W A^T (the fragment-packed weight tile as the
// MFMA A operand, the activation rows as B -- the same lane maps), so lane (c16, g4) holds the 4
// CONSECUTIVE output columns 4 g4 .. 4 g4 + 3 of row c16: epilogues move 16 bytes per row tile
// instead of four scalars.
template <typename T, bool TR = false>
__device__ __forceinline__ void mma_aw(f32x4& acc, const T* A, int SA, int rt, int kf, uint4 wb, int lane) {
  const int r16 = lane & 15, g = lane >> 4;
  if constexpr (sizeof(T) == 2) {
    const bf16x8 av = *(const bf16x8*)(A + (rt * 16 + r16) * SA + kf * 32 + g * 8);
    if constexpr (TR)
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wb), av, acc, 0, 0, 0);
    else
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, __builtin_bit_cast(bf16x8, wb), acc, 0, 0, 0);
  } else {
    const f32x4 av = *(const f32x4*)(A + (rt * 16 + r16) * SA + kf * 16 + g * 4);
    const f32x4 bv = __builtin_bit_cast(f32x4, wb);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if constexpr (TR)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(bv[s], av[s], acc, 0, 0, 0);
      else
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], acc, 0, 0, 0);
    }
  }
}

// C[64 rows][NJ tiles] = A[64][K] x W tiles, K = KT fragment steps starting at step k0.
// Fragments are held in registers in groups of G steps: bf16 the whole K (issued by
// load(0) before the caller's activation staging), f32 (parity mode) in groups of 32 / NJ.
template <typename T, int NJ, int KT, int RT = FRT>
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
      for (int k = 0; k < G; ++k) {
        typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
        const u32x4 v = ggd::G((const u32x4*)W)[((size_t)tiles[j] * kt_total + k0 + g * G + k) * 64 + lane];
        wb[j][k] = make_uint4(v.x, v.y, v.z, v.w);
      }
  }
  __device__ __forceinline__ void load_tile(int j, int lane) {  // group 0 of tile j only
#pragma unroll
    for (int k = 0; k < G; ++k) {
      typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
      const u32x4 v = ggd::G((const u32x4*)W)[((size_t)tiles[j] * kt_total + k0 + k) * 64 + lane];
      wb[j][k] = make_uint4(v.x, v.y, v.z, v.w);
    }
  }
  // k step k of every tile (bf16: group 0 holds the whole K)
  __device__ __forceinline__ void load_step(int k, int lane) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
      const u32x4 v = ggd::G((const u32x4*)W)[((size_t)tiles[j] * kt_total + k0 + k) * 64 + lane];
      wb[j][k] = make_uint4(v.x, v.y, v.z, v.w);
    }
  }
  // group 0 must have been loaded; tiles j >= nj_on are skipped (wave-uniform).  bf16: the A
  // fragments of k step k + 1 are read from LDS before the MFMAs of step k issue, so the LDS
  // latency overlaps the matrix work (one wave per SIMD hides nothing on its own).
  // zero = false: accumulate onto the caller's acc (e.g. residual + bias preloaded)
  // FENCE: -1 the unit's SCHED_FENCE, 0 / 1 this call site's own choice
  // after(k) runs once step k's MFMAs have issued (bf16): e.g. the next GEMM's step k loaded into
  // the registers step k has just freed (WGemm::load_step), a weight stream without a second set
  template <bool TR = false, int FENCE = -1>
  __device__ __forceinline__ void run(f32x4 (&acc)[RT][NJ], const T* A, int SA, int lane, int nj_on = NJ,
                                      bool zero = true) {
    run_then<TR, FENCE>(acc, A, SA, lane, [](int) {}, nj_on, zero);
  }
  template <bool TR = false, int FENCE = -1, typename AF>
  __device__ __forceinline__ void run_then(f32x4 (&acc)[RT][NJ], const T* A, int SA, int lane, AF&& after,
                                           int nj_on = NJ, bool zero = true) {
    constexpr bool FEN = FENCE < 0 ? SCHED_FENCE : FENCE != 0;
    if (zero) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (sizeof(T) == 2) {
      const int r16 = lane & 15, gq = lane >> 4;
      const T* a0 = A + r16 * SA + gq * 8;
      bf16x8 cur[RT], nxt[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) cur[rt] = *(const bf16x8*)(a0 + rt * 16 * SA);
#pragma unroll
      for (int k = 0; k < KT; ++k) {
        if (k + 1 < KT) {
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) nxt[rt] = *(const bf16x8*)(a0 + rt * 16 * SA + (k + 1) * 32);
        }
        // keep step k + 1's LDS reads ahead of step k's MFMAs: left alone, the scheduler (under
        // register pressure) sinks each read next to its MFMA and exposes the LDS latency per step
        if constexpr (FEN) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            if (j < nj_on) {
              if constexpr (TR)
                acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wb[j][k]), cur[rt],
                                                                     acc[rt][j], 0, 0, 0);
              else
                acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[rt], __builtin_bit_cast(bf16x8, wb[j][k]),
                                                                     acc[rt][j], 0, 0, 0);
            }
        if constexpr (FEN) __builtin_amdgcn_sched_barrier(0);
        after(k);
        if (k + 1 < KT) {
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) cur[rt] = nxt[rt];
        }
      }
    } else {
#pragma unroll 1
      for (int g = 0; g < KT / G; ++g) {
        if (g > 0) load(g, lane);
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              if (j < nj_on) mma_aw<T, TR>(acc[rt][j], A, SA, rt, g * G + k, wb[j][k], lane);
      }
    }
  }
};

// ------------------------------------------------------------------------------------------
// LayerNorm (eps 1e-5, two-pass) of the f32 rows Hs[0..L) (stride SH) into a T image
// ------------------------------------------------------------------------------------------
// statistics: LPR lanes per row (4: the generic GEMM's LN prologue order), each summing 64 / LPR
// float4 of the row; rows r < NR are computed for threads r * LPR .. r * LPR + LPR - 1
template <int NR = FR, int LPR = 4>
__device__ __forceinline__ void ln_stats(const float* Hs, int L, float2* st, int tid = ltid()) {
  constexpr int NV = 64 / LPR;
  const int r = tid / LPR, j = tid % LPR;
  if (r >= NR) return;
  const int rr = min(r, L - 1);
  float4 v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = *(const float4*)(Hs + rr * SH + (j + LPR * i) * 4);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  s = group_sum<LPR>(s);
  const float mu = s / (float)FD;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float d0 = v[i].x - mu, d1 = v[i].y - mu, d2 = v[i].z - mu, d3 = v[i].w - mu;
    q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
  }
  q = group_sum<LPR>(q);
  if (j == 0) st[r] = make_float2(mu, 1.0f / sqrtf(q / (float)FD + 1e-5f));
}

// normalize: thread t owns columns 4 (t & 63) .. +3 (gamma / beta preloaded), rows t >> 6 + NW i;
// rows >= L are written as zeros.  All LDS reads are issued before the first write (one wave
// per SIMD hides nothing: a read-use-read loop pays the LDS latency per row).
template <typename T, int NT = NTHREADS, int NR = FR, int SXI = Frag<T>::SX>
__device__ __forceinline__ void ln_apply(const float* Hs, int L, const float2* st, float4 g, float4 bb, T* img,
                                         int tid = ltid()) {
  constexpr int NW = NT / 64, NI = NR / NW;
  const int c4 = (tid & 63) * 4, r0 = tid >> 6;
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
    const float y0 = ok ? (v[i].x - s[i].x) * s[i].y * g.x + bb.x : 0.f;
    const float y1 = ok ? (v[i].y - s[i].x) * s[i].y * g.y + bb.y : 0.f;
    const float y2 = ok ? (v[i].z - s[i].x) * s[i].y * g.z + bb.z : 0.f;
    const float y3 = ok ? (v[i].w - s[i].x) * s[i].y * g.w + bb.w : 0.f;
    if constexpr (sizeof(T) == 2) {  // one 8-byte LDS store per row instead of four 2-byte ones
      const uint32_t lo = pk_bf16(y0, y1);
      const uint32_t hi = pk_bf16(y2, y3);
      *(uint2*)(img + r * SXI + c4) = make_uint2(lo, hi);
    } else {
      *(float4*)(img + r * SXI + c4) = make_float4(y0, y1, y2, y3);
    }
  }
}

// One-pass LayerNorm without the affine (gamma / beta are folded into the consuming Linear at
// finalize, ggd_api.hip frag_from): row r of the f32 image Hs (stride SH) -> (x - mu) / sigma into
// the T image (stride SXI).  Each row is held by 8 lanes, 32 values each, in registers: mean,
// centred variance (two-pass, as torch) and the normalised output need no LDS round trip and no
// barrier between them.  Rows L .. NR - 1 are written as zeros.  The per-value arithmetic runs on
// packed f32 pairs (v_pk_add / v_pk_fma / v_pk_mul_f32) and bf16 pairs are converted with one
// v_cvt_pk_bf16_f32: half the VALU instructions of the scalar form (the LN segments are
// instruction-bound on the 5 waves that hold the 40 rows; measured 0.9 us per LN before).
template <typename T, int NT, int NR, int SXI = Frag<T>::SX>
__device__ __forceinline__ void ln_rows(const float* Hs, int L, T* img, int tid = ltid()) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 h2 __attribute__((ext_vector_type(2)));
  constexpr int RPP = NT / 8;  // rows per pass
  const int j = tid & 7;
#pragma unroll
  for (int r0 = 0; r0 < NR; r0 += RPP) {
    const int r = r0 + (tid >> 3);
    if (r0 + RPP > NR && r >= NR) break;
    if (r < L) {
      f2 v[16];  // columns (j + 8 i) 4 .. + 3 as the pairs v[2 i], v[2 i + 1]
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 t = *(const float4*)(Hs + r * SH + (j + 8 * i) * 4);
        v[2 * i] = f2{t.x, t.y};
        v[2 * i + 1] = f2{t.z, t.w};
      }
      f2 s2 = v[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) s2 += v[i];
      const float mu = group_sum<8>(s2.x + s2.y) * (1.0f / (float)FD);
      const f2 m2 = f2{mu, mu};
      f2 q2 = f2{0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        v[i] -= m2;
        q2 += v[i] * v[i];
      }
      const float rs = __builtin_amdgcn_rsqf(group_sum<8>(q2.x + q2.y) * (1.0f / (float)FD) + 1e-5f);
      const f2 r2 = f2{rs, rs};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c4 = (j + 8 * i) * 4;
        const f2 a = v[2 * i] * r2, b = v[2 * i + 1] * r2;
        if constexpr (sizeof(T) == 2) {
          *(uint2*)(img + r * SXI + c4) = make_uint2(__builtin_bit_cast(uint32_t, __builtin_convertvector(a, h2)),
                                                     __builtin_bit_cast(uint32_t, __builtin_convertvector(b, h2)));
        } else {
          *(float4*)(img + r * SXI + c4) = make_float4(a.x, a.y, b.x, b.y);
        }
      }
    } else if (r < NR) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c4 = (j + 8 * i) * 4;
        if constexpr (sizeof(T) == 2)
          *(uint2*)(img + r * SXI + c4) = make_uint2(0u, 0u);
        else
          *(float4*)(img + r * SXI + c4) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// depthwise 3-tap conv (Primer-EZ, transformer.py:28-44) and attention (transformer.py:88-118)
// ------------------------------------------------------------------------------------------
struct ConvW { float w0, w1, w2, b; };
__device__ __forceinline__ ConvW conv_w(const float* w, const float* b, int c) {
  return ConvW{G(w)[c * 3 + 0], G(w)[c * 3 + 1], G(w)[c * 3 + 2], G(b)[c]};
}
// one output of the 3-tap conv, in ONE fixed operation order (explicit fmaf chain): the
// step-invariant cross-attention memory rows are convolved once per clip batch
// (ca_kv_conv_kernel) with exactly the arithmetic the per-step kernels use for the other rows
__device__ __forceinline__ float conv3(const ConvW& w, float p0, float p1, float p2) {
  return fmaf(w.w2, p2, fmaf(w.w1, p1, fmaf(w.w0, p0, w.b)));
}

// The 3-tap conv over tokens applied to a transposed GEMM's accumulators (WGemm TR): v[rt][r]
// is channel 4 g4 + r of token rt 16 + c16 (bias added).  The neighbour tokens are lanes c16 -/+ 1
// of the same 16-lane DPP row (row_ror 1 / 15); across row tiles, lane 15 of tile rt - 1 /
// lane 0 of tile rt + 1.  Zero padding outside [0, L); tokens >= L come out zero (as conv_rows).
template <int RT>
__device__ __forceinline__ void conv_tokens(f32x4 (&v)[RT], const ConvW (&w)[4], int L, int c16) {
  constexpr int ROR1 = 0x121, ROR15 = 0x12F;  // dst[l] = src[(l - 1) mod 16] / src[(l + 1) mod 16]
  f32x4 pr[RT], nx[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pr[rt][r] = dpp_mov<ROR1>(v[rt][r]);
      nx[rt][r] = dpp_mov<ROR15>(v[rt][r]);
    }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int i = rt * 16 + c16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = c16 == 0 ? (rt > 0 ? pr[rt - 1 < 0 ? 0 : rt - 1][r] : 0.f) : pr[rt][r];
      float n = c16 == 15 ? (rt + 1 < RT ? nx[rt + 1 < RT ? rt + 1 : rt][r] : 0.f) : nx[rt][r];
      n = i + 1 < L ? n : 0.f;
      v[rt][r] = i < L ? conv3(w[r], p, v[rt][r], n) : 0.f;
    }
  }
}
// conv weights of the 4 consecutive channels c0 .. c0 + 3 of a transposed tile's lane
__device__ __forceinline__ void conv_w4(ConvW (&cw)[4], const float* w, const float* b, int c0) {
#pragma unroll
  for (int r = 0; r < 4; ++r) cw[r] = conv_w(w, b, c0 + r);
}
// store the lane's 4 consecutive channels c0 .. c0 + 3 of token i: row-major image (Q / K: 8 or 16
// bytes at i S + c0) or transposed (V^T: four scalars at (c0 + r) S + i)
template <typename T, bool TRANS>
__device__ __forceinline__ void put_tok4(T* img, int S, int i, int c0, const f32x4& v) {
  if constexpr (TRANS) {
#pragma unroll
    for (int r = 0; r < 4; ++r) img[(c0 + r) * S + i] = from_f32<T>(v[r]);
  } else if constexpr (sizeof(T) == 2) {
    *(uint2*)(img + i * S + c0) = make_uint2(pk_bf16(v[0], v[1]),
                                             pk_bf16(v[2], v[3]));
  } else {
    *(float4*)(img + i * S + c0) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// Step-invariant cross-attention K / V of one (layer, clip, head), convolved and in the
// attention-image element order: K [FLK rows][FDK] then V^T [FDK][FLK keys]; rows / keys 0 and 1
// (which see the step token through the conv) and >= Lk are zero here -- the per-step kernels
// fill 0 and 1 (KvFix).  KVC_ELEMS (ggd_kernels.h) elements of T per head.
static_assert(KVC_ELEMS == 2 * FLK * FDK, "kvc block = K [FLK][FDK] + V^T [FDK][FLK]");

// dst rows (or transposed columns) i < 64 = conv over rows i-1, i, i+1 of the f32 source (row
// stride ss, column c = tid & 31 of the thread; zero outside [0, rows)); rows >= `rows` are
// written as zeros, so padded keys / values are finite
template <typename T, bool TRANS, int NR = 64, int NT = NTHREADS, typename SRC = float>
__device__ __forceinline__ void conv_rows(T* dst, int S, const SRC* src, int ss, int rows, ConvW w,
                                          int tid = ltid()) {
  constexpr int RS = NT / 32, NK = NR / RS;  // row stride between a thread's rows, rows per thread
  static_assert(NR % RS == 0, "rows must split over the thread groups");
  const int c = tid & 31, i0 = tid >> 5;
  float p0[NK], p1[NK], p2[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int i = i0 + RS * k;
    p0[k] = to_f32<SRC>(src[min(max(i - 1, 0), rows - 1) * ss + c]);
    p1[k] = to_f32<SRC>(src[min(i, rows - 1) * ss + c]);
    p2[k] = to_f32<SRC>(src[min(i + 1, rows - 1) * ss + c]);
  }
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int i = i0 + RS * k;
    const float v = conv3(w, i > 0 ? p0[k] : 0.f, p1[k], i + 1 < rows ? p2[k] : 0.f);
    const T o = from_f32<T>(i < rows ? v : 0.f);
    if (TRANS)
      dst[c * S + i] = o;
    else
      dst[i * S + c] = o;
  }
}

template <typename T, int QR = FR> struct FAtt {   // QR: query rows of the Q image
  static constexpr int P = 16 / sizeof(T);
  static constexpr int SQ = FDK + P;       // Q / K rows
  static constexpr int SV = FLK + P;       // V^T rows (keys along the row)
  static constexpr int SP = FLK + P;       // per-wave P tile rows
  static constexpr size_t OQ = 0;
  static constexpr size_t OK = OQ + sizeof(T) * QR * SQ;
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

// Whole 16-lane rows of a wave exchanged by gfx950's v_permlane16_swap / v_permlane32_swap (one
// VALU instruction each; lane semantics checked by scripts/permlane_probe.hip): the max / sum of
// x over the wave's 4 lane rows at the same column c16, identical bits in every lane.
__device__ __forceinline__ float lanerow_max4(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const float m = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float lanerow_sum4(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const float s = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// bf16 attention of one 16-query tile with the probabilities kept in registers.  S^T = K Q^T (the
// K tile as the MFMA A operand), so lane (c16, g4) holds the scores of query c16 against keys
// 16 t + 4 g4 .. + 3: the softmax reduces over keys in-lane and across the 4 lane rows, and the
// bf16 P values of key tile t are exactly the B operand (k = 4 g4 .. + 3, n = c16) of
// O^T = V^T P^T on v_mfma_f32_16x16x16_bf16 -- no P tile through LDS, no per-element P stores.
// Output lane map as fattn's: query c16, channels 4 g4 .. + 3 of each 16-channel tile.
// qext (optional): the query rows come from another bf16 image (row stride sqe) instead of the
// attention image's Q
template <int LKT, int QR, bool TO_LDS, int CP>
__device__ __forceinline__ void fattn_regp(unsigned char* att, int Lk, float scale, bf16_t* out, int ldo,
                                           const OutRowsP<CP>& dst, int rt, int lane, const bf16_t* qext = nullptr,
                                           int sqe = 0) {
  using A = FAtt<bf16_t, QR>;
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  const bf16_t* Qm = qext ? qext : (const bf16_t*)(att + A::OQ);
  const int sq = qext ? sqe : A::SQ;
  const bf16_t* Km = (const bf16_t*)(att + A::OK);
  const bf16_t* Vt = (const bf16_t*)(att + A::OV);
  const int c16 = lane & 15, g4 = lane >> 4;
  const bf16x8 qf = *(const bf16x8*)(Qm + (rt * 16 + c16) * sq + g4 * 8);
  f32x4 s[LKT];
#pragma unroll
  for (int t = 0; t < LKT; ++t) {
    const bf16x8 kf = *(const bf16x8*)(Km + (t * 16 + c16) * A::SQ + g4 * 8);
    s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  }
  // base-2 softmax (as fattn): a masked key is -inf after the scaling, its exp2 is 0
  const float sl2 = scale * 1.4426950408889634f;
  float mx = -INFINITY;
#pragma unroll
  for (int t = 0; t < LKT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = t * 16 + 4 * g4 + i < Lk ? s[t][i] * sl2 : -INFINITY;
      s[t][i] = v;
      mx = fmaxf(mx, v);
    }
  mx = lanerow_max4(mx);
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < LKT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s[t][i] = __builtin_amdgcn_exp2f(s[t][i] - mx);
      sum += s[t][i];
    }
  const float inv = __builtin_amdgcn_rcpf(lanerow_sum4(sum));
  s16x4 pb[LKT];
#pragma unroll
  for (int t = 0; t < LKT; ++t) {
    const uint2 u = make_uint2(pk_bf16(s[t][0] * inv, s[t][1] * inv), pk_bf16(s[t][2] * inv, s[t][3] * inv));
    pb[t] = __builtin_bit_cast(s16x4, u);
  }
#pragma unroll
  for (int ct = 0; ct < FDK / 16; ++ct) {
    f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < LKT; ++t) {
      const s16x4 vf = *(const s16x4*)(Vt + (ct * 16 + c16) * A::SV + t * 16 + 4 * g4);
      o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vf, pb[t], o, 0, 0, 0);
    }
    const int q = rt * 16 + c16, d0 = ct * 16 + 4 * g4;
    if constexpr (TO_LDS)
      *(uint2*)(out + q * ldo + d0) = make_uint2(pk_bf16(o[0], o[1]), pk_bf16(o[2], o[3]));
    else
      dst.template put4v<bf16_t>((uint32_t)(q * ldo + d0), o);
  }
}

// O[Lq][32] = softmax(scale Q K^T) V for one head; wave w owns query rows 16w..16w+15.
// LKT = key tiles of 16 (Lk <= 16 LKT, LKT even).  Keys >= Lk are masked by select (their K
// rows may hold anything); V^T columns >= Lk must be finite (zeroed by the caller).
// TO_LDS: `out` is an LDS operand image and every query row (padding included) is written;
// otherwise `out` is global and rows >= Lq are dropped by the bounded buffer stores.
// bf16 runs fattn_regp (P in registers); f32 (the parity precision) keeps the P tile in LDS.
template <typename T, int LKT, int QR = FR, bool TO_LDS = false, int CP = CP_KERNEL>
__device__ __forceinline__ void fattn(unsigned char* att, int Lq, int Lk, float scale, T* out, int ldo,
                                      int tid = ltid(), const bf16_t* qext = nullptr, int sqe = 0) {
  using A = FAtt<T, QR>;
  const T* Qm = (const T*)(att + A::OQ);
  const T* Km = (const T*)(att + A::OK);
  const T* Vt = (const T*)(att + A::OV);
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), c16 = lane & 15, g4 = lane >> 4;
  T* P = (T*)(att + A::OP) + wave * 16 * A::SP;
  const int rt = wave;
  if (rt * 16 >= Lq) return;
  if constexpr (sizeof(T) == 2) {
    const OutRowsP<CP> dst(out, (uint32_t)(sizeof(T) * ((size_t)(Lq - 1) * ldo + FDK)));  // rows >= Lq dropped
    fattn_regp<LKT, QR, TO_LDS, CP>(att, Lk, scale, out, ldo, dst, rt, lane, qext, sqe);
    return;
  }
  f32x4 s[LKT];
#pragma unroll
  for (int t = 0; t < LKT; ++t) {
    s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    att_mma16(s[t], Qm + rt * 16 * A::SQ, A::SQ, Km + t * 16 * A::SQ, A::SQ, 0, lane);
  }
  // softmax in the base-2 domain: exp(scale s - m) = exp2(scale log2(e) s - m'), one v_exp_f32
  // per score (and one v_rcp_f32 per row) instead of the range-reduced library expf / division
  // The lane's 4 rows run as two packed f32 pairs (rows 0-1, 2-3: v_pk_mul / v_pk_add_f32) for
  // the scaling, the sums and the normalisation; per element the operations and their order are
  // the scalar ones.  A masked key is -inf after the scaling, so its exp2 is 0 without a select.
  typedef float f2 __attribute__((ext_vector_type(2)));
  const float sl2 = scale * 1.4426950408889634f;
  const f2 sl = f2{sl2, sl2};
  float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int t = 0; t < LKT; ++t) {
    const bool ok = t * 16 + c16 < Lk;
    const f2 lo = f2{s[t][0], s[t][1]} * sl, hi = f2{s[t][2], s[t][3]} * sl;
    s[t] = ok ? f32x4{lo.x, lo.y, hi.x, hi.y} : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int r = 0; r < 4; ++r) mx[r] = fmaxf(mx[r], s[t][r]);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) mx[r] = group_max<16>(mx[r]);
  f2 sum01 = f2{0.f, 0.f}, sum23 = f2{0.f, 0.f};
#pragma unroll
  for (int t = 0; t < LKT; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) s[t][r] = __builtin_amdgcn_exp2f(s[t][r] - mx[r]);
    sum01 += f2{s[t][0], s[t][1]};
    sum23 += f2{s[t][2], s[t][3]};
  }
  const f2 inv01 = f2{__builtin_amdgcn_rcpf(group_sum<16>(sum01.x)), __builtin_amdgcn_rcpf(group_sum<16>(sum01.y))};
  const f2 inv23 = f2{__builtin_amdgcn_rcpf(group_sum<16>(sum23.x)), __builtin_amdgcn_rcpf(group_sum<16>(sum23.y))};
#pragma unroll
  for (int t = 0; t < LKT; ++t) {
    const f2 lo = f2{s[t][0], s[t][1]} * inv01, hi = f2{s[t][2], s[t][3]} * inv23;
    P[(4 * g4 + 0) * A::SP + t * 16 + c16] = from_f32<T>(lo.x);
    P[(4 * g4 + 1) * A::SP + t * 16 + c16] = from_f32<T>(lo.y);
    P[(4 * g4 + 2) * A::SP + t * 16 + c16] = from_f32<T>(hi.x);
    P[(4 * g4 + 3) * A::SP + t * 16 + c16] = from_f32<T>(hi.y);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const OutRowsP<CP> dst(out, (uint32_t)(sizeof(T) * ((size_t)(Lq - 1) * ldo + FDK)));  // rows >= Lq dropped
  // O^T = V^T P^T per 16-channel tile: lane (query c16, group g4) holds channels 4 g4 .. + 3 of its
  // query row, so the row is written with one 8-byte (bf16) / 16-byte (f32) store per tile
#pragma unroll
  for (int ct = 0; ct < FDK / 16; ++ct) {
    f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k0 = 0; k0 < LKT * 16; k0 += 32) att_mma16(o, Vt + ct * 16 * A::SV, A::SV, P, A::SP, k0, lane);
    const int q = rt * 16 + c16, d0 = ct * 16 + 4 * g4;
    if constexpr (TO_LDS) {
      if constexpr (sizeof(T) == 2)
        *(uint2*)(out + q * ldo + d0) = make_uint2(pk_bf16(o[0], o[1]), pk_bf16(o[2], o[3]));
      else
        *(float4*)(out + q * ldo + d0) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
      dst.template put4v<T>((uint32_t)(q * ldo + d0), o);
    }
  }
}

template <typename T, int CP = CP_KERNEL>
__device__ __forceinline__ void fattn_any(unsigned char* att, int Lq, int Lk, float scale, T* out, int ldo) {
  if (Lk <= 32)
    fattn<T, 2, FR, false, CP>(att, Lq, Lk, scale, out, ldo);
  else
    fattn<T, 4, FR, false, CP>(att, Lq, Lk, scale, out, ldo);
}

// Cross-attention K / V^T images of head hd from the precomputed kvc block (KVC_ELEMS of T):
// load() issues the 16-byte pieces (NT threads, issued early), store() writes them into the
// attention image `att` (FAtt layout) with its row pads.
template <typename T, int NT, int QR = FR> struct KvcStage {
  using A = FAtt<T, QR>;
  static constexpr int PIECES = KVC_ELEMS * (int)sizeof(T) / 16, NV = (PIECES + NT - 1) / NT, PER_ROW_K = FDK * (int)sizeof(T) / 16,
                       PER_ROW_V = FLK * (int)sizeof(T) / 16, K_PIECES = FLK * PER_ROW_K;
  static_assert(PIECES % NT == 0, "whole pieces per thread");
  uint4 v[NV];
  __device__ __forceinline__ void load(const T* src, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
      const u32x4 u = G((const u32x4*)src)[tid + i * NT];
      v[i] = make_uint4(u.x, u.y, u.z, u.w);
    }
  }
  __device__ __forceinline__ void store(unsigned char* att, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int q = tid + i * NT;
      unsigned char* dst;
      if (q < K_PIECES)
        dst = att + A::OK + sizeof(T) * ((q / PER_ROW_K) * A::SQ) + 16 * (q % PER_ROW_K);
      else
        dst = att + A::OV + sizeof(T) * (((q - K_PIECES) / PER_ROW_V) * A::SV) + 16 * ((q - K_PIECES) % PER_ROW_V);
      *(uint4*)dst = v[i];
    }
  }
};

// Rows 0 and 1 of the cross-attention K and V of head hd (the rows whose 3-tap conv reads the
// step token, memory row 0): lane l of the fixing wave handles half l >> 5 (K / V), channel l & 31.
// m0 = the step token's pre-conv K|V row (kv_step[t]), m1 / m2 = the clip's first two speech rows.
struct KvFix {
  float m0, m1, m2;
  __device__ __forceinline__ void load(const float* kv_step_t, const float* kv_mem_b, int Ts, int hd, int l) {
    const int half = l >> 5, c = l & 31, col = half * FD + hd * FDK + c;
    m0 = G(kv_step_t)[col];
    m1 = G(kv_mem_b)[col];
    m2 = G(kv_mem_b)[(size_t)min(1, Ts - 1) * 2 * FD + col];
    if (Ts < 2) m2 = 0.f;
  }
  template <typename T, int QR = FR>
  __device__ __forceinline__ void store(unsigned char* att, const ConvW& ck, const ConvW& cv, int Lk, int l) const {
    using A = FAtt<T, QR>;
    const int half = l >> 5, c = l & 31;
    const ConvW& w = half ? cv : ck;
    const float r0 = conv3(w, 0.f, m0, Lk > 1 ? m1 : 0.f), r1 = conv3(w, m0, m1, Lk > 2 ? m2 : 0.f);
    T* K = (T*)(att + A::OK);
    T* Vt = (T*)(att + A::OV);
    if (half == 0) {
      K[0 * A::SQ + c] = from_f32<T>(r0);
      if (Lk > 1) K[1 * A::SQ + c] = from_f32<T>(r1);
    } else {
      Vt[c * A::SV + 0] = from_f32<T>(r0);
      if (Lk > 1) Vt[c * A::SV + 1] = from_f32<T>(r1);
    }
  }
};

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
  // KE: [Xn][stats][Hs][E (64 x 20 f32: the block's 16 channels)]
  static constexpr size_t E = al16(sizeof(float) * FR * (16 + 4));
  static constexpr size_t KE = IMG + ST + HS + E;
  // KA of layer 0 also stages the emb operand (64 x (128 + PT), aliasing the LN image)
  static constexpr size_t XB = al16(sizeof(T) * FR * (128 + Frag<T>::PT));
  static_assert(XB <= IMG, "emb operand must fit the LN image");
};
static_assert(Plan<float>::KA <= 160 * 1024 && Plan<float>::KB <= 160 * 1024 && Plan<float>::KE <= 160 * 1024 &&
                  Plan<float>::KD <= 160 * 1024,
              "fused LDS plans must fit 160 KiB");

}  // namespace ggd
