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
#include "ggd_common.h"

namespace ggd {

// ---------------------------------------------------------------------------
// GEMM:  out[M][N] = epi( pro(A)[M][K] . W[N][K]^T + b )
//
// One 256-thread workgroup per MT x 64 output tile; K is staged through LDS in 256-wide
// chunks.  Every global load of a chunk (A rows and W rows) is issued back to back into
// registers before any of them is consumed, and chunk c+1 is prefetched into registers
// while the MFMAs of chunk c run -- these small, latency-bound GEMMs are paced by memory
// round trips, not by MFMA throughput.  PRO_LN keeps the tile's f32 rows in registers,
// reduces the row statistics there (4 lanes per row, fixed, so results do not depend on
// the tile height) and normalises on the way into LDS.
// ---------------------------------------------------------------------------
template <typename T> struct Tile;
template <> struct Tile<bf16_t> { static constexpr int PAD = 8; static constexpr int VE = 8; };
template <> struct Tile<float>  { static constexpr int PAD = 4; static constexpr int VE = 4; };

template <typename T, int MT, int PRO> struct ARegs;
template <typename T, int MT> struct ARegs<T, MT, PRO_T> {          // T rows, 16-byte vectors
  static constexpr int VPR = KC / Tile<T>::VE;                      // vectors per row
  static constexpr int N = MT * VPR / NTHREADS;
  uint4 v[N];
};
template <typename T, int MT> struct ARegs<T, MT, PRO_LN> {         // f32 rows, 4 lanes per row
  static constexpr int N = KC / 16;                                 // float4 per lane
  float4 v[N];
  float mu, rs;
};
template <typename T, int MT> struct ARegs<T, MT, PRO_F32> {        // f32, arbitrary lda, k < k_valid
  static constexpr int N = MT * KC / NTHREADS;
  float v[N];
};

template <typename T, int MT, int PRO>
__device__ __forceinline__ void load_a(ARegs<T, MT, PRO>& R, const GemmArgs& a, int m0, int kc0) {
  constexpr int N = ARegs<T, MT, PRO>::N;
  const int tid = threadIdx.x;
  if constexpr (PRO == PRO_T) {
    constexpr int VPR = ARegs<T, MT, PRO>::VPR, VE = Tile<T>::VE;
    const T* A = (const T*)a.A;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int v = tid + i * NTHREADS, r = v / VPR, cv = v % VPR, m = m0 + r;
      R.v[i] = m < a.M ? *(const uint4*)(A + (size_t)m * a.lda + kc0 + cv * VE) : make_uint4(0, 0, 0, 0);
    }
  } else if constexpr (PRO == PRO_LN) {
    const int r = tid >> 2, j = tid & 3, m = m0 + r;
    const bool ok = tid < MT * 4 && m < a.M;
    const float* row = (const float*)a.A + map_row(ok ? m : 0, a.a_len, a.a_stride, a.a_off) * a.lda + kc0;
#pragma unroll
    for (int i = 0; i < N; ++i)
      R.v[i] = ok ? *(const float4*)(row + (j + 4 * i) * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  } else {
    const float* A = (const float*)a.A;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int v = tid + i * NTHREADS, r = v / KC, c = v % KC, m = m0 + r, k = kc0 + c;
      const bool ok = m < a.M && k < a.k_valid;
      const size_t e = ok ? map_row(m, a.a_len, a.a_stride, a.a_off) * a.lda + k : 0;
      R.v[i] = ok ? A[e] : 0.f;
      if (a.a_add) R.v[i] += ok ? a.a_add[e] : 0.f;  // inpaint conditioning: x + proj(pose, mask)
    }
  }
}

// LayerNorm statistics of the registers' rows (two-pass: mean, then centred sum of squares).
template <typename T, int MT>
__device__ __forceinline__ void ln_stats(ARegs<T, MT, PRO_LN>& R, int K) {
  ln_stats4<ARegs<T, MT, PRO_LN>::N>(R.v, (float)K, R.mu, R.rs);
}

// PRO_F32 with a dense A (lda == k_valid, identity row map, one K chunk): the tile's rows are one
// contiguous, 16-byte aligned span of MT * lda floats, loaded as float4 (all loads issued before the
// first use) and scattered into the LDS tile; columns k_valid .. KC - 1 are written as zeros.  The
// emb_x GEMM reads the pose state this way (lda = C = 123: rows are not 16-byte aligned on their
// own, so the per-element path issued MT * KC / NTHREADS scalar loads per thread).
template <typename T, int MT>
__device__ __forceinline__ void stage_f32_span(T* As, const GemmArgs& a, int m0) {
  constexpr int STR = KC + Tile<T>::PAD, NV = (MT * KC / 4 + NTHREADS - 1) / NTHREADS;
  const int lda = a.lda, rows = min(MT, a.M - m0), nv = (rows * lda) >> 2;  // whole float4s
  const float* base = (const float*)a.A + (size_t)m0 * lda;
  const float* add = a.a_add ? a.a_add + (size_t)m0 * lda : nullptr;
  float4 v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int j = min((int)threadIdx.x + i * NTHREADS, max(nv - 1, 0));
    v[i] = *(const float4*)(base + 4 * j);
  }
  if (add) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int j = min((int)threadIdx.x + i * NTHREADS, max(nv - 1, 0));
      const float4 w = *(const float4*)(add + 4 * j);
      v[i].x += w.x; v[i].y += w.y; v[i].z += w.z; v[i].w += w.w;
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int j = (int)threadIdx.x + i * NTHREADS;
    if (j >= nv) continue;
    const float e4[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = 4 * j + q, r = e / lda, c = e - r * lda;
      As[r * STR + c] = from_f32<T>(e4[q]);
    }
  }
  // the tail that is not a whole float4 (rows * lda % 4), zero padding columns and rows >= rows
  for (int e = 4 * nv + (int)threadIdx.x; e < rows * lda; e += NTHREADS) {
    const int r = e / lda, c = e - r * lda;
    As[r * STR + c] = from_f32<T>(base[e] + (add ? add[e] : 0.f));
  }
  const int padc = KC - lda;
  for (int e = threadIdx.x; e < MT * padc; e += NTHREADS) {
    const int r = e / padc, c = lda + e % padc;
    As[r * STR + c] = from_f32<T>(0.f);
  }
  for (int e = threadIdx.x; e < (MT - rows) * lda; e += NTHREADS) {
    const int r = rows + e / lda, c = e % lda;
    As[r * STR + c] = from_f32<T>(0.f);
  }
}

template <typename T, int MT, int PRO>
__device__ __forceinline__ void store_a(const ARegs<T, MT, PRO>& R, const GemmArgs& a, T* As, int kc0) {
  constexpr int STR = KC + Tile<T>::PAD;
  constexpr int N = ARegs<T, MT, PRO>::N;
  const int tid = threadIdx.x;
  if constexpr (PRO == PRO_T) {
    constexpr int VPR = ARegs<T, MT, PRO>::VPR, VE = Tile<T>::VE;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int v = tid + i * NTHREADS, r = v / VPR, cv = v % VPR;
      *(uint4*)(As + r * STR + cv * VE) = R.v[i];
    }
  } else if constexpr (PRO == PRO_LN) {
    if (tid >= MT * 4) return;
    const int r = tid >> 2, j = tid & 3;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int k = (j + 4 * i) * 4;
      const float4 g = *(const float4*)(a.ln_g + kc0 + k);
      const float4 b = *(const float4*)(a.ln_b + kc0 + k);
      const float4 x = R.v[i];
      T* dst = As + r * STR + k;
      dst[0] = from_f32<T>((x.x - R.mu) * R.rs * g.x + b.x);
      dst[1] = from_f32<T>((x.y - R.mu) * R.rs * g.y + b.y);
      dst[2] = from_f32<T>((x.z - R.mu) * R.rs * g.z + b.z);
      dst[3] = from_f32<T>((x.w - R.mu) * R.rs * g.w + b.w);
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int v = tid + i * NTHREADS, r = v / KC, c = v % KC;
      As[r * STR + c] = from_f32<T>(R.v[i]);
    }
  }
}

// rows [r0, r0 + ROWS) x columns [kc0, kc0 + KC) of a row-major T matrix -> LDS tile
// (rows >= nrows read as zero).  All loads of the tile are independent and issue together.
template <typename T, int ROWS>
__device__ __forceinline__ void copy_tile(T* dst, const T* src, int ld, int r0, int nrows, int kc0, int len = 0,
                                          int stride = 0, int off = 0) {
  constexpr int STR = KC + Tile<T>::PAD, VE = Tile<T>::VE, VPR = KC / VE, N = ROWS * VPR / NTHREADS;
  uint4 v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int e = threadIdx.x + i * NTHREADS, r = e / VPR, cv = e % VPR;
    v[i] = r0 + r < nrows ? *(const uint4*)(src + map_row(r0 + r, len, stride, off) * ld + kc0 + cv * VE)
                          : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int e = threadIdx.x + i * NTHREADS, r = e / VPR, cv = e % VPR;
    *(uint4*)(dst + r * STR + cv * VE) = v[i];
  }
}

template <typename T> struct WRegs {
  static constexpr int VPR = KC / Tile<T>::VE;
  static constexpr int N = NT * VPR / NTHREADS;
  uint4 v[N];
};

template <typename T>
__device__ __forceinline__ void load_w(WRegs<T>& R, const GemmArgs& a, int n0, int kc0) {
  constexpr int N = WRegs<T>::N;
  constexpr int VPR = WRegs<T>::VPR, VE = Tile<T>::VE;
  const T* W = (const T*)a.W;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int v = threadIdx.x + i * NTHREADS, r = v / VPR, cv = v % VPR;
    R.v[i] = *(const uint4*)(W + (size_t)(n0 + r) * a.K + kc0 + cv * VE);
  }
}

template <typename T>
__device__ __forceinline__ void store_w(const WRegs<T>& R, T* Ws) {
  constexpr int N = WRegs<T>::N;
  constexpr int STR = KC + Tile<T>::PAD;
  constexpr int VPR = WRegs<T>::VPR, VE = Tile<T>::VE;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int v = threadIdx.x + i * NTHREADS, r = v / VPR, cv = v % VPR;
    *(uint4*)(Ws + r * STR + cv * VE) = R.v[i];
  }
}

// fp8 weight tile (GGD_FP8W): rows [n0, n0 + NT) x columns [kc0, kc0 + KC) of OCP e4m3fn bytes
// -> the bf16 LDS tile.  e4m3 values are exactly representable in bf16 (3 mantissa bits,
// exponents -9 .. 8), so the dequantization is exact: v_cvt_pk_f32_fp8 (OCP on gfx950) and the
// f32 -> bf16 truncation loses nothing; the per-channel scale is applied in the epilogue.
// All 16-byte loads of the tile issue before the first conversion.
__device__ __forceinline__ void copy_tile_w8(bf16_t* dst, const uint8_t* src, int ld, int n0, int kc0) {
  constexpr int STR = KC + Tile<bf16_t>::PAD, VPR = KC / 16, N = NT * VPR / NTHREADS;
  typedef __attribute__((ext_vector_type(2))) float f2;
  uint4 v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int e = threadIdx.x + i * NTHREADS, r = e / VPR, cv = e % VPR;
    v[i] = *(const uint4*)(src + (size_t)(n0 + r) * ld + kc0 + cv * 16);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int e = threadIdx.x + i * NTHREADS, r = e / VPR, cv = e % VPR;
    const unsigned w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
    unsigned o[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f2 lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[q], false);
      const f2 hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[q], true);
      o[2 * q] = (__float_as_uint(lo.x) >> 16) | (__float_as_uint(lo.y) & 0xffff0000u);
      o[2 * q + 1] = (__float_as_uint(hi.x) >> 16) | (__float_as_uint(hi.y) & 0xffff0000u);
    }
    uint4* d = (uint4*)(dst + r * STR + cv * 16);
    d[0] = make_uint4(o[0], o[1], o[2], o[3]);
    d[1] = make_uint4(o[4], o[5], o[6], o[7]);
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
    // f32 operands: each lane reads 4 consecutive k; MFMA step s pairs k = kk + 4*g + s
    // identically for A and W, so every k is used once (a k-permuted f32 fma chain).
#pragma unroll 4
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

template <typename T, int MT, int PRO, int EPI, int NCH, bool W8 = false>
__global__ void __launch_bounds__(NTHREADS) gemm_kernel(GemmArgs a) {
  static_assert(!W8 || sizeof(T) == 2, "fp8 weights feed the bf16 MFMA");
  constexpr int STR = KC + Tile<T>::PAD;
  constexpr int WM = MT / 2, WN = NT / 2;     // 2 x 2 waves
  constexpr int TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) T As[MT * STR];
  __shared__ __attribute__((aligned(16))) T Ws[NT * STR];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  // XCD-aware tile order (T1): workgroups are dealt round-robin over the 8 XCDs; remap so each
  // XCD gets a contiguous run of row-major tiles, i.e. whole row blocks share one L2 and the
  // A rows are fetched once per XCD instead of once per column tile.  Speed only.
  int tile = blockIdx.y * gridDim.x + blockIdx.x;
  if (!a.no_xcd_remap) {
    const int nwg = gridDim.x * gridDim.y, q = nwg / 8, rem = nwg % 8, x = tile % 8, slot = tile / 8;
    tile = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + slot;
  }
  const int n0 = (tile % gridDim.x) * NT, m0 = (tile / gridDim.x) * MT;

  if (a.step_counter && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) atomicAdd(a.step_counter, 1);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // NCH = K / 256 is a template constant.  Each chunk's loads are issued together (one
  // memory round trip) and written to LDS; plain T operands and the weights are copied
  // global -> LDS directly (no register array survives a chunk: a loop-carried staging
  // array is demoted to scratch by the compiler).
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (c > 0) __syncthreads();  // previous chunk's MFMAs are done with the LDS tiles
    if constexpr (PRO == PRO_T) {
      copy_tile<T, MT>(As, (const T*)a.A, a.lda, m0, a.M, c * KC, a.a_len, a.a_stride, a.a_off);
    } else if (PRO == PRO_F32 && NCH == 1 && a.a_len == 0 && a.lda == a.k_valid && a.lda <= KC &&
               ((size_t)m0 * a.lda) % 4 == 0) {
      stage_f32_span<T, MT>(As, a, m0);
    } else {
      ARegs<T, MT, PRO> ra;
      load_a<T, MT, PRO>(ra, a, m0, c * KC);
      if constexpr (PRO == PRO_LN) ln_stats<T, MT>(ra, a.K);
      store_a<T, MT, PRO>(ra, a, As, c * KC);
    }
    if constexpr (W8) copy_tile_w8((bf16_t*)Ws, (const uint8_t*)a.W, a.K, n0, c * KC);
    else copy_tile<T, NT>(Ws, (const T*)a.W, a.K, n0, 1 << 30, c * KC);
    __syncthreads();
    mma_chunk<T, TM, TN>(As, Ws, wr * WM, wc * WN, lane, acc);
  }

  // epilogue: C/D map of the 16x16 MFMA: col = lane & 15, row = 4 * (lane >> 4) + r
  const int g = lane >> 4, c16 = lane & 15;
  float res[TM][TN][4];
  if constexpr (EPI == EPI_RESID) {  // read every residual first: one round trip, not one per store
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wr * WM + i * 16 + g * 4 + r, n = n0 + wc * WN + j * 16 + c16;
          res[i][j][r] = m < a.M ? ((const float*)a.out)[map_row(m, a.o_len, a.o_stride, a.o_off) * a.ldo + n] : 0.f;
        }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wc * WN + j * 16 + c16;
      const float bn = a.bias[n];
      const float sn = W8 ? a.wscale[n] : 1.0f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * WM + i * 16 + g * 4 + r;
        if (m >= a.M) continue;
        const size_t mo = map_row(m, a.o_len, a.o_stride, a.o_off);
        float v = W8 ? acc[i][j][r] * sn + bn : acc[i][j][r] + bn;
        if constexpr (EPI == EPI_T) {
          ((T*)a.out)[mo * a.ldo + n] = from_f32<T>(v);
        } else if constexpr (EPI == EPI_RELU2) {
          v = fmaxf(v, 0.f);
          ((T*)a.out)[mo * a.ldo + n] = from_f32<T>(v * v);
        } else if constexpr (EPI == EPI_F32) {
          if (n < a.n_valid) ((float*)a.out)[mo * a.ldo + n] = v;
        } else if constexpr (EPI == EPI_SILU) {
          ((float*)a.out)[mo * a.ldo + n] = v / (1.0f + expf(-v));
        } else if constexpr (EPI == EPI_RESID) {
          ((float*)a.out)[mo * a.ldo + n] = res[i][j][r] + v;
        } else {  // EPI_PE
          const int pos = (m % a.pe_period) + a.pe_offset;
          ((float*)a.out)[mo * a.ldo + n] = v + a.pe[(size_t)pos * a.N + n];
        }
      }
    }
}

template <typename T, int MT, int PRO, int EPI>
static hipError_t gemm_go(const GemmArgs& a, hipStream_t s) {
  dim3 grid(a.N / NT, (a.M + MT - 1) / MT);
  if constexpr (sizeof(T) == 2) {
    if (a.wscale) {  // fp8 weights: K = 256 (every d_model-input Linear) or 1024 (FFN down)
      switch (a.K / KC) {
        case 1: hipLaunchKernelGGL((gemm_kernel<T, MT, PRO, EPI, 1, true>), grid, dim3(NTHREADS), 0, s, a); break;
        case 4:
          if constexpr (PRO == PRO_T) hipLaunchKernelGGL((gemm_kernel<T, MT, PRO, EPI, 4, true>), grid, dim3(NTHREADS), 0, s, a);
          else return hipErrorInvalidValue;
          break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
  }
  switch (a.K / KC) {
    case 1: hipLaunchKernelGGL((gemm_kernel<T, MT, PRO, EPI, 1>), grid, dim3(NTHREADS), 0, s, a); break;
    case 2:
      if constexpr (PRO != PRO_LN) hipLaunchKernelGGL((gemm_kernel<T, MT, PRO, EPI, 2>), grid, dim3(NTHREADS), 0, s, a);
      break;
    case 3:
      if constexpr (PRO != PRO_LN) hipLaunchKernelGGL((gemm_kernel<T, MT, PRO, EPI, 3>), grid, dim3(NTHREADS), 0, s, a);
      break;
    case 4:
      if constexpr (PRO != PRO_LN) hipLaunchKernelGGL((gemm_kernel<T, MT, PRO, EPI, 4>), grid, dim3(NTHREADS), 0, s, a);
      break;
    case 8:
      if constexpr (PRO == PRO_T) hipLaunchKernelGGL((gemm_kernel<T, MT, PRO, EPI, 8>), grid, dim3(NTHREADS), 0, s, a);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T, int PRO, int EPI>
static hipError_t gemm_mt(const GemmArgs& a, hipStream_t s) {
  // 64-row tiles when that still gives >= ~200 workgroups, else 32-row tiles.
  const long tiles64 = (long)(a.N / NT) * ((a.M + 63) / 64);
  if (a.force_mt == 64 || (a.force_mt == 0 && tiles64 >= 200)) return gemm_go<T, 64, PRO, EPI>(a, s);
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
  if (a.K != KC && a.K != 2 * KC && a.K != 3 * KC && a.K != 4 * KC && !(a.K == 8 * KC && pro == PRO_T))
    return hipErrorInvalidValue;
  if (pro == PRO_LN && a.K != KC) return hipErrorInvalidValue;  // LayerNorm width = one chunk
  if (dtype == 0) {
    if (a.wscale) return hipErrorInvalidValue;  // fp8 weights feed the bf16 MFMA only
    return gemm_pro<float>(pro, epi, a, s);
  }
  return gemm_pro<bf16_t>(pro, epi, a, s);
}

// ---------------------------------------------------------------------------
// attention with fused depthwise sequence conv (transformer.py:28-44, 88-118)
//
// One workgroup per (head, clip).  The head's raw Q / K / V rows are staged into LDS (f32,
// zero halo rows) and the Primer-EZ 3-tap conv writes MFMA-ready operands: Q and K row-major,
// V transposed (so P.V's B operand is a contiguous 16-byte read).  Each wave owns 16-row
// query tiles: S = Q K^T on MFMA (16 x Lk_pad accumulators in registers), softmax on the
// accumulator layout (row reductions over the 16 lanes sharing a row: xor 1, 2, 4, 8),
// P to a per-wave LDS tile, O = P V on MFMA.  bf16: v_mfma_f32_16x16x32_bf16; f32 parity
// mode: v_mfma_f32_16x16x4_f32.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(NTHREADS) attn_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int h = blockIdx.x, b = blockIdx.y;
  const int dk = a.dk, Lq = a.Lq, Lk = a.Lk;
  const AttGeom G = att_geom<T>(Lq, Lk, dk);
  T* Qm = (T*)(smem + G.off_q);
  T* Km = (T*)(smem + G.off_k);
  T* Vt = (T*)(smem + G.off_v);
  T* Pw = (T*)(smem + G.off_p);
  float* raw = (float*)(smem + G.off_raw);
  const int tid = threadIdx.x;

  // zero the padded operand images (rows >= Lq / Lk must be finite zeros)
  {
    uint4* z = (uint4*)smem;
    const int n16 = (int)(G.off_p / 16);
    for (int i = tid; i < n16; i += NTHREADS) z[i] = make_uint4(0, 0, 0, 0);
  }
  const size_t row0 = a.seq_stride ? (size_t)b * a.seq_stride + a.seq_off : (size_t)b * Lq;
  att_stage_rows<T>(raw, a.q, row0, a.ldq, h * dk, Lq, dk);
  __syncthreads();
  att_conv<T, false>(Qm, G.SQ, raw, Lq, dk, a.cw_q, a.cb_q);
  __syncthreads();
  if (!a.cross) {
    att_stage_rows<T>(raw, a.k, row0, a.ldkv, h * dk, Lk, dk);
    __syncthreads();
    att_conv<T, false>(Km, G.SQ, raw, Lk, dk, a.cw_k, a.cb_k);
    __syncthreads();
    att_stage_rows<T>(raw, a.v, row0, a.ldkv, h * dk, Lk, dk);
    __syncthreads();
    att_conv<T, true>(Vt, G.SV, raw, Lk, dk, a.cw_v, a.cb_v);
  } else {
    // memory row 0 = the diffusion-step token of this clip's t; rows 1.. = cached speech K|V
    const int t = a.t_clip ? a.t_clip[b] : a.steps[*a.step_counter].t_orig;
    const float* r0 = a.kv_step + (size_t)t * 2 * a.d;
    for (int half = 0; half < 2; ++half) {
      const int col = half * a.d + h * dk;
      att_stage_rows<float>(raw + dk, a.kv_mem, (size_t)b * (Lk - 1), 2 * a.d, col, Lk - 1, dk);
      for (int c = tid; c < dk; c += NTHREADS) {
        raw[c] = 0.f;
        raw[dk + c] = r0[col + c];
      }
      __syncthreads();
      if (half == 0)
        att_conv<T, false>(Km, G.SQ, raw, Lk, dk, a.cw_k, a.cb_k);
      else
        att_conv<T, true>(Vt, G.SV, raw, Lk, dk, a.cw_v, a.cb_v);
      __syncthreads();
    }
  }
  __syncthreads();

  attn_core<T>(Qm, Km, Vt, Pw, G, Lq, Lk, dk, a.scale, (T*)a.out + row0 * a.ldo + (size_t)h * dk, a.ldo);
}

// ---------------------------------------------------------------------------
// Query-split attention (attn_q_kernel): one workgroup per (head, clip, 64-query block), so a
// 160-frame clip (BASELINE configs[3]) spreads its 10 query tiles over 3 workgroups per head
// instead of serialising them in one, and every wave runs exactly one 16-row query tile.
// Staging skips the f32 raw image: each thread computes the 3-tap conv of its own 16-byte
// channel vectors straight from global rows i-1, i, i+1 (rows outside the sequence are the
// conv's zero padding), all loads of a batch issued before the first use.  The K / V conv is
// recomputed by each query block (L2 hits; a few % of the block's work).
// ---------------------------------------------------------------------------
constexpr int AQ_QT = 64;  // query rows per workgroup: 4 waves x 16

template <typename T>
__host__ __device__ inline AttGeom aq_geom(int Lk, int dk) {
  constexpr int KA = sizeof(T) == 2 ? 32 : 16;
  AttGeom g;
  g.Lqp = AQ_QT;
  g.Lkp = (Lk + KA - 1) / KA * KA;
  g.SQ = dk + AttPad<T>::P;
  g.SV = g.Lkp + AttPad<T>::P;
  g.SP = g.Lkp + AttPad<T>::P;
  g.off_q = 0;
  g.off_k = g.off_q + sizeof(T) * (size_t)AQ_QT * g.SQ;
  g.off_v = g.off_k + sizeof(T) * (size_t)g.Lkp * g.SQ;
  g.off_p = g.off_v + sizeof(T) * (size_t)dk * g.SV;
  g.off_raw = g.off_p;
  g.total = g.off_p + sizeof(T) * (size_t)AQ_QT * g.SP;
  return g;
}

// One 16-byte vector of T channels (VE of them) of sequence row j, as f32.  Rows outside
// [0, len) are the conv's zero padding: their address is redirected to a zeroed global row
// (`zero`), so no per-element select is needed.  Self mode reads T rows
// base[(row0 + j) * ld + col]; memory mode (step_row set) reads f32 rows: j = 0 the step token
// step_row, j >= 1 the cached speech rows base[(row0 + j - 1) * ld + col].
template <typename T> struct AqSrc {
  static constexpr int VE = 16 / sizeof(T);
  const void* base;
  size_t row0;
  int ld, col, len;
  const float* step_row;
  const float* zero;
  __device__ __forceinline__ void load(int j, int cv, float (&o)[VE]) const {
    const bool in = j >= 0 && j < len;
    if (step_row) {
      const float* p = !in ? zero : j == 0 ? step_row + cv * VE
                                           : (const float*)base + (row0 + j - 1) * (size_t)ld + col + cv * VE;
#pragma unroll
      for (int q = 0; q < VE / 4; ++q) {
        const float4 v = *(const float4*)(p + 4 * q);
        o[4 * q] = v.x;
        o[4 * q + 1] = v.y;
        o[4 * q + 2] = v.z;
        o[4 * q + 3] = v.w;
      }
    } else {
      const T* p = in ? (const T*)base + (row0 + j) * (size_t)ld + col + cv * VE : (const T*)zero;
      const uint4 u = *(const uint4*)p;
      if constexpr (sizeof(T) == 2) {
        const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          o[2 * q] = __uint_as_float(w[q] << 16);
          o[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
        }
      } else {
        o[0] = __uint_as_float(u.x);
        o[1] = __uint_as_float(u.y);
        o[2] = __uint_as_float(u.z);
        o[3] = __uint_as_float(u.w);
      }
    }
  }
};

// Conv staging by row strips: thread t owns channel vector cv = t % VPR and the strip of SL
// consecutive rows sid * SL .. (sid = t / VPR), so it loads SL + 2 rows (not 3 SL) and every
// load of the strip issues before the first conv.  SL = ceil(rows / NS) <= SLMAX.
template <typename T, int DK> struct AqStrip {
  static constexpr int VE = 16 / sizeof(T), VPR = DK / VE, NS = NTHREADS / VPR;
  static constexpr int SLMAX = (ATT_LMAX + NS - 1) / NS;
  static_assert(NTHREADS % VPR == 0, "a thread keeps one channel vector");
  float x[SLMAX + 2][VE];
  int r0, sl, rows;
  __device__ __forceinline__ void load(const AqSrc<T>& src, int r0_, int rows_) {
    r0 = r0_;
    rows = rows_;
    sl = (rows + NS - 1) / NS;
    const int cv = (int)threadIdx.x % VPR, sid = (int)threadIdx.x / VPR;
#pragma unroll
    for (int s = 0; s < SLMAX + 2; ++s)
      if (s < sl + 2) src.load(r0 + sid * sl - 1 + s, cv, x[s]);
  }
  // wl: LDS [4][DK] = tap 0, tap 1, tap 2, bias (transformer.py:28-44: out[i] = b + sum_k w_k in[i+k-1])
  template <bool TRANS>
  __device__ __forceinline__ void conv(T* dst, int S, const float* wl) const {
    const int cv = (int)threadIdx.x % VPR, sid = (int)threadIdx.x / VPR;
    float w0[VE], w1[VE], w2[VE], bb[VE];
#pragma unroll
    for (int e = 0; e < VE; ++e) {
      const int c = cv * VE + e;
      w0[e] = wl[c];
      w1[e] = wl[DK + c];
      w2[e] = wl[2 * DK + c];
      bb[e] = wl[3 * DK + c];
    }
#pragma unroll
    for (int s = 0; s < SLMAX; ++s) {
      const int r = sid * sl + s;
      if (s >= sl || r >= rows) continue;
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        const int c = cv * VE + e;
        const float v = bb[e] + w0[e] * x[s][e] + w1[e] * x[s + 1][e] + w2[e] * x[s + 2][e];
        if (TRANS)
          dst[c * S + r] = from_f32<T>(v);
        else
          dst[r * S + c] = from_f32<T>(v);
      }
    }
  }
};

// conv taps [dk][3] + bias [dk] of Q, K, V -> LDS wl[3][4][DK]
template <int DK>
__device__ __forceinline__ void aq_stage_taps(float* wl, const AttnArgs& a) {
  const float* W[3] = {a.cw_q, a.cw_k, a.cw_v};
  const float* B[3] = {a.cb_q, a.cb_k, a.cb_v};
  for (int i = threadIdx.x; i < 3 * 4 * DK; i += NTHREADS) {
    const int m = i / (4 * DK), k = (i / DK) % 4, c = i % DK;
    wl[i] = k < 3 ? W[m][c * 3 + k] : B[m][c];
  }
}

template <typename T, int DK>
__global__ void __launch_bounds__(NTHREADS) attn_q_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int h = blockIdx.x, b = blockIdx.y, q0 = blockIdx.z * AQ_QT;
  const int Lq = a.Lq, Lk = a.Lk;
  const AttGeom G = aq_geom<T>(Lk, DK);
  T* Qm = (T*)(smem + G.off_q);
  T* Km = (T*)(smem + G.off_k);
  T* Vt = (T*)(smem + G.off_v);
  T* Pw = (T*)(smem + G.off_p);
  float* wl = (float*)(smem + G.total);  // conv taps, after the attention images
  const int tid = threadIdx.x;
  const size_t row0 = a.seq_stride ? (size_t)b * a.seq_stride + a.seq_off : (size_t)b * Lq;
  const int qrows = min(AQ_QT, Lq - q0);
  // issue the Q and K strips first: their loads fly while the images are zeroed and the taps staged
  AqSrc<T> sq{a.q, row0, a.ldq, h * DK, Lq, nullptr, a.zero};
  AqSrc<T> sk{a.k, row0, a.ldkv, h * DK, Lk, nullptr, a.zero};
  AqSrc<T> sv{a.v, row0, a.ldkv, h * DK, Lk, nullptr, a.zero};
  if (a.cross) {
    // memory row 0 = the diffusion-step token of this clip's t; rows 1.. = cached speech K|V
    const int t = a.t_clip ? a.t_clip[b] : a.steps[*a.step_counter].t_orig;
    const float* r0 = a.kv_step + (size_t)t * 2 * a.d;
    const size_t mrow0 = (size_t)b * (Lk - 1);
    sk = AqSrc<T>{a.kv_mem, mrow0, 2 * a.d, h * DK, Lk, r0 + h * DK, a.zero};
    sv = AqSrc<T>{a.kv_mem, mrow0, 2 * a.d, a.d + h * DK, Lk, r0 + a.d + h * DK, a.zero};
  }
  AqStrip<T, DK> xq, xk;
  xq.load(sq, q0, qrows);
  xk.load(sk, 0, Lk);
  {  // zero the padded operand images (rows >= Lq / Lk must be finite zeros)
    uint4* z = (uint4*)smem;
    const int n16 = (int)(G.off_p / 16);
    for (int i = tid; i < n16; i += NTHREADS) z[i] = make_uint4(0, 0, 0, 0);
  }
  aq_stage_taps<DK>(wl, a);
  __syncthreads();
  xq.template conv<false>(Qm, G.SQ, wl);
  AqStrip<T, DK> xv;
  xv.load(sv, 0, Lk);
  xk.template conv<false>(Km, G.SQ, wl + 4 * DK);
  xv.template conv<true>(Vt, G.SV, wl + 8 * DK);
  __syncthreads();
  attn_core<T>(Qm, Km, Vt, Pw, G, qrows, Lk, DK, a.scale, (T*)a.out + (row0 + q0) * a.ldo + (size_t)h * DK, a.ldo);
}

size_t attention_lds_bytes(int dtype, const AttnArgs& a) {
  return dtype == 0 ? att_geom<float>(a.Lq, a.Lk, a.dk).total : att_geom<bf16_t>(a.Lq, a.Lk, a.dk).total;
}

hipError_t launch_attention(int dtype, const AttnArgs& a, int n, hipStream_t s) {
  if (a.Lq > ATT_LMAX || a.Lk > ATT_LMAX || (a.dk != 32 && a.dk != 64)) return hipErrorInvalidValue;
  if (attention_clip_supported(dtype, a)) return launch_attention_clip(a, n, s);  // long clips, bf16
  if (a.seq_stride && (a.cross || a.Lq != a.Lk)) return hipErrorInvalidValue;
  const size_t lds = attention_lds_bytes(dtype, a);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)attn_kernel<float>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)attn_kernel<bf16_t>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  // query-split kernel whenever its images fit (every BASELINE.json shape); else one
  // workgroup per (head, clip)
  const size_t lq = (dtype == 0 ? aq_geom<float>(a.Lk, a.dk).total : aq_geom<bf16_t>(a.Lk, a.dk).total) +
                    sizeof(float) * 12 * a.dk;  // + conv taps
  static bool aq_attr = false;
  if (!aq_attr) {
    (void)hipFuncSetAttribute((const void*)attn_q_kernel<float, 32>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)attn_q_kernel<float, 64>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)attn_q_kernel<bf16_t, 32>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)attn_q_kernel<bf16_t, 64>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    aq_attr = true;
  }
  if (lq <= 160 * 1024 && !a.no_qsplit && a.zero) {
    const dim3 gq(a.heads, n, (a.Lq + AQ_QT - 1) / AQ_QT);
    const bool d32 = a.dk == 32;
    if (dtype == 0) {
      if (d32) hipLaunchKernelGGL((attn_q_kernel<float, 32>), gq, dim3(NTHREADS), lq, s, a);
      else hipLaunchKernelGGL((attn_q_kernel<float, 64>), gq, dim3(NTHREADS), lq, s, a);
    } else {
      if (d32) hipLaunchKernelGGL((attn_q_kernel<bf16_t, 32>), gq, dim3(NTHREADS), lq, s, a);
      else hipLaunchKernelGGL((attn_q_kernel<bf16_t, 64>), gq, dim3(NTHREADS), lq, s, a);
    }
    return hipGetLastError();
  }
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  dim3 grid(a.heads, n);
  if (dtype == 0)
    hipLaunchKernelGGL(attn_kernel<float>, grid, dim3(NTHREADS), lds, s, a);
  else
    hipLaunchKernelGGL(attn_kernel<bf16_t>, grid, dim3(NTHREADS), lds, s, a);
  return hipGetLastError();
}

// Speech2GestureModelInpaint's projection input (models/model.py:160-162):
// out[m][0..C) = pose[m][c] * mask[m], out[m][C] = mask[m]; rows m = clip * L + frame
__global__ void inpaint_input_kernel(float* out, const float* pose, const float* mask, int M, int C) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * (C + 1)) return;
  const int m = idx / (C + 1), c = idx % (C + 1);
  const float mk = mask[m];
  out[idx] = c < C ? pose[(size_t)m * C + c] * mk : mk;
}

hipError_t launch_inpaint_input(float* out, const float* pose, const float* mask, int M, int C, hipStream_t s) {
  const int total = M * (C + 1);
  hipLaunchKernelGGL(inpaint_input_kernel, dim3((total + 255) / 256), dim3(256), 0, s, out, pose, mask, M, C);
  return hipGetLastError();
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
    z = philox_normal(((uint64_t)r.seed_hi << 32) | r.seed_lo, r.clip_offset + (uint32_t)b, (uint32_t)r.i, TAG_STEP,
                      (uint32_t)(c * a.L + l));
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

__global__ void init_state_gated_kernel(float* x, const float* xT, uint64_t seed, int64_t clip_offset, int clip0,
                                        int n, int C, int L, const int* gate, int gate_xl) {
  if (!gate_open(gate, gate_xl)) return;
  const int idx = blockIdx.x * NTHREADS + threadIdx.x;
  if (idx >= n * L * C) return;
  const int c = idx % C, bl = idx / C, l = bl % L, b = clip0 + bl / L;
  x[(size_t)clip0 * L * C + idx] = xT ? xT[((size_t)b * C + c) * L + l]
                                      : philox_normal(seed, (uint32_t)(clip_offset + b), 0u, TAG_XT, (uint32_t)(c * L + l));
}

hipError_t launch_init_state_gated(float* x, const float* x_T_ncl, uint64_t seed, int64_t clip_offset, int clip0,
                                   int n, int C, int L, const int* gate, int gate_xl, hipStream_t s) {
  hipLaunchKernelGGL(init_state_gated_kernel, dim3((n * L * C + NTHREADS - 1) / NTHREADS), dim3(NTHREADS), 0, s,
                     x, x_T_ncl, seed, clip_offset, clip0, n, C, L, gate, gate_xl);
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

// ---------------------------------------------------------------------------
// LayerNorm of f32 rows -> T rows (nn.LayerNorm([d]), eps 1e-5; two-pass mean / centred
// variance like PRO_LN), one wave per row.  Used where the normalised width exceeds the GEMM's
// fused LN prologue (d = 512, two-way decoder).
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(NTHREADS) layernorm_kernel(const float* in, int len, int stride, int off,
                                                             const float* g, const float* b, T* out, int M, int d) {
  const int lane = threadIdx.x & 63, m = blockIdx.x * (NTHREADS / 64) + (threadIdx.x >> 6);
  if (m >= M) return;
  const float* row = in + map_row(m, len, stride, off) * d;
  constexpr int PER = 16;  // d <= 1024
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = lane + 64 * i;
    v[i] = k < d ? row[k] : 0.f;
    s += v[i];
  }
  const float mu = wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = lane + 64 * i;
    const float e = k < d ? v[i] - mu : 0.f;
    q += e * e;
  }
  const float rs = 1.0f / sqrtf(wave_sum(q) / (float)d + 1e-5f);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = lane + 64 * i;
    if (k < d) out[(size_t)m * d + k] = from_f32<T>((v[i] - mu) * rs * g[k] + b[k]);
  }
}

hipError_t launch_layernorm(int dtype, const float* in, int len, int stride, int off, const float* g, const float* b,
                            void* out, int M, int d, hipStream_t s) {
  if (d > 1024 || M <= 0) return hipErrorInvalidValue;
  const dim3 grid((M + 3) / 4);
  if (dtype == 0)
    hipLaunchKernelGGL(layernorm_kernel<float>, grid, dim3(NTHREADS), 0, s, in, len, stride, off, g, b, (float*)out, M, d);
  else
    hipLaunchKernelGGL(layernorm_kernel<bf16_t>, grid, dim3(NTHREADS), 0, s, in, len, stride, off, g, b, (bf16_t*)out,
                       M, d);
  return hipGetLastError();
}

__global__ void mem_assemble_kernel(float* h, const float* base, const float* tab, const int* t_clip,
                                    const StepRec* steps, const int* step_counter, int L, int Ts, int d) {
  const int b = blockIdx.y, r = blockIdx.x;  // r = 0: step token, 1..Ts: speech rows
  const int J = L + 1 + Ts;
  float* dst = h + ((size_t)b * J + L + r) * d;
  const float* src;
  if (r == 0) {
    const int t = t_clip ? t_clip[b] : steps[*step_counter].t_orig;
    src = tab + (size_t)t * d;
  } else {
    src = base + ((size_t)b * Ts + r - 1) * d;
  }
  for (int k = threadIdx.x; k < d; k += blockDim.x) dst[k] = src[k];
}

hipError_t launch_mem_assemble(float* h, const float* base, const float* tab, const int* t_clip, const StepRec* steps,
                               const int* step_counter, int n, int L, int Ts, int d, hipStream_t s) {
  hipLaunchKernelGGL(mem_assemble_kernel, dim3(1 + Ts, n), dim3(128), 0, s, h, base, tab, t_clip, steps, step_counter,
                     L, Ts, d);
  return hipGetLastError();
}

}  // namespace ggd
