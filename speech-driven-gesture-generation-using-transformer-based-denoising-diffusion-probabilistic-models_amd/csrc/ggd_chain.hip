// ggd_chain.hip -- row-block chains of the one-way decoder (gfx950): the generic route's
// GEMMs between two attention launches run as ONE launch per row block.
//
// The generic route (ggd_api.hip launch_decoder) spends 8 launches per layer on GEMMs of a few
// GFLOP each; at 32 clips x 160 frames every one of them is latency-bound (8 - 21 us for
// <= 2.7 GFLOP).  A chain keeps a 32-row block of the residual stream h in LDS and runs, in
// order, whichever of these stages its arguments enable (models/nn.py:160-172 DecoderLayer):
//   R  h += A W_r^T + b_r                       attention output projection + residual
//   F  h += relu2(LN_f(h) W_1^T + b_1) W_2^T + b_2   the feed-forward block, hidden rows in LDS
//   P  out = LN_p(h) W_p^T + b_p                the NEXT consumer's projection: cross-attn Q,
//                                               the next layer's self-attn QKV, or out_layers
// so a layer is [self-attn, chain R+P, cross-attn, chain R+F+P]: 4 launches instead of 10.
//
// Weights are read as MFMA B fragments straight from a fragment-packed copy (chain_pack_kernel)
// into registers -- one coalesced 1 KiB load per wave per (16 columns, 64 k), no LDS staging,
// no barrier per tile -- double-buffered so the next tile group's loads fly under this group's
// MFMAs.  fp8 weights (GGD_FP8W) are widened with v_cvt_scalef32_pk_bf16_fp8 (scale 1: exact).
//
// Bit-exact with the per-GEMM route: every output element is the same MFMA chain
// (v_mfma_f32_16x16x32_bf16, k steps of 32 in order, lane k offsets 8 (lane >> 4)), the
// LayerNorm statistics use gemm_kernel's PRO_LN lane split and operation order, and the
// epilogues are the same expressions (tests/test_gpu_parity.py compares the two routes).
#include "ggd_common.h"

namespace ggd {
namespace {

constexpr int CH_MT = 32;           // residual rows per workgroup
constexpr int CH_D = 256;           // d_model
constexpr int CH_FF = 1024;         // feed-forward hidden width
constexpr int HS_STR = CH_D + 16;   // f32 residual rows: the LN lanes (4 rows x 4) hit distinct banks
constexpr int XS_STR = CH_D + 8;    // bf16 A rows (16-byte row pad, as gemm_kernel)
constexpr int HH_STR = CH_FF + 8;   // bf16 hidden rows
constexpr size_t CH_LDS = sizeof(float) * CH_MT * HS_STR + sizeof(bf16_t) * CH_MT * (XS_STR + HH_STR);

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

// 16-byte units per (16-column tile, 256-k chunk): fp8 packs two k steps per unit
template <bool W8> struct Units { static constexpr int U = W8 ? 4 : 8; };
template <bool W8, int TG> struct BBuf { uint4 v[TG][Units<W8>::U]; };

// 8 e4m3 bytes (two dwords, k ascending) -> the bf16x8 B operand
__device__ __forceinline__ bf16x8 fp8x8_bf16(unsigned w0, unsigned w1) {
  const bf16x2 a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)w0, 1.0f, false);
  const bf16x2 b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)w0, 1.0f, true);
  const bf16x2 c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)w1, 1.0f, false);
  const bf16x2 d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)w1, 1.0f, true);
  return bf16x8{a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
}

// Fragment-packed weights: unit u of tile nt (16 output rows of W) at
//   ((nt * units_per_tile + u) * 64 + lane) * 16 bytes, lane = (g << 4) | r16:
//   bf16: 8 values W[nt 16 + r16][32 u + 8 g + e]
//   fp8:  bytes 0-7 W[nt 16 + r16][64 u + 8 g + e], bytes 8-15 W[..][64 u + 32 + 8 g + e]
template <bool W8, int TG>
__device__ __forceinline__ void ch_load(BBuf<W8, TG>& B, const unsigned char* wf, int upt, int nt0, int c, int lane) {
  constexpr int U = Units<W8>::U;
#pragma unroll
  for (int j = 0; j < TG; ++j)
#pragma unroll
    for (int u = 0; u < U; ++u)
      B.v[j][u] = *(const uint4*)(wf + ((size_t)((nt0 + j) * upt + c * U + u) * 64 + lane) * 16);
}

// acc[i][j] += A[16 i + .][256 c + .] . W[16 (nt0 + j) + .][256 c + .]^T over the chunk's 8 k steps
template <bool W8, int TG>
__device__ __forceinline__ void ch_mma(const BBuf<W8, TG>& B, const bf16_t* As, int sa, int c, int lane,
                                       f32x4 (&acc)[2][TG]) {
  const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int k = (c * 8 + q) * 32 + g * 8;
    const bf16x8 a0 = *(const bf16x8*)(As + r16 * sa + k);
    const bf16x8 a1 = *(const bf16x8*)(As + (16 + r16) * sa + k);
#pragma unroll
    for (int j = 0; j < TG; ++j) {
      bf16x8 bw;
      if constexpr (W8) {
        const uint4 u = B.v[j][q >> 1];
        bw = (q & 1) ? fp8x8_bf16(u.z, u.w) : fp8x8_bf16(u.x, u.y);
      } else {
        bw = __builtin_bit_cast(bf16x8, B.v[j][q]);
      }
      acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw, acc[0][j], 0, 0, 0);
      acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw, acc[1][j], 0, 0, 0);
    }
  }
}

// One GEMM of the chain: out[32][npad] = As[32][kpad] . W^T.  Wave w owns tile groups
// (gi * 4 + w) * TG .. + TG - 1 (gi < ng); iterations (group, 256-k chunk) are double-buffered.
// epi(acc, nt0) runs after a group's last chunk.
template <bool W8, int TG, class Epi>
__device__ __forceinline__ void ch_gemm(const bf16_t* As, int sa, const ChainLin& L, int wave, int lane, Epi&& epi) {
  const unsigned char* wf = (const unsigned char*)L.w;
  const int nch = L.kpad / 256, upt = nch * Units<W8>::U;
  const int ng = L.npad / (64 * TG), I = ng * nch;
  auto nt_of = [&](int it) { return ((it / nch) * 4 + wave) * TG; };
  BBuf<W8, TG> b0, b1;
  f32x4 acc[2][TG];
  auto step = [&](const BBuf<W8, TG>& B, int it) {
    const int c = it % nch;
    if (c == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TG; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    ch_mma<W8, TG>(B, As, sa, c, lane, acc);
    if (c == nch - 1) epi(acc, nt_of(it));
  };
  // loads are unconditional (clamped to the last iteration) so the wait counts stay static
  ch_load<W8, TG>(b0, wf, upt, nt_of(0), 0, lane);
  for (int it = 0; it < I; it += 2) {
    const int i1 = min(it + 1, I - 1), i2 = min(it + 2, I - 1);
    ch_load<W8, TG>(b1, wf, upt, nt_of(i1), i1 % nch, lane);
    step(b0, it);
    ch_load<W8, TG>(b0, wf, upt, nt_of(i2), i2 % nch, lane);
    if (it + 1 < I) step(b1, it + 1);
  }
}

template <bool W8, class Epi>
__device__ __forceinline__ void ch_gemm_any(const bf16_t* As, int sa, const ChainLin& L, int wave, int lane, Epi&& epi) {
  constexpr int TGMAX = W8 ? 4 : 2;  // 64 B-operand VGPRs per buffer
  if (L.npad % (64 * TGMAX) == 0) ch_gemm<W8, TGMAX>(As, sa, L, wave, lane, epi);
  else if (L.npad % 128 == 0) ch_gemm<W8, 2>(As, sa, L, wave, lane, epi);
  else ch_gemm<W8, 1>(As, sa, L, wave, lane, epi);
}

// LayerNorm of the 32 LDS residual rows -> bf16 A rows, in gemm_kernel's PRO_LN arithmetic:
// 4 lanes per row, lane j holds float4 columns (j + 4 i) 4, two-pass statistics, xor 1 / 2.
__device__ __forceinline__ void ch_layernorm(const float* hs, const float* gm, const float* bt, bf16_t* xs) {
  const int tid = threadIdx.x;
  if (tid >= CH_MT * 4) return;  // waves 0, 1 (whole waves: the shuffles stay uniform)
  const int r = tid >> 2, j = tid & 3;
  float4 v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = *(const float4*)(hs + r * HS_STR + (j + 4 * i) * 4);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  const float mu = s / (float)CH_D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float d0 = v[i].x - mu, d1 = v[i].y - mu, d2 = v[i].z - mu, d3 = v[i].w - mu;
    q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
  }
  q += __shfl_xor(q, 1);
  q += __shfl_xor(q, 2);
  const float rs = 1.0f / sqrtf(q / (float)CH_D + 1e-5f);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int k = (j + 4 * i) * 4;
    const float4 g = *(const float4*)(gm + k);
    const float4 b = *(const float4*)(bt + k);
    const float4 x = v[i];
    bf16_t* dst = xs + r * XS_STR + k;
    dst[0] = f2bf((x.x - mu) * rs * g.x + b.x);
    dst[1] = f2bf((x.y - mu) * rs * g.y + b.y);
    dst[2] = f2bf((x.z - mu) * rs * g.z + b.z);
    dst[3] = f2bf((x.w - mu) * rs * g.w + b.w);
  }
}

// acc + bias (and the fp8 per-channel scale) of element (i, j, r): gemm_kernel's expression
template <bool W8>
__device__ __forceinline__ float ch_val(const ChainLin& L, float acc, int n) {
  const float bn = L.b[n];
  const float sn = W8 ? L.scale[n] : 1.0f;
  return W8 ? acc * sn + bn : acc + bn;
}

template <bool W8>
__global__ void __launch_bounds__(NTHREADS) chain_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* hs = (float*)smem;
  bf16_t* xs = (bf16_t*)(smem + sizeof(float) * CH_MT * HS_STR);
  bf16_t* hh = xs + CH_MT * XS_STR;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * CH_MT, rows = min(CH_MT, a.M - m0);
  const int g4 = 4 * (lane >> 4), c16 = lane & 15;
  const bool upd = a.r.w || a.f1.w;  // the residual rows change: written back at the end

  // stage the residual rows (rows past M read as zero) and the R operand
#pragma unroll
  for (int i = 0; i < CH_MT * CH_D / 4 / NTHREADS; ++i) {
    const int e = tid + i * NTHREADS, r = e / (CH_D / 4), c4 = e % (CH_D / 4);
    const float4 v = r < rows ? *(const float4*)(a.h + (size_t)(m0 + r) * CH_D + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    *(float4*)(hs + r * HS_STR + 4 * c4) = v;
  }
  if (a.r.w) {
#pragma unroll
    for (int i = 0; i < CH_MT * CH_D / 8 / NTHREADS; ++i) {
      const int e = tid + i * NTHREADS, r = e / (CH_D / 8), cv = e % (CH_D / 8);
      const uint4 v = r < rows ? *(const uint4*)(a.a_in + (size_t)(m0 + r) * CH_D + 8 * cv) : make_uint4(0, 0, 0, 0);
      *(uint4*)(xs + r * XS_STR + 8 * cv) = v;
    }
  }
  __syncthreads();

  // R: h += A W_r^T + b_r  (EPI_RESID)
  if (a.r.w) {
    ch_gemm_any<W8>(xs, XS_STR, a.r, wave, lane, [&](auto& acc, int nt0) {
      constexpr int TG = sizeof(acc[0]) / sizeof(acc[0][0]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TG; ++j) {
          const int n = (nt0 + j) * 16 + c16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* p = hs + (i * 16 + g4 + r) * HS_STR + n;
            *p = *p + ch_val<W8>(a.r, acc[i][j][r], n);
          }
        }
    });
    __syncthreads();
  }

  // F: h += relu2(LN_f(h) W_1^T + b_1) W_2^T + b_2
  if (a.f1.w) {
    ch_layernorm(hs, a.f_g, a.f_b, xs);
    __syncthreads();
    ch_gemm_any<W8>(xs, XS_STR, a.f1, wave, lane, [&](auto& acc, int nt0) {
      constexpr int TG = sizeof(acc[0]) / sizeof(acc[0][0]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TG; ++j) {
          const int n = (nt0 + j) * 16 + c16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = fmaxf(ch_val<W8>(a.f1, acc[i][j][r], n), 0.f);
            hh[(i * 16 + g4 + r) * HH_STR + n] = f2bf(v * v);
          }
        }
    });
    __syncthreads();
    ch_gemm_any<W8>(hh, HH_STR, a.f2, wave, lane, [&](auto& acc, int nt0) {
      constexpr int TG = sizeof(acc[0]) / sizeof(acc[0][0]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TG; ++j) {
          const int n = (nt0 + j) * 16 + c16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* p = hs + (i * 16 + g4 + r) * HS_STR + n;
            *p = *p + ch_val<W8>(a.f2, acc[i][j][r], n);
          }
        }
    });
    __syncthreads();
  }

  // residual rows back to HBM (the P stage below only reads them)
  if (upd) {
#pragma unroll
    for (int i = 0; i < CH_MT * CH_D / 4 / NTHREADS; ++i) {
      const int e = tid + i * NTHREADS, r = e / (CH_D / 4), c4 = e % (CH_D / 4);
      if (r < rows) *(float4*)(a.h + (size_t)(m0 + r) * CH_D + 4 * c4) = *(const float4*)(hs + r * HS_STR + 4 * c4);
    }
  }

  // P: out = LN_p(h) W_p^T + b_p  (EPI_T bf16, or EPI_F32 for out_layers)
  if (a.p.w) {
    ch_layernorm(hs, a.p_g, a.p_b, xs);
    __syncthreads();
    ch_gemm_any<W8>(xs, XS_STR, a.p, wave, lane, [&](auto& acc, int nt0) {
      constexpr int TG = sizeof(acc[0]) / sizeof(acc[0][0]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TG; ++j) {
          const int n = (nt0 + j) * 16 + c16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = i * 16 + g4 + r;
            if (row >= rows) continue;
            const float v = ch_val<W8>(a.p, acc[i][j][r], n);
            if (a.out_f32) {
              if (n < a.n_valid) ((float*)a.out)[(size_t)(m0 + row) * a.ldo + n] = v;
            } else {
              ((bf16_t*)a.out)[(size_t)(m0 + row) * a.ldo + n] = f2bf(v);
            }
          }
        }
    });
  }
}

// row-major W [npad][kpad] (bf16 or e4m3 bytes) -> the fragment-packed copy, one 16-byte unit per thread
template <bool W8>
__global__ void chain_pack_kernel(const unsigned char* __restrict__ src, unsigned char* __restrict__ dst, int npad,
                                  int kpad) {
  const int upt = W8 ? kpad / 64 : kpad / 32;
  const long units = (long)(npad / 16) * upt * 64;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= units) return;
  const int lane = (int)(e % 64), u = (int)((e / 64) % upt), nt = (int)(e / (64 * upt));
  const int row = nt * 16 + (lane & 15), g = lane >> 4;
  uint4 out;
  if constexpr (W8) {
    const unsigned char* r = src + (size_t)row * kpad + 64 * u + 8 * g;
    const uint2 lo = *(const uint2*)r, hi = *(const uint2*)(r + 32);
    out = make_uint4(lo.x, lo.y, hi.x, hi.y);
  } else {
    out = *(const uint4*)(src + ((size_t)row * kpad + 32 * u + 8 * g) * 2);
  }
  *(uint4*)(dst + e * 16) = out;
}

bool lin_ok(const ChainLin& L, int npad, int kpad) {
  return L.w && L.b && L.npad == npad && L.kpad == kpad;
}

}  // namespace

size_t chain_pack_bytes(int w8, int npad, int kpad) { return (size_t)npad * kpad * (w8 ? 1 : 2); }

hipError_t launch_chain_pack(int w8, const void* src, void* dst, int npad, int kpad, hipStream_t s) {
  if (!src || !dst || npad <= 0 || npad % 64 || kpad <= 0 || kpad % 256) return hipErrorInvalidValue;
  const long units = (long)npad * kpad * (w8 ? 1 : 2) / 16;
  const int blocks = (int)((units + 255) / 256);
  if (w8)
    hipLaunchKernelGGL(chain_pack_kernel<true>, dim3(blocks), dim3(256), 0, s, (const unsigned char*)src,
                       (unsigned char*)dst, npad, kpad);
  else
    hipLaunchKernelGGL(chain_pack_kernel<false>, dim3(blocks), dim3(256), 0, s, (const unsigned char*)src,
                       (unsigned char*)dst, npad, kpad);
  return hipGetLastError();
}

hipError_t launch_chain(int w8, const ChainArgs& a, hipStream_t s) {
  // shapes the kernel assumes: d_model 256, FFN hidden 1024, P columns a multiple of 64
  if (a.M <= 0 || !a.h) return hipErrorInvalidValue;
  if (a.r.w && (!a.a_in || !lin_ok(a.r, CH_D, CH_D))) return hipErrorInvalidValue;
  if (a.f1.w && (!a.f_g || !a.f_b || !lin_ok(a.f1, CH_FF, CH_D) || !lin_ok(a.f2, CH_D, CH_FF)))
    return hipErrorInvalidValue;
  if (a.p.w && (!a.p_g || !a.p_b || !a.out || a.p.kpad != CH_D || a.p.npad <= 0 || a.p.npad % 64 ||
                a.ldo < a.p.npad))
    return hipErrorInvalidValue;
  if (w8 && ((a.r.w && !a.r.scale) || (a.f1.w && (!a.f1.scale || !a.f2.scale)) || (a.p.w && !a.p.scale)))
    return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)chain_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)CH_LDS);
    (void)hipFuncSetAttribute((const void*)chain_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)CH_LDS);
    attr = true;
  }
  const dim3 grid((a.M + CH_MT - 1) / CH_MT);
  if (w8) hipLaunchKernelGGL(chain_kernel<true>, grid, dim3(NTHREADS), CH_LDS, s, a);
  else hipLaunchKernelGGL(chain_kernel<false>, grid, dim3(NTHREADS), CH_LDS, s, a);
  return hipGetLastError();
}

}  // namespace ggd
