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
// no barrier per tile -- with two more tile groups' loads in flight under each group's MFMAs;
// 8 waves (two per SIMD) so one wave's widening and waits overlap the other's MFMAs.  fp8 weights (GGD_FP8W) are widened with v_cvt_scalef32_pk_bf16_fp8 (scale 1: exact).
//
// Bit-exact with the per-GEMM route: every output element is the same MFMA chain
// (v_mfma_f32_16x16x32_bf16, k steps of 32 in order, lane k offsets 8 (lane >> 4)), the
// LayerNorm statistics use gemm_kernel's PRO_LN lane split and operation order, and the
// epilogues are the same expressions (tests/test_gpu_parity.py compares the two routes).
#include "ggd_chainlib.h"

namespace ggd {
namespace {

using namespace chainlib;


// The chain's iterations, fixed at compile time: stage, index within the stage, tile-group width,
// groups per wave and 256-k chunks.  R 256 columns, F1 1024, F2 256 (K 1024), P PN columns.
enum { ST_R = 0, ST_F1 = 1, ST_F2 = 2, ST_P = 3 };
struct ChIt { int stage, l, tg, nch; };

template <bool W8, bool HR, bool HF, int PN>
struct ChPlan {
  static constexpr int TGB = W8 ? 2 : 1;               // 8 16-byte units per wave per iteration
  static constexpr int TGP = PN == 128 ? 1 : TGB;      // 128 columns: one tile per wave
  static constexpr int IR = HR ? 2 / TGB : 0;
  static constexpr int IF1 = HF ? 8 / TGB : 0;
  static constexpr int IF2 = HF ? 4 * (2 / TGB) : 0;
  static constexpr int IP = PN ? PN / (128 * TGP) : 0;
  static constexpr int TOTAL = IR + IF1 + IF2 + IP;
  static __host__ __device__ constexpr ChIt at(int it) {
    return it < IR ? ChIt{ST_R, it, TGB, 1}
         : it < IR + IF1 ? ChIt{ST_F1, it - IR, TGB, 1}
         : it < IR + IF1 + IF2 ? ChIt{ST_F2, it - IR - IF1, TGB, 4}
         : ChIt{ST_P, it - IR - IF1 - IF2, TGP, 1};
  }
};

// PRM offsets of the per-column parameters of a stage, and its width
__host__ __device__ constexpr int prm_of(int stage) {
  return stage == ST_R ? PRM_R : stage == ST_F1 ? PRM_F1 : stage == ST_F2 ? PRM_F2 : PRM_P;
}

// Everything one workgroup's iterations share (registers and LDS pointers).
template <bool W8, int TGB>
struct ChCtx {
  const ChainArgs& a;
  float* hs;
  bf16_t* xs;
  bf16_t* hh;
  float* prm;
  int wave, lane, rows, m0, g4, c16;
  unsigned lane16;
  BBuf<W8, TGB> b[CH_DEPTH];
  f32x4 acc[2][TGB];
};

template <bool W8, bool HR, bool HF, int PN, class X>
__device__ __forceinline__ void ch_writeback(X& x) {  // residual rows back to HBM
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < CH_MT * CH_D / 4 / CH_NT; ++i) {
    const int e = tid + i * CH_NT, r = e / (CH_D / 4), c4 = e % (CH_D / 4);
    if (r < x.rows)
      *(float4*)(x.a.h + (size_t)(x.m0 + r) * CH_D + 4 * c4) = *(const float4*)(x.hs + r * HS_STR + 4 * c4);
  }
}

// weight loads of iteration IT into buffer IT % CH_DEPTH
template <bool W8, bool HR, bool HF, int PN, int IT, class X>
__device__ __forceinline__ void ch_issue(X& x) {
  using P = ChPlan<W8, HR, HF, PN>;
  constexpr ChIt d = P::at(IT);
  constexpr int upt = d.nch * Units<W8>::U;
  const void* w = d.stage == ST_R ? x.a.r.w : d.stage == ST_F1 ? x.a.f1.w : d.stage == ST_F2 ? x.a.f2.w : x.a.p.w;
  const unsigned char* wb = (const unsigned char*)w + (size_t)x.wave * d.tg * upt * 1024;
  ch_load<W8, P::TGB>(x.b[IT % CH_DEPTH], wb, x.lane16, (d.l / d.nch) * CH_WAVES * d.tg, d.l % d.nch, upt, d.tg);
}

// iteration IT: prefetch IT + CH_DEPTH - 1, the stage hand-off if IT opens a stage, the MFMAs,
// the epilogue if IT closes a tile group; then iteration IT + 1
template <bool W8, bool HR, bool HF, int PN, int IT, class X>
__device__ __forceinline__ void ch_iter(X& x) {
  using P = ChPlan<W8, HR, HF, PN>;
  constexpr int TGB = P::TGB, D1 = CH_DEPTH - 1;
  constexpr ChIt d = P::at(IT);
  if constexpr (IT + D1 < P::TOTAL) ch_issue<W8, HR, HF, PN, IT + D1>(x);
  if constexpr (d.l == 0 && d.stage == ST_F1) {   // LDS hand-offs; prefetched weights stay in flight
    if constexpr (HR) ch_bar();
    ch_layernorm(x.hs, x.prm + PRM_LN, x.prm + PRM_LN + CH_D, x.xs);
    ch_bar();
  } else if constexpr (d.l == 0 && d.stage == ST_F2) {
    ch_bar();
  } else if constexpr (d.l == 0 && d.stage == ST_P) {
    if constexpr (HR || HF) {
      ch_bar();
      ch_writeback<W8, HR, HF, PN>(x);
    }
    ch_layernorm(x.hs, x.prm + PRM_LN + 2 * CH_D, x.prm + PRM_LN + 3 * CH_D, x.xs);
    ch_bar();
  }
  constexpr int c = d.l % d.nch;
  const int nt0 = ((d.l / d.nch) * CH_WAVES + x.wave) * d.tg;
  if constexpr (c == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < TGB; ++j) x.acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if constexpr (d.stage == ST_F2)
    ch_mma<W8, TGB>(x.b[IT % CH_DEPTH], x.hh, HH_STR, c, x.lane, x.acc, d.tg);
  else
    ch_mma<W8, TGB>(x.b[IT % CH_DEPTH], x.xs, XS_STR, c, x.lane, x.acc, d.tg);
  if constexpr (c == d.nch - 1) {
    // epilogues (C/D map of the 16x16 MFMA: column lane & 15, row 4 (lane >> 4) + r)
    constexpr int np = d.stage == ST_F1 ? CH_FF : d.stage == ST_P ? PN : CH_D;
    const float* pp = x.prm + prm_of(d.stage);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < d.tg; ++j) {
        const int n = (nt0 + j) * 16 + x.c16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + x.g4 + r;
          const float v = ch_val<W8>(pp, np, x.acc[i][j][r], n);
          if constexpr (d.stage == ST_R || d.stage == ST_F2) {   // EPI_RESID
            float* p = x.hs + row * HS_STR + n;
            *p = *p + v;
          } else if constexpr (d.stage == ST_F1) {               // EPI_RELU2
            const float y = fmaxf(v, 0.f);
            x.hh[row * HH_STR + n] = f2bf(y * y);
          } else if (row < x.rows) {                             // EPI_T / EPI_F32
            if (x.a.out_f32) {
              if (n < x.a.n_valid) ((float*)x.a.out)[(size_t)(x.m0 + row) * x.a.ldo + n] = v;
            } else {
              ((bf16_t*)x.a.out)[(size_t)(x.m0 + row) * x.a.ldo + n] = f2bf(v);
            }
          }
        }
      }
  }
  if constexpr (IT + 1 < P::TOTAL) ch_iter<W8, HR, HF, PN, IT + 1>(x);
}

template <bool W8, bool HR, bool HF, int PN>
__global__ void __launch_bounds__(CH_NT) chain_kernel(ChainArgs a) {
  using P = ChPlan<W8, HR, HF, PN>;
  constexpr int D1 = CH_DEPTH - 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  ChCtx<W8, P::TGB> x{a};
  x.hs = (float*)smem;
  x.xs = (bf16_t*)(smem + sizeof(float) * CH_MT * HS_STR);
  x.hh = x.xs + CH_MT * XS_STR;
  x.prm = (float*)(x.hh + CH_MT * HH_STR);
  x.wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  x.lane = lane;
  x.m0 = blockIdx.x * CH_MT;
  x.rows = min(CH_MT, a.M - x.m0);
  x.g4 = 4 * (lane >> 4);
  x.c16 = lane & 15;
  x.lane16 = (unsigned)lane * 16u;
  const int rows = x.rows, m0 = x.m0;

  // the first iterations' weights fly while the rows and parameters are staged
  ch_issue<W8, HR, HF, PN, 0>(x);
  if constexpr (D1 > 1 && P::TOTAL > 1) ch_issue<W8, HR, HF, PN, 1>(x);
  static_assert(CH_DEPTH == 3, "prologue issues CH_DEPTH - 1 iterations");

  {  // staging: every global load issued before the first LDS write (one round trip)
    constexpr int NSEG = 12;
    const float* src[NSEG] = {a.r.b, a.r.scale, a.f1.b, a.f1.scale, a.f2.b, a.f2.scale, a.p.b, a.p.scale,
                              a.f_g, a.f_b, a.p_g, a.p_b};
    constexpr int dst[NSEG] = {PRM_R, PRM_R + CH_D, PRM_F1, PRM_F1 + CH_FF, PRM_F2, PRM_F2 + CH_D, PRM_P, PRM_P + PN,
                               PRM_LN, PRM_LN + CH_D, PRM_LN + 2 * CH_D, PRM_LN + 3 * CH_D};
    constexpr int len[NSEG] = {CH_D, CH_D, CH_FF, CH_FF, CH_D, CH_D, PN, PN, CH_D, CH_D, CH_D, CH_D};
    constexpr bool on[NSEG] = {HR, HR, HF, HF, HF, HF, PN > 0, PN > 0, HF, HF, PN > 0, PN > 0};
    constexpr bool scale[NSEG] = {false, true, false, true, false, true, false, true, false, false, false, false};
    float v[NSEG][2];
#pragma unroll
    for (int sgi = 0; sgi < NSEG; ++sgi)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int e = tid + k * CH_NT;
        v[sgi][k] = 1.0f;
        if (on[sgi] && e < len[sgi] && (W8 || !scale[sgi])) v[sgi][k] = src[sgi][e];
      }
    float4 hv[CH_MT * CH_D / 4 / CH_NT];
#pragma unroll
    for (int i = 0; i < CH_MT * CH_D / 4 / CH_NT; ++i) {
      const int e = tid + i * CH_NT, r = e / (CH_D / 4), c4 = e % (CH_D / 4);
      hv[i] = r < rows ? *(const float4*)(a.h + (size_t)(m0 + r) * CH_D + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    uint4 av[CH_MT * CH_D / 8 / CH_NT];
    if constexpr (HR) {
#pragma unroll
      for (int i = 0; i < CH_MT * CH_D / 8 / CH_NT; ++i) {
        const int e = tid + i * CH_NT, r = e / (CH_D / 8), cv = e % (CH_D / 8);
        av[i] = r < rows ? *(const uint4*)(a.a_in + (size_t)(m0 + r) * CH_D + 8 * cv) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int sgi = 0; sgi < NSEG; ++sgi)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int e = tid + k * CH_NT;
        if (on[sgi] && e < len[sgi]) x.prm[dst[sgi] + e] = v[sgi][k];
      }
#pragma unroll
    for (int i = 0; i < CH_MT * CH_D / 4 / CH_NT; ++i) {
      const int e = tid + i * CH_NT, r = e / (CH_D / 4), c4 = e % (CH_D / 4);
      *(float4*)(x.hs + r * HS_STR + 4 * c4) = hv[i];
    }
    if constexpr (HR) {
#pragma unroll
      for (int i = 0; i < CH_MT * CH_D / 8 / CH_NT; ++i) {
        const int e = tid + i * CH_NT, r = e / (CH_D / 8), cv = e % (CH_D / 8);
        *(uint4*)(x.xs + r * XS_STR + 8 * cv) = av[i];
      }
    }
  }
  ch_bar();
  ch_iter<W8, HR, HF, PN, 0>(x);
  if constexpr (!PN) {
    ch_bar();
    ch_writeback<W8, HR, HF, PN>(x);
  }
}

// row-major W [npad][kpad] (bf16 or e4m3 bytes) -> the fragment-packed copy, one 16-byte unit per thread
// MX: the block-scaled MFMA's B order (ggd_chainlib.h: unit u of chunk c = step u / 2, half u % 2)
template <bool W8, bool MX = false>
__global__ void chain_pack_kernel(const unsigned char* __restrict__ src, unsigned char* __restrict__ dst, int npad,
                                  int kpad) {
  const int upt = W8 ? kpad / 64 : kpad / 32;
  const long units = (long)(npad / 16) * upt * 64;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= units) return;
  const int lane = (int)(e % 64), u = (int)((e / 64) % upt), nt = (int)(e / (64 * upt));
  const int row = nt * 16 + (lane & 15), g = lane >> 4;
  uint4 out;
  if constexpr (MX) {
    const int c = u >> 2, st = (u >> 1) & 1, hf = u & 1;
    out = *(const uint4*)(src + (size_t)row * kpad + 256 * c + 128 * st + 64 * hf + 16 * g);
  } else if constexpr (W8) {
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
  if (w8 == 2)  // e4m3 in the block-scaled MFMA's B order
    hipLaunchKernelGGL((chain_pack_kernel<true, true>), dim3(blocks), dim3(256), 0, s, (const unsigned char*)src,
                       (unsigned char*)dst, npad, kpad);
  else if (w8)
    hipLaunchKernelGGL(chain_pack_kernel<true>, dim3(blocks), dim3(256), 0, s, (const unsigned char*)src,
                       (unsigned char*)dst, npad, kpad);
  else
    hipLaunchKernelGGL(chain_pack_kernel<false>, dim3(blocks), dim3(256), 0, s, (const unsigned char*)src,
                       (unsigned char*)dst, npad, kpad);
  return hipGetLastError();
}

namespace {

template <bool W8, bool HR, bool HF, int PN>
hipError_t chain_go(const ChainArgs& a, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)chain_kernel<W8, HR, HF, PN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)CH_LDS);
    attr = true;
  }
  hipLaunchKernelGGL((chain_kernel<W8, HR, HF, PN>), dim3((a.M + CH_MT - 1) / CH_MT), dim3(CH_NT), CH_LDS, s, a);
  return hipGetLastError();
}

template <bool W8, bool HR, bool HF>
hipError_t chain_pn(const ChainArgs& a, hipStream_t s) {
  switch (a.p.w ? a.p.npad : 0) {
    case 0:
      if constexpr (HR) return chain_go<W8, HR, HF, 0>(a, s);
      break;
    case 128: return chain_go<W8, HR, HF, 128>(a, s);
    case 256: return chain_go<W8, HR, HF, 256>(a, s);
    case 768: return chain_go<W8, HR, HF, 768>(a, s);
    default: break;
  }
  return hipErrorInvalidValue;
}

template <bool W8>
hipError_t chain_stages(const ChainArgs& a, hipStream_t s) {
  if (a.r.w && a.f1.w) return chain_pn<W8, true, true>(a, s);
  if (a.r.w) return chain_pn<W8, true, false>(a, s);
  if (a.f1.w) return hipErrorInvalidValue;  // F without R: not a decoder-layer shape
  return chain_pn<W8, false, false>(a, s);
}

}  // namespace

bool chain_p_supported(int npad) { return npad == 128 || npad == 256 || npad == 768; }

hipError_t launch_chain(int w8, const ChainArgs& a, hipStream_t s) {
  // shapes the kernel assumes: d_model 256, FFN hidden 1024, P 128 / 256 / 768 columns
  if (a.M <= 0 || !a.h) return hipErrorInvalidValue;
  if (a.r.w && (!a.a_in || !lin_ok(a.r, CH_D, CH_D))) return hipErrorInvalidValue;
  if (a.f1.w && (!a.f_g || !a.f_b || !lin_ok(a.f1, CH_FF, CH_D) || !lin_ok(a.f2, CH_D, CH_FF)))
    return hipErrorInvalidValue;
  if (a.p.w && (!a.p_g || !a.p_b || !a.p.b || !a.out || a.p.kpad != CH_D || a.ldo < a.p.npad ||
                !chain_p_supported(a.p.npad)))
    return hipErrorInvalidValue;
  if (w8 && ((a.r.w && !a.r.scale) || (a.f1.w && (!a.f1.scale || !a.f2.scale)) || (a.p.w && !a.p.scale)))
    return hipErrorInvalidValue;
  return w8 ? chain_stages<true>(a, s) : chain_stages<false>(a, s);
}

// ------------------------------------------------------------------------------------------
// One block-scaled fp8 MFMA Linear, exactly as the long-clip loop's MX stages compute it
// (ggd_long.hip: LayerNorm projections and FFN; ggd_chainlib.h ch_mma_mx): the f32 input rows
// quantised to e4m3 with one e8m0 scale per 32 consecutive values (mx_scale_byte / mx_mul /
// mx_pack4), the e4m3 weights in the MX B order (chain_pack_kernel<true, true>), 256-k chunks of two
// v_mfma_scale_f32_16x16x128_f8f6f4 per (row tile, column tile), and the epilogue
// out = acc * wscale[col] + bias[col] (ch_val).  A verification entry (ggd_mx_linear): it pins the
// arithmetic of those stages value by value against a numpy restatement (tests/test_gpu_mx_linear.py).
// One wave per 32 rows x 32 columns; K % 256 == 0, K <= 1024.
// ------------------------------------------------------------------------------------------
namespace {
constexpr int MXL_KMAX = 1024, MXL_STR = MXL_KMAX + 16;
__global__ void __launch_bounds__(64) mx_linear_kernel(int M, int N, int K, const float* __restrict__ a,
                                                       const unsigned char* __restrict__ wpk, const float* __restrict__ wscale,
                                                       const float* __restrict__ bias, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) unsigned char xs8[32 * MXL_STR];
  __shared__ unsigned char sc8[32 * (MXL_KMAX / 32)];
  const int lane = threadIdx.x, m0 = blockIdx.y * 32, t0 = blockIdx.x * 2, nb = K / 32;
  // quantise: lane takes (row, 32-block) pairs; the block max, its scale byte, 8 packed quads
  for (int pr = lane; pr < 32 * nb; pr += 64) {
    const int r = pr / nb, blk = pr - r * nb;
    const float* src = a + (size_t)min(m0 + r, M - 1) * K + blk * 32;
    float v[32];
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      v[i] = src[i];
      m = fmaxf(m, fabsf(v[i]));
    }
    const unsigned sb = mx_scale_byte(m);
    const float mul = mx_mul(sb);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      *(unsigned*)(xs8 + r * MXL_STR + blk * 32 + 4 * q) =
          mx_pack4(v[4 * q] * mul, v[4 * q + 1] * mul, v[4 * q + 2] * mul, v[4 * q + 3] * mul);
    sc8[r * nb + blk] = (unsigned char)sb;
  }
  __syncthreads();
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int upt = K / 64;
  for (int c = 0; c < K / 256; ++c) {
    BBuf<true, 2> B;
    ch_load<true, 2>(B, wpk, (unsigned)lane * 16, t0, c, upt, 2);
    ch_mma_mx<2>(B, xs8, MXL_STR, sc8, nb, c, lane, acc, 2);
  }
  // C layout: row 16 i + 4 (lane >> 4) + r, column 16 (t0 + j) + (lane & 15)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = (t0 + j) * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + 16 * i + 4 * (lane >> 4) + r;
        if (row < M && col < N) out[(size_t)row * N + col] = acc[i][j][r] * wscale[col] + bias[col];
      }
  }
}
}  // namespace

}  // namespace ggd

extern "C" int ggd_mx_linear(int32_t M, int32_t N, int32_t K, const float* a, const uint8_t* w_e4m3, const float* wscale,
                             const float* bias, float* out, void* stream) {
  using namespace ggd;
  if (M <= 0 || N <= 0 || K <= 0 || K % 256 || K > MXL_KMAX || N % 64 || !a || !w_e4m3 || !wscale || !bias || !out)
    return -1;   // GGD_ERR_ARG
  hipStream_t s = (hipStream_t)stream;
  void* pk = nullptr;
  if (hipMalloc(&pk, (size_t)N * K) != hipSuccess) return -3;
  hipError_t e = launch_chain_pack(2, w_e4m3, pk, N, K, s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(mx_linear_kernel, dim3(N / 32, (M + 31) / 32), dim3(64), 0, s, M, N, K, a,
                       (const unsigned char*)pk, wscale, bias, out);
    e = hipGetLastError();
  }
  const hipError_t e2 = hipStreamSynchronize(s);
  (void)hipFree(pk);
  return e == hipSuccess && e2 == hipSuccess ? 0 : -3;
}
