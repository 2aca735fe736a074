// ggd_chainlib.h -- building blocks of the row-block chains (ggd_chain.hip) and the long-clip
// persistent loop (ggd_long.hip): fragment-packed weight loads, the bf16 MFMA chain of one 256-k
// chunk, the PRO_LN-exact LayerNorm of 32 LDS rows and the epilogue parameter expression.
#pragma once
#include "ggd_common.h"

namespace ggd {
namespace chainlib {

constexpr int CH_MT = 32;           // residual rows per workgroup
constexpr int CH_D = 256;           // d_model
constexpr int CH_FF = 1024;         // feed-forward hidden width
constexpr int HS_STR = CH_D + 4;    // f32 residual rows: the MFMA epilogue (rows 4g + r, 16 columns) hits 64 distinct banks
constexpr int XS_STR = CH_D + 8;    // bf16 A rows (16-byte row pad, as gemm_kernel)
constexpr int HH_STR = CH_FF + 8;   // bf16 hidden rows
constexpr int CH_PMAX = 1024;       // P stage: widest projection
constexpr int CH_DEPTH = 3;         // weight tile groups in flight per wave
constexpr int CH_WAVES = 8;         // two waves per SIMD: one's fp8 widening and loads overlap the other's MFMAs
constexpr int CH_NT = 64 * CH_WAVES;
// per-column epilogue parameters and LayerNorm vectors, staged once per workgroup (LDS reads do
// not queue behind the weight prefetch the way global loads would: vmcnt retires in order)
constexpr int PRM_R = 0, PRM_F1 = PRM_R + 2 * CH_D, PRM_F2 = PRM_F1 + 2 * CH_FF, PRM_P = PRM_F2 + 2 * CH_D,
              PRM_LN = PRM_P + 2 * CH_PMAX, PRM_FLOATS = PRM_LN + 4 * CH_D;
constexpr size_t CH_LDS = sizeof(float) * (CH_MT * HS_STR + PRM_FLOATS) + sizeof(bf16_t) * CH_MT * (XS_STR + HH_STR);

// workgroup barrier for LDS hand-offs only: global loads stay in flight across it
__device__ __forceinline__ void ch_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

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
// Loads of one iteration: TG tiles x the chunk's U units.  wb: this wave's first tile of the
// stage (wave-uniform, so the constant offsets fold into the scalar base).
template <bool W8, int TGB>
__device__ __forceinline__ void ch_load(BBuf<W8, TGB>& B, const unsigned char* wb, unsigned lane16, int t0, int c,
                                        int upt, int tg) {
  constexpr int U = Units<W8>::U;
#pragma unroll
  for (int j = 0; j < TGB; ++j)
    if (j < tg)
#pragma unroll
      for (int u = 0; u < U; ++u)
        B.v[j][u] = *(const uint4*)(wb + (size_t)(((t0 + j) * upt + c * U + u) * 1024) + lane16);
  // keep the loads where they are issued: the scheduler would otherwise sink them next to
  // their first use (lower register pressure) and the prefetch distance would collapse
  __builtin_amdgcn_sched_barrier(0);
}

// acc[i][j] += A[16 i + .][256 c + .] . W[16 (nt0 + j) + .][256 c + .]^T over the chunk's 8 k steps
template <bool W8, int TGB>
__device__ __forceinline__ void ch_mma(const BBuf<W8, TGB>& B, const bf16_t* As, int sa, int c, int lane,
                                       f32x4 (&acc)[2][TGB], int tg) {
  const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int k = (c * 8 + q) * 32 + g * 8;
    const bf16x8 a0 = *(const bf16x8*)(As + r16 * sa + k);
    const bf16x8 a1 = *(const bf16x8*)(As + (16 + r16) * sa + k);
#pragma unroll
    for (int j = 0; j < TGB; ++j) {
      if (j >= tg) continue;
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

// LayerNorm of the 32 LDS residual rows -> bf16 A rows, in gemm_kernel's PRO_LN arithmetic:
// 4 lanes per row, lane j holds float4 columns (j + 4 i) 4, two-pass statistics, xor 1 / 2.
// gm, bt: LDS copies of gamma / beta.
// tid: the thread index (a caller inside a persistent loop passes an opaque one)
__device__ __forceinline__ void ch_layernorm(const float* hs, const float* gm, const float* bt, bf16_t* xs,
                                             int tid = threadIdx.x) {
  if (tid >= CH_MT * 4) return;  // waves 0, 1 (whole waves: the shuffles stay uniform)
  const int r = tid >> 2, j = tid & 3;
  float4 v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = *(const float4*)(hs + r * HS_STR + (j + 4 * i) * 4);
  float mu, rs;
  ln_stats4<16>(v, (float)CH_D, mu, rs);
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

// ------------------------------------------------------------------------------------------
// Block-scaled fp8 MFMA (long-clip loop, GGD_ROUTE_FP8_MFMA): v_mfma_scale_f32_16x16x128_f8f6f4
// with e4m3 activations AND e4m3 weights -- K = 128 per instruction at twice the cycles of the
// bf16 16x16x32 form, i.e. 2x the bf16 rate (MI355X_MICROARCH.md:432), and no fp8 -> bf16
// widening of the weights.  Lane map (scripts/mx_probe.hip, profiles/r04l_mx_probe.txt: the one of
// four hypotheses that reproduces exact integer products with non-unit A and B scales): lane l,
// g = l >> 4, holds bytes j < 16 = k 16 g + j and bytes 16 + j = k 64 + 16 g + j of row l & 15 (A)
// / column l & 15 (B); its e8m0 scale operand scales the 32-value block k 32 g .. 32 g + 31 of
// that row / column -- a block whose values other lanes hold.
//   Activations: one e8m0 scale per (row, 32 consecutive k) -- the MX block -- chosen from the
//   block's max |v| = 1.f 2^E as 2^(E - 7), so the block's values land below 256 < 448 (no
//   saturation) and keep e4m3's relative precision down to max / 2^13.
//   Weights: the context's per-output-channel e4m3 quantisation (scale amax / 448, applied in
//   the epilogue exactly as the bf16-widened route), MFMA scale operand 2^0.
// MX weight packing (chain_pack_kernel<true, true>): unit u of a 256-k chunk = MFMA step s = u / 2,
// half h = u % 2: lane (g, r16) bytes e < 16 = W[16 nt + r16][256 c + 128 s + 64 h + 16 g + e], so
// units 2s, 2s + 1 of a lane are its 32 B operand bytes of step s in the MFMA's order.
constexpr int XS8_STR = CH_D + 16;   // fp8 A rows (bytes; 68 dwords: consecutive rows 4 banks apart)
constexpr int HH8_STR = CH_FF + 16;  // fp8 hidden rows (bytes)
typedef int i32x8 __attribute__((ext_vector_type(8)));

// e8m0 block scale byte of a block whose max |v| is m (>= 0): 2^(E - 7) for m = 1.f 2^E, clamped so
// that the quantisation multiplier 2^(7 - E) stays a normal f32
__device__ __forceinline__ unsigned mx_scale_byte(float m) {
  const int be = (int)((__float_as_uint(m) >> 23) & 0xff);
  return (unsigned)min(max(be - 7, 2), 253);
}
// the multiplier that maps the block into e4m3: 2^-(sb - 127)
__device__ __forceinline__ float mx_mul(unsigned sb) { return __uint_as_float((254u - sb) << 23); }
// 4 f32 -> 4 e4m3 bytes (round to nearest even), byte i = value i
__device__ __forceinline__ unsigned mx_pack4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (unsigned)w;
}
// acc[i][j] += A8[16 i + .][256 c + .] . W[16 (nt0 + j) + .][256 c + .]^T over the chunk's 256 k:
// two block-scaled MFMAs per (row tile, column tile).  A8: fp8 rows (stride sa bytes), As8: their
// e8m0 scale bytes [32 rows][nb blocks].  TR: computed transposed (the weights as the MFMA A
// operand), so lane (c16, g4) holds row 16 i + c16, columns 16 (nt0 + j) + 4 g4 .. + 3 -- four
// consecutive columns of one row, what a packed epilogue store wants
template <int TGB, bool TR = false>
__device__ __forceinline__ void ch_mma_mx(const BBuf<true, TGB>& B, const unsigned char* A8, int sa,
                                          const unsigned char* As8, int nb, int c, int lane, f32x4 (&acc)[2][TGB],
                                          int tg) {
  const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int k = 256 * c + 128 * s + 16 * g, blk = 8 * c + 4 * s + g;
    const uint4 p0 = *(const uint4*)(A8 + r16 * sa + k), q0 = *(const uint4*)(A8 + r16 * sa + k + 64);
    const uint4 p1 = *(const uint4*)(A8 + (16 + r16) * sa + k), q1 = *(const uint4*)(A8 + (16 + r16) * sa + k + 64);
    const i32x8 a0 = {(int)p0.x, (int)p0.y, (int)p0.z, (int)p0.w, (int)q0.x, (int)q0.y, (int)q0.z, (int)q0.w};
    const i32x8 a1 = {(int)p1.x, (int)p1.y, (int)p1.z, (int)p1.w, (int)q1.x, (int)q1.y, (int)q1.z, (int)q1.w};
    const int s0 = As8[r16 * nb + blk], s1 = As8[(16 + r16) * nb + blk];
#pragma unroll
    for (int j = 0; j < TGB; ++j) {
      if (j >= tg) continue;
      const uint4 u0 = B.v[j][2 * s], u1 = B.v[j][2 * s + 1];
      const i32x8 bw = {(int)u0.x, (int)u0.y, (int)u0.z, (int)u0.w, (int)u1.x, (int)u1.y, (int)u1.z, (int)u1.w};
      if constexpr (TR) {
        acc[0][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bw, a0, acc[0][j], 0, 0, 0, 127, 0, s0);
        acc[1][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bw, a1, acc[1][j], 0, 0, 0, 127, 0, s1);
      } else {
        acc[0][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a0, bw, acc[0][j], 0, 0, 0, s0, 0, 127);
        acc[1][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a1, bw, acc[1][j], 0, 0, 0, s1, 0, 127);
      }
    }
  }
}

// acc + bias (and the fp8 per-channel scale) of column n: gemm_kernel's expression; prm = the
// stage's LDS parameters [bias[npad] | scale[npad]]
template <bool W8>
__device__ __forceinline__ float ch_val(const float* prm, int npad, float acc, int n) {
  const float bn = prm[n];
  const float sn = W8 ? prm[npad + n] : 1.0f;
  return W8 ? acc * sn + bn : acc + bn;
}

}  // namespace chainlib
}  // namespace ggd
