// ggd_cliptiles.h -- the query tiles of the whole-clip attention (clips of >= 96 frames), shared
// by attn_clip_kernel (ggd_attn.hip, the launch route) and the long-clip loop (ggd_long.hip), so
// the two routes compute the same bits.  transformer.py:19-44 (softmax(Q K^T / sqrt(dk)) V).
#pragma once
#include "ggd_common.h"

namespace ggd {

// One wave per 16-query tile (tiles rt = wave, wave + NW, ...); Q / K rows of stride SQ (bf16),
// V^T [32][SV], the wave's P tile [16][SP]; LKT 16-key tiles (Lk padded to 32), keys >= Lk masked.
// Softmax in the base-2 domain (one v_exp_f32 per score) with the lane's 4 query rows as two packed
// f32 pairs for the scaling, the sums and the normalisation (per element the scalar operations and
// order); a masked key is -inf after the scaling, so its exp2 is 0 without a select.  O^T = V^T P^T
// per 16-channel tile: a lane holds 4 consecutive channels of one query row (one 8-byte store).
template <int LKT, int NW, int SQ>
__device__ __forceinline__ void clip_attn_tiles(const bf16_t* Qm, const bf16_t* Km, const bf16_t* Vt, bf16_t* P,
                                                int SV, int SP, int Lq, int Lk, float sl2, bf16_t* out, int ldo,
                                                int wave, int lane) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const int c16 = lane & 15, g4 = lane >> 4;
  const f2 sl = f2{sl2, sl2};
  for (int rt = wave; rt * 16 < Lq; rt += NW) {
    const bf16x8 qa = *(const bf16x8*)(Qm + (rt * 16 + c16) * SQ + g4 * 8);
    bf16x8 kb[LKT];
#pragma unroll
    for (int t = 0; t < LKT; ++t) kb[t] = *(const bf16x8*)(Km + (t * 16 + c16) * SQ + g4 * 8);
    f32x4 s[LKT];
#pragma unroll
    for (int t = 0; t < LKT; ++t)
      s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kb[t], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
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
    const f2 inv01 = f2{1.0f / group_sum<16>(sum01.x), 1.0f / group_sum<16>(sum01.y)};
    const f2 inv23 = f2{1.0f / group_sum<16>(sum23.x), 1.0f / group_sum<16>(sum23.y)};
#pragma unroll
    for (int t = 0; t < LKT; ++t) {
      const f2 lo = f2{s[t][0], s[t][1]} * inv01, hi = f2{s[t][2], s[t][3]} * inv23;
      P[(4 * g4 + 0) * SP + t * 16 + c16] = f2bf(lo.x);
      P[(4 * g4 + 1) * SP + t * 16 + c16] = f2bf(lo.y);
      P[(4 * g4 + 2) * SP + t * 16 + c16] = f2bf(hi.x);
      P[(4 * g4 + 3) * SP + t * 16 + c16] = f2bf(hi.y);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    constexpr int KS = LKT / 2;  // 32-key steps of P V
    bf16x8 pa[KS], vb[2][KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      pa[k] = *(const bf16x8*)(P + c16 * SP + k * 32 + g4 * 8);
      vb[0][k] = *(const bf16x8*)(Vt + c16 * SV + k * 32 + g4 * 8);
      vb[1][k] = *(const bf16x8*)(Vt + (16 + c16) * SV + k * 32 + g4 * 8);
    }
    f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) o[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vb[ct][k], pa[k], o[ct], 0, 0, 0);
    const int i = rt * 16 + c16;
    if (i < Lq) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
        *(uint2*)(out + (size_t)i * ldo + ct * 16 + 4 * g4) = make_uint2(pk_bf16(o[ct][0], o[ct][1]),
                                                                         pk_bf16(o[ct][2], o[ct][3]));
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace ggd
