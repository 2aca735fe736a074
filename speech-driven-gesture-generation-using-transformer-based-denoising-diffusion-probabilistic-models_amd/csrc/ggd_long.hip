// ggd_long.hip -- the long-clip reverse loop as ONE persistent launch (gfx950; bf16 activations,
// bf16 or fp8 weights): the route of BASELINE configs[3] (32 clips x 160 frames, DDPM 1000).
//
// The launch route (ggd_chain.hip + ggd_attn.hip) runs a denoise step as 19 kernels; at 32 clips
// a kernel boundary costs a few microseconds of fill / drain and cold loads, a third of the step.
// Here 8 workgroups per clip run every step of the loop inside one launch and meet at barriers
// of their clip group only (clips are independent): per layer
//   self-attention   part p = head p                      (qkv rows -> att rows)
//   chain A          parts p < L / 32: row block p         R(o_sa) + P(LN2, q_ca)      -> q rows
//   cross-attention  part p = head p                      (q rows, speech memory -> att rows)
//   chain B          row blocks                            R(o_ca) + F + P(next LN1, qkv)
// and at the last layer chain B ends the step: P(out_layers) into LDS, the posterior update of
// the block's frames (counter or injected noise), then the next step's emb_x + PE and LN1 + QKV.
// A row block's residual rows stay resident in LDS for the whole loop (no h traffic at all).
//
// The chain and attention bodies are those of the launch route (ggd_chainlib.h; same MFMA chains
// and epilogue expressions, so the two routes agree bit for bit -- tests/test_gpu_parity.py),
// with the hand-off rows read past the CU's L1 (sc1) since other workgroups wrote them.
// Placement and barriers follow ggd_mega.hip: a clip group lives on one XCD (XCC-id tickets,
// grid padded to whole XCDs; a launch that cannot be placed leaves before any work with status 3
// and the host runs the launch route), hand-off stores stay in that XCD's L2, every wait is
// bounded (status 1).
#include "ggd_chainlib.h"
#include "ggd_fusedlib.h"
#include "ggd_cliptiles.h"

namespace ggd {
namespace {

using namespace chainlib;

// weight tile groups in flight per wave.  Round 5, A/B on one box (profiles/r05y4_c4_depth_ab.txt,
// r05y6_c4w_depth_ab.txt): 2 -> 156.1-157.0 ms per C4 launch, 3 -> 159.0-159.5, 4 -> 163.0 (fp8 MFMA
// route; widened route 163.5-164.4 vs 164.7-165.7 at 3): the loop sits at the 256-VGPR limit, and
// the 32 registers of the third group cost more than its prefetch distance buys (4 spills).
constexpr int LK_DEPTH = 2;
constexpr int LK_ARRIVE = 128, LK_FLAGS = 256;  // ctl: tickets [x * 16], arrivals, group flag lines [g * 32]

__device__ __forceinline__ unsigned lk_add(unsigned* p, unsigned v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned lk_load(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// thread 0: (group << 3 | part), -2 (idle surplus), -1 (status set).  Group g lives on XCD g % 8.
__device__ int lk_role(unsigned* ctl, int* status, int nwg, int G) {
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 7;
  const int t = (int)lk_add(ctl + xcc * 16, 1u);
  __hip_atomic_fetch_add(ctl + LK_ARRIVE, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned t_res = wait_t0();
  while (__hip_atomic_load(ctl + LK_ARRIVE, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nwg) {
    if (wait_expired(t_res)) {
      atomicMax(status, 2);
      return -1;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  auto slots = [&](int x) { return x < G ? 8 * ((G - 1 - x) / 8 + 1) : 0; };
  for (int x = 0; x < 8; ++x)  // every workgroup reads the same final counts: one launch-wide verdict
    if ((int)lk_load(ctl + x * 16) < slots(x)) {
      atomicMax(status, 3);
      return -1;
    }
  if (t >= slots((int)xcc)) return -2;
  return (((int)xcc + 8 * (t >> 3)) << 3) | (t & 7);
}

// barrier of the clip group's 8 workgroups (one L2): each publishes its epoch in its word of the
// group's flag line after its stores have drained; wave 0 polls the 8 words with sc1 loads.
// prefetch: the next phase's loads that do not depend on the other workgroups' stores (weights,
// parameters, cached keys), issued after the drain so that they are in flight across the wait;
// the polling wave issues its share after its poll (a poll load would retire behind them)
__device__ __forceinline__ void lk_nop() {}
template <typename F = void (*)()>
__device__ __forceinline__ bool lk_sync(unsigned* flags, int part, unsigned epoch, int* status, int* s_ok,
                                        F&& prefetch = lk_nop) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const __amdgpu_buffer_rsrc_t r = uni_rsrc(flags, 32u);
    __builtin_amdgcn_raw_buffer_store_b32(epoch, r, part * 4, 0, 0);
  }
  if (threadIdx.x >= 64) prefetch();
  if (threadIdx.x < 64) {
    const __amdgpu_buffer_rsrc_t r = uni_rsrc(flags, 32u);
    const int off = (threadIdx.x & 7) * 4;
    int ok = 1;
    const unsigned t0 = wait_t0();
    for (int spin = 0;; ++spin) {
      const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, CP_COH);
      if (__ballot(v < epoch) == 0) break;
      if ((spin & 255) == 255) {
        const bool expired = wait_expired(t0);
        if (expired || __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          if (threadIdx.x == 0) status_leave(status, expired);
          ok = 0;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (threadIdx.x == 0) *s_ok = ok;
    prefetch();
  }
  bar_lds();
  return *s_ok != 0;
}

// ------------------------------------------------------------------------------------------
// LDS: [hs: the row block's residual rows, resident] [scratch: chain xs | hh | prm, or attention]
// ------------------------------------------------------------------------------------------
constexpr size_t LK_HS = sizeof(float) * CH_MT * HS_STR;
constexpr int EPS_STR = 132;  // f32 eps rows of the out_layers projection (in the hh region)

// ------------------------------------------------------------------------------------------
// chain phases: a compile-time list of GEMM stages
// ------------------------------------------------------------------------------------------
enum { SK_E = 0, SK_R, SK_F1, SK_F2, SK_P, SK_PO, SK_P2 };
struct Stg { int kind, ncols, nch; };
enum { K_A = 0, K_B, K_BL, K_BLL };  // chain A, chain B, chain B ending a step, ending the loop

template <int KIND> struct LkPlan;
template <> struct LkPlan<K_A> {
  static constexpr int NS = 2;
  static constexpr Stg s[NS] = {{SK_R, 256, 1}, {SK_P, 256, 1}};
};
template <> struct LkPlan<K_B> {
  static constexpr int NS = 4;
  static constexpr Stg s[NS] = {{SK_R, 256, 1}, {SK_F1, 1024, 1}, {SK_F2, 256, 4}, {SK_P, 768, 1}};
};
template <> struct LkPlan<K_BL> {
  static constexpr int NS = 6;
  static constexpr Stg s[NS] = {{SK_R, 256, 1}, {SK_F1, 1024, 1}, {SK_F2, 256, 4}, {SK_PO, 128, 1},
                                {SK_E, 256, 1},  {SK_P2, 768, 1}};
};
template <> struct LkPlan<K_BLL> {
  static constexpr int NS = 4;
  static constexpr Stg s[NS] = {{SK_R, 256, 1}, {SK_F1, 1024, 1}, {SK_F2, 256, 4}, {SK_PO, 128, 1}};
};

template <bool W8, int KIND>
struct LkGeo {
  using PL = LkPlan<KIND>;
  static constexpr int TGB = W8 ? 2 : 1;
  static constexpr int tg(int i) { return PL::s[i].ncols == 128 ? 1 : TGB; }
  static constexpr int iters(int i) { return PL::s[i].ncols / (16 * CH_WAVES * tg(i)) * PL::s[i].nch; }
  static constexpr int first(int i) { return i == 0 ? 0 : first(i - 1) + iters(i - 1); }
  static constexpr int TOTAL = first(PL::NS - 1) + iters(PL::NS - 1);
  static constexpr int stage_of(int it, int i = 0) { return it < first(i) + iters(i) ? i : stage_of(it, i + 1); }
  static constexpr int prm(int i) { return i == 0 ? 0 : prm(i - 1) + 2 * PL::s[i - 1].ncols; }  // bias | scale
  static constexpr int PRM_LN0 = prm(PL::NS - 1) + 2 * PL::s[PL::NS - 1].ncols;
  static constexpr int ln(int i) { return PRM_LN0 + 2 * CH_D * i; }                            // gamma | beta
  static constexpr int PRM_TOTAL = PRM_LN0 + 2 * CH_D * PL::NS;
  static constexpr size_t LDS = LK_HS + sizeof(bf16_t) * CH_MT * (XS_STR + HH_STR) + sizeof(float) * (PRM_TOTAL + 2 * CH_MT);
};

// ch_layernorm with the statistics on two waves (gemm_kernel's PRO_LN lanes and order) and the
// normalisation on all eight: the same values, a quarter of the per-thread element work.
// st: LDS [32][mu, rs]
__device__ __forceinline__ void lk_layernorm(const float* hs, const float* gm, const float* bt, bf16_t* xs, float* st) {
  const int tid = ltid();
  if (tid < CH_MT * 4) {
    const int r = tid >> 2, j = tid & 3;
    float4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = *(const float4*)(hs + r * HS_STR + (j + 4 * i) * 4);
    float mu, rs;
    ln_stats4<16>(v, (float)CH_D, mu, rs);
    if (j == 0) {
      st[2 * r] = mu;
      st[2 * r + 1] = rs;
    }
  }
  ch_bar();
  for (int e = tid; e < CH_MT * CH_D / 4; e += CH_NT) {
    const int r = e / (CH_D / 4), k = (e % (CH_D / 4)) * 4;
    const float mu = st[2 * r], rs = st[2 * r + 1];
    const float4 x = *(const float4*)(hs + r * HS_STR + k);
    const float4 g = *(const float4*)(gm + k);
    const float4 b = *(const float4*)(bt + k);
    // one 8-byte LDS store of the 4 bf16 values (two v_cvt_pk_bf16_f32)
    *(uint2*)(xs + r * XS_STR + k) = make_uint2(pk_bf16((x.x - mu) * rs * g.x + b.x, (x.y - mu) * rs * g.y + b.y),
                                                pk_bf16((x.z - mu) * rs * g.z + b.z, (x.w - mu) * rs * g.w + b.w));
  }
}

// lk_layernorm into the block-scaled fp8 A image (MX stages): the same statistics and normalised
// values, then per (row, 32 columns) the e8m0 block scale over the 8 lanes that hold the block
// (a wave covers one row per pass) and 4 e4m3 bytes per lane.  xs8: [32][XS8_STR] bytes, sc: [32][8]
__device__ __forceinline__ void lk_layernorm_mx(const float* hs, const float* gm, const float* bt, unsigned char* xs8,
                                                unsigned char* sc, float* st) {
  const int tid = ltid();
  if (tid < CH_MT * 4) {
    const int r = tid >> 2, j = tid & 3;
    float4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = *(const float4*)(hs + r * HS_STR + (j + 4 * i) * 4);
    float mu, rs;
    ln_stats4<16>(v, (float)CH_D, mu, rs);
    if (j == 0) {
      st[2 * r] = mu;
      st[2 * r + 1] = rs;
    }
  }
  ch_bar();
  static_assert(CH_MT * CH_D / 4 % CH_NT == 0 && CH_NT % (CH_D / 4) == 0, "a wave pass is one whole row");
#pragma unroll
  for (int i = 0; i < CH_MT * CH_D / 4 / CH_NT; ++i) {
    const int e = tid + i * CH_NT, r = e / (CH_D / 4), k = (e % (CH_D / 4)) * 4;
    const float mu = st[2 * r], rs = st[2 * r + 1];
    const float4 x = *(const float4*)(hs + r * HS_STR + k);
    const float4 g = *(const float4*)(gm + k);
    const float4 b = *(const float4*)(bt + k);
    const float y0 = (x.x - mu) * rs * g.x + b.x, y1 = (x.y - mu) * rs * g.y + b.y;
    const float y2 = (x.z - mu) * rs * g.z + b.z, y3 = (x.w - mu) * rs * g.w + b.w;
    const float m = group_max<8>(fmaxf(fmaxf(fabsf(y0), fabsf(y1)), fmaxf(fabsf(y2), fabsf(y3))));
    const unsigned sb = mx_scale_byte(m);
    const float mul = mx_mul(sb);
    *(unsigned*)(xs8 + r * XS8_STR + k) = mx_pack4(y0 * mul, y1 * mul, y2 * mul, y3 * mul);
    if ((tid & 7) == 0) sc[r * (CH_D / 32) + k / 32] = (unsigned char)sb;
  }
}

// stage arguments and layers live in constant memory: field reads are scalar loads
typedef const __attribute__((address_space(4))) ChainStage* cst_t;
typedef const __attribute__((address_space(4))) LongArgs cla_T;  // the kernel's argument block, in place
typedef const __attribute__((address_space(4))) LongLayer* cll_t;

constexpr int LK_UPD_NW = (128 * (CH_MT / 4) + CH_NT - 1) / CH_NT;  // update items per thread (C <= 128)
template <bool W8, int TGB>
struct LkCtx {
  cla_T& a;
  cst_t sa;
  float* hs;
  bf16_t* xs;
  bf16_t* hh;
  float* prm;
  int wave, lane, g4, c16, b, part, it;  // it: the loop iteration (update, noise)
  unsigned lane16;
  BBuf<W8, TGB> bb[LK_DEPTH];
  f32x4 acc[2][TGB];
  float uxo[LK_UPD_NW][4], uz[LK_UPD_NW][4];  // the update's x (and injected noise), loaded at PO (lk_update_load)
};

template <bool W8, int KIND, int IT, class X>
__device__ __forceinline__ void lk_issue(X& x) {
  using GE = LkGeo<W8, KIND>;
  constexpr int si = GE::stage_of(IT), l = IT - GE::first(si), tg = GE::tg(si), nch = LkPlan<KIND>::s[si].nch;
  constexpr int upt = nch * Units<W8>::U;
  const unsigned char* wb = (const unsigned char*)x.sa[si].w.w + (size_t)x.wave * tg * upt * 1024;
  ch_load<W8, GE::TGB>(x.bb[IT % LK_DEPTH], wb, x.lane16, (l / nch) * CH_WAVES * tg, l % nch, upt, tg);
}

// The update's loads: a thread's <= 2 items' x (and injected noise), issued at the start of the PO
// stage so that they land during LN_out and out_layers (round 6: loaded inside the update they cost a
// memory round trip after the eps rows were ready)
template <class X>
__device__ __forceinline__ void lk_update_load(X& x) {
  cla_T& a = x.a;
  const int C = a.C, L = a.L, l0 = x.part * CH_MT, NWI = C * (CH_MT / 4);
  const float* xg = a.x + ((size_t)x.b * L + l0) * C;
#pragma unroll
  for (int k = 0; k < LK_UPD_NW; ++k) {
    const int w = min(ltid() + k * CH_NT, NWI - 1);  // clamped: a thread past the items loads a valid one
    const int c = w / (CH_MT / 4), q4 = (w % (CH_MT / 4)) * 4, l = l0 + q4;
#pragma unroll
    for (int i = 0; i < 4; ++i) x.uxo[k][i] = ld_f32<CP_COH>(xg, (uint32_t)((q4 + i) * C + c));
    if (a.noise) {
#pragma unroll
      for (int i = 0; i < 4; ++i) x.uz[k][i] = a.noise[(size_t)x.it * a.n * C * L + ((size_t)x.b * C + c) * L + l + i];
    }
  }
}

// one work item = channel c x 4 consecutive frames: one Philox call gives their 4 normals
// (counter quad (c L + l) / 4, update_kernel's element -> quad map; L and l0 are multiples of 32);
// x / injected noise from lk_update_load
template <class X>
__device__ __forceinline__ void lk_update(X& x, bool to_xs) {
  cla_T& a = x.a;
  const int C = a.C, L = a.L, l0 = x.part * CH_MT, NWI = C * (CH_MT / 4);
  constexpr int NW = LK_UPD_NW;
  const StepRec r = a.steps[x.it];
  const float* eps = (const float*)x.hh;
  float* xg = a.x + ((size_t)x.b * L + l0) * C;
  const uint64_t seed = ((uint64_t)r.seed_hi << 32) | r.seed_lo;
  auto& xo = x.uxo;
  auto& z = x.uz;
  if (!a.noise) {
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int w = min(ltid() + k * CH_NT, NWI - 1);
      const int c = w / (CH_MT / 4), l = l0 + (w % (CH_MT / 4)) * 4;
      philox_normal4(seed, r.clip_offset + (uint32_t)x.b, (uint32_t)r.i, TAG_STEP, (uint32_t)(c * L + l) >> 2, z[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int w = ltid() + k * CH_NT;
    if (w >= NWI) continue;
    const int c = w / (CH_MT / 4), q4 = (w % (CH_MT / 4)) * 4, l = l0 + q4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = q4 + i;
      const float ev = eps[rr * EPS_STR + c];
      const UpdOut o = upd_math(r, a.alg, xo[k][i], ev, false, 0.f, false, 0.f, 0.f, 0.f, z[k][i]);
      xg[rr * C + c] = o.xn;
      if (a.extras && x.it == a.k0 + a.n_steps - 1) {  // the last iteration's p_sample dict entries
        const size_t plane = (size_t)a.n * C * L, ncl = ((size_t)x.b * C + c) * L + l + i;
        a.extras[0 * plane + ncl] = o.mean;
        a.extras[1 * plane + ncl] = r.var;
        a.extras[2 * plane + ncl] = r.logvar;
        a.extras[3 * plane + ncl] = ev;
        a.extras[4 * plane + ncl] = o.x0;
        a.extras[5 * plane + ncl] = o.raw;
      }
      if (to_xs) x.xs[rr * XS_STR + c] = f2bf(o.xn);
    }
  }
  if (to_xs)  // emb_x's K padding: columns C .. 255 of the A rows are zero
    for (int e = ltid(); e < CH_MT * (CH_D - C); e += CH_NT) {
      const int rr = e / (CH_D - C), c = C + e % (CH_D - C);
      x.xs[rr * XS_STR + c] = 0;
    }
}

// MX (w8 = 2): the FFN and LayerNorm-projection stages run on block-scaled fp8 MFMA; their A images
// live in the xs / hh regions as e4m3 bytes, the e8m0 block scales behind the fp8 hidden rows
// (the attention output projections, out_layers and emb_x keep the bf16-widened route)
constexpr size_t LK_HSC = (size_t)CH_MT * HH8_STR;           // hh region: hidden block scales [32][32]
constexpr size_t LK_XSC = LK_HSC + (size_t)CH_MT * (CH_FF / 32);  //            LN block scales [32][8]
static_assert(LK_XSC + CH_MT * (CH_D / 32) <= sizeof(bf16_t) * CH_MT * HH_STR, "MX images fit the hh region");
static_assert(CH_MT * XS8_STR <= sizeof(bf16_t) * CH_MT * XS_STR, "fp8 A rows fit the xs region");
static_assert(LK_XSC >= sizeof(float) * CH_MT * EPS_STR, "eps rows (out_layers) stay clear of the LN scales");
// (the attention out-projections -- stage R, A = the hand-off rows quantised as they are staged -- on
// block-scaled fp8 MFMA too measured slower: 164 vs 158 ms per C4 launch, round 4)
// The FFN-up stage's epilogue on the MX route: ReLU^2 of the transposed accumulators into the
// block-scaled fp8 hidden image.  Lane (c16, g4) holds row 16 i + c16, columns 16 (nt0 + j) + 4 g4
// .. + 3; a 32-column block is the lane's two tiles x the 4 lane rows of its row (permlane swaps,
// lanerow_max4), one 4-byte store per (row, tile), the block's scale byte by the g4 = 0 lane.
// pp: the stage's LDS parameters [bias[NP] | scale[NP]]; hh8: [32][HH8_STR] e4m3 rows, their e8m0
// scales [32][CH_FF / 32] at LK_HSC.  Also run on its own by ggd_mx_ffn_up (the verification entry).
template <int NP>
__device__ __forceinline__ void lk_relu2_mx(const f32x4 (&acc)[2][2], const float* pp, int nt0, int c16, int g4,
                                            unsigned char* hh8) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = i * 16 + c16;
    float y[2][4], m = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = fmaxf(ch_val<true>(pp, NP, acc[i][j][r], (nt0 + j) * 16 + 4 * g4 + r), 0.f);
        y[j][r] = v * v;
        m = fmaxf(m, y[j][r]);
      }
    const unsigned sb = mx_scale_byte(lanerow_max4(m));
    const float mul = mx_mul(sb);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      *(unsigned*)(hh8 + row * HH8_STR + (nt0 + j) * 16 + 4 * g4) =
          mx_pack4(y[j][0] * mul, y[j][1] * mul, y[j][2] * mul, y[j][3] * mul);
    if (g4 == 0) hh8[LK_HSC + row * (CH_FF / 32) + nt0 / 2] = (unsigned char)sb;
  }
}

template <int KIND, int si, bool MX>
constexpr bool lk_mx() {
  constexpr int k = LkPlan<KIND>::s[si].kind;
  return MX && (k == SK_F1 || k == SK_F2 || k == SK_P || k == SK_P2);
}

template <bool W8, int KIND, int IT, bool MX, class X>
__device__ __forceinline__ void lk_iter(X& x) {
  using GE = LkGeo<W8, KIND>;
  using PL = LkPlan<KIND>;
  constexpr int TGB = GE::TGB, D1 = LK_DEPTH - 1;
  constexpr int si = GE::stage_of(IT), l = IT - GE::first(si), tg = GE::tg(si), nch = PL::s[si].nch;
  constexpr int kind = PL::s[si].kind;
  constexpr bool mx = lk_mx<KIND, si, MX>();
  static_assert(!MX || W8, "block-scaled fp8 needs e4m3 weights");
  unsigned char* const xs8 = (unsigned char*)x.xs;
  unsigned char* const hh8 = (unsigned char*)x.hh;
  if constexpr (IT + D1 < GE::TOTAL) lk_issue<W8, KIND, IT + D1>(x);
  if constexpr (kind == SK_PO && l == 0) lk_update_load(x);
  if constexpr (l == 0 && si > 0) {  // stage hand-offs (LDS); the prefetched weights stay in flight
    ch_bar();
    if constexpr (kind == SK_F1 || kind == SK_P || kind == SK_PO || kind == SK_P2) {
      if constexpr (mx)
        lk_layernorm_mx(x.hs, x.prm + GE::ln(si), x.prm + GE::ln(si) + CH_D, xs8, hh8 + LK_XSC, x.prm + GE::PRM_TOTAL);
      else
        lk_layernorm(x.hs, x.prm + GE::ln(si), x.prm + GE::ln(si) + CH_D, x.xs, x.prm + GE::PRM_TOTAL);
      ch_bar();
    } else if constexpr (kind == SK_E) {  // after out_layers: the update, its x rows feed emb_x
      lk_update(x, true);
      ch_bar();
    }
  }
  constexpr int c = l % nch;
  const int nt0 = ((l / nch) * CH_WAVES + x.wave) * tg;
  if constexpr (c == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < TGB; ++j) x.acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  [[maybe_unused]] float pev[2][TGB][4];
  if constexpr (kind == SK_E) {  // the PE rows of the epilogue, in flight across the MFMAs
    const int L = x.a.L, l0 = x.part * CH_MT;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < tg; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          pev[i][j][r] = x.a.pe[(size_t)((l0 + i * 16 + x.g4 + r) % L) * CH_D + (nt0 + j) * 16 + x.c16];
  }
  if constexpr (mx) {
    if constexpr (kind == SK_F2)
      ch_mma_mx<TGB>(x.bb[IT % LK_DEPTH], hh8, HH8_STR, hh8 + LK_HSC, CH_FF / 32, c, x.lane, x.acc, tg);
    else if constexpr (kind == SK_F1)  // transposed: the ReLU^2 epilogue quantises 4 columns of a row per lane
      ch_mma_mx<TGB, true>(x.bb[IT % LK_DEPTH], xs8, XS8_STR, hh8 + LK_XSC, CH_D / 32, c, x.lane, x.acc, tg);
    else
      ch_mma_mx<TGB>(x.bb[IT % LK_DEPTH], xs8, XS8_STR, hh8 + LK_XSC, CH_D / 32, c, x.lane, x.acc, tg);
  } else if constexpr (kind == SK_F2) {
    ch_mma<W8, TGB>(x.bb[IT % LK_DEPTH], x.hh, HH_STR, c, x.lane, x.acc, tg);
  } else {
    ch_mma<W8, TGB>(x.bb[IT % LK_DEPTH], x.xs, XS_STR, c, x.lane, x.acc, tg);
  }
  if constexpr (c == nch - 1 && mx && kind == SK_F1) {  // ReLU^2 hidden rows -> e4m3 + block scales
    static_assert(tg == 2 && TGB == 2, "a lane's two column tiles are one 32-column block");
    lk_relu2_mx<PL::s[si].ncols>(x.acc, x.prm + GE::prm(si), nt0, x.c16, x.g4 >> 2, hh8);  // x.g4 = 4 (lane >> 4)
  } else if constexpr (c == nch - 1) {
    constexpr int np = PL::s[si].ncols;
    const float* pp = x.prm + GE::prm(si);
    const int L = x.a.L, l0 = x.part * CH_MT;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < tg; ++j) {
        const int n = (nt0 + j) * 16 + x.c16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + x.g4 + r;
          const float v = ch_val<W8>(pp, np, x.acc[i][j][r], n);
          if constexpr (kind == SK_R || kind == SK_F2) {          // EPI_RESID
            float* p = x.hs + row * HS_STR + n;
            *p = *p + v;
          } else if constexpr (kind == SK_F1) {                   // EPI_RELU2
            const float y = fmaxf(v, 0.f);
            x.hh[row * HH_STR + n] = f2bf(y * y);
          } else if constexpr (kind == SK_E) {                    // EPI_PE: h = emb_x(x) + PE[frame]
            x.hs[row * HS_STR + n] = v + pev[i][j][r];
          } else if constexpr (kind == SK_PO) {                   // eps rows -> LDS (the update reads them)
            ((float*)x.hh)[row * EPS_STR + n] = v;
          } else {                                                 // EPI_T: hand-off rows
            ((bf16_t*)x.sa[si].out)[((size_t)x.b * L + l0 + row) * x.sa[si].ldo + n] = f2bf(v);
          }
        }
      }
  }
  if constexpr (IT + 1 < GE::TOTAL) lk_iter<W8, KIND, IT + 1, MX>(x);
}

// one chain phase of row block `part` of clip b
template <bool W8, int KIND, bool MX>
__device__ __forceinline__ void lk_chain(cla_T& a, cst_t sa, int b, int part, int it,
                                                   unsigned char* smem) {
  using GE = LkGeo<W8, KIND>;
  using PL = LkPlan<KIND>;
  const int tid = ltid(), lane = tid & 63;  // opaque: nothing thread-derived is hoisted across phases
  LkCtx<W8, GE::TGB> x{a, sa};
  x.hs = (float*)smem;
  x.xs = (bf16_t*)(smem + LK_HS);
  x.hh = x.xs + CH_MT * XS_STR;
  x.prm = (float*)(x.hh + CH_MT * HH_STR);
  x.wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  x.lane = lane;
  x.g4 = 4 * (lane >> 4);
  x.c16 = lane & 15;
  x.lane16 = (unsigned)lane * 16u;
  x.b = b;
  x.part = part;
  x.it = it;
  // Parameters (bias | scale per stage, LayerNorm vectors) and the first stage's A rows (the attention
  // output rows of the block, written by the head parts): every load is issued before the first LDS
  // store -- one memory round trip, not one per stage and pass (round 6: the prologue took 3.4 us of
  // chain B at 4 stages and 5.9 us at 6, profiles/r06aa_long_chain_stamps.txt) -- then the first
  // iteration's weights, which arrive while the rows are stored.
  constexpr int NPJ = 2;  // passes of CH_NT columns per stage (ncols <= 1024)
  float pv[PL::NS][2][NPJ], lv[PL::NS][2];
#pragma unroll
  for (int si = 0; si < PL::NS; ++si) {
    const float* wb = sa[si].w.b;
    const float* ws = sa[si].w.scale;
    const int np = PL::s[si].ncols;
#pragma unroll
    for (int j = 0; j < NPJ; ++j) {
      const int e = min(tid + j * CH_NT, np - 1);  // clamped: a thread past the stage loads a valid element
      pv[si][0][j] = wb[e];
      pv[si][1][j] = W8 ? ws[e] : 1.0f;
    }
    const float* lg = sa[si].ln_g;
    if (lg) {
      const int t = min(tid, CH_D - 1);
      lv[si][0] = lg[t];
      lv[si][1] = sa[si].ln_b[t];
    }
  }
  static_assert(PL::s[0].kind == SK_R, "every chain phase opens with the attention output projection");
  constexpr int NV = CH_MT * CH_D / 8 / CH_NT;
  uint4 v[NV];
  {
    const bf16_t* src = (const bf16_t*)a.att + ((size_t)b * a.L + part * CH_MT) * CH_D;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + i * CH_NT, r = e / (CH_D / 8), cv = e % (CH_D / 8);
      v[i] = ld_16B<CP_XL>(src, (uint32_t)((r * CH_D + 8 * cv) * 2));
    }
  }
  lk_issue<W8, KIND, 0>(x);
  if constexpr (LK_DEPTH > 2 && GE::TOTAL > 1) lk_issue<W8, KIND, 1>(x);
  if constexpr (LK_DEPTH > 3 && GE::TOTAL > 2) lk_issue<W8, KIND, 2>(x);
  static_assert(LK_DEPTH >= 2 && LK_DEPTH <= 4, "the prologue issues LK_DEPTH - 1 iterations");
  static_assert(NPJ * CH_NT >= CH_FF && CH_NT >= CH_D, "prologue passes");
#pragma unroll
  for (int si = 0; si < PL::NS; ++si) {
    const int np = PL::s[si].ncols;
#pragma unroll
    for (int j = 0; j < NPJ; ++j) {
      const int e = tid + j * CH_NT;
      if (e < np) {
        x.prm[GE::prm(si) + e] = pv[si][0][j];
        x.prm[GE::prm(si) + np + e] = pv[si][1][j];
      }
    }
    if (sa[si].ln_g && tid < CH_D) {
      x.prm[GE::ln(si) + tid] = lv[si][0];
      x.prm[GE::ln(si) + CH_D + tid] = lv[si][1];
    }
  }
  {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + i * CH_NT, r = e / (CH_D / 8), cv = e % (CH_D / 8);
      if constexpr (lk_mx<KIND, 0, MX>()) {  // e4m3 rows + the block scales: a block is 4 lanes' pieces
        // max |v| on the bf16 bits (non-negative bf16 order as integers: v_pk_max_u16), then two
        // values at a time into e4m3 (few live registers beside the weight groups in flight)
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        const unsigned w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        u16x2 mm = {0, 0};
#pragma unroll
        for (int q = 0; q < 4; ++q) mm = __builtin_elementwise_max(mm, __builtin_bit_cast(u16x2, w[q] & 0x7fff7fffu));
        const unsigned mb = (unsigned)max(mm.x, mm.y) << 16;
        const unsigned sb = mx_scale_byte(group_max<4>(__uint_as_float(mb)));
        const float mul = mx_mul(sb);
        auto lo = [&](int q) { return __uint_as_float(w[q] << 16) * mul; };
        auto hi = [&](int q) { return __uint_as_float(w[q] & 0xffff0000u) * mul; };
        int o0 = __builtin_amdgcn_cvt_pk_fp8_f32(lo(0), hi(0), 0, false);
        o0 = __builtin_amdgcn_cvt_pk_fp8_f32(lo(1), hi(1), o0, true);
        int o1 = __builtin_amdgcn_cvt_pk_fp8_f32(lo(2), hi(2), 0, false);
        o1 = __builtin_amdgcn_cvt_pk_fp8_f32(lo(3), hi(3), o1, true);
        unsigned char* xs8 = (unsigned char*)x.xs;
        *(uint2*)(xs8 + r * XS8_STR + 8 * cv) = make_uint2((unsigned)o0, (unsigned)o1);
        if ((cv & 3) == 0) ((unsigned char*)x.hh)[LK_XSC + r * (CH_D / 32) + cv / 4] = (unsigned char)sb;
      } else {
        *(uint4*)(x.xs + r * XS_STR + 8 * cv) = v[i];
      }
    }
  }
  ch_bar();
  lk_iter<W8, KIND, 0, MX>(x);
  if constexpr (KIND == K_BLL) {  // the last step: update only
    ch_bar();
    lk_update(x, false);
  }
}

// ------------------------------------------------------------------------------------------
// attention phase: head `head` of clip b over all its frames (ggd_attn.hip with 8 waves; the
// Q / K / V rows another workgroup wrote are read past L1)
// ------------------------------------------------------------------------------------------
constexpr int LA_SQ = 40;                    // Q / K operand row stride (bf16, 16-byte pad)

// Raw conv inputs: NM bf16 hand-off images of `rows` rows x 32 channels into LDS [NM][rows + 2][32]
// (rows 0 and rows + 1 are the conv's zero padding), each 16-byte unit loaded once (no halo
// re-reads); load() issues them, store() writes them after the phase's other loads are issued
// (lk_attn).  src[m] = base + col[m] (row stride ld).
constexpr int LA_RAW_UNITS = (3 * ATT_LMAX * 4 + CH_NT - 1) / CH_NT;  // units per thread (max)
// raw row stride (bf16): 32 channels + 8 pad, so that the 16 lanes (4 runs of 4 rows x 4 channel
// groups) of one LDS pass of la_conv_runs hit 16 distinct 16-byte bank slots
constexpr int LA_RS = 40;
template <int NM> struct LaRaw {
  uint4 v[LA_RAW_UNITS];
  __device__ __forceinline__ void load(const void* base, size_t row0, int ld, const int (&col)[3], int rows) {
    const int tid = ltid(), per = rows * 4, total = NM * per;
#pragma unroll
    for (int i = 0; i < LA_RAW_UNITS; ++i) {
      const int u = min(tid + i * CH_NT, total - 1), m = u / per, r = (u % per) / 4, cv = u % 4;
      v[i] = ld_16B<CP_XL>(base, (uint32_t)(((row0 + r) * (size_t)ld + col[m] + cv * 8) * 2));
    }
  }
  __device__ __forceinline__ void store(int rows, bf16_t* raw) const {
    const int tid = ltid(), per = rows * 4, total = NM * per;
#pragma unroll
    for (int i = 0; i < LA_RAW_UNITS; ++i) {
      const int u = tid + i * CH_NT;
      if (u >= total) continue;
      const int m = u / per, r = (u % per) / 4, cv = u % 4;
      *(uint4*)(raw + ((size_t)m * (rows + 2) + r + 1) * LA_RS + cv * 8) = v[i];
    }
    for (int u = tid; u < NM * 2 * 4; u += CH_NT) {  // halo rows
      const int m = u / 8, h = (u / 4) % 2, cv = u % 4;
      *(uint4*)(raw + ((size_t)m * (rows + 2) + h * (rows + 1)) * LA_RS + cv * 8) = make_uint4(0, 0, 0, 0);
    }
  }
};

// The NM convs of an attention phase (raw image m -> operand image m: out[i] = b + w0 in[i-1] + w1 in[i]
// + w2 in[i+1], LaStrip::conv's expression; matrix 2 of 3 written as V^T): thread (matrix m, run of 4
// rows, 8-channel group cv) reads the 6 raw rows its 4 outputs need and its 32 taps once, and writes
// a row's 8 channels as one 16-byte store (a V^T channel's 4 rows as one 8-byte store).  16
// consecutive lanes are 4 runs x 4 channel groups: with the 80-byte raw rows (LA_RS) each LDS pass
// touches 16 distinct bank slots.  Round 6: one element per (row, channel group) re-read the taps for
// every row and took 2.0 us per self-attention phase (profiles/r06ae_c4_barrier_prefetch_ab.txt).
// rows % 4 == 0 (whole row blocks).  wl = [m][w0 | w1 | w2 | b][32]
template <int NM>
__device__ __forceinline__ void la_conv_runs(const bf16_t* raw, int rows, const float* wl, bf16_t* const (&dst)[3],
                                             const int (&S)[3]) {
  for (int u = ltid(); u < NM * rows; u += CH_NT) {
    const int m = u / rows, r = u % rows, cv = r % 4, i0 = (r / 4) * 4;
    const float* w = wl + m * 128 + cv * 8;
    const float4 w0a = *(const float4*)(w), w0b = *(const float4*)(w + 4);
    const float4 w1a = *(const float4*)(w + 32), w1b = *(const float4*)(w + 36);
    const float4 w2a = *(const float4*)(w + 64), w2b = *(const float4*)(w + 68);
    const float4 bba = *(const float4*)(w + 96), bbb = *(const float4*)(w + 100);
    const float w0[8] = {w0a.x, w0a.y, w0a.z, w0a.w, w0b.x, w0b.y, w0b.z, w0b.w};
    const float w1[8] = {w1a.x, w1a.y, w1a.z, w1a.w, w1b.x, w1b.y, w1b.z, w1b.w};
    const float w2[8] = {w2a.x, w2a.y, w2a.z, w2a.w, w2b.x, w2b.y, w2b.z, w2b.w};
    const float bb[8] = {bba.x, bba.y, bba.z, bba.w, bbb.x, bbb.y, bbb.z, bbb.w};
    const bf16_t* src = raw + ((size_t)m * (rows + 2) + i0) * LA_RS + cv * 8;
    float x[6][8];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const uint4 q = *(const uint4*)(src + (size_t)k * LA_RS);
      const unsigned e4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[k][2 * e] = __uint_as_float(e4[e] << 16);
        x[k][2 * e + 1] = __uint_as_float(e4[e] & 0xffff0000u);
      }
    }
    float y[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) y[q][e] = bb[e] + w0[e] * x[q][e] + w1[e] * x[q + 1][e] + w2[e] * x[q + 2][e];
    bf16_t* out = dst[m];
    if (NM == 3 && m == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        *(uint2*)(out + (size_t)(cv * 8 + e) * S[2] + i0) = make_uint2(pk_bf16(y[0][e], y[1][e]), pk_bf16(y[2][e], y[3][e]));
    } else {
      const int so = m == 0 ? S[0] : S[1];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *(uint4*)(out + (size_t)(i0 + q) * so + cv * 8) = make_uint4(pk_bf16(y[q][0], y[q][1]), pk_bf16(y[q][2], y[q][3]),
                                                                    pk_bf16(y[q][4], y[q][5]), pk_bf16(y[q][6], y[q][7]));
    }
  }
}

// the query tiles of one wave, LKT (16-key tiles, Lk padded to 32) fixed at compile time: every
// LDS fragment of a matrix product is read before its MFMAs (no per-tile branch between them)
template <int LKT>
__device__ __forceinline__ void lk_attn_tiles(const bf16_t* Qm, const bf16_t* Km, const bf16_t* Vt, bf16_t* P, int SV,
                                              int SP, int Lq, int Lk, float sl2, bf16_t* out, int wave, int lane) {
  clip_attn_tiles<LKT, CH_WAVES, LA_SQ>(Qm, Km, Vt, P, SV, SP, Lq, Lk, sl2, out, CH_D, wave, lane);
}

// An attention phase's loads that need nothing from the phase before it, issued by lk_sync's
// prefetch hook (round 6): the conv taps and biases [m][w0 | w1 | w2 | b][32] (threads < 384), and for
// the cross-attention the layer's cached convolved memory keys 2 .. (K rows, V^T rows: step-invariant,
// ggd_set_memory) and the inputs of the step-dependent keys 0, 1 (thread t < 64: K[t / 32][t % 32],
// thread 64 + c: the V^T pair of channel c)
constexpr int LA_KU = (ATT_LMAX * 4 + CH_NT - 1) / CH_NT;      // K units (rows 2 .. Lk_pad - 1) per thread
constexpr int LA_VU = (32 * ATT_LMAX / 8 + CH_NT - 1) / CH_NT;  // V^T units per thread
template <bool CROSS> struct LaPre {
  float wv;
  uint4 kv[CROSS ? LA_KU : 1], vv[CROSS ? LA_VU : 1];
  float x0, x1, x2, w0, w1, w2, wb0;
  __device__ __forceinline__ void load(cla_T& a, cll_t lyp, int b, int head, int t_orig) {
    const __attribute__((address_space(4))) LongLayer& Ly = *lyp;
    const int tid = ltid();
    static_assert(12 * 32 <= CH_NT, "one tap per thread");
    wv = 0.f;
    if (tid < 12 * 32) {
      const int m = tid / 128, k = (tid / 32) % 4, c = tid % 32;
      const float* w = CROSS ? (m == 0 ? Ly.ca_qw : m == 1 ? Ly.ca_kw : Ly.ca_vw) : (m == 0 ? Ly.sa_qw : m == 1 ? Ly.sa_kw : Ly.sa_vw);
      const float* bb = CROSS ? (m == 0 ? Ly.ca_qb : m == 1 ? Ly.ca_kb : Ly.ca_vb) : (m == 0 ? Ly.sa_qb : m == 1 ? Ly.sa_kb : Ly.sa_vb);
      wv = k < 3 ? w[c * 3 + k] : bb[c];
    }
    if constexpr (CROSS) {
      const int Lk = 1 + a.Ts, Lkp = (Lk + 31) / 32 * 32, kpr = Lkp / 8;
      const bf16_t* kc = Ly.kvc + ((size_t)b * CH_WAVES + head) * 2 * Lkp * 32;
      const bf16_t* vc = kc + Lkp * 32;
#pragma unroll
      for (int i = 0; i < LA_KU; ++i) {
        const int u = min(tid + i * CH_NT, (Lkp - 2) * 4 - 1), r = 2 + u / 4, cv = u % 4;
        kv[i] = *(const uint4*)(kc + r * 32 + cv * 8);
      }
#pragma unroll
      for (int i = 0; i < LA_VU; ++i) {
        const int u = min(tid + i * CH_NT, 32 * kpr - 1), c = u / kpr, kb = u % kpr;
        vv[i] = *(const uint4*)(vc + c * Lkp + kb * 8);
      }
      const float* r0 = Ly.kv_step + (size_t)t_orig * 2 * CH_D;
      const float* m0 = Ly.kv_mem + (size_t)b * (Lk - 1) * 2 * CH_D;
      x0 = x1 = x2 = w0 = w1 = w2 = wb0 = 0.f;
      if (tid < 96) {
        const bool isv = tid >= 64;
        const int c = isv ? tid - 64 : tid % 32, col = (isv ? CH_D : 0) + head * 32 + c;
        x0 = r0[col];
        x1 = m0[col];
        x2 = Lk > 2 ? m0[2 * CH_D + col] : 0.f;
        const float* w = isv ? Ly.ca_vw : Ly.ca_kw;
        w0 = w[c * 3];
        w1 = w[c * 3 + 1];
        w2 = w[c * 3 + 2];
        wb0 = isv ? Ly.ca_vb[c] : Ly.ca_kb[c];
      }
    }
  }
};

template <bool CROSS>
__device__ __forceinline__ void lk_attn(cla_T& a, cll_t lyp, int b, int head, const LaPre<CROSS>* pre,
                                                  unsigned char* scratch, unsigned long long* sub = nullptr) {
  // sub (diagnostics): realtime stamps after staging, after the convs, after the query tiles
  const __attribute__((address_space(4))) LongLayer& Ly = *lyp;
  const int Lq = a.L, Lk = CROSS ? 1 + a.Ts : a.L, tid = ltid(), lane = tid & 63, wave = tid >> 6;
  const int Lkp = (Lk + 31) / 32 * 32, SV = Lkp + 8, SP = Lkp + 8, Lqp = (Lq + 15) / 16 * 16;
  bf16_t* Qm = (bf16_t*)scratch;
  bf16_t* Km = Qm + Lqp * LA_SQ;
  bf16_t* Vt = Km + Lkp * LA_SQ;
  bf16_t* Pall = Vt + 32 * SV;
  float* wl = (float*)(Pall + CH_WAVES * 16 * SP);
  bf16_t* raw = Pall;  // the raw conv inputs share the P tiles' region (dead until the tiles)
  const size_t row0 = (size_t)b * Lq;
  // Staging: every global load of the phase is issued before the first LDS store (one memory round
  // trip; round 6 -- the separate load / store passes cost 2.3 us self, 2.7 us cross before the convs).
  // The cross-attention's taps, cached keys and memory rows are in flight since the barrier (pre).
  float wv = 0.f;
  if constexpr (CROSS) {
    wv = pre->wv;
  } else if (tid < 12 * 32) {  // conv taps and biases [m][w0 | w1 | w2 | b][32]
    const int m = tid / 128, k = (tid / 32) % 4, c = tid % 32;
    const float* w = m == 0 ? Ly.sa_qw : m == 1 ? Ly.sa_kw : Ly.sa_vw;
    const float* bb = m == 0 ? Ly.sa_qb : m == 1 ? Ly.sa_kb : Ly.sa_vb;
    wv = k < 3 ? w[c * 3 + k] : bb[c];
  }
  float k0 = 0.f, k1 = 0.f;  // CROSS: the step-dependent keys 0, 1 of thread t < 96's K / V channel
  if constexpr (CROSS) {
    // keys >= 2 from the step-invariant convolved cache (ggd_set_memory); keys 0 and 1 depend on the
    // step token (memory row 0) and are convolved here, in the cache kernel's expression
    const int colq[3] = {head * 32, 0, 0};
    LaRaw<1> rq;
    rq.load(a.q, row0, CH_D, colq, Lq);
    const int kpr = Lkp / 8;  // 16-byte units per V^T row
    rq.store(Lq, raw);
#pragma unroll
    for (int i = 0; i < LA_KU; ++i) {
      const int u = tid + i * CH_NT;
      if (u >= (Lkp - 2) * 4) continue;
      const int r = 2 + u / 4, cv = u % 4;
      *(uint4*)(Km + r * LA_SQ + cv * 8) = pre->kv[i];
    }
    k0 = pre->wb0 + pre->w0 * 0.f + pre->w1 * pre->x0 + pre->w2 * pre->x1;  // key 0 (LaStrip::conv's expression)
    k1 = pre->wb0 + pre->w0 * pre->x0 + pre->w1 * pre->x1 + pre->w2 * pre->x2;  // key 1
#pragma unroll
    for (int i = 0; i < LA_VU; ++i) {
      const int u = tid + i * CH_NT;
      if (u >= 32 * kpr) continue;
      const int c = u / kpr, kb = u % kpr;
      *(uint4*)(Vt + c * SV + kb * 8) = pre->vv[i];
    }
    if (tid < 64) Km[(tid / 32) * LA_SQ + tid % 32] = f2bf(tid < 32 ? k0 : k1);  // (V^T's pair: after the barrier)
  } else {
    const int cols[3] = {head * 32, CH_D + head * 32, 2 * CH_D + head * 32};
    LaRaw<3> rr;
    rr.load(a.qkv, row0, 3 * CH_D, cols, Lq);  // self: Lk = Lq
    rr.store(Lq, raw);
  }
  if (tid < 12 * 32) wl[tid] = wv;
  if constexpr (!CROSS) {
    for (int i = tid; i < (Lkp - Lk) * 32; i += CH_NT) {
      const int r = Lk + i / 32, c = i % 32;
      Km[r * LA_SQ + c] = 0;
      Vt[c * SV + r] = 0;
    }
  }
  bar_lds();
  if (sub && tid == 0) sub[0] = __builtin_amdgcn_s_memrealtime();
  // V^T keys 0, 1 of channel tid - 64, over the cached row's first pair, once that copy (another
  // thread's) has landed; the tiles read them after the conv barrier below
  if (CROSS && tid >= 64 && tid < 96) *(unsigned*)(Vt + (tid - 64) * SV) = pk_bf16(k0, k1);
  {
    bf16_t* const cd[3] = {Qm, Km, Vt};
    const int cs[3] = {LA_SQ, LA_SQ, SV};
    la_conv_runs<CROSS ? 1 : 3>(raw, Lq, wl, cd, cs);  // self: Lk = Lq
  }
  bar_lds();
  if (sub && tid == 0) sub[1] = __builtin_amdgcn_s_memrealtime();
  bf16_t* P = Pall + wave * 16 * SP;
  bf16_t* out = (bf16_t*)a.att + row0 * CH_D + (size_t)head * 32;
  const float sl2 = a.scale * 1.4426950408889634f;  // softmax on exp2: e^(s - m) = 2^((s - m) log2 e)
  switch (Lkp / 16) {  // long_loop_supported: 96 <= Lk_pad <= 192
    case 6: lk_attn_tiles<6>(Qm, Km, Vt, P, SV, SP, Lq, Lk, sl2, out, wave, lane); break;
    case 8: lk_attn_tiles<8>(Qm, Km, Vt, P, SV, SP, Lq, Lk, sl2, out, wave, lane); break;
    case 10: lk_attn_tiles<10>(Qm, Km, Vt, P, SV, SP, Lq, Lk, sl2, out, wave, lane); break;
    default: lk_attn_tiles<12>(Qm, Km, Vt, P, SV, SP, Lq, Lk, sl2, out, wave, lane); break;
  }
  if (sub && tid == 0) sub[2] = __builtin_amdgcn_s_memrealtime();  // wave 0's tiles done
}

// convolved memory keys 2 .. Lk - 1 of one layer (the expression of LaStrip::conv); one workgroup
// per (head, clip): K [Lk_pad][32] then V^T [32][Lk_pad], bf16, other keys zero
__global__ void lk_kv_cache_kernel(const float* __restrict__ kv_mem, const float* __restrict__ kw,
                                   const float* __restrict__ kb, const float* __restrict__ vw,
                                   const float* __restrict__ vb, int Ts, int Lkp, bf16_t* __restrict__ out) {
  const int h = blockIdx.x, b = blockIdx.y, heads = gridDim.x, Lk = 1 + Ts;
  bf16_t* kc = out + ((size_t)b * heads + h) * 2 * Lkp * 32;
  bf16_t* vc = kc + Lkp * 32;
  const float* m0 = kv_mem + (size_t)b * Ts * 2 * CH_D;
  for (int e = threadIdx.x; e < 2 * Lkp * 32; e += blockDim.x) {
    const bool isv = e >= Lkp * 32;
    const int i = isv ? e - Lkp * 32 : e;
    const int j = isv ? i % Lkp : i / 32, c = isv ? i / Lkp : i % 32;  // key, channel
    float v = 0.f;
    if (j >= 2 && j < Lk) {
      const int col = (isv ? CH_D : 0) + h * 32 + c;
      const float* w = isv ? vw : kw;
      const float bb = isv ? vb[c] : kb[c];
      const float x0 = m0[(size_t)(j - 2) * 2 * CH_D + col], x1 = m0[(size_t)(j - 1) * 2 * CH_D + col];
      const float x2 = j + 1 < Lk ? m0[(size_t)j * 2 * CH_D + col] : 0.f;
      v = bb + w[c * 3] * x0 + w[c * 3 + 1] * x1 + w[c * 3 + 2] * x2;
    }
    (isv ? vc : kc)[i] = j >= 2 && j < Lk ? f2bf(v) : (bf16_t)0;
  }
}

// One attention phase (Lk keys, nm raw conv inputs: 3 self, 1 cross): Q | K | V^T | P tiles (the raw
// inputs, nm x (L + 2) rows of LA_RS, in the P region: lk_attn places them there) | taps
size_t lk_attn_lds(int L, int Lk, int nm) {
  const int Lkp = (Lk + 31) / 32 * 32, Lqp = (L + 15) / 16 * 16;
  const size_t p = std::max((size_t)CH_WAVES * 16 * (Lkp + 8), (size_t)nm * (L + 2) * LA_RS);
  return 2 * ((size_t)Lqp * LA_SQ + (size_t)Lkp * LA_SQ + 32 * (size_t)(Lkp + 8) + p) + sizeof(float) * 12 * 32;
}
// the raw conv inputs fit the P region (lk_attn's layout)
static bool lk_raw_fits(int L, int Lk, int nm) {
  const int Lkp = (Lk + 31) / 32 * 32;
  return (size_t)nm * (L + 2) * LA_RS <= (size_t)CH_WAVES * 16 * (Lkp + 8);
}

// ------------------------------------------------------------------------------------------
// the persistent loop
// ------------------------------------------------------------------------------------------
template <bool W8, bool MX>
__global__ void __launch_bounds__(CH_NT) lk_kernel(LongArgs args, int G) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int s_role, s_ok;
  cla_T& a = *(const __attribute__((address_space(4))) LongArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  if (threadIdx.x == 0) s_role = lk_role(a.ctl, a.status, gridDim.x, G);
  __syncthreads();
  const int role = s_role;
  if (role < 0) return;
  const int grp = role >> 3, part = role & 7, b = a.clip0 + grp, NB = a.L / CH_MT, NL = a.n_layers;
  unsigned* flags = a.ctl + LK_FLAGS + grp * 32;
  unsigned epoch = 0;
  unsigned long long* stamps = role == 0 ? a.stamps : nullptr;
  if (stamps && threadIdx.x == 0) stamps[0] = __builtin_amdgcn_s_memrealtime();
  auto stamp = [&]() {
    if (stamps && threadIdx.x == 0 && epoch < LONG_STAMPS) stamps[epoch] = __builtin_amdgcn_s_memrealtime();
  };
  const cll_t lay = (cll_t)a.layers;
  const cst_t st = (cst_t)a.stages;
  const bool rows = part < NB;
  if (rows) {  // the block's residual rows (h = emb_x(x_T) + PE; its LN1 + QKV rows are in qkv)
    float* hs = (float*)smem;
    const float* hg = a.h + ((size_t)b * a.L + part * CH_MT) * CH_D;
    for (int e = ltid(); e < CH_MT * CH_D / 4; e += CH_NT) {
      const int r = e / (CH_D / 4), c4 = e % (CH_D / 4);
      *(float4*)(hs + r * HS_STR + 4 * c4) = *(const float4*)(hg + r * CH_D + 4 * c4);
    }
  }
  __syncthreads();
  for (int k = 0; k < a.n_steps; ++k) {
    const int it = a.k0 + k;
    const int t_orig = a.steps[it].t_orig;
    for (int li = 0; li < NL; ++li) {
      const cst_t sl = st + 2 + LONG_STAGES_PER_LAYER * li;
      lk_attn<false>(a, lay + li, b, part, nullptr, smem + LK_HS, stamps && k == 1 && li == 0 ? stamps + 56 : nullptr);
      if (!lk_sync(flags, part, ++epoch, a.status, &s_ok)) return;
      stamp();
      if (rows) lk_chain<W8, K_A, MX>(a, sl, b, part, it, smem);         // R(o_sa) + P(LN2, q_ca)
      {  // (the cross-attention's step-invariant keys and taps: loaded at the barrier)
        LaPre<true> pc;
        if (!lk_sync(flags, part, ++epoch, a.status, &s_ok, [&] { pc.load(a, lay + li, b, part, t_orig); })) return;
        stamp();
        lk_attn<true>(a, lay + li, b, part, &pc, smem + LK_HS, stamps && k == 1 && li == 0 ? stamps + 60 : nullptr);
      }
      if (!lk_sync(flags, part, ++epoch, a.status, &s_ok)) return;
      stamp();
      if (rows) {
        if (li + 1 < NL)
          lk_chain<W8, K_B, MX>(a, sl + 2, b, part, it, smem);             // R(o_ca) + F + P(next LN1, QKV)
        else if (k + 1 < a.n_steps)
          lk_chain<W8, K_BL, MX>(a, sl + 2, b, part, it, smem);            // ... + out_layers, update, emb_x, LN1 + QKV
        else
          lk_chain<W8, K_BLL, MX>(a, sl + 2, b, part, it, smem);           // ... + out_layers, update
      }
      if (k + 1 < a.n_steps || li + 1 < NL)
        if (!lk_sync(flags, part, ++epoch, a.status, &s_ok)) return;
      stamp();
    }
  }
}

template <bool W8>
size_t lk_lds(int L, int Lk) {
  size_t m = LkGeo<W8, K_BL>::LDS;
  m = std::max(m, LkGeo<W8, K_B>::LDS);
  m = std::max(m, LK_HS + lk_attn_lds(L, L, 3));  // self-attention
  return std::max(m, LK_HS + lk_attn_lds(L, Lk, 1));  // cross-attention
}

// Verification kernel (ggd_mx_layernorm): lk_layernorm_mx -- the long loop's LayerNorm into the
// block-scaled fp8 A image of its MX stages (LN2 / LN3 / LN1 before the Q, FFN-up and QKV
// projections) -- on one 32-row block given as f32 rows, the fp8 rows and e8m0 scale bytes copied out
// as the stage's MFMAs read them.  One workgroup of the loop's shape (8 waves).
__global__ void __launch_bounds__(CH_NT) lk_ln_mx_probe_kernel(const float* __restrict__ rows, const float* __restrict__ gm,
                                                            const float* __restrict__ bt, unsigned char* __restrict__ codes,
                                                            unsigned char* __restrict__ scales) {
  __shared__ __attribute__((aligned(16))) float hs[CH_MT * HS_STR];
  __shared__ __attribute__((aligned(16))) unsigned char xs8[CH_MT * XS8_STR];
  __shared__ unsigned char sc[CH_MT * (CH_D / 32)];
  __shared__ float st[2 * CH_MT];
  __shared__ __attribute__((aligned(16))) float prm[2 * CH_D];
  for (int e = threadIdx.x; e < CH_MT * CH_D; e += CH_NT) hs[(e / CH_D) * HS_STR + e % CH_D] = rows[e];
  for (int e = threadIdx.x; e < CH_D; e += CH_NT) {
    prm[e] = gm[e];
    prm[CH_D + e] = bt[e];
  }
  __syncthreads();
  lk_layernorm_mx(hs, prm, prm + CH_D, xs8, sc, st);
  __syncthreads();
  for (int e = threadIdx.x; e < CH_MT * CH_D; e += CH_NT) codes[e] = xs8[(e / CH_D) * XS8_STR + e % CH_D];
  for (int e = threadIdx.x; e < CH_MT * (CH_D / 32); e += CH_NT) scales[e] = sc[e];
}

// Verification kernel (ggd_mx_ffn_up): the long loop's FFN-up stage on the MX route -- the
// transposed block-scaled MFMA (ch_mma_mx<2, true>) over one 32-row block of an e4m3 A image with
// its e8m0 scales, then lk_relu2_mx -- with the loop's wave -> column-tile map (iteration l: tiles
// 16 l + 2 wave, + 1) and weight fragment addressing (lk_issue).  The hidden codes and scale bytes
// are copied out as the FFN-down stage reads them.  One workgroup of the loop's shape (8 waves).
__global__ void __launch_bounds__(CH_NT) lk_ffn_up_mx_probe_kernel(const unsigned char* __restrict__ a_codes,
                                                                const unsigned char* __restrict__ a_scales,
                                                                const unsigned char* __restrict__ wpk,
                                                                const float* __restrict__ wscale,
                                                                const float* __restrict__ bias,
                                                                unsigned char* __restrict__ h_codes,
                                                                unsigned char* __restrict__ h_scales) {
  __shared__ __attribute__((aligned(16))) unsigned char xs8[CH_MT * XS8_STR];
  __shared__ unsigned char sc[CH_MT * (CH_D / 32)];
  __shared__ __attribute__((aligned(16))) unsigned char hh8[LK_HSC + CH_MT * (CH_FF / 32)];
  __shared__ __attribute__((aligned(16))) float prm[2 * CH_FF];
  for (int e = threadIdx.x; e < CH_MT * CH_D; e += CH_NT) xs8[(e / CH_D) * XS8_STR + e % CH_D] = a_codes[e];
  for (int e = threadIdx.x; e < CH_MT * (CH_D / 32); e += CH_NT) sc[e] = a_scales[e];
  for (int e = threadIdx.x; e < CH_FF; e += CH_NT) {
    prm[e] = bias[e];
    prm[CH_FF + e] = wscale[e];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int TG = 2, UPT = Units<true>::U;  // one 256-k chunk: 4 units per tile
  const unsigned char* wb = wpk + (size_t)wave * TG * UPT * 1024;
  for (int l = 0; l < CH_FF / (16 * CH_WAVES * TG); ++l) {
    BBuf<true, TG> B;
    ch_load<true, TG>(B, wb, (unsigned)lane * 16, l * CH_WAVES * TG, 0, UPT, TG);
    f32x4 acc[2][TG];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < TG; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    ch_mma_mx<TG, true>(B, xs8, XS8_STR, sc, CH_D / 32, 0, lane, acc, TG);
    lk_relu2_mx<CH_FF>(acc, prm, (l * CH_WAVES + wave) * TG, lane & 15, lane >> 4, hh8);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < CH_MT * CH_FF; e += CH_NT) h_codes[e] = hh8[(e / CH_FF) * HH8_STR + e % CH_FF];
  for (int e = threadIdx.x; e < CH_MT * (CH_FF / 32); e += CH_NT) h_scales[e] = hh8[LK_HSC + e];
}

}  // namespace

bool long_loop_supported(int dtype, int d_model, int heads, int L, int Ts, int C, int out_npad) {
  const size_t lds = std::max(lk_lds<true>(L, 1 + Ts), lk_lds<false>(L, 1 + Ts));
  const int lkp = (1 + Ts + 31) / 32 * 32;  // memory keys, padded (whole-clip tiles: 96 .. 192)
  return dtype != 0 && d_model == CH_D && heads == 8 && L % CH_MT == 0 && L / CH_MT <= 8 && L >= 96 &&
         lk_raw_fits(L, L, 3) && lk_raw_fits(L, 1 + Ts, 1) &&
         L <= ATT_LMAX && lkp >= 96 && lkp <= ATT_LMAX && C <= 128 && out_npad == 128 && lds <= 160 * 1024 - 256;
}

size_t long_kv_cache_bytes(int n, int Ts, int heads) {
  const int Lkp = (1 + Ts + 31) / 32 * 32;
  return (size_t)n * heads * 2 * Lkp * 32 * sizeof(bf16_t);
}

hipError_t launch_long_kv_cache(const float* kv_mem, const float* kw, const float* kb, const float* vw, const float* vb,
                                int n, int Ts, int heads, bf16_t* out, hipStream_t s) {
  if (n <= 0 || heads != CH_WAVES) return hipErrorInvalidValue;
  hipLaunchKernelGGL(lk_kv_cache_kernel, dim3(heads, n), dim3(256), 0, s, kv_mem, kw, kb, vw, vb, Ts,
                     (1 + Ts + 31) / 32 * 32, out);
  return hipGetLastError();
}

int long_loop_capacity() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipGetLastError();
  return std::min(32, cus / 8);
}

hipError_t launch_long_loop(int w8, const LongArgs& a, int G, hipStream_t s) {
  if (G < 1 || G > long_loop_capacity() || 64 * ((G + 7) / 8) > 8 * long_loop_capacity()) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(a.ctl, 0, sizeof(unsigned) * LONG_CTL_WORDS, s);
  if (e != hipSuccess) return e;
  const size_t lds = w8 ? lk_lds<true>(a.L, 1 + a.Ts) : lk_lds<false>(a.L, 1 + a.Ts);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)lk_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 256);
    (void)hipFuncSetAttribute((const void*)lk_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 256);
    (void)hipFuncSetAttribute((const void*)lk_kernel<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 256);
    (void)hipGetLastError();
    attr = true;
  }
  const int nwg = 64 * ((G + 7) / 8);
  if (w8 == 2) hipLaunchKernelGGL((lk_kernel<true, true>), dim3(nwg), dim3(CH_NT), lds, s, a, G);
  else if (w8) hipLaunchKernelGGL((lk_kernel<true, false>), dim3(nwg), dim3(CH_NT), lds, s, a, G);
  else hipLaunchKernelGGL((lk_kernel<false, false>), dim3(nwg), dim3(CH_NT), lds, s, a, G);
  return hipGetLastError();
}

}  // namespace ggd

extern "C" int ggd_mx_layernorm(const float* rows, const float* gamma, const float* beta, uint8_t* codes, uint8_t* scales,
                                void* stream) {
  if (!rows || !gamma || !beta || !codes || !scales) return -1;  // GGD_ERR_ARG
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(ggd::lk_ln_mx_probe_kernel, dim3(1), dim3(ggd::chainlib::CH_NT), 0, s, rows, gamma, beta, codes, scales);
  hipError_t e = hipGetLastError();
  const hipError_t e2 = hipStreamSynchronize(s);
  return e == hipSuccess && e2 == hipSuccess ? 0 : -3;
}

extern "C" int ggd_mx_ffn_up(const uint8_t* a_codes, const uint8_t* a_scales, const uint8_t* w_e4m3, const float* wscale,
                             const float* bias, uint8_t* h_codes, uint8_t* h_scales, void* stream) {
  using namespace ggd;
  using namespace ggd::chainlib;
  if (!a_codes || !a_scales || !w_e4m3 || !wscale || !bias || !h_codes || !h_scales) return -1;  // GGD_ERR_ARG
  hipStream_t s = (hipStream_t)stream;
  void* pk = nullptr;
  if (hipMalloc(&pk, (size_t)CH_FF * CH_D) != hipSuccess) return -3;
  hipError_t e = launch_chain_pack(2, w_e4m3, pk, CH_FF, CH_D, s);  // the MX B order, as the context packs wmx
  if (e == hipSuccess) {
    hipLaunchKernelGGL(lk_ffn_up_mx_probe_kernel, dim3(1), dim3(CH_NT), 0, s, a_codes, a_scales,
                       (const unsigned char*)pk, wscale, bias, h_codes, h_scales);
    e = hipGetLastError();
  }
  const hipError_t e2 = hipStreamSynchronize(s);
  (void)hipFree(pk);
  return e == hipSuccess && e2 == hipSuccess ? 0 : -3;
}
