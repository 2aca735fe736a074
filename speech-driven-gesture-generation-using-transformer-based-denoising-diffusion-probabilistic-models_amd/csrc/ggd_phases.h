// ggd_phases.h -- the five phases of one denoise step of the one-way decoder, per clip group
// (8 workgroups of 512 threads per clip).  Instantiated twice: as one launch per phase
// (ggd_fused.hip, CP_KERNEL) and inside the persistent step loop (ggd_mega.hip, CP_COH).
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
#pragma once
#include "ggd_fusedlib.h"

// KE rows phase (round 4, both measured on one box, profiles/r04m_c2_ab.txt): the last layer's
// FFN-down reduction runs inside KE for each block's rows (one clip-group barrier and the KD phase
// fewer per step: 75.07 -> 74.21 ms per C2 launch), and the update threads take channel t % 128
// (coalesced x access; 74.85 ms).  The per-GEMM k-step fences (WGemm::run FENCE) follow the unit's
// GGD_SCHED_FENCE except KA's QKV tile, whose fence is per unit (ggd_mega.hip: none, r05w10)
#ifndef GGD_MK_FENCE_QKV
#define GGD_MK_FENCE_QKV -1
#endif

namespace ggd {

constexpr int FT = 512;  // threads of the fused kernels: 8 waves, two per SIMD

// a step record through the global view (see G in ggd_fusedlib.h)
__device__ __forceinline__ StepRec ld_rec(const StepRec* p) {
  static_assert(sizeof(StepRec) % 4 == 0, "step records are whole dwords");
  StepRec r;
  unsigned* d = (unsigned*)&r;
  const gptr<unsigned> src = G((const unsigned*)p);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(StepRec) / 4); ++i) d[i] = src[i];
  return r;
}

__device__ __forceinline__ float bias_at(const float4& b, int r) { return r == 0 ? b.x : r == 1 ? b.y : r == 2 ? b.z : b.w; }

// Residual rows resident in LDS (persistent loop, bf16): a workgroup keeps its clip's f32
// residual rows (Hs, at LDS offset 0) from KA through KB and KC to KD -- KB and KC compute the
// full rows redundantly anyway -- so only KA / KE gather them and only KD publishes them.
// (As separate launches, or with f32 images that do not fit beside them, Hs is re-read.)
template <typename T, int CP> struct Res {
  static constexpr bool ON = CP != CP_KERNEL && sizeof(T) == 2;
  static constexpr size_t BASE = ON ? Plan<T>::HS : 0;  // start of the phase-private LDS
};

// Hs[i][n] += A[i] . W[n] + bias[n] for all row tiles; wave w owns the NJ column tiles
// NJ w .. NJ w + NJ - 1.  Computed transposed (WGemm TR): lane (c16, g4) of tile (rt, j) holds
// row rt 16 + c16, columns 16 (NJ w + j) + 4 g4 .. + 3, so the accumulators start from one
// float4 of Hs + bias and the epilogue is one float4 store (no dependent read-modify-write).
template <typename T, int KT, int NJ, int RT, typename AF>
__device__ __forceinline__ void residual_gemm_then(float* Hs, const T* A, int SA, WGemm<T, NJ, KT, RT>& g,
                                                   const float4 (&bias)[NJ], int lane, int wave, AF&& after);
template <typename T, int KT, int NJ, int RT>
__device__ __forceinline__ void residual_gemm(float* Hs, const T* A, int SA, WGemm<T, NJ, KT, RT>& g,
                                              const float4 (&bias)[NJ], int lane, int wave) {
  residual_gemm_then<T, KT, NJ, RT>(Hs, A, SA, g, bias, lane, wave, [](int) {});
}
// residual_gemm with WGemm::run_then's per-k-step hook
template <typename T, int KT, int NJ, int RT, typename AF>
__device__ __forceinline__ void residual_gemm_then(float* Hs, const T* A, int SA, WGemm<T, NJ, KT, RT>& g,
                                                   const float4 (&bias)[NJ], int lane, int wave, AF&& after) {
  const int c16 = lane & 15, g4 = lane >> 4;
  f32x4 acc[RT][NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = (NJ * wave + j) * 16 + 4 * g4;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const float4 h = *(const float4*)(Hs + (rt * 16 + c16) * SH + col);
      acc[rt][j] = f32x4{h.x + bias[j].x, h.y + bias[j].y, h.z + bias[j].z, h.w + bias[j].w};
    }
  }
  g.template run_then<true, -1>(acc, A, SA, lane, after, NJ, false);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = (NJ * wave + j) * 16 + 4 * g4;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      *(float4*)(Hs + (rt * 16 + c16) * SH + col) = make_float4(acc[rt][j][0], acc[rt][j][1], acc[rt][j][2], acc[rt][j][3]);
  }
}

// rows [0, L) of Hs -> global rows, shared by the 8 workgroups of a clip: workgroup `part`
// writes rows r with r % 8 == part (every row once; bounded 16-byte stores, no branch)
template <int CP>
__device__ __forceinline__ void store_rows(float* dst, const float* Hs, int L, int part) {
  const OutRowsP<CP> out(dst, (uint32_t)(sizeof(float) * L * FD));
  static_assert(FR / 8 * 64 == FT, "one 16-byte piece per thread");
  const int idx = ltid(), r = (idx >> 6) * 8 + part, c = (idx & 63) * 4;
  out.put4((uint32_t)(r * FD + c), *(const float4*)(Hs + min(r, L - 1) * SH + c));
}

// ------------------------------------------------------------------------------------------
// The weight fragments a phase streams into registers, separable from the phase: the kernels
// load them at their start; the persistent loop issues them while the clip group meets at the
// barrier in front of the phase, so the weight stream overlaps the wait.
// ------------------------------------------------------------------------------------------
// one 16-column tile over K = 256 per wave: KA's QKV tile and KE's output tile share the type,
// so the persistent loop carries ONE set of registers for "the next phase's tile" across layers
// on = false: the wave computes nothing with the tile (KA: waves 6-7; KE: waves >= RT) and loads nothing
template <typename T, int RT> struct Pre1 {
  WGemm<T, 1, FD / Frag<T>::KF, RT> g;
  bool on;
  __device__ __forceinline__ Pre1(const void* w, int tile, bool on_) : g(w, FD / Frag<T>::KF, 0), on(on_) {
    g.tiles[0] = tile;
  }
  __device__ __forceinline__ void load(int lane) {
    if (on) g.load(0, lane);
  }
  __device__ __forceinline__ int loads() const { return on ? decltype(g)::G : 0; }  // vector loads per load()
};
template <typename T, int RT> using KAPre = Pre1<T, RT>;
template <typename T, int RT> using KEPre = Pre1<T, RT>;
template <typename T, int RT, typename FA>  // QKV of head h: waves 0-5 one tile each
__device__ __forceinline__ KAPre<T, RT> ka_pre(const FA& a, int h, int wave) {
  return KAPre<T, RT>(a.w.qkv, h * 6 + min(wave, 5), wave < 6);
}
template <typename T, int RT, typename FA>  // output channel tile p (waves 0 .. RT-1, one row tile each)
__device__ __forceinline__ KEPre<T, RT> ke_pre(const FA& a, int p, int wave) {
  return KEPre<T, RT>(a.w_out, p, wave < RT);
}
template <typename T, int RT> struct KBPre {  // SA out-projection, all 16 tiles (2 per wave)
  WGemm<T, 2, FD / Frag<T>::KF, RT> go;
  template <typename FA>
  __device__ __forceinline__ KBPre(const FA& a, int wave) : go(a.w.o_sa, FD / Frag<T>::KF, 0) {
    go.tiles[0] = 2 * wave;
    go.tiles[1] = 2 * wave + 1;
  }
  __device__ __forceinline__ void load(int lane) { go.load(0, lane); }
  __device__ __forceinline__ void load_tile(int j, int lane) { go.load_tile(j, lane); }
  static constexpr int LOADS = 2 * decltype(go)::G;  // vector loads per load()
  static constexpr int TILE_LOADS = decltype(go)::G;
};
template <typename T, int RT> struct KCPre {  // CA out-projection (the FFN-up tile loads in the phase)
  WGemm<T, 2, FD / Frag<T>::KF, RT> go;
  template <typename FA>
  __device__ __forceinline__ KCPre(const FA& a, int c, int wave) : go(a.w.o_ca, FD / Frag<T>::KF, 0) {
    (void)c;
    go.tiles[0] = 2 * wave;
    go.tiles[1] = 2 * wave + 1;
  }
  __device__ __forceinline__ void load(int lane) { go.load(0, lane); }
  __device__ __forceinline__ void load_tile(int j, int lane) { go.load_tile(j, lane); }
  static constexpr int LOADS = 2 * decltype(go)::G;
  static constexpr int TILE_LOADS = decltype(go)::G;
};
template <typename T, int RT> struct KDPre {  // the FFN-down column reduce streams no weights
  template <typename FA>
  __device__ __forceinline__ KDPre(const FA&, int, int) {}
  __device__ __forceinline__ void load(int) {}
};

// The persistent loop hands KA and KB a hook that issues the NEXT phase's weight fragments right
// behind the attention: the waves the attention leaves idle (it runs on one wave per 16 query rows)
// get there as it starts, so their share of the 128 KiB out-projection stream runs under the
// attention instead of at the barrier (issuing the whole stream earlier, from every wave, stalls
// the issuing waves' own work: measured).  One load site per wave keeps the registers unspilled.
// Separate launches pass none.
struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};

// ------------------------------------------------------------------------------------------
// KA: [emb_x + PE (layer 0)] + LN1 + QKV(head) + conv + self-attention      grid (heads, clips)
// ------------------------------------------------------------------------------------------
// EMB = false (the persistent loop): layer 0's residual rows come from the KE rows phase, the x ->
// emb path is not compiled in
template <typename T, int RT, int CP, bool EMB = true, typename FA, typename H = NoHook, typename H0 = NoHook>
__device__ __forceinline__ void ka_phase(const FA& a, int h, int b, unsigned char* smem, KAPre<T, RT>& pre,
                                         H&& hook = H(), H0&& hook0 = H0()) {
  using PL = Plan<T>;
  constexpr int KT = FD / Frag<T>::KF, SY = 96 + 4;
  const int tid = ltid(), lane = tid & 63, wave = tid >> 6;
  const int L = a.L, c16 = lane & 15, g4 = lane >> 4;
  using R = Res<T, CP>;
  unsigned char* pv = smem + R::BASE;
  T* Xn = (T*)pv;
  float2* st = (float2*)(pv + PL::IMG);
  unsigned char* un = pv + PL::IMG + PL::ST;
  float* Hs = R::ON ? (float*)smem : (float*)un;
  float* Y = (float*)un;
  unsigned char* att = un + PL::Y_KA;
  static_assert(R::BASE + PL::IMG + PL::ST + PL::Y_KA + FAtt<T>::BYTES <= 160 * 1024 - 256, "KA LDS");
  const auto& w = a.w;

  STAMP(0);
  const bool emb = EMB && a.x_emb != nullptr;  // layer 0: h = emb_x(x) + PE computed here
  glds_rows<FT, CP>(Hs, sizeof(float) * SH, emb ? a.pe : a.h + (size_t)b * L * FD, sizeof(float) * FD, L, 1);
  constexpr int KTE = 128 / Frag<T>::KF, SB = 128 + Frag<T>::PT, NXV = FR * 128 / FT;
  WGemm<T, 2, KTE, RT> ge(a.w_emb, KTE, 0);
  float4 be[2];
  float xv[NXV];
  if (emb) {
    ge.tiles[0] = 2 * wave;
    ge.tiles[1] = 2 * wave + 1;
    ge.load(0, lane);
    be[0] = ld_f4(a.b_emb + (2 * wave) * 16 + 4 * g4);
    be[1] = ld_f4(a.b_emb + (2 * wave + 1) * 16 + 4 * g4);
    const int C = a.C;
#pragma unroll
    for (int i = 0; i < NXV; ++i) {
      const int idx = tid + i * FT, l = idx >> 7, c = idx & 127;
      xv[i] = ld_f32<CP>(a.x_emb, (uint32_t)(((size_t)b * L + min(l, L - 1)) * C + min(c, C - 1)));
    }
  }
  // QKV of head h: packed as 6 tiles [q0 q1 k0 k1 v0 v1]; waves 0-5 own one tile each
  const int nq = wave < 6 ? 1 : 0;
  auto& gm = pre.g;
  const float4 bias = ld_f4(w.qkv_b + h * 96 + min(wave, 5) * 16 + 4 * g4);
  // the conv of the wave's tile (0-1 Q, 2-3 K, 4-5 V): channels c0 .. c0 + 3 of the head
  const int kind = min(wave, 5) >> 1, c0 = (wave & 1) * 16 + 4 * g4;
  ConvW cw[4];
  conv_w4(cw, kind == 0 ? w.sa_qw : kind == 1 ? w.sa_kw : w.sa_vw, kind == 0 ? w.sa_qb : kind == 1 ? w.sa_kb : w.sa_vb,
          c0);
  __syncthreads();  // LDS-DMA rows and every operand above have landed
  if (emb) {
    // Xb = bf16(x) (channels >= C zero; aliases the LN image), Hs = PE + Xb W_emb^T + b
    T* Xb = Xn;
#pragma unroll
    for (int i = 0; i < NXV; ++i) {
      const int idx = tid + i * FT, l = idx >> 7, c = idx & 127;
      Xb[l * SB + c] = from_f32<T>(c < a.C ? xv[i] : 0.f);
    }
    bar_lds();
    residual_gemm<T, KTE, 2, RT>(Hs, Xb, SB, ge, be, lane, wave);
    bar_lds();
    if (!R::ON) store_rows<CP>(a.h + (size_t)b * L * FD, Hs, L, h);  // the residual rows KB reads
  }
  ln_rows<T, FT, RT * 16>(Hs, L, Xn);
  bar_lds();
  STAMP(1);
  // (kernel path) Hs is dead from here: the attention images overlay it.  The QKV tile of each
  // wave is convolved over tokens in registers (conv_tokens) and written straight into the Q, K
  // (row-major) or V^T image; waves 6-7 zero the V^T keys past the row tiles.
  using AT = FAtt<T>;
  {
    f32x4 acc[RT][1];
    gm.template run<true, GGD_MK_FENCE_QKV>(acc, Xn, Frag<T>::SX, lane, nq);
    if (nq) {
      f32x4 v[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        v[rt] = f32x4{acc[rt][0][0] + bias.x, acc[rt][0][1] + bias.y, acc[rt][0][2] + bias.z, acc[rt][0][3] + bias.w};
      conv_tokens<RT>(v, cw, L, c16);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        if (kind == 0) put_tok4<T, false>((T*)(att + AT::OQ), AT::SQ, rt * 16 + c16, c0, v[rt]);
        else if (kind == 1) put_tok4<T, false>((T*)(att + AT::OK), AT::SQ, rt * 16 + c16, c0, v[rt]);
        else put_tok4<T, true>((T*)(att + AT::OV), AT::SV, rt * 16 + c16, c0, v[rt]);
      }
    } else if constexpr (RT * 16 < FLK) {
      constexpr int NK = FLK - RT * 16;
      T* Vt = (T*)(att + AT::OV);
      for (int e = tid - 6 * 64; e < FDK * NK; e += 2 * 64) Vt[(e / NK) * AT::SV + RT * 16 + e % NK] = from_f32<T>(0.f);
    }
  }
  bar_lds();
  STAMP(2);
  STAMP(3);
  hook0();  // before the attention: all waves (the attention waves issue only part of their stream here)
  fattn_any<T, CP>(att, L, L, a.scale, (T*)a.o_sa + (size_t)b * L * FD + h * FDK, FD);
  asm volatile("" ::: "memory");  // the hook's loads stay behind every store above (mk_sync counts them)
  hook();
  STAMP_END(4);
}

// ------------------------------------------------------------------------------------------
// KB: SA out-proj + residual + LN2 + cross-attn Q(head) + conv + cross-attention  (heads, clips)
// ------------------------------------------------------------------------------------------
template <typename T, int RT, int CP, typename FA, typename H = NoHook, typename H0 = NoHook>
__device__ __forceinline__ void kb_phase(const FA& a, int h, int b, int it, unsigned char* smem, KBPre<T, RT>& pre,
                                         H&& hook = H(), H0&& hook0 = H0()) {
  using PL = Plan<T>;
  using AT = FAtt<T>;
  constexpr int KT = FD / Frag<T>::KF, SYQ = FDK + 4;
  const int tid = ltid(), lane = tid & 63, wave = tid >> 6;
  const int L = a.L, Lk = 1 + a.Ts, c16 = lane & 15, g4 = lane >> 4;
  using R = Res<T, CP>;
  unsigned char* pv = smem + R::BASE;
  T* Ax = (T*)pv;                     // O_sa image, then LN2(h) image
  float2* st = (float2*)(pv + PL::IMG);
  unsigned char* un = pv + PL::IMG + PL::ST;
  float* Hs = R::ON ? (float*)smem : (float*)un;
  float* Yq = (float*)un;
  unsigned char* att = un + PL::YQ + PL::RAW;
  static_assert(R::BASE + PL::IMG + PL::ST + PL::YQ + PL::RAW + FAtt<T>::BYTES <= 160 * 1024 - 256, "KB LDS");
  const auto& w = a.w;
  const size_t row0 = (size_t)b * L;

  STAMP(0);
  const int span_slot = it * a.span_stride + a.span_layer;
  SPAN_BEGIN(span_slot);
  const int t = a.t_clip ? a.t_clip[b] : G(a.steps)[it].t_orig;
  if (!R::ON) glds_rows<FT, CP>(Hs, sizeof(float) * SH, a.h + row0 * FD, sizeof(float) * FD, L, 1);
  ImgStage<T, FT, CP> so;
  so.load(Ax, (const T*)a.o_sa + row0 * FD, L);
  auto& go = pre.go;
  float4 bo[2];
  bo[0] = ld_f4(w.o_sa_b + (2 * wave) * 16 + 4 * g4);
  bo[1] = ld_f4(w.o_sa_b + (2 * wave + 1) * 16 + 4 * g4);
  so.store(Ax, L);
  __syncthreads();  // LDS-DMA rows and every operand above have landed
  STAMP(1);
  // cross-attn query of head h: waves 0, 1 own tiles 2h, 2h + 1 of the natural packing
  WGemm<T, 1, KT, RT> gq(w.q_ca, KT, 0);
  gq.tiles[0] = 2 * h + (wave & 1);
  if (wave < 2) gq.load(0, lane);
  const float4 bq = ld_f4(w.q_ca_b + h * FDK + (wave & 1) * 16 + 4 * g4);
  const int cq0 = (wave & 1) * 16 + 4 * g4;  // the query channels of the lane (waves 0-1)
  ConvW cq[4];
  conv_w4(cq, w.ca_qw, w.ca_qb, cq0);
  const ConvW ck = conv_w(w.ca_kw, w.ca_kb, tid & 31), cv = conv_w(w.ca_vw, w.ca_vb, tid & 31);
  // memory K / V of head h: the step-invariant rows come convolved and in image order from the
  // kvc block (set_memory), rows 0 / 1 (the step token's conv reach) are computed by wave 7
  residual_gemm<T, KT, 2, RT>(Hs, Ax, Frag<T>::SX, go, bo, lane, wave);
  // issued after the out-projection: the fix-up rows need t (a two-load dependent chain), which
  // must not stall it; the loads complete under LN2
  KvcStage<T, FT> kvs;
  kvs.load((const T*)w.kvc + ((size_t)b * (FD / FDK) + h) * KVC_ELEMS, tid);
  KvFix fx;
  if (wave == FT / 64 - 1) fx.load(w.kv_step + (size_t)t * 2 * FD, w.kv_mem + (size_t)b * a.Ts * 2 * FD, a.Ts, h, lane);
  bar_lds();
  STAMP(2);
  if (!R::ON) store_rows<CP>(a.h_out + row0 * FD, Hs, L, h);
  ln_rows<T, FT, RT * 16>(Hs, L, Ax);
  // resident rows: the attention images do not overlay Hs, so the memory K / V pieces (loads in
  // flight since the out-projection) are staged before LN2's barrier and the step-token rows fixed
  // right after it
  if constexpr (R::ON) kvs.store(att, tid);
  bar_lds();
  STAMP(3);
  // (kernel path) Hs is dead: the attention images overlay it
  if constexpr (!R::ON) kvs.store(att, tid);
  if (wave < 2) {  // the head's query, convolved over tokens in registers, into the Q image
    f32x4 acc[RT][1];
    gq.template run<true, -1>(acc, Ax, Frag<T>::SX, lane);
    f32x4 v[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      v[rt] = f32x4{acc[rt][0][0] + bq.x, acc[rt][0][1] + bq.y, acc[rt][0][2] + bq.z, acc[rt][0][3] + bq.w};
    conv_tokens<RT>(v, cq, L, c16);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) put_tok4<T, false>((T*)(att + AT::OQ), AT::SQ, rt * 16 + c16, cq0, v[rt]);
  }
  if constexpr (!R::ON) bar_lds();  // every staged piece has landed before the fix-up overwrites some
  STAMP(4);
  if (wave == FT / 64 - 1) fx.store<T>(att, ck, cv, Lk, lane);
  bar_lds();
  STAMP(5);
  hook0();
  fattn_any<T, CP>(att, L, Lk, a.scale, (T*)a.o_ca + row0 * FD + h * FDK, FD);
  asm volatile("" ::: "memory");
  hook();
  STAMP_END(6);
  SPAN_END(span_slot);
}

// ------------------------------------------------------------------------------------------
// KC: CA out-proj + residual + LN3 + FFN-up chunk c (128 hidden) + ReLU^2 + that chunk's share of
// FFN-down (hidden chunk x W2[:, chunk]^T, all 256 output columns): a partial sum per chunk in T
// (bf16 loops: bf16 partials, half the hand-off bytes of f32), reduced in f32 by KD.  The hidden
// chunk never leaves LDS.                                                grid (8 chunks, clips)
// ------------------------------------------------------------------------------------------
template <typename T, int RT, int CP, typename FA>
__device__ __forceinline__ void kc_phase(const FA& a, int c, int b, unsigned char* smem, KCPre<T, RT>& pre) {
  using PL = Plan<T>;
  constexpr int KT = FD / Frag<T>::KF;
  const int tid = ltid(), lane = tid & 63, wave = tid >> 6;
  const int L = a.L, c16 = lane & 15, g4 = lane >> 4;
  using R = Res<T, CP>;
  unsigned char* pv = smem + R::BASE;
  T* Ax = (T*)pv;
  float2* st = (float2*)(pv + PL::IMG);
  float* Hs = R::ON ? (float*)smem : (float*)(pv + PL::IMG + PL::ST);
  const auto& w = a.w;
  const size_t row0 = (size_t)b * L;
  const int h = c;  // STAMP uses (h, b)

  STAMP(0);
  if (!R::ON) glds_rows<FT, CP>(Hs, sizeof(float) * SH, a.h + row0 * FD, sizeof(float) * FD, L, 1);
  ImgStage<T, FT, CP> so;
  so.load(Ax, (const T*)a.o_ca + row0 * FD, L);
  auto& go = pre.go;
  float4 bo[2];
  bo[0] = ld_f4(w.o_ca_b + (2 * wave) * 16 + 4 * g4);
  bo[1] = ld_f4(w.o_ca_b + (2 * wave + 1) * 16 + 4 * g4);
  so.store(Ax, L);
  __syncthreads();  // LDS-DMA rows and every operand above have landed
  STAMP(1);
  WGemm<T, 1, KT, RT> gf(w.ff1, KT, 0);  // in flight across the out-projection
  gf.tiles[0] = 8 * c + wave;
  gf.load(0, lane);
  const float4 bf = ld_f4(w.ff1_b + (8 * c + wave) * 16 + 4 * g4);
  residual_gemm<T, KT, 2, RT>(Hs, Ax, Frag<T>::SX, go, bo, lane, wave);
  // FFN-down fragments of the chunk (k steps c KC .. c KC + KC - 1, column tiles 2w, 2w + 1): in
  // flight across LN3 and FFN-up, in the registers the out-projection has just released
  constexpr int KC = 128 / Frag<T>::KF, KTT = 4 * FD / Frag<T>::KF, SHC = 128 + Frag<T>::PT;
  WGemm<T, 2, KC, RT> gd(w.ff2, KTT, c * KC);
  gd.tiles[0] = 2 * wave;
  gd.tiles[1] = 2 * wave + 1;
  gd.load(0, lane);
  bar_lds();
  STAMP(2);
  if (!R::ON) store_rows<CP>(a.h_out + row0 * FD, Hs, L, c);
  ln_rows<T, FT, RT * 16>(Hs, L, Ax);
  bar_lds();
  STAMP(3);
  // hidden chunk image (overlays the dead Hs on the kernel path; beside the resident rows otherwise)
  T* Hc = (T*)(pv + PL::IMG + PL::ST);
  {
    f32x4 acc[RT][1];
    gf.template run<true, -1>(acc, Ax, Frag<T>::SX, lane);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const float v0 = fmaxf(acc[rt][0][0] + bf.x, 0.f), v1 = fmaxf(acc[rt][0][1] + bf.y, 0.f);
      const float v2 = fmaxf(acc[rt][0][2] + bf.z, 0.f), v3 = fmaxf(acc[rt][0][3] + bf.w, 0.f);
      put_tok4<T, false>(Hc, SHC, rt * 16 + c16, wave * 16 + 4 * g4, f32x4{v0 * v0, v1 * v1, v2 * v2, v3 * v3});
    }
  }
  bar_lds();
  STAMP(4);
  {
    f32x4 acc[RT][2];
    gd.template run<true, -1>(acc, Hc, SHC, lane);
    const OutRowsP<CP> out((T*)a.ffp + ((size_t)b * 8 + c) * L * FD, (uint32_t)(sizeof(T) * L * FD));
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        out.template put4v<T>((uint32_t)((rt * 16 + c16) * FD + (2 * wave + j) * 16 + 4 * g4), acc[rt][j]);
  }
  STAMP_END(5);
}

// ------------------------------------------------------------------------------------------
// KD: columns [32 p, 32 p + 32) of h += sum over the 8 chunks of KC's FFN-down partials + b2, in
// place.  Thread (row tid / 8, column quad tid % 8): 8 partial float4 in flight, added in chunk
// order (deterministic).                                          grid (8 column chunks, clips)
// ------------------------------------------------------------------------------------------
template <typename T, int RT, int CP, typename FA>
__device__ __forceinline__ void kd_phase(const FA& a, int p, int b, unsigned char* smem, KDPre<T, RT>& pre) {
  (void)pre;
  const int tid = ltid(), L = a.L;
  const int row = min(tid >> 3, L - 1), col = 32 * p + 4 * (tid & 7);  // rows >= L: clamped loads, dropped store
  const auto& w = a.w;
  const size_t row0 = (size_t)b * L;
  const int h = p;  // STAMP uses (h, b)

  STAMP(0);
  float4 part[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint32_t off = (uint32_t)(sizeof(T) * ((((size_t)b * 8 + c) * L + row) * FD + col));
    if constexpr (sizeof(T) == 2) {
      const uint2 u = ld_8B<CP>(a.ffp, off);
      part[c] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                            __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
    } else {
      const uint4 u = ld_16B<CP>(a.ffp, off);
      part[c] = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
    }
  }
  float4 res;
  if constexpr (Res<T, CP>::ON) {  // the residual rows KC left in LDS
    res = *(const float4*)((const float*)smem + row * SH + col);
  } else {
    const uint4 u = ld_16B<CP>(a.h, (uint32_t)(sizeof(float) * ((row0 + row) * FD + col)));
    res = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
  }
  const float4 bias = ld_f4(w.ff2_b + col);
  float4 y = part[0];
#pragma unroll
  for (int c = 1; c < 8; ++c) {
    y.x += part[c].x;
    y.y += part[c].y;
    y.z += part[c].z;
    y.w += part[c].w;
  }
  STAMP(1);
  const OutRowsP<CP> out(a.h + row0 * FD, (uint32_t)(sizeof(float) * L * FD));
  out.put4((uint32_t)((tid >> 3) * FD + col),
           make_float4(res.x + (y.x + bias.x), res.y + (y.y + bias.y), res.z + (y.z + bias.z), res.w + (y.w + bias.w)));
  STAMP_END(3);
}

// ------------------------------------------------------------------------------------------
// KE: LN_out + out-proj of 16 channels (eps) [+ diffusion update of those channels]
// grid (8 channel blocks, clips).  Block p owns pose channels [16p, 16p + 16): wave w < RT computes
// eps for row tile w; the update of the block's L x 16 elements is one Philox quad per thread of
// the other waves.
// The next step's emb_x + PE is computed by that step's first KA (x_emb).
// ------------------------------------------------------------------------------------------
template <typename T, int RT, int CP, typename FA>
__device__ __forceinline__ void ke_phase(const FA& a, int p, int b, int k, unsigned char* smem, KEPre<T, RT>& pre) {
  using PL = Plan<T>;
  constexpr int KT = FD / Frag<T>::KF, SE = 16 + 4;
  const int tid = ltid(), lane = tid & 63, wave = tid >> 6;
  const int L = a.L, C = a.C, c16 = lane & 15, g4 = lane >> 4, LC = L * C;
  T* Xn = (T*)smem;
  float2* st = (float2*)(smem + PL::IMG);
  float* Hs = (float*)(smem + PL::IMG + PL::ST);
  float* E = (float*)(smem + PL::IMG + PL::ST + PL::HS);
  const size_t row0 = (size_t)b * L;
  const int c0 = 16 * p, cn = max(0, min(16, C - c0));       // the block's channels
  const int e0 = c0 * L, ne = cn * L;                         // its elements, reference (C, L) order
  const int h = p;                                            // STAMP uses (h, b)

  STAMP(0);
  glds_rows<FT, CP>(Hs, sizeof(float) * SH, a.h + row0 * FD, sizeof(float) * FD, L, 1);
  WGemm<T, 1, KT, 1> go(a.w_out, KT, 0);  // waves 0..RT-1: row tile w of channel tile p (prefetched)
  go.tiles[0] = p;
#pragma unroll
  for (int k = 0; k < KT; ++k) go.wb[0][k] = pre.g.wb[0][k];
  const float4 bo = ld_f4(a.b_out + p * 16 + 4 * g4);
  // the thread's quad: elements e0 + 4 qi .. + 3 (issued now, consumed after the GEMM).  The quads
  // live on the waves the out-projection leaves idle (ut = tid - 64 RT; 64 (8 - RT) >= 4 L / 4), so
  // their Philox normals are drawn while waves 0 .. RT-1 run the GEMM.  With L % 4 == 0 a quad is 4
  // frames of one channel and 16 consecutive threads take the block's 16 channels at the same
  // frames (qi = channel (L / 4) + frame quad): each x store of a wave covers 4 frame rows x 64 bytes
  // instead of 64 scattered rows.  The Philox counter stays the quad's index in (C, L) order.
  const int ut = tid - 64 * RT;
  const bool q4 = (L & 3) == 0;
  const int qi = q4 ? (ut & 15) * (L >> 2) + (ut >> 4) : ut;
  const bool upd = a.do_update && ut >= 0 && (q4 ? (ut & 15) < cn && (ut >> 4) < (L >> 2) : 4 * ut < ne);
  StepRec rec{};
  float xq[4] = {0.f, 0.f, 0.f, 0.f}, zq[4] = {0.f, 0.f, 0.f, 0.f};
  float mq[4] = {0.f, 0.f, 0.f, 0.f}, pq[4] = {0.f, 0.f, 0.f, 0.f}, tq[4] = {0.f, 0.f, 0.f, 0.f};
  int cc0 = 0, l0 = 0;
  const bool inp = a.inp_mask != nullptr;
  const size_t plane = (size_t)a.n * LC;
  if (a.do_update) {
    rec = ld_rec(a.steps + k);
    const int e = min(e0 + 4 * max(qi, 0), e0 + max(ne, 1) - 1);  // tail threads (no valid element) load clamped addresses
    cc0 = e / L;
    l0 = e - cc0 * L;
    int cc = cc0, l = l0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t gi = (row0 + l) * C + min(cc, C - 1);
      xq[u] = ld_f32<CP>(a.x, (uint32_t)gi);
      if (a.noise) zq[u] = G(a.noise)[(size_t)k * plane + (size_t)b * LC + min(e + u, LC - 1)];
      if (inp) {
        mq[u] = G(a.inp_mask)[row0 + l];
        pq[u] = G(a.inp_pose)[gi];
        tq[u] = G(a.trans)[l];
      }
      if (++l == L) { l = 0; ++cc; }
    }
  }
  __syncthreads();  // LDS-DMA rows and every operand above have landed
  ln_rows<T, FT, RT * 16>(Hs, L, Xn);
  bar_lds();
  STAMP(1);
  static_assert(64 * (FT / 64 - RT) * 4 >= 16 * RT * 16, "the idle waves hold every update quad");
  if (wave < RT) {
    f32x4 acc[1][1];
    go.template run<true>(acc, Xn + wave * 16 * Frag<T>::SX, Frag<T>::SX, lane);
    *(float4*)(E + (wave * 16 + c16) * SE + 4 * g4) =
        make_float4(acc[0][0][0] + bo.x, acc[0][0][1] + bo.y, acc[0][0][2] + bo.z, acc[0][0][3] + bo.w);
  } else if (upd && !a.noise) {
    philox_normal4(((uint64_t)rec.seed_hi << 32) | rec.seed_lo, rec.clip_offset + (uint32_t)b, (uint32_t)rec.i,
                   TAG_STEP, (uint32_t)((e0 >> 2) + qi), zq);
  }
  bar_lds();
  STAMP(2);
  if (upd) {
    const OutRowsP<CP> xo(a.x, (uint32_t)(sizeof(float) * plane));
    int cc = cc0, l = l0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + 4 * qi + u;
      if (e < e0 + ne) {
        const float ev = E[l * SE + (cc - c0)];
        const UpdOut o = upd_math(rec, a.alg, xq[u], ev, false, 0.f, inp, mq[u], pq[u], tq[u], zq[u]);
        xo.template put<float>((uint32_t)((row0 + l) * C + cc), o.xn);
        if (a.extras && (a.extras_k < 0 || k == a.extras_k)) {
          const size_t ncl = (size_t)b * LC + e;
          a.extras[0 * plane + ncl] = o.mean;
          a.extras[1 * plane + ncl] = rec.var;
          a.extras[2 * plane + ncl] = rec.logvar;
          a.extras[3 * plane + ncl] = ev;
          a.extras[4 * plane + ncl] = o.x0;
          a.extras[5 * plane + ncl] = o.raw;
        }
      }
      if (++l == L) { l = 0; ++cc; }
    }
  } else if (!a.do_update && a.do_out) {
    for (int i = tid; i < ne; i += FT) {
      const int e = e0 + i, cc = e / L, l = e - cc * L;
      a.eps_out[(size_t)b * LC + e] = E[l * SE + (cc - c0)];
    }
  }
  STAMP_END(3);
}

// ------------------------------------------------------------------------------------------
// KE by frame rows (the persistent loop, round 4).  Workgroup p of clip b owns frames
// [r0, r1) = [p L / 8, (p + 1) L / 8) (<= 8 rows: one MFMA row tile) and runs, for those rows,
//   the last layer's FFN-down reduction (KD) for its rows: no KD phase and barrier in front of KE;
//   LN_out + eps of all C channels (wave w: channel tile w) -> E (LDS);
//   the DDPM / DDIM update of every element of its frames: the Philox quads keep the reference's
//   (C, L) element order (a quad is 4 consecutive elements of a channel's frames), one quad per
//   thread -- thread (channel c = t % 128, k = t / 128 < 3) draws quad (c L + r0) / 4 + k and updates the elements of
//   it that are channel c's frames in [r0, r1) (a quad that straddles two blocks is drawn by both,
//   each keeping its own elements; a quad that straddles two channels by both channels' threads);
//   emb_x + PE of the updated rows -> the next step's layer-0 residual rows h.
// The next step's KA of layer 0 then stages h like every other layer (no x -> emb path in front
// of it: 16 dword loads per thread, the operand image, a 3-row-tile GEMM and two barriers).
// ------------------------------------------------------------------------------------------
template <typename T> struct KerPlan {
  static constexpr int SE = 128 + 4, SB = 128 + Frag<T>::PT;
  static constexpr size_t HS = al16(sizeof(float) * 8 * SH);                  // the block's h rows
  static constexpr size_t XN = al16(sizeof(T) * 16 * Frag<T>::SX);            // LN_out image
  static constexpr size_t E = al16(sizeof(float) * 16 * SE);                  // eps [row][channel]
  static constexpr size_t XB = al16(sizeof(T) * 16 * SB);                     // emb operand
  static constexpr size_t BYTES = HS + XN + E + XB;
};
template <typename T, int RT, typename FA>  // channel tile = wave (the tiles past C load nothing)
__device__ __forceinline__ KEPre<T, RT> ker_pre(const FA& a, int wave) {
  return KEPre<T, RT>(a.w_out, wave, 16 * wave < a.C);
}

// h rows [r0, r0 + R) of clip b = PE + b_emb + Xb W_emb^T (Xb: the rows' x in bf16 / f32, 16 x 128,
// zero past C and R); wave w owns columns 32 w .. 32 w + 31.  ge: the wave's two W_emb tiles (loaded).
template <typename T, int CP, typename FA>
__device__ __forceinline__ void emb_rows_store(const FA& a, int b, int r0, int R, const T* Xb,
                                               WGemm<T, 2, 128 / Frag<T>::KF, 1>& ge, const float4 (&pe)[2],
                                               int lane, int wave) {
  const int c16 = lane & 15, g4 = lane >> 4;
  f32x4 acc[1][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) acc[0][j] = f32x4{pe[j].x, pe[j].y, pe[j].z, pe[j].w};
  ge.template run<true, -1>(acc, Xb, KerPlan<T>::SB, lane, 2, false);
  const OutRowsP<CP> ho(a.h + ((size_t)b * a.L + r0) * FD, (uint32_t)(sizeof(float) * R * FD));  // rows >= R dropped
#pragma unroll
  for (int j = 0; j < 2; ++j)
    ho.put4((uint32_t)(c16 * FD + (2 * wave + j) * 16 + 4 * g4),
            make_float4(acc[0][j][0], acc[0][j][1], acc[0][j][2], acc[0][j][3]));
}

// LayerNorm (no affine, as ln_rows) of R <= 8 f32 rows Hs (stride SH) into the 16-row T image:
// wave w normalises row w with all 64 lanes (4 columns each; sums over 16 lanes by DPP, then across
// the wave's 4 lane rows), so the few rows of a block cost one short pass instead of 32 values per
// lane on one wave; rows R .. 15 are written as zeros (waves w and w + 8)
template <typename T>
__device__ __forceinline__ void ln_rows_wave(const float* Hs, int R, T* img, int lane, int wave) {
  const int c4 = 4 * lane;
  const float4 v = *(const float4*)(Hs + min(wave, 7) * SH + c4);
  const float mu = lanerow_sum4(group_sum<16>((v.x + v.y) + (v.z + v.w))) * (1.0f / (float)FD);
  const float d0 = v.x - mu, d1 = v.y - mu, d2 = v.z - mu, d3 = v.w - mu;
  const float q = lanerow_sum4(group_sum<16>((d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3)));
  const float rs = __builtin_amdgcn_rsqf(q * (1.0f / (float)FD) + 1e-5f);
  const bool on = wave < R;  // a row past R holds stale LDS (maybe a NaN pattern): zeros, not 0 * x
  const float y0 = on ? d0 * rs : 0.f, y1 = on ? d1 * rs : 0.f, y2 = on ? d2 * rs : 0.f, y3 = on ? d3 * rs : 0.f;
  constexpr int SXI = Frag<T>::SX;
  if constexpr (sizeof(T) == 2) {
    *(uint2*)(img + wave * SXI + c4) = make_uint2(pk_bf16(y0, y1), pk_bf16(y2, y3));
    *(uint2*)(img + (wave + 8) * SXI + c4) = make_uint2(0u, 0u);
  } else {
    *(float4*)(img + wave * SXI + c4) = make_float4(y0, y1, y2, y3);
    *(float4*)(img + (wave + 8) * SXI + c4) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// the lane's PE + b_emb initial accumulators of emb_rows_store (row r0 + c16, clamped)
template <typename FA>
__device__ __forceinline__ void emb_init(const FA& a, int r0, int lane, int wave, float4 (&pe)[2]) {
  const int c16 = lane & 15, g4 = lane >> 4, r = min(r0 + c16, a.L - 1);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = (2 * wave + j) * 16 + 4 * g4;
    const float4 p = ld_f4(a.pe + (size_t)r * FD + col), bb = ld_f4(a.b_emb + col);
    pe[j] = make_float4(p.x + bb.x, p.y + bb.y, p.z + bb.z, p.w + bb.w);
  }
}

// the persistent loop's prologue: the first step's layer-0 residual rows from the initial x
template <typename T, int CP, typename FA>
__device__ __forceinline__ void emb_prologue(const FA& a, int p, int b, unsigned char* smem) {
  using KP = KerPlan<T>;
  constexpr int KTE = 128 / Frag<T>::KF;
  const int tid = ltid(), lane = tid & 63, wave = tid >> 6;
  const int L = a.L, C = a.C, r0 = p * L / 8, R = (p + 1) * L / 8 - r0;
  T* Xb = (T*)(smem + KP::HS + KP::XN + KP::E);
  WGemm<T, 2, KTE, 1> ge(a.w_emb, KTE, 0);
  ge.tiles[0] = 2 * wave;
  ge.tiles[1] = 2 * wave + 1;
  ge.load(0, lane);
  float4 pe[2];
  emb_init(a, r0, lane, wave, pe);
  float xv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // 16 rows x 128 channels, 4 per thread
    const int idx = tid + i * FT, l = idx >> 7, c = idx & 127;
    xv[i] = ld_f32<CP>(a.x, (uint32_t)(((size_t)b * L + r0 + min(l, R - 1)) * C + min(c, C - 1)));
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + i * FT, l = idx >> 7, c = idx & 127;
    Xb[l * KP::SB + c] = from_f32<T>(l < R && c < C ? xv[i] : 0.f);
  }
  __syncthreads();
  emb_rows_store<T, CP>(a, b, r0, R, Xb, ge, pe, lane, wave);
}

template <typename T, int RT, int CP, typename FA>
__device__ __forceinline__ void ker_phase(const FA& a, int p, int b, int k, unsigned char* smem, KEPre<T, RT>& pre) {
  using KP = KerPlan<T>;
  constexpr int KT = FD / Frag<T>::KF, KTE = 128 / Frag<T>::KF, SE = KP::SE, SB = KP::SB;
  const int tid = ltid(), lane = tid & 63, wave = tid >> 6;
  const int L = a.L, C = a.C, c16 = lane & 15, g4 = lane >> 4, LC = L * C;
  const int r0 = p * L / 8, R = (p + 1) * L / 8 - r0;
  using RS = Res<T, CP>;
  unsigned char* kb = smem + RS::BASE;  // behind the resident residual rows (KC left them there)
  float* Hs = (float*)kb;
  T* Xn = (T*)(kb + KP::HS);
  float* E = (float*)(kb + KP::HS + KP::XN);
  T* Xb = (T*)(kb + KP::HS + KP::XN + KP::E);
  static_assert(RS::BASE + KP::BYTES <= 160 * 1024 - 256, "KE rows LDS");
  const size_t row0 = (size_t)b * L;
  const int h = p;  // STAMP uses (h, b)

  STAMP(0);
  // the last layer's KD for the block's rows only: h = h_KC + (sum of the 8 FFN-down partials in
  // chunk order + b2), kd_phase's arithmetic; thread (row i = tid / 64, columns 4 (tid % 64) ..)
  const int si = tid >> 6, sc = 4 * (tid & 63), srow = min(r0 + max(min(si, R - 1), 0), L - 1);  // R = 0 when L < 8
  float4 part[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint32_t off = (uint32_t)(sizeof(T) * ((((size_t)b * 8 + c) * L + srow) * FD + sc));
    if constexpr (sizeof(T) == 2) {
      const uint2 u = ld_8B<CP>(a.ffp, off);
      part[c] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                            __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
    } else {
      const uint4 u = ld_16B<CP>(a.ffp, off);
      part[c] = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
    }
  }
  float4 sres = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (RS::ON) {
    sres = *(const float4*)((const float*)smem + srow * SH + sc);
  } else {
    const uint4 u = ld_16B<CP>(a.h, (uint32_t)(sizeof(float) * ((row0 + srow) * FD + sc)));
    sres = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
  }
  const float4 sb2 = ld_f4(a.ff2_b + sc);
  WGemm<T, 1, KT, 1> go(a.w_out, KT, 0);  // wave w: channel tile w (prefetched at the barrier)
  go.tiles[0] = wave;
#pragma unroll
  for (int kk = 0; kk < KT; ++kk) go.wb[0][kk] = pre.g.wb[0][kk];
  const float4 bo = ld_f4(a.b_out + wave * 16 + 4 * g4);
  // the thread's quad (see above); its elements' state / noise loads are issued now.  Thread t
  // takes channel t % 128 and the (t / 128)-th quad of it: with L % 4 == 0 every lane of a wave
  // then holds the same frames, so each x store / load of the wave covers one frame row's
  // consecutive channels (a few cache lines) instead of 64 scattered rows (C <= 128, E's rows)
  const int uc = tid & 127, qi = ((uc * L + r0) >> 2) + (tid >> 7);
  const bool qon = uc < C && tid < 3 * 128;
  StepRec rec = ld_rec(a.steps + k);
  float xq[4] = {0.f, 0.f, 0.f, 0.f}, zq[4] = {0.f, 0.f, 0.f, 0.f};
  float mq[4] = {0.f, 0.f, 0.f, 0.f}, pq[4] = {0.f, 0.f, 0.f, 0.f}, tq[4] = {0.f, 0.f, 0.f, 0.f};
  int ul[4];
  bool uok[4];
  const bool inp = a.inp_mask != nullptr;
  const size_t plane = (size_t)a.n * LC;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    // element e = 4 qi + u is frame e - uc L of channel uc when that lies in [r0, r0 + R) (the quad
    // starts at most 3 elements before the channel's frame r0: no division needed)
    const int e = 4 * qi + u, lr = e - uc * L, l = min(max(lr, 0), L - 1);
    ul[u] = l;
    uok[u] = qon && lr >= r0 && lr < r0 + R;
    const size_t gi = (row0 + l) * C + min(uc, C - 1);
    xq[u] = ld_f32<CP>(a.x, (uint32_t)gi);
    if (a.noise) zq[u] = G(a.noise)[(size_t)k * plane + (size_t)b * LC + min(e, LC - 1)];
    if (inp) {
      mq[u] = G(a.inp_mask)[row0 + l];
      pq[u] = G(a.inp_pose)[gi];
      tq[u] = G(a.trans)[l];
    }
  }
  // emb operand pads: channels C..127 of every row and rows R..15 (the update fills the rest)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + i * FT, l = idx >> 7, c = idx & 127;
    if (l >= R || c >= C) Xb[l * SB + c] = from_f32<T>(0.f);
  }
  __syncthreads();  // every operand above has landed
  if (si < R) {
    float4 y = part[0];
#pragma unroll
    for (int c = 1; c < 8; ++c) {
      y.x += part[c].x;
      y.y += part[c].y;
      y.z += part[c].z;
      y.w += part[c].w;
    }
    *(float4*)(Hs + si * SH + sc) =
        make_float4(sres.x + (y.x + sb2.x), sres.y + (y.y + sb2.y), sres.z + (y.z + sb2.z), sres.w + (y.w + sb2.w));
  }
  bar_lds();
  // the emb operands, in flight across LN_out, eps and the update (issued after the wait above, so
  // that it does not hold for them)
  WGemm<T, 2, KTE, 1> ge(a.w_emb, KTE, 0);
  ge.tiles[0] = 2 * wave;
  ge.tiles[1] = 2 * wave + 1;
  ge.load(0, lane);
  float4 pe[2];
  emb_init(a, r0, lane, wave, pe);
  ln_rows_wave<T>(Hs, R, Xn, lane, wave);
  bar_lds();
  STAMP(1);
  if (16 * wave < C) {
    f32x4 acc[1][1];
    go.template run<true, -1>(acc, Xn, Frag<T>::SX, lane);
    *(float4*)(E + c16 * SE + 16 * wave + 4 * g4) =
        make_float4(acc[0][0][0] + bo.x, acc[0][0][1] + bo.y, acc[0][0][2] + bo.z, acc[0][0][3] + bo.w);
  }
  if (qon && !a.noise)
    philox_normal4(((uint64_t)rec.seed_hi << 32) | rec.seed_lo, rec.clip_offset + (uint32_t)b, (uint32_t)rec.i,
                   TAG_STEP, (uint32_t)qi, zq);
  bar_lds();
  STAMP(2);
  {
    const OutRowsP<CP> xo(a.x, (uint32_t)(sizeof(float) * plane));
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (!uok[u]) continue;
      const int l = ul[u], e = 4 * qi + u;
      const float ev = E[(l - r0) * SE + uc];
      const UpdOut o = upd_math(rec, a.alg, xq[u], ev, false, 0.f, inp, mq[u], pq[u], tq[u], zq[u]);
      xo.template put<float>((uint32_t)((row0 + l) * C + uc), o.xn);
      Xb[(l - r0) * SB + uc] = from_f32<T>(o.xn);
      if (a.extras && (a.extras_k < 0 || k == a.extras_k)) {
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
  bar_lds();
  STAMP(3);
  emb_rows_store<T, CP>(a, b, r0, R, Xb, ge, pe, lane, wave);
  STAMP_END(4);
}

}  // namespace ggd
