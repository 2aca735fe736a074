// ggd_rows.hip -- the clip-group reverse loop (C2 / C3) with the decoder split by ROW BLOCKS
// wherever its work is row-local (round 5).
//
// ggd_mega.hip splits every phase of a layer by head or by FFN chunk, so the two attention
// out-projections and the three LayerNorms of a layer run on all 40 rows in every one of the 8
// workgroups of a clip (8x redundant, on 48-row MFMA tiles).  Here only the two phases that need
// a whole sequence stay split by head / chunk; everything between them is row-local and runs on
// the workgroup's own rows [r0, r1) = [p L / 8, (p + 1) L / 8) (5 rows at L = 40):
//
//   KA (head h)    LN1 image of all rows (published by KD) -> QKV of head h + 3-tap conv + self-attn
//                  -> o_sa[:, head h]                                              (transformer.py:88-118)
//   KB (rows p)    o_sa rows r0-1 .. r1 (the conv halo) -> SA out-proj + residual -> LN2 -> query of
//                  EVERY head (wave w: head w) + conv -> cross-attention of head w for the block's
//                  queries against the cached memory K / V (registers, no LDS image) -> CA out-proj +
//                  residual -> LN3 of the own rows -> LN3 image rows      (nn.py:159-167, 213)
//   KC (chunk c)   LN3 image of all rows -> FFN-up chunk + ReLU^2 -> FFN-down partial   (transformer.py:151-154)
//   KD (rows p)    sum of the 8 partials + b2 + residual -> h rows -> LN1 of the next layer in
//                  registers (wave w: row w) -> LN1 image rows                     (nn.py:170-172)
//   KE (rows p)    the last layer's KD + LN_out + eps + update + emb_x + PE (ggd_phases.h ker_phase)
//                  + LN1 of the next step's layer 0
//
// Four clip-group barriers per layer, as before (16 per step), but per workgroup and layer the
// out-projections run on ONE 16-row tile instead of three (the halo rows r0 - 1 and r1 are
// recomputed so that the query conv sees its neighbours), the LayerNorms on <= 10 rows instead
// of 40, and KC / KA start from a staged LN image instead of residual rows + LayerNorm.
// The residual rows of the block stay in LDS (Hr, 16 rows at offset 0) from KD to KB to KD.
// Hand-off buffers: o_sa (FusedArgs::o_sa), the LN1 / LN3 images (FusedArgs::o_ca: the
// cross-attention output never leaves its workgroup here), FFN-down partials (ffp), h rows (h).
// bf16 only (f32 parity mode keeps ggd_mega.hip).
#include "ggd_megasync.h"

namespace ggd {
namespace {

using T = bf16_t;
constexpr int SX = Frag<T>::SX;     // operand image row stride (elements)
constexpr int KT = FD / Frag<T>::KF;  // k steps of a 256-wide GEMM (8)

// LDS plan (bytes)
template <int RT> struct RowPlan {
  static constexpr size_t HR = al16(sizeof(float) * 16 * SH);        // resident rows: image row i = token r0 - 1 + i
  static constexpr size_t XN = al16(sizeof(T) * RT * 16 * SX);       // LN image of the clip's rows (KA / KC)
  static constexpr size_t IMG16 = al16(sizeof(T) * 16 * SX);         // a 16-row operand image (KB)
  static constexpr size_t FIX = sizeof(float) * 8 * 128;             // KB: per head K rows 0-1 [2][32], V [32][2]
  static constexpr size_t CQ = sizeof(float4) * FDK;                 // KB: the query conv taps (w0, w1, w2, b) per channel
  static constexpr size_t KA = HR + XN + FAtt<T, RT * 16>::BYTES;  // Q image: the clip's RT row tiles only
  static constexpr size_t KB = HR + 2 * IMG16 + FIX + CQ;
  static constexpr size_t HC = al16(sizeof(T) * RT * 16 * (128 + Frag<T>::PT));
  static constexpr size_t KC = HR + XN + HC;
  static constexpr size_t KE = HR + KerPlan<T>::BYTES;
  // KB's CA out-projection fragments, k steps 0 .. GCK - 1 of every wave's two tiles, copied into
  // LDS by LDS-DMA in the KA in front (no registers: the loop is at ~240 VGPRs), clear of KA's and
  // KB's own regions
  // GCK: 5 of the 8 k steps at L <= 48 (80 KiB), as many as fit at RT = 4.  Measured (C2 mr_kernel,
  // one box, two rounds each, profiles/r06g_c2_rows_dma_ab.txt, r06h_c2_rows_dma_ab.txt): 4 / 5 / 6
  // k steps 68.17 / 67.68-67.82 / 68.21-68.26 ms per launch (KA's own intake starts to show at 6);
  // moving query k steps into LDS instead (0-4 of them, the rest of the budget CA) 67.7-68.6 ms
  static constexpr size_t GC = al16(KA > KB ? KA : KB);
  static constexpr int FREE_K = (int)((160 * 1024 - 256 - GC) / (8 * 2 * 1024));  // k steps of 16 KiB that fit
  static constexpr int GCK = 5 < FREE_K ? 5 : FREE_K;
  static constexpr size_t GC_BYTES = 8 * 2 * GCK * 1024;
  static_assert(KA <= 160 * 1024 - 256 && KB <= 160 * 1024 - 256 && KC <= 160 * 1024 - 256 &&
                    KE <= 160 * 1024 - 256 && GC + GC_BYTES <= 160 * 1024 - 256 && GCK >= 1, "row-block loop LDS");
};

// LDS-DMA of this wave's CA out-projection tiles 2 wave, 2 wave + 1, k steps 0 .. GCK - 1 (fragment
// [tile][k step][lane][16 B]) into the GC region: [wave][tile j][k step] x 1 KiB, lane l at 16 l.
// Written as asm: the compiler treats a builtin LDS-DMA as a store that may alias every later LDS
// access and drains it (vmcnt(0)) at the next one -- measured: KA's staging waited for the whole
// copy (+0.7 us).  hipcc does not count asm loads either, so nothing waits for these until the
// KA -> KB barrier's vmcnt drain (every load issued after them is drained there too).
__device__ __forceinline__ void glds16_asm(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
template <int NK>
__device__ __forceinline__ void w2_dma_range(const void* w, unsigned char* dst, int wave, int lane, int p0, int p1) {
  typedef __attribute__((address_space(3))) unsigned char lds_u8;
  const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_u8*)(dst + wave * 2 * NK * 1024));
#pragma unroll
  for (int q = 0; q < 2 * NK; ++q) {
    if (q < p0 || q >= p1) continue;
    const int j = q / NK, k = q % NK;
    glds16_asm((const char*)w + ((size_t)((2 * wave + j) * KT + k) * 64 + lane) * 16, base + (j * NK + k) * 1024);
  }
}
// this wave's two tiles' k step k from such a copy
template <int NK, int J>
__device__ __forceinline__ void w2_lds_step(WGemm<T, J, KT, 1>& g, const unsigned char* src, int wave, int lane, int k) {
#pragma unroll
  for (int j = 0; j < 2; ++j) g.wb[j][k] = *(const uint4*)(src + ((wave * 2 + j) * NK + k) * 1024 + lane * 16);
}

// 8 bytes through the global view
__device__ __forceinline__ uint2 ld_g8(const T* p) {
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
  const u32x2 v = *G((const u32x2*)p);
  return make_uint2(v.x, v.y);
}

// NR rows (tokens tk0 + r, clamped into [0, L)) of a bf16 [rows][256] block -> LDS image (stride SX)
template <int NR, int CP> struct RowsStage {
  static constexpr int NV = NR * 32 / FT;  // 16-byte pieces per thread
  static_assert(NR * 32 % FT == 0, "whole pieces per thread");
  uint4 v[NV];
  __device__ __forceinline__ void load(const T* src, int tk0, int L) {
    const int tid = ltid();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = tid + i * FT, r = idx >> 5, c = idx & 31;
      v[i] = ld_16B<CP>(src, (uint32_t)(sizeof(T) * ((size_t)min(max(tk0 + r, 0), L - 1) * FD + c * 8)));
    }
  }
  __device__ __forceinline__ void store(T* img) const {
    const int tid = ltid();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = tid + i * FT, r = idx >> 5, c = idx & 31;
      *(uint4*)(img + r * SX + c * 8) = v[i];
    }
  }
};

// LayerNorm without the affine (folded into the consuming Linear at finalize) of one 256-wide row
// held by a whole wave (lane: columns 4 lane .. + 3): sums over 16 lanes by DPP, then across the
// wave's 4 lane rows (ln_rows_wave's arithmetic)
__device__ __forceinline__ float4 ln_wave(const float4 v) {
  const float mu = lanerow_sum4(group_sum<16>((v.x + v.y) + (v.z + v.w))) * (1.0f / (float)FD);
  const float d0 = v.x - mu, d1 = v.y - mu, d2 = v.z - mu, d3 = v.w - mu;
  const float q = lanerow_sum4(group_sum<16>((d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3)));
  const float rs = __builtin_amdgcn_rsqf(q * (1.0f / (float)FD) + 1e-5f);
  return make_float4(d0 * rs, d1 * rs, d2 * rs, d3 * rs);
}

// LN of Hr rows [i0, i0 + n) into the LDS image rows of the same index (wave w: rows w, w + 8);
// the other rows of the 16-row image are zeros
__device__ __forceinline__ void ln16_img(const float* Hr, int i0, int n, T* img, int lane, int wave) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = wave + 8 * k;
    const bool on = i >= i0 && i < i0 + n;
    const float4 y = ln_wave(*(const float4*)(Hr + i * SH + 4 * lane));
    *(uint2*)(img + i * SX + 4 * lane) = on ? make_uint2(pk_bf16(y.x, y.y), pk_bf16(y.z, y.w)) : make_uint2(0u, 0u);
  }
}

// Hr row (1 + w) of the block, w < R (wave w), normalised -> global LN image row r0 + w
template <int CP>
__device__ __forceinline__ void ln_publish_row(const float* Hr, int R, T* img_rows, int lane, int wave) {
  if (wave >= R) return;  // wave-uniform
  const float4 y = ln_wave(*(const float4*)(Hr + (1 + wave) * SH + 4 * lane));
  const OutRowsP<CP> out(img_rows, (uint32_t)(sizeof(T) * R * FD));
  out.template put4v<T>((uint32_t)(wave * FD + 4 * lane), f32x4{y.x, y.y, y.z, y.w});
}

// ------------------------------------------------------------------------------------------
// KA: LN1 image -> QKV of head h + conv + self-attention (ka_phase without the residual rows)
// ------------------------------------------------------------------------------------------
// step(k): issued after the QKV GEMM's k step k (the next phases' weight streams, spread over the GEMM
// instead of issued in one batch in front of the GEMM / the attention: 67.78 -> 67.52 ms per C2
// launch with KE's emb loads behind LN_out, one box, profiles/r06l_c2_rows_issue_ab.txt); hook: after
// the attention
template <int RT, int CP, typename FA, typename H, typename HS, typename H0>
__device__ __forceinline__ void ka_rows(const FA& a, int h, int b, unsigned char* smem, Pre1<T, RT>& pre, H&& hook,
                                        HS&& step, H0&& hook0) {
  using RP = RowPlan<RT>;
  const int tid = ltid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = a.L, c16 = lane & 15, g4 = lane >> 4;
  T* Xn = (T*)(smem + RP::HR);
  unsigned char* att = smem + RP::HR + RP::XN;
  const auto& w = a.w;
  STAMP(0);
  RowsStage<RT * 16, CP> so;
  so.load((const T*)a.o_ca + (size_t)b * L * FD, 0, L);
  const int nq = wave < 6 ? 1 : 0;
  auto& gm = pre.g;
  const float4 bias = ld_f4(w.qkv_b + h * 96 + min(wave, 5) * 16 + 4 * g4);
  const int kind = min(wave, 5) >> 1, c0 = (wave & 1) * 16 + 4 * g4;
  ConvW cw[4];
  conv_w4(cw, kind == 0 ? w.sa_qw : kind == 1 ? w.sa_kw : w.sa_vw, kind == 0 ? w.sa_qb : kind == 1 ? w.sa_kb : w.sa_vb,
          c0);
  so.store(Xn);
  bar_lds();
  STAMP(1);
  // (the QKV GEMM's step hook issues KB's SA out-projection tile 0 and the LDS-DMA of most of KB's CA
  // out-projection weights: KB's operand intake is its bound, round 6)
  using AT = FAtt<T, RT * 16>;
  {
    f32x4 acc[RT][1];
    gm.template run_then<true>(acc, Xn, SX, lane, [&](int k) { step(k); }, nq);
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
  hook0();
  if (L <= 32)
    fattn<T, 2, RT * 16, false, CP>(att, L, L, a.scale, (T*)a.o_sa + (size_t)b * L * FD + h * FDK, FD);
  else
    fattn<T, 4, RT * 16, false, CP>(att, L, L, a.scale, (T*)a.o_sa + (size_t)b * L * FD + h * FDK, FD);
  asm volatile("" ::: "memory");  // the hook's loads stay behind every store above (mk_sync counts them)
  hook();
  STAMP_END(3);
}

// KB's SA out-projection tiles 2w, 2w + 1 (tile 0 issued inside KA's QKV GEMM, tile 1 after its
// attention) and its query tiles of head w (issued in KA before the attention, where the registers are
// free: C2 mr_kernel 67.87 -> 67.58 ms against streaming them into the registers KB's SA out-projection
// frees; 2 / 4 / 6 of the 8 k steps early: 68.6-68.9 / 68.5 / 68.0-68.2 ms, one box,
// profiles/r06n_c2_rows_qhead_ab.txt).  All of it lands before KB's staging does (vector loads
// complete in issue order), so it must be in flight early: KA's QKV GEMM and attention cover it.
struct KBRPre {
  WGemm<T, 2, KT, 1> go, gq;
  template <typename FA>
  __device__ __forceinline__ KBRPre(const FA& a, int wave) : go(a.w.o_sa, KT, 0), gq(a.w.q_ca, KT, 0) {
    go.tiles[0] = 2 * wave;
    go.tiles[1] = 2 * wave + 1;
    gq.tiles[0] = 2 * wave;
    gq.tiles[1] = 2 * wave + 1;
  }
  __device__ __forceinline__ void load_q(int lane) { gq.load(0, lane); }
  __device__ __forceinline__ void load_tile(int j, int lane) { go.load_tile(j, lane); }
  __device__ __forceinline__ void load_tile_step(int j, int k, int lane) {
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
    const u32x4 v = ggd::G((const u32x4*)go.W)[((size_t)go.tiles[j] * KT + k) * 64 + lane];
    go.wb[j][k] = make_uint4(v.x, v.y, v.z, v.w);
  }
  static constexpr int TILE_LOADS = decltype(go)::G;
};

// ------------------------------------------------------------------------------------------
// KB (rows p): SA out-proj + residual + LN2 + query (all heads) + conv + cross-attention +
// CA out-proj + residual + LN3 -> LN3 image rows.  Image row i of Hr / the operand images is token
// r0 - 1 + i: rows 1 .. R are the block, rows 0 and R + 1 its conv halo (recomputed here from the
// neighbours' published h rows), rows past R + 1 are don't-care (every GEMM is row-independent and
// every row that reaches a valid output is finite: staged rows are clamped copies).
// ------------------------------------------------------------------------------------------
template <int RT, int LKT, int CP, typename FA>
__device__ __forceinline__ void kb_rows(const FA& a, int p, int b, int t_orig, unsigned char* smem, KBRPre& pre) {
  using RP = RowPlan<RT>;
  const int tid = ltid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), c16 = lane & 15, g4 = lane >> 4;
  const int L = a.L, Ts = a.Ts, Lk = 1 + Ts;
  const int r0 = p * L / 8, R = (p + 1) * L / 8 - r0;
  float* Hr = (float*)smem;
  T* Oi = (T*)(smem + RP::HR);                 // o_sa rows, then the cross-attention output rows
  T* Xi = (T*)(smem + RP::HR + RP::IMG16);     // LN2 image
  float* fix = (float*)(smem + RP::HR + 2 * RP::IMG16) + wave * 128;  // head w: K [2][32], V [32][2]
  float4* cqs = (float4*)(smem + RP::HR + 2 * RP::IMG16 + RP::FIX);    // query conv taps [32]
  const auto& w = a.w;
  const size_t row0 = (size_t)b * L;
  STAMP(0);
  // ---- loads, in the order they are needed (vector loads retire in issue order, so a load issued
  // behind a weight stream is not usable before the whole stream has landed): the staging, then the
  // small operands of LN2 / the step-token fix / the query epilogue, the memory K / V fragments and
  // last the CA out-projection weights not in LDS (round 5 issued the conv taps behind the query
  // weight stream: the SA out-projection segment waited for it, 3.3 us)
  RowsStage<16, CP> so;
  so.load((const T*)a.o_sa + row0 * FD, r0 - 1, L);
  const int hs = (tid >> 6) & 1, hc = 4 * (tid & 63);  // halo residual rows: tokens r0 - 1 / r1 (tid < 128)
  const uint4 hv = ld_16B<CP>(a.h, (uint32_t)(sizeof(float) * ((row0 + min(max(hs ? r0 + R : r0 - 1, 0), L - 1)) * FD + hc)));
  float4 bo[2];
  bo[0] = ld_f4(w.o_sa_b + (2 * wave) * 16 + 4 * g4);
  bo[1] = ld_f4(w.o_sa_b + (2 * wave + 1) * 16 + 4 * g4);
  // memory rows 0 / 1 of head w see the step token through the conv: lane l fixes K (l < 32) or V
  // (l >= 32) channel l & 31 (KvFix's arithmetic); t_orig comes from the step loop (one load per step)
  KvFix fx;
  fx.load(w.kv_step + (size_t)t_orig * 2 * FD, w.kv_mem + (size_t)b * Ts * 2 * FD, Ts, wave, lane);
  const ConvW ckv = conv_w(lane < 32 ? w.ca_kw : w.ca_vw, lane < 32 ? w.ca_kb : w.ca_vb, lane & 31);
  const ConvW cqv = conv_w(w.ca_qw, w.ca_qb, tid & 31);  // (stored by threads 0-31)
  float4 bq[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bq[j] = ld_f4(w.q_ca_b + wave * FDK + j * 16 + 4 * g4);
  __builtin_amdgcn_sched_barrier(0);  // the staging and the small operands first: loads retire in issue order
  so.store(Oi);
  if (tid < 128) *(uint4*)(Hr + (hs ? R + 1 : 0) * SH + hc) = hv;
  bar_lds();
  STAMP(1);
  // ---- SA out-projection + residual (rows 0 .. 15); the query tiles of head w (q_ca tiles 2w, 2w + 1)
  // were issued in KA
  auto& gq = pre.gq;
  residual_gemm<T, KT, 2, 1>(Hr, Oi, SX, pre.go, bo, lane, wave);
  // memory K / V^T fragments of head w (kvc block: K [64][32] | V^T [32][64], keys 0 / 1 zero): the
  // lane's query dims are {4 g4 .. + 3} u {16 + 4 g4 .. + 3} (the transposed query GEMM's lane map),
  // so its K fragment holds those dims of key 16 t + c16 -- the contraction runs in that order
  const T* kvh = (const T*)w.kvc + ((size_t)b * (FD / FDK) + wave) * KVC_ELEMS;
  uint2 kf[LKT][2], vf[2][LKT];
#pragma unroll
  for (int t = 0; t < LKT; ++t) {
    kf[t][0] = ld_g8(kvh + (t * 16 + c16) * FDK + 4 * g4);
    kf[t][1] = ld_g8(kvh + (t * 16 + c16) * FDK + 16 + 4 * g4);
  }
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int t = 0; t < LKT; ++t) vf[ct][t] = ld_g8(kvh + FLK * FDK + (ct * 16 + c16) * FLK + t * 16 + 4 * g4);
  if (tid < FDK) cqs[tid] = make_float4(cqv.w0, cqv.w1, cqv.w2, cqv.b);
  bar_lds();
  STAMP(2);
  // ---- LN2 of rows 0 .. R + 1; the step-token rows of head w's memory K / V (wave-local LDS)
  ln16_img(Hr, 0, R + 2, Xi, lane, wave);
  {
    const float v0 = conv3(ckv, 0.f, fx.m0, Lk > 1 ? fx.m1 : 0.f), v1 = conv3(ckv, fx.m0, fx.m1, Lk > 2 ? fx.m2 : 0.f);
    if (lane < 32) {
      fix[lane] = v0;
      fix[32 + lane] = v1;
    } else {
      *(float2*)(fix + 64 + 2 * (lane - 32)) = make_float2(v0, v1);
    }
  }
  bar_lds();
  STAMP(3);
  // ---- query of head w (transposed: lane = image row c16, channels 16 j + 4 g4 ..) + conv over tokens
  // the CA out-projection tiles go into the query's registers as the query GEMM frees them: k steps
  // < GCK from the LDS copy KA made, the rest streamed from L2, in flight across the conv and the attention
  f32x4 q[1][2];
  WGemm<T, 2, KT, 1> gc(w.o_ca, KT, 0);
  gc.tiles[0] = 2 * wave;
  gc.tiles[1] = 2 * wave + 1;
  gq.template run_then<true>(q, Xi, SX, lane, [&](int k) {
    if (k < RP::GCK) w2_lds_step<RP::GCK>(gc, smem + RP::GC, wave, lane, k);  // DMA'd in KA (drained by the KA -> KB barrier)
    else gc.load_step(k, lane);
  });
  {
    constexpr int ROR1 = 0x121, ROR15 = 0x12F;  // lanes c16 - 1 / c16 + 1 of the 16-lane row
    const int tk = r0 - 1 + c16;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float4 bb = bq[j];
      f32x4 v = f32x4{q[0][j][0] + bb.x, q[0][j][1] + bb.y, q[0][j][2] + bb.z, q[0][j][3] + bb.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float4 cw = cqs[j * 16 + 4 * g4 + r];
        float pv = dpp_mov<ROR1>(v[r]), nv = dpp_mov<ROR15>(v[r]);
        pv = tk >= 1 ? pv : 0.f;
        nv = tk + 1 < L ? nv : 0.f;
        q[0][j][r] = conv3(ConvW{cw.x, cw.y, cw.z, cw.w}, pv, v[r], nv);
      }
    }
  }
  // the step-token fix of the K / V^T fragments (key tile 0: keys 0 / 1)
  if (c16 < 2) {
    const float4 a0 = *(const float4*)(fix + c16 * 32 + 4 * g4), a1 = *(const float4*)(fix + c16 * 32 + 16 + 4 * g4);
    kf[0][0] = make_uint2(pk_bf16(a0.x, a0.y), pk_bf16(a0.z, a0.w));
    kf[0][1] = make_uint2(pk_bf16(a1.x, a1.y), pk_bf16(a1.z, a1.w));
  }
  if (g4 == 0) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const float2 f = *(const float2*)(fix + 64 + 2 * (ct * 16 + c16));
      vf[ct][0].x = pk_bf16(f.x, f.y);
    }
  }
  // the CA out-projection's bias (its loads complete under the attention)
  float4 bc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bc[j] = ld_f4(w.o_ca_b + (2 * wave + j) * 16 + 4 * g4);
  // ---- cross-attention of head w for the 16 image rows (fattn_regp with Q, K, V^T in registers)
  {
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    const uint4 qu = make_uint4(pk_bf16(q[0][0][0], q[0][0][1]), pk_bf16(q[0][0][2], q[0][0][3]),
                                pk_bf16(q[0][1][0], q[0][1][1]), pk_bf16(q[0][1][2], q[0][1][3]));
    const bf16x8 qf = __builtin_bit_cast(bf16x8, qu);
    f32x4 s[LKT];
#pragma unroll
    for (int t = 0; t < LKT; ++t) {
      const uint4 ku = make_uint4(kf[t][0].x, kf[t][0].y, kf[t][1].x, kf[t][1].y);
      s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ku), qf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
    const float sl2 = a.scale * 1.4426950408889634f;
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
    for (int t = 0; t < LKT; ++t)
      pb[t] = __builtin_bit_cast(s16x4, make_uint2(pk_bf16(s[t][0] * inv, s[t][1] * inv), pk_bf16(s[t][2] * inv, s[t][3] * inv)));
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < LKT; ++t) o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, vf[ct][t]), pb[t], o, 0, 0, 0);
      *(uint2*)(Oi + c16 * SX + wave * FDK + ct * 16 + 4 * g4) = make_uint2(pk_bf16(o[0], o[1]), pk_bf16(o[2], o[3]));
    }
  }
  bar_lds();
  STAMP(4);
  // ---- CA out-projection + residual, LN3 of the block's rows -> LN3 image rows
  residual_gemm<T, KT, 2, 1>(Hr, Oi, SX, gc, bc, lane, wave);
  bar_lds();
  ln_publish_row<CP>(Hr, R, (T*)a.o_ca + (row0 + r0) * FD, lane, wave);
  STAMP_END(5);
}

// KC's FFN-up tile (8 c + w), prefetched at the barrier in front of it
template <int RT> struct KCRPre {
  WGemm<T, 1, KT, RT> gf;
  template <typename FA>
  __device__ __forceinline__ KCRPre(const FA& a, int c, int wave) : gf(a.w.ff1, KT, 0) {
    gf.tiles[0] = 8 * c + wave;
  }
  __device__ __forceinline__ void load(int lane) { gf.load(0, lane); }
};

// ------------------------------------------------------------------------------------------
// KC (chunk c): LN3 image -> FFN-up chunk + ReLU^2 (in LDS) -> its FFN-down partial (kc_phase's tail)
// ------------------------------------------------------------------------------------------
template <int RT, int CP, typename FA>
__device__ __forceinline__ void kc_rows(const FA& a, int c, int b, unsigned char* smem, KCRPre<RT>& pre) {
  using RP = RowPlan<RT>;
  const int tid = ltid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = a.L, c16 = lane & 15, g4 = lane >> 4;
  T* Ax = (T*)(smem + RP::HR);
  T* Hc = (T*)(smem + RP::HR + RP::XN);
  const auto& w = a.w;
  const int h = c;  // STAMP uses (h, b)
  (void)h;
  STAMP(0);
  RowsStage<RT * 16, CP> so;
  so.load((const T*)a.o_ca + (size_t)b * L * FD, 0, L);
  constexpr int KC = 128 / Frag<T>::KF, KTT = 4 * FD / Frag<T>::KF, SHC = 128 + Frag<T>::PT;
  WGemm<T, 2, KC, RT> gd(w.ff2, KTT, c * KC);  // in flight across FFN-up
  gd.tiles[0] = 2 * wave;
  gd.tiles[1] = 2 * wave + 1;
  gd.load(0, lane);
  const float4 bf = ld_f4(w.ff1_b + (8 * c + wave) * 16 + 4 * g4);
  so.store(Ax);
  bar_lds();
  STAMP(1);
  {
    f32x4 acc[RT][1];
    pre.gf.template run<true>(acc, Ax, SX, lane);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const float v0 = fmaxf(acc[rt][0][0] + bf.x, 0.f), v1 = fmaxf(acc[rt][0][1] + bf.y, 0.f);
      const float v2 = fmaxf(acc[rt][0][2] + bf.z, 0.f), v3 = fmaxf(acc[rt][0][3] + bf.w, 0.f);
      put_tok4<T, false>(Hc, SHC, rt * 16 + c16, wave * 16 + 4 * g4, f32x4{v0 * v0, v1 * v1, v2 * v2, v3 * v3});
    }
  }
  bar_lds();
  STAMP(2);
  {
    f32x4 acc[RT][2];
    gd.template run<true>(acc, Hc, SHC, lane);
    const OutRowsP<CP> out((T*)a.ffp + ((size_t)b * 8 + c) * L * FD, (uint32_t)(sizeof(T) * L * FD));
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        out.template put4v<T>((uint32_t)((rt * 16 + c16) * FD + (2 * wave + j) * 16 + 4 * g4), acc[rt][j]);
  }
  STAMP_END(3);
}

// ------------------------------------------------------------------------------------------
// KD (rows p): h = x2 + (sum of the 8 FFN-down partials in chunk order + b2) for the block's rows,
// wave w = row r0 + w, lane = 4 columns: h rows -> global (the neighbours' KB halo) and Hr (this
// workgroup's next KB); LN1 of the next layer in registers -> LN1 image row.  No LDS barrier.
// ------------------------------------------------------------------------------------------
template <int CP, typename FA>
__device__ __forceinline__ void kd_rows(const FA& a, int p, int b, unsigned char* smem) {
  const int tid = ltid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = a.L, r0 = p * L / 8, R = (p + 1) * L / 8 - r0;
  const int h = p;  // STAMP uses (h, b)
  (void)h;
  STAMP(0);
  if (wave >= R) return;  // wave-uniform
  float* Hr = (float*)smem;
  const size_t row0 = (size_t)b * L;
  const int row = r0 + wave, col = 4 * lane;
  float4 part[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint2 u = ld_8B<CP>(a.ffp, (uint32_t)(sizeof(T) * ((((size_t)b * 8 + c) * L + row) * FD + col)));
    part[c] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                          __uint_as_float(u.y & 0xffff0000u));
  }
  const float4 bias = ld_f4(a.w.ff2_b + col);
  const float4 res = *(const float4*)(Hr + (1 + wave) * SH + col);
  float4 y = part[0];
#pragma unroll
  for (int c = 1; c < 8; ++c) {
    y.x += part[c].x;
    y.y += part[c].y;
    y.z += part[c].z;
    y.w += part[c].w;
  }
  const float4 hn = make_float4(res.x + (y.x + bias.x), res.y + (y.y + bias.y), res.z + (y.z + bias.z), res.w + (y.w + bias.w));
  *(float4*)(Hr + (1 + wave) * SH + col) = hn;
  const OutRowsP<CP> ho(a.h + (row0 + r0) * FD, (uint32_t)(sizeof(float) * R * FD));
  ho.put4((uint32_t)(wave * FD + col), hn);
  const float4 n = ln_wave(hn);
  const OutRowsP<CP> xo((T*)a.o_ca + (row0 + r0) * FD, (uint32_t)(sizeof(T) * R * FD));
  xo.template put4v<T>((uint32_t)(wave * FD + col), f32x4{n.x, n.y, n.z, n.w});
  STAMP(1);
}

// The emb rows of the block (emb_rows_store's GEMM) also into Hr rows 1 .. R, then LN1 of them into
// the LN1 image rows (the first step's prologue and KE)
template <int CP, typename FA>
__device__ __forceinline__ void emb_rows_publish(const FA& fe, T* xn, int b, int r0, int R, const T* Xb,
                                                 WGemm<T, 2, 128 / Frag<T>::KF, 1>& ge, const float4 (&pe)[2], float* Hr,
                                                 int lane, int wave) {
  const int c16 = lane & 15, g4 = lane >> 4;
  f32x4 acc[1][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) acc[0][j] = f32x4{pe[j].x, pe[j].y, pe[j].z, pe[j].w};
  ge.template run<true>(acc, Xb, KerPlan<T>::SB, lane, 2, false);
  const OutRowsP<CP> ho(fe.h + ((size_t)b * fe.L + r0) * FD, (uint32_t)(sizeof(float) * R * FD));  // rows >= R dropped
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = (2 * wave + j) * 16 + 4 * g4;
    const float4 v = make_float4(acc[0][j][0], acc[0][j][1], acc[0][j][2], acc[0][j][3]);
    ho.put4((uint32_t)(c16 * FD + col), v);
    if (c16 < R) *(float4*)(Hr + (1 + c16) * SH + col) = v;
  }
  bar_lds();
  ln_publish_row<CP>(Hr, R, xn + ((size_t)b * fe.L + r0) * FD, lane, wave);
}

// the first step's layer-0 rows: emb_prologue's arithmetic + Hr + LN1 image
template <int RT, int CP, typename FA>
__device__ __forceinline__ void emb_prologue_rows(const FA& a, T* xn, int p, int b, unsigned char* smem) {
  using KP = KerPlan<T>;
  using RP = RowPlan<RT>;
  constexpr int KTE = 128 / Frag<T>::KF;
  const int tid = ltid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = a.L, C = a.C, r0 = p * L / 8, R = (p + 1) * L / 8 - r0;
  float* Hr = (float*)smem;
  T* Xb = (T*)(smem + RP::HR + KP::HS + KP::XN + KP::E);
  WGemm<T, 2, KTE, 1> ge(a.w_emb, KTE, 0);
  ge.tiles[0] = 2 * wave;
  ge.tiles[1] = 2 * wave + 1;
  ge.load(0, lane);
  float4 pe[2];
  emb_init(a, r0, lane, wave, pe);
  float xv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + i * FT, l = idx >> 7, c = idx & 127;
    xv[i] = ld_f32<CP>(a.x, (uint32_t)(((size_t)b * L + r0 + min(l, R - 1)) * C + min(c, C - 1)));
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + i * FT, l = idx >> 7, c = idx & 127;
    Xb[l * KP::SB + c] = from_f32<T>(l < R && c < C ? xv[i] : 0.f);
  }
  __syncthreads();
  emb_rows_publish<CP>(a, xn, b, r0, R, Xb, ge, pe, Hr, lane, wave);
}

// ------------------------------------------------------------------------------------------
// KE (rows p): ker_phase (ggd_phases.h) with the residual rows from Hr, and the next step's layer-0
// rows also into Hr + LN1 image
// ------------------------------------------------------------------------------------------
template <int RT, int CP, typename FA>
__device__ __forceinline__ void ke_rows(const FA& a, T* xn, int p, int b, int k, unsigned char* smem, Pre1<T, RT>& pre) {
  using KP = KerPlan<T>;
  using RP = RowPlan<RT>;
  constexpr int KTE = 128 / Frag<T>::KF, SE = KP::SE, SB = KP::SB;
  const int tid = ltid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = a.L, C = a.C, c16 = lane & 15, g4 = lane >> 4, LC = L * C;
  const int r0 = p * L / 8, R = (p + 1) * L / 8 - r0;
  float* Hr = (float*)smem;
  unsigned char* kb = smem + RP::HR;
  float* Hs = (float*)kb;
  T* Xn = (T*)(kb + KP::HS);
  float* E = (float*)(kb + KP::HS + KP::XN);
  T* Xb = (T*)(kb + KP::HS + KP::XN + KP::E);
  const size_t row0 = (size_t)b * L;
  const int h = p;  // STAMP uses (h, b)
  (void)h;
  STAMP(0);
  // the last layer's KD for the block's rows (kd_rows' arithmetic): thread (row si = tid / 64, columns sc)
  const int si = tid >> 6, sc = 4 * (tid & 63), srow = r0 + min(si, max(R - 1, 0));
  float4 part[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint2 u = ld_8B<CP>(a.ffp, (uint32_t)(sizeof(T) * ((((size_t)b * 8 + c) * L + srow) * FD + sc)));
    part[c] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                          __uint_as_float(u.y & 0xffff0000u));
  }
  const float4 sres = *(const float4*)(Hr + (1 + min(si, 15)) * SH + sc);
  const float4 sb2 = ld_f4(a.ff2_b + sc);
  WGemm<T, 1, KT, 1> go(a.w_out, KT, 0);  // wave w: channel tile w (prefetched at the barrier)
  go.tiles[0] = wave;
#pragma unroll
  for (int kk = 0; kk < KT; ++kk) go.wb[0][kk] = pre.g.wb[0][kk];
  const float4 bo = ld_f4(a.b_out + wave * 16 + 4 * g4);
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
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + i * FT, l = idx >> 7, c = idx & 127;
    if (l >= R || c >= C) Xb[l * SB + c] = from_f32<T>(0.f);
  }
  __syncthreads();
  STAMP(1);
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
  STAMP(2);
  WGemm<T, 2, KTE, 1> ge(a.w_emb, KTE, 0);
  ge.tiles[0] = 2 * wave;
  ge.tiles[1] = 2 * wave + 1;
  float4 pe[2];
  emb_init(a, r0, lane, wave, pe);
  ln_rows_wave<T>(Hs, R, Xn, lane, wave);
  ge.load(0, lane);
  bar_lds();
  STAMP(3);
  if (16 * wave < C) {
    f32x4 acc[1][1];
    go.template run<true>(acc, Xn, SX, lane);
    *(float4*)(E + c16 * SE + 16 * wave + 4 * g4) =
        make_float4(acc[0][0][0] + bo.x, acc[0][0][1] + bo.y, acc[0][0][2] + bo.z, acc[0][0][3] + bo.w);
  }
  if (qon && !a.noise)
    philox_normal4(((uint64_t)rec.seed_hi << 32) | rec.seed_lo, rec.clip_offset + (uint32_t)b, (uint32_t)rec.i,
                   TAG_STEP, (uint32_t)qi, zq);
  bar_lds();
  STAMP(4);
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
  STAMP(5);
  emb_rows_publish<CP>(a, xn, b, r0, R, Xb, ge, pe, Hr, lane, wave);
  STAMP_END(6);
}

template <int RT, int LKT, int CPV>
__global__ void __launch_bounds__(FT) mr_kernel(MegaArgs m, int G) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int s_role, s_ok;
  if (m.gate && ggd::G(m.gate)[0] != 3) return;  // gated re-run: the XCD-local launch placed (or failed otherwise)
  if (m.sim_unresident == 1) {  // test hook: as if the workgroups were never all resident
    if (threadIdx.x == 0) atomicMax(m.status, 2);
    return;
  }
  if (threadIdx.x == 0) s_role = CPV == CP_XL ? mk_role_xl(m, gridDim.x, G) : mk_role(m, gridDim.x);
  __syncthreads();
  const int role = s_role;
  if (role < 0) return;
  if (m.sim_unresident == 2 && (role & 1)) {  // test hook: odd parts report 2, the rest wait in a barrier
    if (threadIdx.x == 0) atomicMax(m.status, 2);
    return;
  }
  const int grp = role >> 3, b = m.clip0 + grp, part = role & 7, lane = ltid() & 63, wave = __builtin_amdgcn_readfirstlane(ltid() >> 6);
  unsigned* ctr = m.ctl + MK_GROUP + grp * 16;
  unsigned* flags = m.ctl + MK_FLAGS + grp * 32;
  unsigned epoch = 0;
  if (m.stamps && role == 0 && threadIdx.x == 0) m.stamps[2 * 17 * MEGA_STAMP_STEPS] = __builtin_amdgcn_s_memtime();
  typedef const __attribute__((address_space(4))) FusedArgs* cfa_t;
  typedef const __attribute__((address_space(4))) FinalArgs* cfe_t;
  const int NL = m.n_layers;
  cfa_t fa0 = (cfa_t)m.fa;
  cfe_t fe = (cfe_t)m.fe;
  T* xn = (T*)fa0[0].o_ca;  // the LN1 / LN3 image rows
  emb_prologue_rows<RT, CPV>(*fe, xn, part, b, smem);
  Pre1<T, RT> pn = ka_pre<T, RT>(fa0[0], part, wave);
  if (!mk_sync<CPV>(ctr, flags, part, ++epoch, m.status, &s_ok, nullptr, [&] { pn.load(lane); })) return;
  for (int k = 0; k < m.n_steps; ++k) {
    const int it = m.k0 + k;
    unsigned long long* st = (m.stamps && role == 0 && k < MEGA_STAMP_STEPS) ? m.stamps : nullptr;
    unsigned long long* ar = (m.stamps && grp == 0 && k < MEGA_STAMP_STEPS) ? m.stamps + 2 * 17 * MEGA_STAMP_STEPS + 1 : nullptr;
    // the step token's original t (KB's memory-row fix): one load per step
    const int t_orig = __builtin_amdgcn_readfirstlane(fa0[0].t_clip ? ggd::G(fa0[0].t_clip)[b] : ggd::G(fa0[0].steps)[it].t_orig);
    for (int li = 0; li < NL; ++li) {
      cfa_t f = fa0 + 4 * li;
      asm volatile("" : "+s"(f));  // per-layer arguments are re-read, not held across the loop
      KBRPre pb(f[0], wave);
      ka_rows<RT, CPV>(f[0], part, b, smem, pn, [&] { pb.load_tile(1, lane); },
                       [&](int k) {  // QKV k step k: the LDS-DMA pieces of it and tile 0's k step k
                         constexpr int NP = 2 * RowPlan<RT>::GCK;
                         w2_dma_range<RowPlan<RT>::GCK>(f[0].w.o_ca, smem + RowPlan<RT>::GC, wave, lane, k * NP / 8,
                                                        (k + 1) * NP / 8);
                         pb.load_tile_step(0, k, lane);
                       },
                       [&] { pb.load_q(lane); });
      if (!mk_sync<CPV, KBRPre::TILE_LOADS>(ctr, flags, part, ++epoch, m.status, &s_ok, st, [] {}, ar)) return;
      // (the four per-layer argument blocks differ only in h / h_out, which these phases read as f[1] /
      // f[3] hold them: h; and in the phase-stamp pointer of the diagnostics)
      kb_rows<RT, LKT, CPV>(f[1], part, b, t_orig, smem, pb);
      KCRPre<RT> pc(f[0], part, wave);
      if (!mk_sync<CPV>(ctr, flags, part, ++epoch, m.status, &s_ok, st, [&] { pc.load(lane); }, ar)) return;
      kc_rows<RT, CPV>(f[2], part, b, smem, pc);
      // the next phase after KD / KE is a KA: its QKV tile (or KE's output tile) is issued here, in
      // flight across the short KD
      pn = li + 1 < NL ? ka_pre<T, RT>(f[4], part, wave) : ker_pre<T, RT>(*fe, wave);
      if (!mk_sync<CPV>(ctr, flags, part, ++epoch, m.status, &s_ok, st, [&] { pn.load(lane); }, ar)) return;
      if (li + 1 < NL) {
        kd_rows<CPV>(f[3], part, b, smem);
        if (!mk_sync<CPV>(ctr, flags, part, ++epoch, m.status, &s_ok, st, [] {}, ar)) return;
      }
    }
    ke_rows<RT, CPV>(*fe, xn, part, b, it, smem, pn);
    pn = ka_pre<T, RT>(fa0[0], part, wave);
    if (!mk_sync<CPV>(ctr, flags, part, ++epoch, m.status, &s_ok, st, [&] { pn.load(lane); }, ar)) return;
  }
}

constexpr size_t MR_LDS = 160 * 1024 - 256;  // one workgroup per CU, as the head / chunk loop

template <int RT, int LKT>
hipError_t launch_rows_t(const MegaArgs& a, int n, bool xl, hipStream_t s) {
  const int G = n, nwg = xl ? 64 * ((G + 7) / 8) : 8 * G;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)mr_kernel<RT, LKT, CP_XL>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)mr_kernel<RT, LKT, CP_COH>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
    attr = true;
  }
  if (xl)
    hipLaunchKernelGGL((mr_kernel<RT, LKT, CP_XL>), dim3(nwg), dim3(FT), MR_LDS, s, a, G);
  else
    hipLaunchKernelGGL((mr_kernel<RT, LKT, CP_COH>), dim3(nwg), dim3(FT), MR_LDS, s, a, G);
  return hipGetLastError();
}

}  // namespace

// shapes the row-block loop runs: bf16, every part owns >= 1 row, <= 8 rows (one 16-row tile with
// the halo), memory keys <= 64
bool rows_supported(int dtype, int L, int Ts) { return dtype != 0 && L >= 8 && L <= 64 && 1 + Ts <= 64; }

hipError_t launch_rows(int dtype, int L, int Ts, const MegaArgs& a, int n, bool xl, hipStream_t s) {
  if (!rows_supported(dtype, L, Ts) || n < 1 || n > mega_capacity(dtype, L)) return hipErrorInvalidValue;
  if (xl && (a.placement != 0 || 64 * ((n + 7) / 8) > 8 * mega_capacity(dtype, L))) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(a.ctl, 0, sizeof(unsigned) * MEGA_CTL_WORDS, s);
  if (e != hipSuccess) return e;
  const bool rt3 = L <= 48, k2 = 1 + Ts <= 32;
  if (rt3) return k2 ? launch_rows_t<3, 2>(a, n, xl, s) : launch_rows_t<3, 4>(a, n, xl, s);
  return k2 ? launch_rows_t<4, 2>(a, n, xl, s) : launch_rows_t<4, 4>(a, n, xl, s);
}

}  // namespace ggd
