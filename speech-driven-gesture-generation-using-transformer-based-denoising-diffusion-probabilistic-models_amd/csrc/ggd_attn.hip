// ggd_attn.hip -- whole-clip attention for long clips (gfx950, bf16): one workgroup per
// (head, clip) with one wave per 16-query tile.
//
// MultiHeadAttention with the Primer-EZ depthwise convs (models/modules/transformer.py:19-44,
// 88-118).  The query-split kernel (ggd_kernels.hip attn_q_kernel) gives each 64-query block its
// own workgroup, so at L = 160 every (head, clip) stages and convolves its K and V three times
// and runs four waves over 16-query tiles; here the clip's Q, K and V are staged once, each of
// the NW waves owns one 16-query tile, and the softmax exponentials run on v_exp_f32
// (exp2 of a log2(e)-scaled argument) instead of the libm expf sequence.
//
//   staging   thread t: channel vector t % 4 (8 channels, 16 bytes of bf16), a strip of
//             consecutive rows; all loads of Q, K and V issue before the first conv
//   per wave  S = Q K^T (MFMA 16x16x32, 16 x Lk_pad in registers), row softmax on the
//             accumulator layout (DPP reductions over the 16 lanes of a row), P to the wave's
//             LDS tile, O = P V (MFMA over 32-key steps), bf16 rows out
#include "ggd_common.h"
#include "ggd_cliptiles.h"

namespace ggd {
namespace {

constexpr int AC_NW = 10;            // waves: one 16-query tile each at L = 160
constexpr int AC_NT = 64 * AC_NW;
constexpr int AC_DK = 32;            // head width (d_model 256 / 8 heads)
constexpr int AC_VPR = AC_DK / 8;    // 16-byte channel vectors per row
constexpr int AC_NS = AC_NT / AC_VPR;  // row strips
constexpr int AC_SQ = AC_DK + 8;     // Q / K row stride (bf16, 16-byte pad)

struct AcGeom {
  int Lqp, Lkp, SV, SP;
  size_t off_k, off_v, off_p, off_w, total;
};

__host__ __device__ inline AcGeom ac_geom(int Lq, int Lk) {
  AcGeom g;
  g.Lqp = (Lq + 15) / 16 * 16;
  g.Lkp = (Lk + 31) / 32 * 32;           // P V runs 32-key MFMA steps
  g.SV = g.Lkp + 8;
  g.SP = g.Lkp + 8;
  g.off_k = 2 * (size_t)g.Lqp * AC_SQ;
  g.off_v = g.off_k + 2 * (size_t)g.Lkp * AC_SQ;
  g.off_p = g.off_v + 2 * (size_t)AC_DK * g.SV;
  g.off_w = g.off_p + 2 * (size_t)AC_NW * 16 * g.SP;
  g.total = g.off_w + sizeof(float) * 12 * AC_DK;  // conv taps of Q, K, V: [3][w0, w1, w2, b][DK]
  return g;
}

// 8 channels (one 16-byte bf16 vector, or 32 bytes of f32) of conv-input row j as f32; rows
// outside [0, len) are the conv's zero padding.  Self mode: bf16 rows base[(row0 + j) ld + col];
// memory mode (step_row set): j = 0 the f32 step-token row, j >= 1 f32 rows base[(row0 + j - 1) ld + col].
struct AcSrc {
  const void* base;
  size_t row0;
  int ld, col, len;
  const float* step_row;
  // the load is always issued (on a clamped row) and the value selected after, so the loads of a
  // strip are in flight together (a load under a divergent branch is waited for before the join)
  __device__ __forceinline__ void load(int j, int cv, float (&o)[8]) const {
    const bool in = j >= 0 && j < len;
    const int jj = in ? j : 0;
    if (step_row) {  // uniform
      const float* p = jj == 0 ? step_row + cv * 8 : (const float*)base + (row0 + jj - 1) * (size_t)ld + col + cv * 8;
      const float4 u = *(const float4*)p, v = *(const float4*)(p + 4);
      const float t[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = in ? t[e] : 0.f;
    } else {
      const uint4 u = *(const uint4*)((const bf16_t*)base + (row0 + jj) * (size_t)ld + col + cv * 8);
      const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        o[2 * q] = in ? __uint_as_float(w[q] << 16) : 0.f;
        o[2 * q + 1] = in ? __uint_as_float(w[q] & 0xffff0000u) : 0.f;
      }
    }
  }
};

constexpr int AC_SLMAX = (ATT_LMAX + AC_NS - 1) / AC_NS;   // rows per strip (2 at 192 rows)

// a thread's strip: rows sid * sl - 1 .. sid * sl + sl of channel vector cv (halo included)
struct AcStrip {
  float x[AC_SLMAX + 2][8];
  int sl, rows;
  __device__ __forceinline__ void load(const AcSrc& src, int rows_) {
    rows = rows_;
    sl = (rows + AC_NS - 1) / AC_NS;
    const int cv = (int)threadIdx.x % AC_VPR, sid = (int)threadIdx.x / AC_VPR;
#pragma unroll
    for (int s = 0; s < AC_SLMAX + 2; ++s)
      if (s < sl + 2) src.load(sid * sl - 1 + s, cv, x[s]);
  }
  // out[i] = b + w0 in[i-1] + w1 in[i] + w2 in[i+1] (transformer.py:28-44); wl = [w0|w1|w2|b][DK]
  template <bool TRANS>
  __device__ __forceinline__ void conv(bf16_t* dst, int S, const float* wl) const {
    const int cv = (int)threadIdx.x % AC_VPR, sid = (int)threadIdx.x / AC_VPR;
#pragma unroll
    for (int s = 0; s < AC_SLMAX; ++s) {
      const int r = sid * sl + s;
      if (s >= sl || r >= rows) continue;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = cv * 8 + e;
        const float v = wl[3 * AC_DK + c] + wl[c] * x[s][e] + wl[AC_DK + c] * x[s + 1][e] + wl[2 * AC_DK + c] * x[s + 2][e];
        if (TRANS)
          dst[c * S + r] = f2bf(v);
        else
          dst[r * S + c] = f2bf(v);
      }
    }
  }
};

// one wave's 16-query tiles with LKT 16-key tiles (Lk padded to 32) fixed at compile time: every
// LDS fragment of a matrix product is read before its MFMAs
template <int LKT>
__device__ __forceinline__ void ac_tiles(const bf16_t* Qm, const bf16_t* Km, const bf16_t* Vt, bf16_t* P, int SV, int SP,
                                         int Lq, int Lk, float sl2, bf16_t* out, int ldo, int wave, int lane) {
  clip_attn_tiles<LKT, AC_NW, AC_SQ>(Qm, Km, Vt, P, SV, SP, Lq, Lk, sl2, out, ldo, wave, lane);
}

__global__ void __launch_bounds__(AC_NT) attn_clip_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int h = blockIdx.x, b = blockIdx.y, Lq = a.Lq, Lk = a.Lk;
  const AcGeom G = ac_geom(Lq, Lk);
  bf16_t* Qm = (bf16_t*)smem;
  bf16_t* Km = (bf16_t*)(smem + G.off_k);
  bf16_t* Vt = (bf16_t*)(smem + G.off_v);
  float* wl = (float*)(smem + G.off_w);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t row0 = (size_t)b * Lq;

  AcSrc sq{a.q, row0, a.ldq, h * AC_DK, Lq, nullptr};
  AcSrc sk{a.k, row0, a.ldkv, h * AC_DK, Lk, nullptr};
  AcSrc sv{a.v, row0, a.ldkv, h * AC_DK, Lk, nullptr};
  if (a.cross) {  // memory row 0 = the step token of this clip's t; rows 1.. = cached speech K|V
    const int t = a.t_clip ? a.t_clip[b] : a.steps[*a.step_counter].t_orig;
    const float* r0 = a.kv_step + (size_t)t * 2 * a.d;
    const size_t mrow0 = (size_t)b * (Lk - 1);
    sk = AcSrc{a.kv_mem, mrow0, 2 * a.d, h * AC_DK, Lk, r0 + h * AC_DK};
    sv = AcSrc{a.kv_mem, mrow0, 2 * a.d, a.d + h * AC_DK, Lk, r0 + a.d + h * AC_DK};
  }
  AcStrip xq, xk, xv;  // every load of the three strips in flight together
  xq.load(sq, Lq);
  xk.load(sk, Lk);
  xv.load(sv, Lk);
  {  // conv taps; zero K rows and V^T columns in [Lk, Lk_pad) (P V multiplies them by P = 0)
    for (int i = tid; i < 12 * AC_DK; i += AC_NT) {
      const int m = i / (4 * AC_DK), k = (i / AC_DK) % 4, c = i % AC_DK;
      const float* w = m == 0 ? a.cw_q : m == 1 ? a.cw_k : a.cw_v;
      const float* bb = m == 0 ? a.cb_q : m == 1 ? a.cb_k : a.cb_v;
      wl[i] = k < 3 ? w[c * 3 + k] : bb[c];
    }
    for (int i = tid; i < (G.Lkp - Lk) * AC_DK; i += AC_NT) {
      const int r = Lk + i / AC_DK, c = i % AC_DK;
      Km[r * AC_SQ + c] = 0;
      Vt[c * G.SV + r] = 0;
    }
  }
  __syncthreads();
  xq.conv<false>(Qm, AC_SQ, wl);
  xk.conv<false>(Km, AC_SQ, wl + 4 * AC_DK);
  xv.conv<true>(Vt, G.SV, wl + 8 * AC_DK);
  __syncthreads();

  // per wave: 16-query tiles rt = wave, wave + NW, ...; the key-tile count is a template constant
  bf16_t* P = (bf16_t*)(smem + G.off_p) + wave * 16 * G.SP;
  bf16_t* out = (bf16_t*)a.out + row0 * a.ldo + (size_t)h * AC_DK;
  const float sl2 = a.scale * 1.4426950408889634f;  // softmax on exp2: e^(s - m) = 2^((s - m) log2 e)
  switch (G.Lkp / 16) {  // attention_clip_supported: 1 <= Lk <= 192
    case 2: ac_tiles<2>(Qm, Km, Vt, P, G.SV, G.SP, Lq, Lk, sl2, out, a.ldo, wave, lane); break;
    case 4: ac_tiles<4>(Qm, Km, Vt, P, G.SV, G.SP, Lq, Lk, sl2, out, a.ldo, wave, lane); break;
    case 6: ac_tiles<6>(Qm, Km, Vt, P, G.SV, G.SP, Lq, Lk, sl2, out, a.ldo, wave, lane); break;
    case 8: ac_tiles<8>(Qm, Km, Vt, P, G.SV, G.SP, Lq, Lk, sl2, out, a.ldo, wave, lane); break;
    case 10: ac_tiles<10>(Qm, Km, Vt, P, G.SV, G.SP, Lq, Lk, sl2, out, a.ldo, wave, lane); break;
    default: ac_tiles<12>(Qm, Km, Vt, P, G.SV, G.SP, Lq, Lk, sl2, out, a.ldo, wave, lane); break;
  }
}

}  // namespace

bool attention_clip_supported(int dtype, const AttnArgs& a) {
  return dtype != 0 && a.dk == AC_DK && !a.seq_stride && !a.no_qsplit && !a.no_clip && a.Lq >= 96 && a.Lq <= ATT_LMAX &&
         a.Lk >= 1 && a.Lk <= ATT_LMAX && ac_geom(a.Lq, a.Lk).total <= 160 * 1024;
}

hipError_t launch_attention_clip(const AttnArgs& a, int n, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_clip_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(attn_clip_kernel, dim3(a.heads, n), dim3(AC_NT), ac_geom(a.Lq, a.Lk).total, s, a);
  return hipGetLastError();
}

}  // namespace ggd
