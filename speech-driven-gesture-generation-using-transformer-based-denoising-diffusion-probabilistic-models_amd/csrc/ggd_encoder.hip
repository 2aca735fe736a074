// ggd_encoder.hip -- the HA2G speech encoder (models/modules/ha2g/speech_encoder.py:9-61) as
// hand-written gfx950 kernels behind the ggd_enc_* entry points of include/ggd.h.
//
// Runs ONCE per clip (the reference recomputes it inside every denoise step, model.py:95-96;
// in eval mode it is a pure function of the clip's audio).  Pipeline per chunk of clips:
//
//   STFT     one workgroup per frame: pre-emphasis (ha2g/model/utils.py:22-38) + centre reflect
//            pad + Hann window, 1024-point radix-2 FFT in LDS (f64-exact twiddles),
//            power re^2 + im^2 of the 513 one-sided bins                             -> f32 [n*F][516]
//   mel      power x HTK filterbank (f32 MFMA GEMM)                                   -> f32 [n*F][128]
//   inorm    +1e-6, InstanceNorm1d(128) over frames (speech_encoder.py:28,57-58)     -> f32 [n][128][F]
//   conv1    3x3 1->32 + bias, ReLU, BN (ResNetSE34V2.py:118-126) on VALU             -> f32 NHWC [n][128][F][32]
//   blocks   SE-ResNet [3,4,6,3] x [32,64,128,256] (ResNetBlocks.py:7-37,81-96):
//              conv3x3(s)+ReLU+BN | conv3x3+BN | [1x1(s)+BN downsample] | SE mean+fc+ReLU+fc+sigmoid |
//              relu(v * se + residual)
//   heads    low conv2x2 / mid shuffle2+conv3x3 / high shuffle4+conv3x3, ReLU, BN, flatten (c*H + h),
//            Linear -> 32, wav_proj Linear 32 -> d (ResNetSE34V2.py:157-188, speech_encoder.py:59-61)
//
// Activations between the kernels are bf16 in bf16 contexts (the convolutions round their inputs to
// bf16 anyway: storing them so halves every activation byte moved -- conv inputs / outputs, the SE
// squeeze, the SE apply, the shuffles) and f32 in f32 contexts.
//
// Convolutions are implicit GEMMs on MFMA: rows = output pixels (NHWC, channels innermost),
// columns = output channels, K = taps x input channels in chunks of 32.  Every lane reads its
// own operand fragment straight from global memory (8 consecutive channels of one pixel, 8
// consecutive input channels of one filter tap), so there is no LDS staging and no barrier:
// neighbouring taps re-read the same lines from L1 / L2.  bf16 contexts multiply on
// v_mfma_f32_16x16x32_bf16 (activations rounded to bf16 at the load, f32 accumulate); f32
// contexts on v_mfma_f32_16x16x4_f32 with the 32-channel chunk split into 8 k steps (lane group
// g owns channels 8g .. 8g+7, step s multiplies channel 8g+s), i.e. exact f32 products.  Each
// output element is one lane's fixed-order accumulation, so a clip's features do not depend on
// the batch it is encoded in.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/ggd.h"
#include "ggd_common.h"

using namespace ggd;

namespace {

constexpr int NFFT = 1024, HOP = 512, NBIN = NFFT / 2 + 1, NMEL = 128;
constexpr int POW_LD = 516;     // 513 power bins, rows 16-byte aligned
constexpr int CONV_TPB = 256;   // 4 waves; a wave owns 32 output pixels
constexpr int SE_SLICES = 64;   // pixel slices of the SE squeeze's first stage

// ------------------------------------------------------------------------------------------
// front end
// ------------------------------------------------------------------------------------------
// Mel power spectrum of frame (clip b, frame f): torch.stft(n_fft 1024, hop 512, Hann window,
// center=True, pad_mode='reflect', onesided) |X_k|^2 (speech_encoder.py:18-26), then the HTK mel
// filterbank.  The frame is loaded in bit-reversed order, then 10 radix-2 decimation-in-time stages
// run in LDS (512 butterflies per stage over 256 threads); tw[t] = exp(-2 pi i t / 1024), t < 512,
// rounded once from f64.  LDS index i + i / 32 (one float2 of padding per 32): the bit-reversed
// stores and the short-stride butterflies of the first stages hit distinct banks (2-dword pairs of
// 32 lanes; 32-way conflicts on the unpadded stores).
// Round 5: the filterbank product is done here instead of by a GEMM over the written-out power
// rows: each triangular filter is nonzero on a short band of bins (fb_lo[m] .. + fb_n[m], the
// band's values packed at fb_off[m], made at finalize from the loaded matrix), so mel bin m is a
// short f32 sum over that band in ascending bin order -- 1-2 % of the dense GEMM's work and no
// power rows in HBM.
__device__ __forceinline__ int fft_ix(int i) { return i + (i >> 5); }
__global__ void __launch_bounds__(256) enc_stft_mel_kernel(const float* __restrict__ wav, const float* __restrict__ window,
                                                           const float2* __restrict__ tw, const int* __restrict__ fb_lo,
                                                           const int* __restrict__ fb_n, const int* __restrict__ fb_off,
                                                           const float* __restrict__ fb_val, float* __restrict__ mel,
                                                           int Tw, int F, float coef) {
  __shared__ float2 a[NFFT + NFFT / 32];
  __shared__ float pwr[POW_LD];
  const int fr = blockIdx.x, b = fr / F, f = fr - b * F;
  const float* x = wav + (size_t)b * Tw;
  for (int k = threadIdx.x; k < NFFT; k += blockDim.x) {
    // centre reflect padding of n_fft / 2 (torch.stft center=True, pad_mode='reflect')
    int src = f * HOP + k - NFFT / 2;
    if (src < 0) src = -src;
    if (src >= Tw) src = 2 * (Tw - 1) - src;
    // pre-emphasis y[j] = x[j] - c x[j - 1], reflect-padded on the left: y[0] = x[0] - c x[1]
    const int prev = src == 0 ? 1 : src - 1;
    a[fft_ix(__brev((unsigned)k) >> 22)] = make_float2((x[src] - coef * x[prev]) * window[k], 0.f);
  }
  __syncthreads();
#pragma unroll 1
  for (int st = 1; st <= 10; ++st) {
    const int half = 1 << (st - 1), stride = NFFT >> st;
    for (int j = threadIdx.x; j < NFFT / 2; j += blockDim.x) {
      const int pos = j & (half - 1), i1 = ((j >> (st - 1)) << st) + pos, i2 = i1 + half;
      const float2 w = tw[pos * stride], u = a[fft_ix(i1)], v = a[fft_ix(i2)];
      const float2 t = make_float2(v.x * w.x - v.y * w.y, v.x * w.y + v.y * w.x);
      a[fft_ix(i1)] = make_float2(u.x + t.x, u.y + t.y);
      a[fft_ix(i2)] = make_float2(u.x - t.x, u.y - t.y);
    }
    __syncthreads();
  }
  for (int k = threadIdx.x; k < NBIN; k += blockDim.x) {
    const float2 v = a[fft_ix(k)];
    pwr[k] = v.x * v.x + v.y * v.y;
  }
  __syncthreads();
  if (threadIdx.x < NMEL) {
    const int m = threadIdx.x, lo = fb_lo[m], n = fb_n[m];
    const float* wv = fb_val + fb_off[m];
    float acc = 0.f;
    for (int j = 0; j < n; ++j) acc += pwr[lo + j] * wv[j];
    mel[(size_t)fr * NMEL + m] = acc;
  }
}

// Power spectrum rows for the dense mel GEMM (the training front end, ggd_enc_frontend: its image
// feeds the train-mode encoder and is kept as it was measured against the oracle).  Frame (clip b,
// frame f): torch.stft(n_fft 1024, hop 512, Hann window,
// center=True, pad_mode='reflect', onesided) |X_k|^2 (speech_encoder.py:18-26).  The frame is loaded
// in bit-reversed order, then 10 radix-2 decimation-in-time stages run in LDS (512 butterflies
// per stage over 256 threads); tw[t] = exp(-2 pi i t / 1024), t < 512, rounded once from f64.
__global__ void __launch_bounds__(256) enc_stft_power_kernel(const float* __restrict__ wav, const float* __restrict__ window,
                                                             const float2* __restrict__ tw, float* __restrict__ pw, int Tw,
                                                             int F, float coef) {
  __shared__ float2 a[NFFT];
  const int fr = blockIdx.x, b = fr / F, f = fr - b * F;
  const float* x = wav + (size_t)b * Tw;
  for (int k = threadIdx.x; k < NFFT; k += blockDim.x) {
    // centre reflect padding of n_fft / 2 (torch.stft center=True, pad_mode='reflect')
    int src = f * HOP + k - NFFT / 2;
    if (src < 0) src = -src;
    if (src >= Tw) src = 2 * (Tw - 1) - src;
    // pre-emphasis y[j] = x[j] - c x[j - 1], reflect-padded on the left: y[0] = x[0] - c x[1]
    const int prev = src == 0 ? 1 : src - 1;
    a[__brev((unsigned)k) >> 22] = make_float2((x[src] - coef * x[prev]) * window[k], 0.f);
  }
  __syncthreads();
#pragma unroll 1
  for (int st = 1; st <= 10; ++st) {
    const int half = 1 << (st - 1), stride = NFFT >> st;
    for (int j = threadIdx.x; j < NFFT / 2; j += blockDim.x) {
      const int pos = j & (half - 1), i1 = ((j >> (st - 1)) << st) + pos, i2 = i1 + half;
      const float2 w = tw[pos * stride], u = a[i1], v = a[i2];
      const float2 t = make_float2(v.x * w.x - v.y * w.y, v.x * w.y + v.y * w.x);
      a[i1] = make_float2(u.x + t.x, u.y + t.y);
      a[i2] = make_float2(u.x - t.x, u.y - t.y);
    }
    __syncthreads();
  }
  for (int k = threadIdx.x; k < POW_LD; k += blockDim.x) {
    float p = 0.f;
    if (k < NBIN) p = a[k].x * a[k].x + a[k].y * a[k].y;
    pw[(size_t)fr * POW_LD + k] = p;
  }
}

// +1e-6, instance norm over frames per (clip, mel bin) -> image [n][128][F]; one workgroup per clip
__global__ void __launch_bounds__(4 * NMEL) enc_inorm_kernel(const float* __restrict__ mel, float* __restrict__ img,
                                                             int F) {
  // four frame groups per mel bin (frames gr, gr + 4, ...), added in group order
  __shared__ float red[4][NMEL];
  const int b = blockIdx.x, m = threadIdx.x % NMEL, gr = threadIdx.x / NMEL;
  const float* src = mel + (size_t)b * F * NMEL + m;
  float s = 0.f;
  for (int f = gr; f < F; f += 4) s += src[(size_t)f * NMEL] + 1e-6f;
  red[gr][m] = s;
  __syncthreads();
  const float mean = ((red[0][m] + red[1][m]) + (red[2][m] + red[3][m])) / (float)F;
  __syncthreads();
  float v = 0.f;
  for (int f = gr; f < F; f += 4) {
    const float d = (src[(size_t)f * NMEL] + 1e-6f) - mean;
    v += d * d;
  }
  red[gr][m] = v;
  __syncthreads();
  const float inv = 1.0f / sqrtf(((red[0][m] + red[1][m]) + (red[2][m] + red[3][m])) / (float)F + 1e-5f);
  float* dst = img + ((size_t)b * NMEL + m) * F;
  for (int f = gr; f < F; f += 4) dst[f] = ((src[(size_t)f * NMEL] + 1e-6f) - mean) * inv;
}

// conv1 (1 -> 32, 3x3, pad 1) + bias, ReLU, BN; one thread per (pixel, 8 output channels)
template <typename TA>
__global__ void enc_conv1_kernel(const float* __restrict__ img, const float* __restrict__ w,
                                 const float* __restrict__ bias, const float* __restrict__ s,
                                 const float* __restrict__ t, TA* __restrict__ out, int n, int H, int W) {
  __shared__ float ws[32 * 9], bs[32], ss[32], ts[32];
  for (int i = threadIdx.x; i < 32 * 9; i += blockDim.x) ws[i] = w[i];
  if (threadIdx.x < 32) {
    bs[threadIdx.x] = bias[threadIdx.x];
    ss[threadIdx.x] = s[threadIdx.x];
    ts[threadIdx.x] = t[threadIdx.x];
  }
  __syncthreads();
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x, total = (size_t)n * H * W * 4;
  if (idx >= total) return;
  const int cg = (int)(idx & 3);
  const size_t p = idx >> 2;
  const int x = (int)(p % W), y = (int)((p / W) % H), b = (int)(p / ((size_t)W * H));
  float tap[9];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int iy = y + ky - 1, ix = x + kx - 1;
      tap[ky * 3 + kx] = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? img[((size_t)b * H + iy) * W + ix] : 0.f;
    }
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cg * 8 + j;
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < 9; ++q) acc += ws[c * 9 + q] * tap[q];
    o[j] = fmaxf(acc + bs[c], 0.f) * ss[c] + ts[c];
  }
  if constexpr (sizeof(TA) == 2) {
    uint4 u;
    u.x = pk_bf16(o[0], o[1]);
    u.y = pk_bf16(o[2], o[3]);
    u.z = pk_bf16(o[4], o[5]);
    u.w = pk_bf16(o[6], o[7]);
    *(uint4*)(out + p * 32 + cg * 8) = u;
  } else {
    float4* dst = (float4*)(out + p * 32 + cg * 8);
    dst[0] = make_float4(o[0], o[1], o[2], o[3]);
    dst[1] = make_float4(o[4], o[5], o[6], o[7]);
  }
}

// ------------------------------------------------------------------------------------------
// implicit-GEMM convolution
// ------------------------------------------------------------------------------------------
enum { CONV_BN = 0, CONV_RELU_BN = 1 };

// activation element access (f32 or bf16 tensors)
__device__ __forceinline__ void act_load8(const float* p, float (&v)[8]) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void act_load8(const bf16_t* p, float (&v)[8]) {
  const uint4 u = *(const uint4*)p;
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ float act_ld(const float* p) { return *p; }
__device__ __forceinline__ float act_ld(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ void act_st(float* p, float v) { *p = v; }
__device__ __forceinline__ void act_st(bf16_t* p, float v) { *p = f2bf(v); }
enum { LAYOUT_NHWC = 0, LAYOUT_NWCH = 1 };

struct ConvArgs {
  const void* in;           // NHWC [N][H][W][Cin] (Cin a multiple of 32), f32 or bf16 (in_bf16)
  const void* w;            // T [Cout_pad][KH * KW][Cin]
  const void* wp;           // bf16 plane-major copy for enc_conv_nhwc_kernel: [Cin / 32][4][Cout_pad][TAPSP][8]
  const float *bias, *s, *t;  // [Cout_pad]: BN folded to y = x * s + t
  void* out;                // f32 or bf16 (out_bf16)
  int N, H, W, Cin, Ho, Wo, Cout_pad, Cvalid, KH, KW, stride, pad, mode, layout, in_bf16, out_bf16;
  float* se_part;           // LDS kernel, non-null: the SE squeeze's partial sums of the f32 outputs,
                            // one row of Cout_pad per (image, output tile): [N][tiles][Cout_pad]
};

template <typename T> struct ConvB;
template <> struct ConvB<bf16_t> {
  bf16x8 v;
  __device__ __forceinline__ void load(const bf16_t* p) { v = *(const bf16x8*)p; }
};
template <> struct ConvB<float> {
  float v[8];
  __device__ __forceinline__ void load(const float* p) {
    const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
};

struct ConvA {
  float v[8];
};

__device__ __forceinline__ void mma(f32x4& acc, const ConvA& a, const ConvB<bf16_t>& b) {
  bf16x8 av;
#pragma unroll
  for (int i = 0; i < 8; ++i) av[i] = (__bf16)a.v[i];
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b.v, acc, 0, 0, 0);
}
__device__ __forceinline__ void mma(f32x4& acc, const ConvA& a, const ConvB<float>& b) {
#pragma unroll
  for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[s], b.v[s], acc, 0, 0, 0);
}

template <typename T, int NJ>
struct ConvStage {
  ConvA a[2];
  ConvB<T> b[NJ];
};

template <typename T, int NJ, typename TI, typename TO>
__global__ void __launch_bounds__(CONV_TPB) enc_conv_kernel(ConvArgs a) {
  const TI* in = (const TI*)a.in;
  TO* out = (TO*)a.out;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r16 = lane & 15, g = lane >> 4;
  const int HWo = a.Ho * a.Wo, P = a.N * HWo;
  const int p0 = blockIdx.x * 128 + wave * 32, n0 = blockIdx.y * (NJ * 16);
  // this lane's A pixels (row tiles 0, 1): clamped into the image; `ok` masks the padding
  int base[2], iy0[2], ix0[2];
  bool pv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = p0 + i * 16 + r16;
    pv[i] = p < P;
    const int pc = min(p, P - 1), b = pc / HWo, rem = pc - b * HWo, oy = rem / a.Wo, ox = rem - oy * a.Wo;
    base[i] = b * a.H * a.W;
    iy0[i] = oy * a.stride - a.pad;
    ix0[i] = ox * a.stride - a.pad;
  }
  const int taps = a.KH * a.KW, cch = a.Cin >> 5, nk = taps * cch;
  const T* wb = (const T*)a.w + (size_t)(n0 + r16) * taps * a.Cin + g * 8;
  const size_t wj = (size_t)16 * taps * a.Cin;  // next column tile

  auto fetch = [&](int kk, ConvStage<T, NJ>& st) {
    const int tap = kk / cch, c0 = (kk - tap * cch) << 5, ky = tap / a.KW, kx = tap - ky * a.KW;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int iy = iy0[i] + ky, ix = ix0[i] + kx;
      const bool ok = pv[i] && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
      const int pix = base[i] + min(max(iy, 0), a.H - 1) * a.W + min(max(ix, 0), a.W - 1);
      float u[8];
      act_load8(in + (size_t)pix * a.Cin + c0 + g * 8, u);
      const float m = ok ? 1.f : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) st.a[i].v[e] = u[e] * m;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) st.b[j].load(wb + j * wj + (size_t)tap * a.Cin + c0);
  };

  f32x4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  ConvStage<T, NJ> cur, nxt;
  fetch(0, cur);
  for (int kk = 0; kk < nk; ++kk) {
    if (kk + 1 < nk) fetch(kk + 1, nxt);  // next chunk in flight under this chunk's MFMAs
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) mma(acc[i][j], cur.a[i], cur.b[j]);
    cur = nxt;
  }

  // epilogue: C/D layout of the 16x16 MFMA -- column = lane & 15, row = 4 (lane >> 4) + r
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int co = n0 + j * 16 + r16;
    const float bi = a.bias[co], sc = a.s[co], sh = a.t[co];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = p0 + i * 16 + 4 * g + r;
        if (p >= P) continue;
        float v = acc[i][j][r];
        v = a.mode == CONV_RELU_BN ? fmaxf(v + bi, 0.f) * sc + sh : (v + bi) * sc + sh;
        if (a.layout == LAYOUT_NHWC) {
          act_st(out + (size_t)p * a.Cout_pad + co, v);
        } else if (co < a.Cvalid) {
          const int b = p / HWo, rem = p - b * HWo, oy = rem / a.Wo, ox = rem - oy * a.Wo;
          act_st(out + (((size_t)b * a.Wo + ox) * a.Cvalid + co) * a.Ho + oy, v);
        }
      }
  }
}

// ------------------------------------------------------------------------------------------
// squeeze-excitation, residual, pixel shuffle, heads
// ------------------------------------------------------------------------------------------
// SE squeeze, stage 1: grid (clips, S slices); each workgroup sums its slice of the clip's pixels
// for every channel -> part[clip][slice][C] (fixed partition and order: deterministic)
template <typename TA>
__global__ void __launch_bounds__(256) enc_se_sum_kernel(const TA* __restrict__ v, int HW, int C,
                                                         float* __restrict__ part) {
  __shared__ float red[256];
  const int b = blockIdx.x, sl = blockIdx.y, S = gridDim.y, tid = threadIdx.x;
  const int stripes = 256 / C, c = tid % C, st = tid / C;
  const int p0 = (int)((long)HW * sl / S), p1 = (int)((long)HW * (sl + 1) / S);
  const TA* src = v + (size_t)b * HW * C;
  // four independent partial sums keep four loads in flight per thread (fixed order per clip)
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (st < stripes) {
    int p = p0 + st;
    for (; p + 3 * stripes < p1; p += 4 * stripes) {
      s0 += act_ld(src + (size_t)p * C + c);
      s1 += act_ld(src + (size_t)(p + stripes) * C + c);
      s2 += act_ld(src + (size_t)(p + 2 * stripes) * C + c);
      s3 += act_ld(src + (size_t)(p + 3 * stripes) * C + c);
    }
    for (; p < p1; p += stripes) s0 += act_ld(src + (size_t)p * C + c);
  }
  red[tid] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (tid < C) {
    float tot = 0.f;
    for (int k = 0; k < stripes; ++k) tot += red[k * C + tid];
    part[((size_t)b * S + sl) * C + tid] = tot;
  }
}

// stage 2, one workgroup per clip: y[c] = sigmoid(fc2(relu(fc0(mean_hw(v)))))  (ResNetBlocks.py:81-96)
// from the squeeze's partial-sum rows (S per clip, added in a fixed order: deterministic).  A
// separate launch: recomputing it in every workgroup of the channel scale below (measured, r03k)
// put three dependent load rounds in front of every one of them and was slower than this launch.
__global__ void __launch_bounds__(256) enc_se_kernel(const float* __restrict__ part, int S, int HW, int C,
                                                     const float* __restrict__ w0, const float* __restrict__ b0,
                                                     const float* __restrict__ w2, const float* __restrict__ b2,
                                                     float* __restrict__ y) {
  __shared__ float mean[256], hid[32], red[256];
  const int b = blockIdx.x, tid = threadIdx.x;
  {  // 256 / C stripes of the S rows, then the stripes in order
    const int stripes = 256 / C, c = tid % C, st = tid / C;
    float s0 = 0.f, s1 = 0.f;
    int k = st;
    for (; k + stripes < S; k += 2 * stripes) {
      s0 += part[((size_t)b * S + k) * C + c];
      s1 += part[((size_t)b * S + k + stripes) * C + c];
    }
    if (k < S) s0 += part[((size_t)b * S + k) * C + c];
    red[tid] = s0 + s1;
    __syncthreads();
    if (tid < C) {
      float tot = 0.f;
      for (int j = 0; j < stripes; ++j) tot += red[j * C + tid];
      mean[tid] = tot / (float)HW;
    }
  }
  __syncthreads();
  // fc.0 (C -> C / 8 <= 32): eight lanes per hidden unit, each a strided eighth of the dot product
  const int Ch = C / 8, u = tid >> 3, q = tid & 7;
  float a0 = 0.f;
  if (u < Ch)
    for (int k = q; k < C; k += 8) a0 += w0[u * C + k] * mean[k];
  a0 = group_sum<8>(a0);
  if (u < Ch && q == 0) hid[u] = fmaxf(a0 + b0[u], 0.f);
  __syncthreads();
  if (tid < C) {
    float a = b2[tid];
    for (int k = 0; k < Ch; ++k) a += w2[tid * Ch + k] * hid[k];
    y[(size_t)b * C + tid] = 1.0f / (1.0f + expf(-a));
  }
}

// out = relu(v * y[clip][c] + res), NHWC; 8 consecutive channels per thread
template <typename TA>
__global__ void enc_se_apply_kernel(const TA* __restrict__ v, const float* __restrict__ y,
                                    const TA* __restrict__ res, TA* __restrict__ out, int HW, int C,
                                    size_t total8) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total8) return;
  const size_t e = idx * 8;
  const int c = (int)(e % C);
  const size_t b = e / ((size_t)HW * C);
  float a[8], r[8];
  act_load8(v + e, a);
  act_load8(res + e, r);
  const float* ys = y + b * C + c;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = fmaxf(a[i] * ys[i] + r[i], 0.f);
  if constexpr (sizeof(TA) == 2) {
    uint4 u;
    u.x = pk_bf16(a[0], a[1]);
    u.y = pk_bf16(a[2], a[3]);
    u.z = pk_bf16(a[4], a[5]);
    u.w = pk_bf16(a[6], a[7]);
    *(uint4*)(out + e) = u;
  } else {
    *(float4*)(out + e) = make_float4(a[0], a[1], a[2], a[3]);
    *(float4*)(out + e + 4) = make_float4(a[4], a[5], a[6], a[7]);
  }
}

// PixelShuffle(r): in NHWC [n][H][W][C r^2] -> out NHWC [n][H r][W r][Cp] (channels >= C zero);
// one thread per 8 consecutive output channels (one 16- / 32-byte store), Cp % 8 == 0
template <typename TA>
__global__ void enc_shuffle_kernel(const TA* __restrict__ in, TA* __restrict__ out, int n, int H, int W,
                                   int C, int r, int Cp) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int Ho = H * r, Wo = W * r, C8 = Cp / 8;
  if (idx >= (size_t)n * Ho * Wo * C8) return;
  const int c0 = (int)(idx % C8) * 8;
  const size_t p = idx / C8;
  const int x = (int)(p % Wo), yy = (int)((p / Wo) % Ho), b = (int)(p / ((size_t)Wo * Ho));
  const int h = yy / r, i = yy - h * r, w = x / r, j = x - w * r;
  const TA* src = in + (((size_t)b * H + h) * W + w) * (C * r * r) + i * r + j;
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = c0 + k < C ? act_ld(src + (c0 + k) * r * r) : 0.f;
  TA* dst = out + p * Cp + c0;
  if constexpr (sizeof(TA) == 2) {
    uint4 o;
    o.x = pk_bf16(v[0], v[1]);
    o.y = pk_bf16(v[2], v[3]);
    o.z = pk_bf16(v[4], v[5]);
    o.w = pk_bf16(v[6], v[7]);
    *(uint4*)dst = o;
  } else {
    *(float4*)dst = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(dst + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// The heads' Linear pair z = Wp (W1 a + b1) + bp (speech_encoder.py: fc_low / fc_mid / fc_high, then
// wav_proj_layer) for 16 (clip, time) rows per workgroup: a = the row's K = C x H conv features,
// read from the NHWC f32 conv output [clip][h][w][Cp] in (h, c) order -- W1's columns are permuted
// to that order at finalize (the reference flattens (c, h)).  W1 a on v_mfma_f32_16x16x4_f32 (f32 products, f32 accumulation): wave w
// takes the 16-deep K steps w, w + 8, ...; lane (row r16, group g) feeds k = 16 s + 4 g + i of step s
// to MFMA i (the same permutation for A and B); the 8 waves' partial sums are added in wave order.
// The 32 -> d projection follows from LDS.  K % 16 == 0.
constexpr int HFC_WAVES = 8, HFC_DEPTH = 4;  // K split over 8 waves; 4 K steps of loads in flight per wave
__global__ void __launch_bounds__(64 * HFC_WAVES) enc_head_fc_kernel(const float* __restrict__ feat, int M, int K,
                                                                     int Hh, int Wo, int Cp, int lc,
                                                                     const float* __restrict__ w1,
                                                                     const float* __restrict__ b1,
                                                                     const float* __restrict__ wp,
                                                                     const float* __restrict__ bp,
                                                                     float* __restrict__ z, int d, int zrows,
                                                                     int zld, int zoff) {
  __shared__ float red[HFC_WAVES][16][33], h1[16][33];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const int row0 = blockIdx.x * 16;
  const int row = min(row0 + r16, M - 1), rb = row / Wo, cm = (1 << lc) - 1;
  // (h, c) of k = 16 st + 4 g: h = k >> lc, c = k & cm (4 consecutive channels: C % 4 == 0)
  const float* a0 = feat + ((size_t)rb * Hh * Wo + (row - rb * Wo)) * Cp;
  auto aptr = [&](int st) { const int k = st * 16 + 4 * g; return a0 + (size_t)(k >> lc) * Wo * Cp + (k & cm); };
  const float* wa = w1 + (size_t)r16 * K + 4 * g;
  const float* wb = w1 + (size_t)(16 + r16) * K + 4 * g;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const int steps = K / 16, nst = steps > wave ? (steps - wave + HFC_WAVES - 1) / HFC_WAVES : 0;
  float4 xa[HFC_DEPTH], xw0[HFC_DEPTH], xw1[HFC_DEPTH];
  auto load = [&](int p, int i) __attribute__((always_inline)) {
    const int st = wave + i * HFC_WAVES;
    xa[p] = *(const float4*)aptr(st);
    xw0[p] = *(const float4*)(wa + st * 16);
    xw1[p] = *(const float4*)(wb + st * 16);
  };
#pragma unroll
  for (int p = 0; p < HFC_DEPTH; ++p)
    if (p < nst) load(p, p);
  for (int i0 = 0; i0 < nst; i0 += HFC_DEPTH) {
#pragma unroll
    for (int p = 0; p < HFC_DEPTH; ++p) {
      const int i = i0 + p;
      if (i < nst) {
        const float4 ca = xa[p], c0 = xw0[p], c1 = xw1[p];
        if (i + HFC_DEPTH < nst) load(p, i + HFC_DEPTH);  // refill the slot HFC_DEPTH steps ahead
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ca.x, c0.x, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ca.x, c1.x, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ca.y, c0.y, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ca.y, c1.y, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ca.z, c0.z, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ca.z, c1.z, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ca.w, c0.w, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ca.w, c1.w, acc1, 0, 0, 0);
      }
    }
  }
  // C layout: row 4 g + i, column r16 (tile 0) / 16 + r16 (tile 1)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    red[wave][4 * g + i][r16] = acc0[i];
    red[wave][4 * g + i][16 + r16] = acc1[i];
  }
  __syncthreads();
  for (int e = tid; e < 16 * 32; e += 64 * HFC_WAVES) {
    const int r = e >> 5, j = e & 31;
    float t = red[0][r][j];
#pragma unroll
    for (int w = 1; w < HFC_WAVES; ++w) t += red[w][r][j];
    h1[r][j] = t + b1[j];
  }
  __syncthreads();
  for (int o = tid; o < d; o += 64 * HFC_WAVES) {
    float wr[32];
#pragma unroll
    for (int j = 0; j < 32; j += 4) {
      const float4 t = *(const float4*)(wp + (size_t)o * 32 + j);
      wr[j] = t.x;
      wr[j + 1] = t.y;
      wr[j + 2] = t.z;
      wr[j + 3] = t.w;
    }
    const float bo = bp[o];
    for (int r = 0; r < 16 && row0 + r < M; ++r) {
      float v = bo;
#pragma unroll
      for (int j = 0; j < 32; ++j) v += wr[j] * h1[r][j];
      // row (clip c, token t) of the level -> z row c zrows + zoff + t, zld floats apart: the
      // separate (N, T, d) tensor, or its place in the decoder's speech memory (see MemMap)
      const int gr = row0 + r, c = gr / Wo;
      z[((size_t)c * zrows + zoff + (gr - c * Wo)) * zld + o] = v;
    }
  }
}

// the left padding of a level in the s2g_v2 speech memory (model.py:97-104: F.pad on time before the
// feature concat): rows [0, npad) of columns [0, d) of every clip's (zrows x zld) block
__global__ void enc_zpad_kernel(float* __restrict__ z, int npad, int d, int zrows, int zld) {
  const int c = blockIdx.x;
  for (int e = threadIdx.x; e < npad * d; e += blockDim.x) z[((size_t)c * zrows + e / d) * zld + e % d] = 0.f;
}

inline unsigned blocks_for(size_t n, int tpb) { return (unsigned)((n + tpb - 1) / tpb); }

// ------------------------------------------------------------------------------------------
// LDS-tiled implicit-GEMM convolution (bf16 contexts): a workgroup owns a TH x TW block of
// output pixels of ONE image (128 pixels = 4 waves x 2 row tiles of 16) and NJ x 16 output
// channels.  Per 32-channel input chunk it stages, once, the input patch the block's taps touch
// ((TH-1)s+KH rows x (TW-1)s+KW columns, bf16, zeros outside the image) and the chunk's filter
// taps (NJ*16 x KH*KW x 32 bf16); every tap's A fragment is then an LDS read of the shifted
// patch position.  enc_conv_kernel fetches each input value from L1/L2 once per tap and each
// filter fragment once per wave; here both are fetched once per workgroup and chunk.  The
// accumulation order of an output element is fixed (chunk, tap, 32 channels): batch-invariant.
// ------------------------------------------------------------------------------------------
// diagnostics: GGD_ENC_CONV_DIRECT=1 routes bf16 contexts back to enc_conv_kernel (A/B timing)
static const bool conv_no_lds = std::getenv("GGD_ENC_CONV_DIRECT") != nullptr;
constexpr int CL_PX = 128;     // output pixels per workgroup
constexpr int CL_CS = 32 + 8;  // bf16 stride of one patch position / one filter tap in LDS
constexpr int CL_PMAX = 18;    // patch float4 per thread (npos * 8 <= 18 * 256: 3x3 stride 2, 16-wide tiles)
constexpr int CL_PMIN = 8;     // ... for the stride-1 shapes (npos <= 256)
constexpr int CL_TAPS_MAX = 9;

struct ConvLdsGeom {
  int TW, TH, PH, PW, taps;
  size_t patch_bytes, w_bytes;
};
__host__ __device__ inline ConvLdsGeom conv_lds_geom(const ConvArgs& a, int TW, int NJ) {
  ConvLdsGeom g;
  g.TW = TW;
  g.TH = CL_PX / TW;
  g.PH = (g.TH - 1) * a.stride + a.KH;
  g.PW = (g.TW - 1) * a.stride + a.KW;
  g.taps = a.KH * a.KW;
  g.patch_bytes = (size_t)g.PH * g.PW * CL_CS * 2;
  g.w_bytes = (size_t)NJ * 16 * g.taps * CL_CS * 2;
  return g;
}

template <int NJ, int PM, typename TI, typename TO>
__global__ void __launch_bounds__(CONV_TPB) enc_conv_lds_kernel(ConvArgs a, int TW) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // an input piece is one 16-byte load: 4 f32 or 8 bf16 channels; QP pieces per 32-channel chunk
  constexpr int CPP = 16 / (int)sizeof(TI), QP = 32 / CPP;
  const TI* in = (const TI*)a.in;
  TO* out = (TO*)a.out;
  const ConvLdsGeom G = conv_lds_geom(a, TW, NJ);
  bf16_t* patch = (bf16_t*)smem;
  bf16_t* wl = (bf16_t*)(smem + G.patch_bytes);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const int tw_n = (a.Wo + G.TW - 1) / G.TW, th_n = (a.Ho + G.TH - 1) / G.TH, per = tw_n * th_n;
  const int b = blockIdx.x / per, tix = blockIdx.x - b * per;
  const int oh0 = (tix / tw_n) * G.TH, ow0 = (tix - (tix / tw_n) * tw_n) * G.TW, n0 = blockIdx.y * (NJ * 16);
  const int ih0 = oh0 * a.stride - a.pad, iw0 = ow0 * a.stride - a.pad;
  int pbase[2];  // patch position of tap (0, 0) for this lane's A pixels (row tiles 0, 1)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = wave * 32 + i * 16 + r16, ty = q / G.TW, tx = q - ty * G.TW;
    pbase[i] = ty * a.stride * G.PW + tx * a.stride;
  }
  f32x4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16_t* W = (const bf16_t*)a.w;
  const int cch = a.Cin >> 5, npos = G.PH * G.PW;
  // the next chunk's patch and filter taps are fetched into registers while this chunk's MFMAs
  // run (PM / WMAX pieces per thread bound them; launch_conv checks the shape fits)
  constexpr int WMAX = (NJ * 16 * CL_TAPS_MAX * 4 + CONV_TPB - 1) / CONV_TPB;
  const int np8 = npos * QP, nw = NJ * 16 * G.taps * 4;
  uint4 xr[PM];
  bf16x8 wr[WMAX];  // native vectors (HIP's uint4 struct copies keep the array in scratch)
  uint32_t okm = 0;  // bit k: patch piece k lies inside the image (else it stages as zero)
  auto fetch = [&](int ck) __attribute__((always_inline)) {
    okm = 0;
#pragma unroll
    for (int k = 0; k < PM; ++k) {
      const int v = tid + k * CONV_TPB;
      {
        const int vc = min(v, np8 - 1);
        const int pos = vc / QP, q4 = vc % QP, py = pos / G.PW, px = pos - py * G.PW;
        const int ih = ih0 + py, iw = iw0 + px;
        const bool ok = ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
        const int ihc = min(max(ih, 0), a.H - 1), iwc = min(max(iw, 0), a.W - 1);
        xr[k] = *(const uint4*)(in + (((size_t)b * a.H + ihc) * a.W + iwc) * a.Cin + ck * 32 + q4 * CPP);
        okm |= (ok && v < np8) ? (1u << k) : 0u;
      }
    }
#pragma unroll
    for (int k = 0; k < WMAX; ++k) {
      const int v = min(tid + k * CONV_TPB, nw - 1);  // clamped: every wr[k] is defined (no scratch)
      const int q8 = v & 3, nt = v >> 2, n = nt / G.taps, tap = nt - n * G.taps;
      wr[k] = *(const bf16x8*)(W + ((size_t)(n0 + n) * G.taps + tap) * a.Cin + ck * 32 + q8 * 8);
    }
  };
  auto put = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < PM; ++k) {
      const int v = tid + k * CONV_TPB;
      if (v < np8) {
        const int pos = v / QP, q4 = v % QP;
        const bool ok = (okm >> k) & 1u;
        if constexpr (sizeof(TI) == 2) {  // 8 bf16 channels as they are
          *(uint4*)(patch + pos * CL_CS + q4 * 8) = ok ? xr[k] : make_uint4(0u, 0u, 0u, 0u);
        } else {
          const uint32_t lo = pk_bf16(__uint_as_float(xr[k].x), __uint_as_float(xr[k].y));
          const uint32_t hi = pk_bf16(__uint_as_float(xr[k].z), __uint_as_float(xr[k].w));
          *(uint2*)(patch + pos * CL_CS + q4 * 4) = ok ? make_uint2(lo, hi) : make_uint2(0u, 0u);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < WMAX; ++k) {
      const int v = tid + k * CONV_TPB;
      if (v < nw) {
        const int q8 = v & 3, nt = v >> 2, n = nt / G.taps, tap = nt - n * G.taps;
        *(bf16x8*)(wl + (n * G.taps + tap) * CL_CS + q8 * 8) = wr[k];
      }
    }
  };
  fetch(0);
  for (int ck = 0; ck < cch; ++ck) {
    if (ck > 0) __syncthreads();  // the previous chunk's MFMAs are done with the LDS images
    put();
    __syncthreads();
    if (ck + 1 < cch) fetch(ck + 1);
    for (int tap = 0; tap < G.taps; ++tap) {
      const int ky = tap / a.KW, kx = tap - ky * a.KW, toff = ky * G.PW + kx;
      bf16x8 av[2], bv[NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = *(const bf16x8*)(patch + (pbase[i] + toff) * CL_CS + g * 8);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bv[j] = *(const bf16x8*)(wl + ((j * 16 + r16) * G.taps + tap) * CL_CS + g * 8);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  }
  // epilogue: C/D layout of the 16x16 MFMA -- column = lane & 15, row = 4 (lane >> 4) + r
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int co = n0 + j * 16 + r16;
    const float bi = a.bias[co], sc = a.s[co], sh = a.t[co];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = wave * 32 + i * 16 + 4 * g + r, ty = q / G.TW, tx = q - ty * G.TW;
        const int oh = oh0 + ty, ow = ow0 + tx;
        if (oh >= a.Ho || ow >= a.Wo) continue;
        const int p = (b * a.Ho + oh) * a.Wo + ow;
        float v = acc[i][j][r];
        v = a.mode == CONV_RELU_BN ? fmaxf(v + bi, 0.f) * sc + sh : (v + bi) * sc + sh;
        if (a.layout == LAYOUT_NHWC) {
          act_st(out + (size_t)p * a.Cout_pad + co, v);
        } else if (co < a.Cvalid) {
          act_st(out + (((size_t)b * a.Wo + ow) * a.Cvalid + co) * a.Ho + oh, v);
        }
      }
  }
  if (a.se_part) {
    // SE squeeze of this tile (ResNetBlocks.py:81-96, the mean's first stage): per output channel the
    // sum of the tile's valid f32 outputs, in a fixed order (lane rows, lane groups, waves) -> one
    // [Cout_pad] row per (image, tile); enc_se_kernel adds the tiles of an image in tile order
    __syncthreads();  // every wave is past the MMA loop: the patch / filter images are free
    float* red = (float*)smem;  // [4 waves][NJ * 16]
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int co = n0 + j * 16 + r16;
      const float bi = a.bias[co], sc = a.s[co], sh = a.t[co];
      float cs = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = wave * 32 + i * 16 + 4 * g + r, ty = q / G.TW, tx = q - ty * G.TW;
          float v = acc[i][j][r];
          v = a.mode == CONV_RELU_BN ? fmaxf(v + bi, 0.f) * sc + sh : (v + bi) * sc + sh;
          cs += (oh0 + ty < a.Ho && ow0 + tx < a.Wo) ? v : 0.f;
        }
      cs += __shfl_xor(cs, 16);
      cs += __shfl_xor(cs, 32);
      if (g == 0) red[wave * NJ * 16 + j * 16 + r16] = cs;
    }
    __syncthreads();
    if (tid < NJ * 16)
      a.se_part[((size_t)b * per + tix) * a.Cout_pad + n0 + tid] =
          (red[tid] + red[NJ * 16 + tid]) + (red[2 * NJ * 16 + tid] + red[3 * NJ * 16 + tid]);
  }
}

// ------------------------------------------------------------------------------------------
// The residual tower's convolutions (NHWC bf16 in / out; 3x3 stride 1 and 2, the 1x1 stride-2
// downsample), with the tile geometry fixed at compile time.  Same tiling as enc_conv_lds_kernel
// (128 output pixels x NJ 16 output channels per 256-thread workgroup, per 32-channel chunk the
// patch and the filter taps staged in LDS, the next chunk in registers), and:
//   * the geometry is constexpr: every index split is a shift / multiply (the runtime version
//     spent ~2x its MFMA time on integer division in the staging and the epilogue), and the
//     per-piece source offsets are computed once, each chunk adding 32 channels;
//   * a 1x1 strided conv stages only the pixels it reads (a TH x TW image, not the stride-2 span);
//   * the product is computed transposed (A = filter taps, B = patch), so a lane holds 4
//     consecutive output channels of one pixel: one 8-byte store per (pixel tile, channel tile)
//     instead of four 2-byte stores, and the SE squeeze reduces over the 16 pixel lanes by DPP.
//   * round 5: the LDS images are PLANE-major -- 16-byte piece q (channels 8q..8q+7) of every patch
//     position / filter row in plane q, 64 B per position instead of 80 -- so that every ds_read_b128
//     lane group (16 lanes, 16 distinct pixels or filter rows) and every ds_write_b128 group (8
//     consecutive positions of one plane) covers 64 distinct banks: conflict-free.  The 80-byte rows
//     cost 2x on the tap reads (PMC r05e: SQ_LDS_BANK_CONFLICT = 49 % of SQ_LDS_IDX_ACTIVE) and
//     25 % more LDS per workgroup (2 instead of 3 workgroups per CU on the 64-channel convs, 1
//     instead of 2 on the stride-2 ones).  For that: a stride-2 3x3 patch stores its columns by
//     parity (even | odd), so a row of output pixels reads consecutive positions at every tap; an
//     8-wide tile pads the patch row so its two pixel rows sit 8 positions (32 banks) apart; the
//     filter rows of one output channel are padded to an odd count (TAPSP) and come from a
//     plane-major copy of the weights (EConv::wp, made at finalize).  The MFMA sequence and its
//     operands are unchanged.  scripts/conv_lds_sim.py checks the addressing and the bank cycles
//     of every compiled shape on the CPU.
// ------------------------------------------------------------------------------------------
template <int TW, int KS, int ST> struct CGeo {
  static constexpr int TH = CL_PX / TW;
  static constexpr int PH = KS == 1 ? TH : (TH - 1) * ST + KS;  // 1x1: only the pixels read
  static constexpr int PW = KS == 1 ? TW : (TW - 1) * ST + KS;
  static constexpr int PS = KS == 1 ? 1 : ST;                   // patch rows / columns per output pixel
  static constexpr int SS = KS == 1 ? ST : 1;                   // source step per patch position
  static constexpr bool DI = KS > 1 && ST == 2;                 // columns stored by parity
  static constexpr int HALF = (PW + 1) / 2;
  static constexpr int PWC = DI ? 2 * HALF : PW;                // stored columns
  static constexpr int pws() {  // row stride (positions): TW = 8 puts a wave's 2 pixel rows 8 slots apart
    int w = PWC;
    if (TW == 8)
      while ((PS * w) % 16 != 8) ++w;
    return w;
  }
  static constexpr int PWS = pws();
  static constexpr int NPOS = (PH * PWS + 15) / 16 * 16;        // positions per plane (256-byte planes)
  static constexpr int TAPS = KS * KS, TAPSP = TAPS | 1;        // filter rows per output channel (odd)
  static constexpr size_t PATCH_BYTES = (size_t)4 * NPOS * 16;
  // stored column of patch column px
  static __host__ __device__ constexpr int col(int px) { return DI ? (px & 1) * HALF + (px >> 1) : px; }
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t conv_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}

// workgroups per CU the LDS image allows (5 at most; 4 for the f32-output head convs, whose
// epilogue does not fit 96 VGPRs): the kernel's register budget is set to match
template <int NJ, int TW, int KS, int ST, typename TO> constexpr int conv_occ() {
  using GE = CGeo<TW, KS, ST>;
  const size_t lds = GE::PATCH_BYTES + (size_t)4 * NJ * 16 * GE::TAPSP * 16;
  const int n = (int)((160 * 1024) / lds), cap = sizeof(TO) == 4 ? 4 : 5;
  return n > cap ? cap : n;
}

template <int NJ, int TW, int KS, int ST, typename TO>
__global__ void __launch_bounds__(CONV_TPB, (conv_occ<NJ, TW, KS, ST, TO>())) enc_conv_nhwc_kernel(ConvArgs a) {
  using GE = CGeo<TW, KS, ST>;
  constexpr int NP = GE::NPOS * 4, PM = (NP + CONV_TPB - 1) / CONV_TPB;     // patch pieces
  constexpr int NWQ = NJ * 16 * GE::TAPSP, NW = 4 * NWQ, WM = (NW + CONV_TPB - 1) / CONV_TPB;  // filter pieces
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const bf16_t* in = (const bf16_t*)a.in;
  TO* out = (TO*)a.out;
  bf16_t* patch = (bf16_t*)smem;                       // [4][NPOS][8]
  bf16_t* wl = (bf16_t*)(smem + GE::PATCH_BYTES);      // [4][NJ 16][TAPSP][8]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const int tw_n = (a.Wo + TW - 1) / TW, th_n = (a.Ho + GE::TH - 1) / GE::TH, per = tw_n * th_n;
  const int b = blockIdx.x / per, tix = blockIdx.x - b * per, tyi = tix / tw_n;
  const int oh0 = tyi * GE::TH, ow0 = (tix - tyi * tw_n) * TW, n0 = blockIdx.y * (NJ * 16);
  const int ih0 = oh0 * ST - a.pad, iw0 = ow0 * ST - a.pad;
  int pbase[2];  // stored position of tap (0, 0) for this lane's pixel in pixel tiles 0, 1
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = wave * 32 + i * 16 + r16, ty = q / TW, tx = q % TW;
    pbase[i] = ty * GE::PS * GE::PWS + tx;
  }
  // chunk-0 element offsets of this thread's pieces (chunk ck adds 32 ck / 4 Cout_pad TAPSP 8 ck).
  // Patch piece v: position p = 8 (v >> 5) + (v & 7) of plane q = (v >> 3) & 3 -- 8 consecutive lanes
  // write 8 consecutive positions of one plane; a wave's 64 lanes read 16 whole pixels.
  uint32_t poff[PM], woff[WM];  // BYTE offsets from the chunk's uniform base (saddr + voffset loads)
  int pdst[PM];
  uint32_t okm = 0;  // bit k: patch piece k lies inside the image (else it stages as zero)
#pragma unroll
  for (int k = 0; k < PM; ++k) {
    const int v = tid + k * CONV_TPB, vc = min(v, NP - 1);
    const int p = (vc >> 5) * 8 + (vc & 7), q = (vc >> 3) & 3, py = p / GE::PWS, pc = p % GE::PWS;
    const int px = GE::DI ? (pc < GE::HALF ? 2 * pc : 2 * (pc - GE::HALF) + 1) : pc;
    const int ih = ih0 + py * GE::SS, iw = iw0 + px * GE::SS;
    const bool ok = py < GE::PH && px < GE::PW && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
    const int ihc = min(max(ih, 0), a.H - 1), iwc = min(max(iw, 0), a.W - 1);
    poff[k] = (uint32_t)(((b * a.H + ihc) * a.W + iwc) * a.Cin + q * 8) * 2u;
    pdst[k] = (q * GE::NPOS + p) * 8;
    okm |= (ok && v < NP) ? (1u << k) : 0u;
  }
  const bf16_t* W = (const bf16_t*)a.wp;
  const int wstep = 4 * a.Cout_pad * GE::TAPSP * 8;  // elements per 32-channel chunk of the plane-major copy
#pragma unroll
  for (int k = 0; k < WM; ++k) {
    const int v = min(tid + k * CONV_TPB, NW - 1);  // clamped: every register is defined
    const int q = v / NWQ, r = v - q * NWQ;
    woff[k] = (uint32_t)(((q * a.Cout_pad + n0) * GE::TAPSP + r) * 8) * 2u;
  }
  f32x4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int cch = a.Cin >> 5;
  // buffer loads: uniform base + 32-bit lane offset + the chunk's scalar offset (no 64-bit address math)
  const __amdgpu_buffer_rsrc_t rin = conv_rsrc(in), rw = conv_rsrc(W);
  bf16x8 xr[PM], wr[WM];
  auto fetch = [&](int ck) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < PM; ++k)
      xr[k] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rin, (int)poff[k], ck * 64, 0));
#pragma unroll
    for (int k = 0; k < WM; ++k)
      wr[k] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, (int)woff[k], ck * wstep * 2, 0));
  };
  auto put = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < PM; ++k) {
      const int v = tid + k * CONV_TPB;
      if (v < NP) {
        const bf16x8 z = {};
        *(bf16x8*)(patch + pdst[k]) = ((okm >> k) & 1u) ? xr[k] : z;
      }
    }
#pragma unroll
    for (int k = 0; k < WM; ++k) {
      const int v = tid + k * CONV_TPB;
      if (v < NW) *(bf16x8*)(wl + v * 8) = wr[k];
    }
  };
  // this lane's LDS read bases (plane g): its two pixels' tap-(0, 0) positions, its filter row
  const bf16_t* pl[2] = {patch + (g * GE::NPOS + pbase[0]) * 8, patch + (g * GE::NPOS + pbase[1]) * 8};
  const bf16_t* wlb = wl + (g * NWQ + r16 * GE::TAPSP) * 8;
  fetch(0);
  for (int ck = 0; ck < cch; ++ck) {
    if (ck > 0) __syncthreads();  // the previous chunk's MFMAs are done with the LDS images
    put();
    __syncthreads();
    if (ck + 1 < cch) fetch(ck + 1);
#pragma unroll
    for (int tap = 0; tap < GE::TAPS; ++tap) {
      const int toff = (tap / KS) * GE::PWS + GE::col(tap % KS);  // compile-time: the ds_read offset field
      bf16x8 bv[2], av[NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i) bv[i] = *(const bf16x8*)(pl[i] + toff * 8);
#pragma unroll
      for (int j = 0; j < NJ; ++j) av[j] = *(const bf16x8*)(wlb + (j * 16 * GE::TAPSP + tap) * 8);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[j], bv[i], acc[i][j], 0, 0, 0);
    }
  }
  // epilogue: lane (pixel r16 of tile i, group g) holds output channels 16 j + 4 g .. + 3
  float cs[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[j][r] = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int co = n0 + j * 16 + 4 * g;
    const float4 bi = *(const float4*)(a.bias + co), sc = *(const float4*)(a.s + co), sh = *(const float4*)(a.t + co);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = wave * 32 + i * 16 + r16, oh = oh0 + q / TW, ow = ow0 + q % TW;
      const bool okp = oh < a.Ho && ow < a.Wo;
      float v[4] = {acc[i][j][0] + bi.x, acc[i][j][1] + bi.y, acc[i][j][2] + bi.z, acc[i][j][3] + bi.w};
      if (a.mode == CONV_RELU_BN) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      v[0] = v[0] * sc.x + sh.x;
      v[1] = v[1] * sc.y + sh.y;
      v[2] = v[2] * sc.z + sh.z;
      v[3] = v[3] * sc.w + sh.w;
      if (okp) {
        TO* dst = out + (((size_t)b * a.Ho + oh) * a.Wo + ow) * a.Cout_pad + co;
        if constexpr (sizeof(TO) == 2) {
          const uint32_t lo = pk_bf16(v[0], v[1]);
          const uint32_t hi = pk_bf16(v[2], v[3]);
          *(uint2*)dst = make_uint2(lo, hi);
        } else {
          *(float4*)dst = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[j][r] += okp ? v[r] : 0.f;
    }
  }
  if (a.se_part) {
    // SE squeeze of this tile (ResNetBlocks.py:81-96, the mean's first stage): per output channel
    // the sum of the tile's valid f32 outputs in a fixed order (pixel tiles, 16 pixel lanes, waves)
    // -> one [Cout_pad] row per (image, tile); enc_se_kernel adds the tiles in tile order
    __syncthreads();  // every wave is past the MMA loop: the patch / filter images are free
    float* red = (float*)smem;  // [4 waves][NJ * 16]
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float t = group_sum<16>(cs[j][r]);
        if (r16 == 0) red[wave * NJ * 16 + j * 16 + 4 * g + r] = t;
      }
    __syncthreads();
    if (tid < NJ * 16)
      a.se_part[((size_t)b * per + tix) * a.Cout_pad + n0 + tid] =
          (red[tid] + red[NJ * 16 + tid]) + (red[2 * NJ * 16 + tid] + red[3 * NJ * 16 + tid]);
  }
}

template <int NJ, int TW, int KS, int ST, typename TO>
hipError_t launch_conv_nhwc(const ConvArgs& a, hipStream_t s) {
  using GE = CGeo<TW, KS, ST>;
  constexpr size_t lds = GE::PATCH_BYTES + (size_t)4 * NJ * 16 * GE::TAPSP * 16;
  static_assert(lds <= 96 * 1024, "conv tile LDS");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)enc_conv_nhwc_kernel<NJ, TW, KS, ST, TO>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    attr = true;
  }
  const dim3 grid(a.N * ((a.Ho + GE::TH - 1) / GE::TH) * ((a.Wo + TW - 1) / TW), a.Cout_pad / (NJ * 16));
  hipLaunchKernelGGL((enc_conv_nhwc_kernel<NJ, TW, KS, ST, TO>), grid, dim3(CONV_TPB), lds, s, a);
  return hipGetLastError();
}

// the compile-time-geometry kernel for this shape, or nullptr (then the runtime-geometry kernel):
// the tower's convs (bf16 out) and the heads' (f32 out: 2x2 on the layer-2 map, 3x3 after the
// pixel shuffles)
typedef hipError_t (*ConvLaunch)(const ConvArgs&, hipStream_t);
ConvLaunch conv_nhwc_for(const ConvArgs& a) {
  if (!a.in_bf16 || !a.wp || a.layout != LAYOUT_NHWC || conv_no_lds || a.KH != a.KW) return nullptr;
  const int nj = a.Cout_pad % 64 == 0 ? 4 : 2, TW = a.Wo >= 16 ? 16 : a.Wo >= 8 ? 8 : 0;
  const int shape = a.KH * 10 + a.stride;
#define GGD_CONV_CASE(NJ_, TW_, KS_, ST_, TO_)                                             \
  if (nj == NJ_ && TW == TW_ && shape == KS_ * 10 + ST_ && (sizeof(TO_) == 2) == (a.out_bf16 != 0)) \
    return launch_conv_nhwc<NJ_, TW_, KS_, ST_, TO_>;
  GGD_CONV_CASE(4, 16, 3, 1, bf16_t) GGD_CONV_CASE(4, 8, 3, 1, bf16_t)
  GGD_CONV_CASE(2, 16, 3, 1, bf16_t) GGD_CONV_CASE(2, 8, 3, 1, bf16_t)
  GGD_CONV_CASE(4, 16, 3, 2, bf16_t) GGD_CONV_CASE(4, 8, 3, 2, bf16_t)
  GGD_CONV_CASE(4, 16, 1, 2, bf16_t) GGD_CONV_CASE(4, 8, 1, 2, bf16_t)
  GGD_CONV_CASE(4, 16, 2, 1, float) GGD_CONV_CASE(2, 16, 3, 1, float)
#undef GGD_CONV_CASE
  return nullptr;
}

// tile width of the LDS path for this shape, or 0 when the shape takes the direct kernel
int conv_lds_tw(int dtype, const ConvArgs& a) {
  if (dtype != GGD_BF16 || conv_no_lds) return 0;
  if (conv_nhwc_for(a)) return a.Wo >= 16 ? 16 : 8;
  const int nj = a.Cout_pad % 64 == 0 ? 4 : 2;
  const int TW = a.Wo >= 16 ? 16 : a.Wo >= 8 ? 8 : 4;
  const ConvLdsGeom G = conv_lds_geom(a, TW, nj);
  const int qp = a.in_bf16 ? 4 : 8;  // input pieces per patch position
  const bool fits = G.patch_bytes + G.w_bytes <= 96 * 1024 && G.PH * G.PW * qp <= CL_PMAX * CONV_TPB &&
                    G.taps <= CL_TAPS_MAX;
  return fits ? TW : 0;
}

// output tiles per image of the LDS path (the rows of ConvArgs::se_part per image)
int conv_lds_tiles(int Ho, int Wo) {
  const int TW = Wo >= 16 ? 16 : Wo >= 8 ? 8 : 4, TH = CL_PX / TW;
  return ((Ho + TH - 1) / TH) * ((Wo + TW - 1) / TW);
}

template <typename TI, typename TO>
hipError_t launch_conv_t(int dtype, const ConvArgs& a, hipStream_t s) {
  const int P = a.N * a.Ho * a.Wo;
  const int nj = a.Cout_pad % 64 == 0 ? 4 : 2;
  const dim3 grid(blocks_for(P, 128), a.Cout_pad / (nj * 16));
  if (a.se_part && !conv_lds_tw(dtype, a)) return hipErrorInvalidValue;  // only the LDS paths squeeze
  if (dtype == GGD_BF16)
    if (const ConvLaunch f = conv_nhwc_for(a)) return f(a, s);
  {
    const int TW = conv_lds_tw(dtype, a);
    const ConvLdsGeom G = conv_lds_geom(a, TW ? TW : 4, nj);
    const size_t lds = G.patch_bytes + G.w_bytes;
    const int qp = 32 / (16 / (int)sizeof(TI));
    if (TW) {
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)enc_conv_lds_kernel<4, CL_PMAX, TI, TO>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        (void)hipFuncSetAttribute((const void*)enc_conv_lds_kernel<2, CL_PMAX, TI, TO>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        (void)hipFuncSetAttribute((const void*)enc_conv_lds_kernel<4, CL_PMIN, TI, TO>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        (void)hipFuncSetAttribute((const void*)enc_conv_lds_kernel<2, CL_PMIN, TI, TO>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        attr = true;
      }
      const int blocks = a.N * ((a.Ho + G.TH - 1) / G.TH) * ((a.Wo + TW - 1) / TW);
      const dim3 gl(blocks, a.Cout_pad / (nj * 16));
      const bool small = G.PH * G.PW * qp <= CL_PMIN * CONV_TPB;
      if (nj == 4 && small) hipLaunchKernelGGL((enc_conv_lds_kernel<4, CL_PMIN, TI, TO>), gl, dim3(CONV_TPB), lds, s, a, TW);
      else if (nj == 4) hipLaunchKernelGGL((enc_conv_lds_kernel<4, CL_PMAX, TI, TO>), gl, dim3(CONV_TPB), lds, s, a, TW);
      else if (small) hipLaunchKernelGGL((enc_conv_lds_kernel<2, CL_PMIN, TI, TO>), gl, dim3(CONV_TPB), lds, s, a, TW);
      else hipLaunchKernelGGL((enc_conv_lds_kernel<2, CL_PMAX, TI, TO>), gl, dim3(CONV_TPB), lds, s, a, TW);
      return hipGetLastError();
    }
  }
  if (dtype == GGD_BF16) {
    if (nj == 4) hipLaunchKernelGGL((enc_conv_kernel<bf16_t, 4, TI, TO>), grid, dim3(CONV_TPB), 0, s, a);
    else hipLaunchKernelGGL((enc_conv_kernel<bf16_t, 2, TI, TO>), grid, dim3(CONV_TPB), 0, s, a);
  } else {
    if (nj == 4) hipLaunchKernelGGL((enc_conv_kernel<float, 4, TI, TO>), grid, dim3(CONV_TPB), 0, s, a);
    else hipLaunchKernelGGL((enc_conv_kernel<float, 2, TI, TO>), grid, dim3(CONV_TPB), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_conv(int dtype, const ConvArgs& a, hipStream_t s) {
  const int P = a.N * a.Ho * a.Wo;
  const int nj = a.Cout_pad % 64 == 0 ? 4 : 2;
  if (a.Cin % 32 || a.Cout_pad % (nj * 16) || P <= 0) return hipErrorInvalidValue;
  if (dtype != GGD_BF16 && (a.in_bf16 || a.out_bf16)) return hipErrorInvalidValue;  // f32 contexts stay f32
  if (a.in_bf16 && a.out_bf16) return launch_conv_t<bf16_t, bf16_t>(dtype, a, s);
  if (a.in_bf16) return launch_conv_t<bf16_t, float>(dtype, a, s);
  if (a.out_bf16) return launch_conv_t<float, bf16_t>(dtype, a, s);
  return launch_conv_t<float, float>(dtype, a, s);
}

struct EConv {            // one convolution + its folded BN epilogue
  int cin = 0, cin_pad = 0, cout = 0, cout_pad = 0, kh = 0, kw = 0, stride = 1, pad = 0;
  void* w = nullptr;      // T [cout_pad][kh*kw][cin_pad]
  void* wp = nullptr;     // bf16 contexts: plane-major copy [cin_pad / 32][4][cout_pad][taps | 1][8] (ConvArgs::wp)
  float *bias = nullptr, *s = nullptr, *t = nullptr;
};

struct EBlock {
  EConv c1, c2, ds;
  bool has_ds = false;
  int planes = 0;
  float *se_w0 = nullptr, *se_b0 = nullptr, *se_w2 = nullptr, *se_b2 = nullptr;
};

struct EHead {
  EConv conv;
  int shuffle = 1, K = 0;
  float *fc_w = nullptr, *fc_b = nullptr;
};

}  // namespace

struct ggd_enc {
  int device = 0, dtype = GGD_BF16, d_model = 0, wav_len = 0, max_batch = 0, chunk = 0;
  int F = 0;                                  // spectrogram frames
  int H[5] = {}, W[5] = {};                   // feature map sizes after conv1 / layer1..4
  int t_low = 0, t_mid = 0, t_high = 0;
  std::string err;
  std::map<std::string, std::vector<float>> staged;
  std::vector<void*> allocs;
  bool finalized = false;
  // weights
  float *window = nullptr, *twiddle = nullptr, *fb_val = nullptr, *fbT = nullptr, *zeros = nullptr;
  int *fb_lo = nullptr, *fb_n = nullptr, *fb_off = nullptr;  // the filterbank's nonzero band per mel bin
  float coef = 0.97f;
  float *c1_w = nullptr, *c1_b = nullptr, *c1_s = nullptr, *c1_t = nullptr;
  std::vector<EBlock> blocks;
  EHead head[3];
  float *proj_w = nullptr, *proj_b = nullptr;
  // workspaces (chunk clips)
  float *pw = nullptr, *mel = nullptr, *img = nullptr;
  void *buf[4] = {}, *feat[3] = {}, *sbuf = nullptr;   // activations: bf16 in bf16 contexts, else f32
  float *se_y = nullptr, *se_part = nullptr, *hbuf = nullptr;
  size_t asz = 4;                                     // bytes per activation element
};

namespace {

int efail(ggd_enc* e, int code, const std::string& msg) {
  if (e) e->err = msg;
  return code;
}

#define ENC_TRY(e, expr)                                                                      \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) return efail(e, GGD_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

template <typename P>
hipError_t ealloc(ggd_enc* e, P** p, size_t bytes) {
  void* q = nullptr;
  hipError_t r = hipMalloc(&q, std::max<size_t>(bytes, 16));
  if (r != hipSuccess) return r;
  e->allocs.push_back(q);
  *p = (P*)q;
  return hipSuccess;
}

hipError_t upload(ggd_enc* e, float** dst, const std::vector<float>& v) {
  hipError_t r = ealloc(e, dst, sizeof(float) * v.size());
  if (r != hipSuccess) return r;
  return hipMemcpy(*dst, v.data(), sizeof(float) * v.size(), hipMemcpyHostToDevice);
}

const std::string PFX = "speech_encoder.", FE = "speech_encoder.wav_encoder.feat_extractor.";

// torch conv2d output size
int conv_out(int n, int k, int s, int p) { return (n + 2 * p - k) / s + 1; }

}  // namespace

extern "C" {

int ggd_enc_create(int device, int32_t d_model, int32_t wav_len, int32_t max_batch, int32_t dtype, ggd_enc** out) {
  if (!out) return GGD_ERR_ARG;
  *out = nullptr;
  ggd_enc* e = new ggd_enc();
  *out = e;
  if (d_model <= 0 || wav_len < NFFT || max_batch <= 0) return efail(e, GGD_ERR_ARG, "bad encoder geometry");
  if (dtype != GGD_F32 && dtype != GGD_BF16) return efail(e, GGD_ERR_UNSUPPORTED, "unsupported dtype");
  e->device = device;
  e->d_model = d_model;
  e->wav_len = wav_len;
  e->max_batch = max_batch;
  e->dtype = dtype;
  e->chunk = std::min(max_batch, 128);
  e->F = 1 + wav_len / HOP;
  e->H[0] = NMEL;
  e->W[0] = e->F;
  e->H[1] = NMEL;
  e->W[1] = e->F;
  for (int l = 2; l <= 4; ++l) {
    e->H[l] = conv_out(e->H[l - 1], 3, 2, 1);
    e->W[l] = conv_out(e->W[l - 1], 3, 2, 1);
  }
  e->t_low = e->W[2] - 1;          // conv 2x2, no padding
  e->t_mid = e->W[3] * 2 - 2;      // pixel shuffle x2, conv 3x3
  e->t_high = e->W[4] * 4 - 2;     // pixel shuffle x4, conv 3x3
  return GGD_OK;                   // no device call before ggd_enc_finalize (geometry is host-only)
}

int ggd_enc_destroy(ggd_enc* e) {
  if (!e) return GGD_OK;
  if (!e->allocs.empty()) {
    (void)hipSetDevice(e->device);
    (void)hipDeviceSynchronize();
    for (void* p : e->allocs) (void)hipFree(p);
  }
  delete e;
  return GGD_OK;
}

const char* ggd_enc_last_error(const ggd_enc* e) { return e ? e->err.c_str() : "null encoder context"; }

int ggd_enc_lengths(const ggd_enc* e, int32_t* t_low, int32_t* t_mid, int32_t* t_high) {
  if (!e || !t_low || !t_mid || !t_high) return GGD_ERR_ARG;
  *t_low = e->t_low;
  *t_mid = e->t_mid;
  *t_high = e->t_high;
  return GGD_OK;
}

int ggd_enc_load_weight(ggd_enc* e, const char* name, const float* host, int64_t numel) {
  if (!e || !name || (!host && numel > 0) || numel < 0) return efail(e, GGD_ERR_ARG, "null argument");
  const std::string n(name);
  if (n.compare(0, PFX.size(), PFX) != 0) return GGD_IGNORED;
  e->staged[n].assign(host, host + numel);
  e->finalized = false;
  return GGD_OK;
}

}  // extern "C"

namespace {

int need(ggd_enc* e, const std::string& name, size_t numel, const std::vector<float>** out) {
  auto it = e->staged.find(name);
  if (it == e->staged.end()) return efail(e, GGD_ERR_NAME, "missing encoder weight " + name);
  if (it->second.size() != numel)
    return efail(e, GGD_ERR_NAME, "encoder weight " + name + " has " + std::to_string(it->second.size()) +
                                      " elements, expected " + std::to_string(numel));
  *out = &it->second;
  return GGD_OK;
}

#define NEED(name, numel, ptr)                     \
  do {                                             \
    int _r = need(e, (name), (numel), &(ptr));     \
    if (_r) return _r;                             \
  } while (0)

// BatchNorm2d (eval) folded to y = x * s + t; bias of the preceding conv kept apart (ReLU sits
// between them in the ReLU-then-BN blocks)
int fold_bn(ggd_enc* e, const std::string& bn, int c, int cpad, std::vector<float>& s, std::vector<float>& t) {
  const std::vector<float> *g, *b, *rm, *rv;
  NEED(bn + ".weight", c, g);
  NEED(bn + ".bias", c, b);
  NEED(bn + ".running_mean", c, rm);
  NEED(bn + ".running_var", c, rv);
  s.assign(cpad, 0.f);
  t.assign(cpad, 0.f);
  for (int i = 0; i < c; ++i) {
    const double sc = (double)(*g)[i] / std::sqrt((double)(*rv)[i] + 1e-5);
    s[i] = (float)sc;
    t[i] = (float)((double)(*b)[i] - (double)(*rm)[i] * sc);
  }
  return GGD_OK;
}

int make_conv(ggd_enc* e, EConv& cv, const std::string& conv, const std::string& bn, int cin, int cout, int k,
              int stride, int pad, bool bias) {
  cv.cin = cin;
  cv.cin_pad = (cin + 31) / 32 * 32;
  cv.cout = cout;
  cv.cout_pad = cout <= 32 ? 32 : (cout + 63) / 64 * 64;
  cv.kh = cv.kw = k;
  cv.stride = stride;
  cv.pad = pad;
  const std::vector<float>* w;
  NEED(conv + ".weight", (size_t)cout * cin * k * k, w);
  std::vector<float> bb(cv.cout_pad, 0.f), s, t;
  if (bias) {
    const std::vector<float>* b;
    NEED(conv + ".bias", cout, b);
    std::copy(b->begin(), b->end(), bb.begin());
  }
  int r = fold_bn(e, bn, cout, cv.cout_pad, s, t);
  if (r) return r;
  // [cout][cin][ky][kx] -> [cout_pad][ky * k + kx][cin_pad]
  const int taps = k * k;
  std::vector<float> p((size_t)cv.cout_pad * taps * cv.cin_pad, 0.f);
  for (int o = 0; o < cout; ++o)
    for (int i = 0; i < cin; ++i)
      for (int q = 0; q < taps; ++q) p[((size_t)o * taps + q) * cv.cin_pad + i] = (*w)[((size_t)o * cin + i) * taps + q];
  if (e->dtype == GGD_BF16) {
    std::vector<uint16_t> h(p.size());
    for (size_t i = 0; i < p.size(); ++i) {  // round to nearest even
      uint32_t u;
      std::memcpy(&u, &p[i], 4);
      h[i] = (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
    }
    ENC_TRY(e, ealloc(e, &cv.w, h.size() * 2));
    ENC_TRY(e, hipMemcpy(cv.w, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    const int tp = taps | 1, cch = cv.cin_pad / 32;
    std::vector<uint16_t> hp((size_t)cch * 4 * cv.cout_pad * tp * 8, 0);
    for (int ck = 0; ck < cch; ++ck)
      for (int q = 0; q < 4; ++q)
        for (int o = 0; o < cv.cout_pad; ++o)
          for (int tap = 0; tap < taps; ++tap)
            for (int el = 0; el < 8; ++el)
              hp[((((size_t)ck * 4 + q) * cv.cout_pad + o) * tp + tap) * 8 + el] =
                  h[((size_t)o * taps + tap) * cv.cin_pad + ck * 32 + q * 8 + el];
    ENC_TRY(e, ealloc(e, &cv.wp, hp.size() * 2));
    ENC_TRY(e, hipMemcpy(cv.wp, hp.data(), hp.size() * 2, hipMemcpyHostToDevice));
  } else {
    ENC_TRY(e, ealloc(e, &cv.w, p.size() * 4));
    ENC_TRY(e, hipMemcpy(cv.w, p.data(), p.size() * 4, hipMemcpyHostToDevice));
  }
  ENC_TRY(e, upload(e, &cv.bias, bb));
  ENC_TRY(e, upload(e, &cv.s, s));
  ENC_TRY(e, upload(e, &cv.t, t));
  return GGD_OK;
}

int make_lin(ggd_enc* e, const std::string& name, int out, int in, float** w, float** b) {
  const std::vector<float> *pw, *pb;
  NEED(name + ".weight", (size_t)out * in, pw);
  NEED(name + ".bias", out, pb);
  ENC_TRY(e, upload(e, w, *pw));
  ENC_TRY(e, upload(e, b, *pb));
  return GGD_OK;
}

ConvArgs conv_args(ggd_enc* e, const EConv& cv, const void* in, int n, int H, int W, void* out, int mode, int layout,
                   bool out_act) {
  ConvArgs a{};
  a.in = in;
  a.in_bf16 = e->asz == 2;
  a.out_bf16 = out_act && e->asz == 2;   // the heads' outputs feed f32 Linear layers
  a.w = cv.w;
  a.wp = cv.wp;
  a.bias = cv.bias;
  a.s = cv.s;
  a.t = cv.t;
  a.out = out;
  a.N = n;
  a.H = H;
  a.W = W;
  a.Cin = cv.cin_pad;
  a.Ho = conv_out(H, cv.kh, cv.stride, cv.pad);
  a.Wo = conv_out(W, cv.kw, cv.stride, cv.pad);
  a.Cout_pad = cv.cout_pad;
  a.Cvalid = cv.cout;
  a.KH = cv.kh;
  a.KW = cv.kw;
  a.stride = cv.stride;
  a.pad = cv.pad;
  a.mode = mode;
  a.layout = layout;
  return a;
}

// se_S non-null: squeeze into e->se_part in the epilogue when the shape takes the LDS path, and
// return its rows per image there (0: not squeezed, the caller runs enc_se_sum_kernel)
int run_conv(ggd_enc* e, const EConv& cv, const void* in, int n, int H, int W, void* out, int mode, int layout,
             hipStream_t s, bool out_act = true, int* se_S = nullptr) {
  ConvArgs a = conv_args(e, cv, in, n, H, W, out, mode, layout, out_act);
  if (se_S) {
    *se_S = 0;
    if (conv_lds_tw(e->dtype, a) && layout == LAYOUT_NHWC) {
      a.se_part = e->se_part;
      *se_S = conv_lds_tiles(a.Ho, a.Wo);
    }
  }
  ENC_TRY(e, launch_conv(e->dtype, a, s));
  return GGD_OK;
}

}  // namespace

extern "C" {

int ggd_enc_finalize(ggd_enc* e) {
  if (!e) return GGD_ERR_ARG;
  ENC_TRY(e, hipSetDevice(e->device));
  const std::vector<float> *win, *fb, *pre;
  NEED(PFX + "wav2spec.1.spectrogram.window", NFFT, win);
  NEED(PFX + "wav2spec.1.mel_scale.fb", (size_t)NBIN * NMEL, fb);
  NEED(PFX + "wav2spec.0.flipped_filter", 2, pre);
  e->coef = -(*pre)[0];
  // FFT twiddles exp(-2 pi i t / n_fft), t < n_fft / 2, as (re, im) pairs
  std::vector<float> tw((size_t)NFFT, 0.f);
  for (int t = 0; t < NFFT / 2; ++t) {
    const double ang = 2.0 * M_PI * (double)t / NFFT;
    tw[2 * t] = (float)std::cos(ang);
    tw[2 * t + 1] = (float)(-std::sin(ang));
  }
  ENC_TRY(e, upload(e, &e->twiddle, tw));
  ENC_TRY(e, upload(e, &e->window, *win));
  {  // each mel filter's band of nonzero bins [lo, lo + n) and its values (any matrix works: a dense
     // column is a band of all 513 bins)
    std::vector<int> lo(NMEL), cnt(NMEL), off(NMEL);
    std::vector<float> val;
    for (int m = 0; m < NMEL; ++m) {
      int first = -1, last = -1;
      for (int f = 0; f < NBIN; ++f)
        if ((*fb)[(size_t)f * NMEL + m] != 0.f) {
          if (first < 0) first = f;
          last = f;
        }
      lo[m] = first < 0 ? 0 : first;
      cnt[m] = first < 0 ? 0 : last - first + 1;
      off[m] = (int)val.size();
      for (int f = lo[m]; f < lo[m] + cnt[m]; ++f) val.push_back((*fb)[(size_t)f * NMEL + m]);
    }
    val.push_back(0.f);
    ENC_TRY(e, upload(e, &e->fb_val, val));
    ENC_TRY(e, ealloc(e, &e->fb_lo, sizeof(int) * NMEL));
    ENC_TRY(e, ealloc(e, &e->fb_n, sizeof(int) * NMEL));
    ENC_TRY(e, ealloc(e, &e->fb_off, sizeof(int) * NMEL));
    ENC_TRY(e, hipMemcpy(e->fb_lo, lo.data(), sizeof(int) * NMEL, hipMemcpyHostToDevice));
    ENC_TRY(e, hipMemcpy(e->fb_n, cnt.data(), sizeof(int) * NMEL, hipMemcpyHostToDevice));
    ENC_TRY(e, hipMemcpy(e->fb_off, off.data(), sizeof(int) * NMEL, hipMemcpyHostToDevice));
  }
  std::vector<float> fbT((size_t)NMEL * 768, 0.f);  // the dense matrix of the training front end's GEMM
  for (int m = 0; m < NMEL; ++m)
    for (int f = 0; f < NBIN; ++f) fbT[(size_t)m * 768 + f] = (*fb)[(size_t)f * NMEL + m];
  ENC_TRY(e, upload(e, &e->fbT, fbT));
  ENC_TRY(e, upload(e, &e->zeros, std::vector<float>(NMEL, 0.f)));

  // conv1 + bn1
  {
    const std::vector<float> *w, *b;
    NEED(FE + "conv1.weight", 32 * 9, w);
    NEED(FE + "conv1.bias", 32, b);
    std::vector<float> s, t;
    int r = fold_bn(e, FE + "bn1", 32, 32, s, t);
    if (r) return r;
    ENC_TRY(e, upload(e, &e->c1_w, *w));
    ENC_TRY(e, upload(e, &e->c1_b, *b));
    ENC_TRY(e, upload(e, &e->c1_s, s));
    ENC_TRY(e, upload(e, &e->c1_t, t));
  }
  e->blocks.clear();
  int inplanes = 32;
  const int planes_l[4] = {32, 64, 128, 256}, nblk[4] = {3, 4, 6, 3}, stride_l[4] = {1, 2, 2, 2};
  for (int l = 0; l < 4; ++l)
    for (int bi = 0; bi < nblk[l]; ++bi) {
      const std::string q = FE + "layer" + std::to_string(l + 1) + "." + std::to_string(bi) + ".";
      EBlock B;
      B.planes = planes_l[l];
      const int st = bi == 0 ? stride_l[l] : 1;
      int r = make_conv(e, B.c1, q + "conv1", q + "bn1", inplanes, B.planes, 3, st, 1, false);
      if (!r) r = make_conv(e, B.c2, q + "conv2", q + "bn2", B.planes, B.planes, 3, 1, 1, false);
      if (r) return r;
      B.has_ds = e->staged.count(q + "downsample.0.weight") != 0;
      if (B.has_ds) {
        r = make_conv(e, B.ds, q + "downsample.0", q + "downsample.1", inplanes, B.planes, 1, st, 0, false);
        if (r) return r;
      } else if (st != 1 || inplanes != B.planes) {
        return efail(e, GGD_ERR_NAME, "missing " + q + "downsample.0.weight");
      }
      r = make_lin(e, q + "se.fc.0", B.planes / 8, B.planes, &B.se_w0, &B.se_b0);
      if (!r) r = make_lin(e, q + "se.fc.2", B.planes, B.planes / 8, &B.se_w2, &B.se_b2);
      if (r) return r;
      e->blocks.push_back(B);
      inplanes = B.planes;
    }
  // heads: (conv, bn, fc, shuffle, channels in / out, kernel)
  const char* hn[3] = {"low", "mid", "high"};
  const int hc[3] = {64, 32, 16}, hk[3] = {2, 3, 3}, hs[3] = {1, 2, 4};
  const int hh[3] = {conv_out(e->H[2], 2, 1, 0), conv_out(e->H[3] * 2, 3, 1, 0), conv_out(e->H[4] * 4, 3, 1, 0)};
  for (int i = 0; i < 3; ++i) {
    EHead& h = e->head[i];
    h.shuffle = hs[i];
    int r = make_conv(e, h.conv, FE + "conv_" + hn[i], FE + "bn_" + hn[i], hc[i], hc[i], hk[i], 1, 0, true);
    if (r) return r;
    h.K = hc[i] * hh[i];
    {  // fc_* columns from the reference's (c, h) flatten order to the kernel's (h, c) order
      const std::vector<float> *pw, *pb;
      NEED(FE + "fc_" + hn[i] + ".weight", (size_t)32 * h.K, pw);
      NEED(FE + "fc_" + hn[i] + ".bias", 32, pb);
      std::vector<float> wt((size_t)32 * h.K);
      for (int j = 0; j < 32; ++j)
        for (int c = 0; c < hc[i]; ++c)
          for (int y = 0; y < hh[i]; ++y)
            wt[(size_t)j * h.K + (size_t)y * hc[i] + c] = (*pw)[(size_t)j * h.K + (size_t)c * hh[i] + y];
      ENC_TRY(e, upload(e, &h.fc_w, wt));
      ENC_TRY(e, upload(e, &h.fc_b, *pb));
    }
  }
  {
    int r = make_lin(e, PFX + "wav_proj_layer", e->d_model, 32, &e->proj_w, &e->proj_b);
    if (r) return r;
  }
  // workspaces for one chunk of clips
  const size_t n = e->chunk, F = e->F;
  e->asz = e->dtype == GGD_BF16 ? 2 : 4;
  ENC_TRY(e, ealloc(e, &e->pw, sizeof(float) * n * F * POW_LD));
  ENC_TRY(e, ealloc(e, &e->mel, sizeof(float) * n * F * NMEL));
  ENC_TRY(e, ealloc(e, &e->img, sizeof(float) * n * F * NMEL));
  size_t big = 0;
  for (int l = 1; l <= 4; ++l) big = std::max(big, (size_t)e->H[l] * e->W[l] * planes_l[l - 1]);
  for (int i = 0; i < 4; ++i) ENC_TRY(e, ealloc(e, &e->buf[i], e->asz * n * big));
  for (int i = 0; i < 3; ++i)
    ENC_TRY(e, ealloc(e, &e->feat[i], e->asz * n * e->H[i + 2] * e->W[i + 2] * planes_l[i + 1]));
  ENC_TRY(e, ealloc(e, &e->se_y, sizeof(float) * n * 256));
  int se_rows = SE_SLICES;
  for (int l = 1; l <= 4; ++l) se_rows = std::max(se_rows, conv_lds_tiles(e->H[l], e->W[l]));
  ENC_TRY(e, ealloc(e, &e->se_part, sizeof(float) * n * se_rows * 256));
  ENC_TRY(e, ealloc(e, &e->sbuf, e->asz * n * 32 *
                                    std::max((size_t)e->H[3] * 2 * e->W[3] * 2, (size_t)e->H[4] * 4 * e->W[4] * 4)));
  size_t hb = 0;
  for (int i = 0; i < 3; ++i) hb = std::max(hb, (size_t)e->head[i].K * (size_t)(e->W[2] + e->W[4] * 4));
  ENC_TRY(e, ealloc(e, &e->hbuf, sizeof(float) * n * hb));
  e->staged.clear();
  e->finalized = true;
  return GGD_OK;
}

int ggd_enc_frontend(ggd_enc* e, const float* wav, int32_t n, float* img, void* stream) {
  if (!e || !wav || !img) return efail(e, GGD_ERR_ARG, "null argument");
  if (!e->finalized) return efail(e, GGD_ERR_STATE, "encoder weights not finalized");
  if (n <= 0 || n > e->max_batch) return efail(e, GGD_ERR_ARG, "batch outside [1, max_batch]");
  ENC_TRY(e, hipSetDevice(e->device));
  hipStream_t s = (hipStream_t)stream;
  const int F = e->F;
  for (int c0 = 0; c0 < n; c0 += e->chunk) {
    const int m = std::min(e->chunk, n - c0);
    hipLaunchKernelGGL(enc_stft_power_kernel, dim3(m * F), dim3(256), 0, s, wav + (size_t)c0 * e->wav_len, e->window,
                       (const float2*)e->twiddle, e->pw, e->wav_len, F, e->coef);
    ENC_TRY(e, hipGetLastError());
    GemmArgs g{};
    g.M = m * F;
    g.bias = e->zeros;
    g.N = NMEL;
    g.K = 768;
    g.k_valid = NBIN;
    g.A = e->pw;
    g.lda = POW_LD;
    g.W = e->fbT;
    g.out = e->mel;
    g.ldo = NMEL;
    g.n_valid = NMEL;
    ENC_TRY(e, launch_gemm(GGD_F32, PRO_F32, EPI_F32, g, s));
    hipLaunchKernelGGL(enc_inorm_kernel, dim3(m), dim3(4 * NMEL), 0, s, e->mel, img + (size_t)c0 * NMEL * F, F);
    ENC_TRY(e, hipGetLastError());
  }
  return GGD_OK;
}

}  // extern "C"

namespace {
// Where the heads write token t of clip c of level l: z[l] + ((c rows + off[l] + t) ld + col)
// floats (col folded into z[l]); pad[l] rows in front of the level are zeroed (s2g_v2 memory)
struct MemMap {
  float* z[3];
  int rows, ld, off[3], pad[3];
};

int enc_run(ggd_enc* e, const float* wav, int32_t n, const MemMap& mm, hipStream_t s);
}  // namespace

extern "C" {

int ggd_enc_run(ggd_enc* e, const float* wav, int32_t n, float* z_low, float* z_mid, float* z_high, void* stream) {
  if (!e || !wav || !z_low || !z_mid || !z_high) return efail(e, GGD_ERR_ARG, "null argument");
  if (!e->finalized) return efail(e, GGD_ERR_STATE, "encoder weights not finalized");
  MemMap mm{};  // three separate (N, T_l, d) tensors: rows = 0 -> each level's own T_l
  float* z[3] = {z_low, z_mid, z_high};
  for (int l = 0; l < 3; ++l) mm.z[l] = z[l];
  mm.ld = e->d_model;
  return enc_run(e, wav, n, mm, (hipStream_t)stream);
}

int ggd_enc_run_memory(ggd_enc* e, const float* wav, int32_t n, int32_t layout, float* mem, void* stream) {
  if (!e || !wav || !mem) return efail(e, GGD_ERR_ARG, "null argument");
  if (!e->finalized) return efail(e, GGD_ERR_STATE, "encoder weights not finalized");
  const int d = e->d_model, t[3] = {e->t_low, e->t_mid, e->t_high};
  MemMap mm{};
  if (layout == GGD_MEM_BLEND) {  // (N, Tmax, 3d): level l in columns [l d, l d + d), left-zero-padded
    const int tm = std::max(t[0], std::max(t[1], t[2]));
    mm.rows = tm;
    mm.ld = 3 * d;
    for (int l = 0; l < 3; ++l) {
      mm.z[l] = mem + (size_t)l * d;
      mm.pad[l] = mm.off[l] = tm - t[l];
    }
  } else if (layout == GGD_MEM_CONCAT) {  // (N, T_low + T_mid + T_high, d): levels one after another
    mm.rows = t[0] + t[1] + t[2];
    mm.ld = d;
    for (int l = 0, o = 0; l < 3; o += t[l], ++l) {
      mm.z[l] = mem;
      mm.off[l] = o;
      mm.pad[l] = 0;
    }
  } else {
    return efail(e, GGD_ERR_ARG, "unknown memory layout");
  }
  return enc_run(e, wav, n, mm, (hipStream_t)stream);
}

}  // extern "C"

namespace {
int enc_run(ggd_enc* e, const float* wav, int32_t n, const MemMap& mm, hipStream_t s) {
  if (n <= 0 || n > e->max_batch) return efail(e, GGD_ERR_ARG, "batch outside [1, max_batch]");
  ENC_TRY(e, hipSetDevice(e->device));
  const int F = e->F, d = e->d_model;
  for (int c0 = 0; c0 < n; c0 += e->chunk) {
    const int m = std::min(e->chunk, n - c0);
    const float* w = wav + (size_t)c0 * e->wav_len;
    // front end: STFT power, then the mel GEMM
    hipLaunchKernelGGL(enc_stft_mel_kernel, dim3(m * F), dim3(256), 0, s, w, e->window, (const float2*)e->twiddle,
                       e->fb_lo, e->fb_n, e->fb_off, e->fb_val, e->mel, e->wav_len, F, e->coef);
    ENC_TRY(e, hipGetLastError());
    hipLaunchKernelGGL(enc_inorm_kernel, dim3(m), dim3(4 * NMEL), 0, s, e->mel, e->img, F);
    ENC_TRY(e, hipGetLastError());
    const size_t n1 = (size_t)m * e->H[1] * e->W[1] * 4;
    const bool hb = e->asz == 2;
    if (hb)
      hipLaunchKernelGGL(enc_conv1_kernel<bf16_t>, dim3(blocks_for(n1, 256)), dim3(256), 0, s, e->img, e->c1_w, e->c1_b,
                         e->c1_s, e->c1_t, (bf16_t*)e->buf[0], m, e->H[1], e->W[1]);
    else
      hipLaunchKernelGGL(enc_conv1_kernel<float>, dim3(blocks_for(n1, 256)), dim3(256), 0, s, e->img, e->c1_w, e->c1_b,
                         e->c1_s, e->c1_t, (float*)e->buf[0], m, e->H[1], e->W[1]);
    ENC_TRY(e, hipGetLastError());
    // residual tower: x is the current input; u, v, r are the scratch buffers other than x
    const void* x = e->buf[0];
    int H = e->H[1], W = e->W[1], bidx = 0;
    const int nblk[4] = {3, 4, 6, 3};
    for (int l = 0; l < 4; ++l)
      for (int bi = 0; bi < nblk[l]; ++bi, ++bidx) {
        const EBlock& B = e->blocks[bidx];
        void* sc[3];
        for (int i = 0, k = 0; i < 4 && k < 3; ++i)
          if (e->buf[i] != x) sc[k++] = e->buf[i];
        void *u = sc[0], *v = sc[1], *r = sc[2];
        const int Ho = conv_out(H, 3, B.c1.stride, 1), Wo = conv_out(W, 3, B.c1.stride, 1);
        int S = 0;  // the squeeze's partial-sum rows per image (conv2's tiles when its epilogue sums)
        int rc = run_conv(e, B.c1, x, m, H, W, u, CONV_RELU_BN, LAYOUT_NHWC, s);
        if (!rc) rc = run_conv(e, B.c2, u, m, Ho, Wo, v, CONV_BN, LAYOUT_NHWC, s, true, &S);
        const void* res = x;
        if (!rc && B.has_ds) {
          rc = run_conv(e, B.ds, x, m, H, W, r, CONV_BN, LAYOUT_NHWC, s);
          res = r;
        }
        if (rc) return rc;
        if (!S) {
          S = std::max(1, std::min(SE_SLICES, Ho * Wo / 64));
          if (hb)
            hipLaunchKernelGGL(enc_se_sum_kernel<bf16_t>, dim3(m, S), dim3(256), 0, s, (const bf16_t*)v, Ho * Wo,
                               B.planes, e->se_part);
          else
            hipLaunchKernelGGL(enc_se_sum_kernel<float>, dim3(m, S), dim3(256), 0, s, (const float*)v, Ho * Wo,
                               B.planes, e->se_part);
          ENC_TRY(e, hipGetLastError());
        }
        // the block output goes to u (consumed by conv2 already), or to the saved feature map
        // of layers 2..4 that the heads read
        void* o = (bi == nblk[l] - 1 && l >= 1) ? e->feat[l - 1] : u;
        hipLaunchKernelGGL(enc_se_kernel, dim3(m), dim3(256), 0, s, e->se_part, S, Ho * Wo, B.planes, B.se_w0,
                           B.se_b0, B.se_w2, B.se_b2, e->se_y);
        ENC_TRY(e, hipGetLastError());
        const size_t tot8 = (size_t)m * Ho * Wo * B.planes / 8;
        if (hb)
          hipLaunchKernelGGL(enc_se_apply_kernel<bf16_t>, dim3(blocks_for(tot8, 256)), dim3(256), 0, s, (const bf16_t*)v,
                             e->se_y, (const bf16_t*)res, (bf16_t*)o, Ho * Wo, B.planes, tot8);
        else
          hipLaunchKernelGGL(enc_se_apply_kernel<float>, dim3(blocks_for(tot8, 256)), dim3(256), 0, s, (const float*)v,
                             e->se_y, (const float*)res, (float*)o, Ho * Wo, B.planes, tot8);
        ENC_TRY(e, hipGetLastError());
        x = o;
        H = Ho;
        W = Wo;
      }
    // heads: each level's tokens straight into their place (MemMap)
    const int tl[3] = {e->t_low, e->t_mid, e->t_high};
    for (int i = 0; i < 3; ++i) {
      const EHead& h = e->head[i];
      const void* fin = e->feat[i];
      int Hh = e->H[i + 2], Wh = e->W[i + 2];
      if (h.shuffle > 1) {
        const int C = h.conv.cin, r = h.shuffle;
        const size_t tot = (size_t)m * Hh * r * Wh * r * (h.conv.cin_pad / 8);
        if (hb)
          hipLaunchKernelGGL(enc_shuffle_kernel<bf16_t>, dim3(blocks_for(tot, 256)), dim3(256), 0, s, (const bf16_t*)fin,
                             (bf16_t*)e->sbuf, m, Hh, Wh, C, r, h.conv.cin_pad);
        else
          hipLaunchKernelGGL(enc_shuffle_kernel<float>, dim3(blocks_for(tot, 256)), dim3(256), 0, s, (const float*)fin,
                             (float*)e->sbuf, m, Hh, Wh, C, r, h.conv.cin_pad);
        ENC_TRY(e, hipGetLastError());
        fin = e->sbuf;
        Hh *= r;
        Wh *= r;
      }
      int rc = run_conv(e, h.conv, fin, m, Hh, Wh, e->hbuf, CONV_RELU_BN, LAYOUT_NHWC, s, false);
      if (rc) return rc;
      const int Wo = conv_out(Wh, h.conv.kw, 1, 0);
      if (Wo != tl[i]) return efail(e, GGD_ERR_STATE, "head length mismatch");
      const int Ho = conv_out(Hh, h.conv.kh, 1, 0), C = h.conv.cout;
      if (h.K % 16 || h.K != C * Ho || (C & (C - 1)) || C % 4) return efail(e, GGD_ERR_STATE, "head feature shape");
      const int zrows = mm.rows ? mm.rows : tl[i];
      float* zc = mm.z[i] + (size_t)c0 * zrows * mm.ld;
      hipLaunchKernelGGL(enc_head_fc_kernel, dim3((m * Wo + 15) / 16), dim3(64 * HFC_WAVES), 0, s, e->hbuf, m * Wo, h.K, Ho, Wo,
                         h.conv.cout_pad, __builtin_ctz(C), h.fc_w, h.fc_b, e->proj_w, e->proj_b, zc, d, zrows, mm.ld,
                         mm.off[i]);
      ENC_TRY(e, hipGetLastError());
      if (mm.pad[i] > 0) {
        hipLaunchKernelGGL(enc_zpad_kernel, dim3(m), dim3(256), 0, s, zc, mm.pad[i], d, zrows, mm.ld);
        ENC_TRY(e, hipGetLastError());
      }
    }
  }
  return GGD_OK;
}
}  // namespace
