// ggd_train.hip -- f32 forward / backward / optimizer kernels of the training path (gfx950).
//
// The reference trains in fp32 with PyTorch autograd (models/trainer.py:131-248 ->
// gaussian_diffusion.py:531-569 training_losses -> model.py:81-117 -> nn.py:154-228 ->
// transformer.py:8-154), AdamW (model_creation.py:176-178) and DDP's NCCL all-reduce
// (trainer.py:83, utils/pytorch_ddp.py:18).  Here every op of the decoder step has a
// hand-written forward and backward kernel; the host (…_amd/training.py) chains them through
// torch.autograd.Function and owns the buffers.  Layout: token-major rows [clip][frame][feature].
//
//   tgemm_kernel<TA, TB, GM>  C = alpha op(A) op(B) + beta C (+ bias): Linear forward (NT), dX (NN),
//                         dW (TN) on v_mfma_f32_16x16x4_f32 (exact f32 products), 64 x 64 tiles
//                         (split-K with a fixed-order slice reduction when few tiles cover a long K);
//                         GM != 0: the encoder's convolutions as implicit GEMMs (forward, dgrad,
//                         wgrad), the conv operand gathered from the NHWC image while it is staged
//   colsum_partial / _final  bias and LayerNorm affine gradients: two-stage column sums
//   ln_fwd / ln_bwd       LayerNorm (eps 1e-5) with saved mean / rstd
//   seqconv_fwd / _bwd / _param_grad  SpatialDepthWiseConv (3 taps along frames, per d_k channel,
//                         shared by heads and clips: transformer.py:19-44)
//   attn_fwd / attn_bwd   softmax(Q K^T scale) V per (clip, head), P recomputed in backward
//   ew_kernel             ReLU^2 / SiLU forward and backward, add
//   qsample / mse         x_t = sqrt(abar) x0 + sqrt(1 - abar) eps; per-clip MSE and its gradient
//   sumsq / adamw / scale grad norm, torch.optim.AdamW's update order, clipping
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "../../include/ggd_train.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TT = 256;  // threads per block of the element / row kernels

// ------------------------------------------------------------------------------------------
// GEMM: C[M][N] = alpha sum_k opA[m][k] opB[k][n] + beta C[m][n] + bias[n]
//   opA[m][k] = TA ? A[k lda + m] : A[m lda + k];  opB[k][n] = TB ? B[n ldb + k] : B[k ldb + n]
// 256 threads = 4 waves in 2 x 2, each 32 x 32 of the 64 x 64 tile (2 x 2 MFMA 16 x 16 blocks);
// K in chunks of 16 staged through LDS as [row][k] images (stride 17: conflict-free columns).
// ------------------------------------------------------------------------------------------
constexpr int GT = 64, GK = 16, GS = GK + 1;

// Implicit-GEMM convolutions (NHWC activations, nn.Conv2d, ha2g/model/ResNetBlocks.py:21-37): the
// conv operand is gathered from the image while it is staged, instead of through an im2col copy.
//   G_CONV_A   forward:  A[m = (n, oh, ow)][k = (ky, kx, c)] = x[n][oh s - pad + ky][ow s - pad + kx][c]
//   G_DCONV_A  dgrad:    A[m = (n, ih, iw)][k = (ky, kx, co)] = dy[n][(ih + pad - ky) / s][(iw + pad - kx) / s][co]
//                        where the division is exact and in range (the adjoint of the forward gather)
//   G_CONV_B   wgrad:    B[k = (n, oh, ow)][j = (ky, kx, c)] = the forward gather, K = output pixels
// (0 outside the image).  The gathered axis (c / co) must be a multiple of 4: a thread stages 4
// consecutive k (A) or j (B) of one tap -- one 16-byte load.
struct ConvGeo { int H, W, C, KH, KW, st, pad, Ho, Wo, Co; };
constexpr int G_PLAIN = 0, G_CONV_A = 1, G_DCONV_A = 2, G_CONV_B = 3;

__device__ __forceinline__ float4 ld4(const float* p) { return *(const float4*)p; }

// Split-K (part != null): slice blockIdx.z covers k in [z kchunk, (z + 1) kchunk) and stores its
// raw f32 accumulators to part[z][M][N]; splitk_reduce_kernel adds the slices in a fixed order.
template <bool TA, bool TB, int GM = G_PLAIN>
__global__ void __launch_bounds__(256) tgemm_kernel(int M, int N, int K, float alpha, const float* __restrict__ A, int lda,
                                                    const float* __restrict__ B, int ldb, float beta, float* C, int ldc,
                                                    const float* __restrict__ bias, int kchunk, float* part,
                                                    ConvGeo cg = ConvGeo{}) {
  __shared__ float As[GT * GS], Bs[GT * GS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
  const int kbeg = blockIdx.z * kchunk, kend = min(K, kbeg + kchunk);
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the thread's fixed gather coordinates: the pixel of its A row (G_CONV_A / G_DCONV_A) or the tap
  // and channel of its 4 B columns (G_CONV_B)
  int gp_n = 0, gp_y = 0, gp_x = 0, gt_ky = 0, gt_kx = 0, gt_c = 0;
  if constexpr (GM == G_CONV_A || GM == G_DCONV_A) {
    const int gm = m0 + (tid >> 2);
    const int ww = GM == G_CONV_A ? cg.Wo : cg.W, hh = GM == G_CONV_A ? cg.Ho : cg.H;
    gp_x = gm % ww;
    gp_y = (gm / ww) % hh;
    gp_n = gm / (ww * hh);
  } else if constexpr (GM == G_CONV_B) {
    const int gn = n0 + (tid & 15) * 4, t = gn / cg.C;
    gt_c = gn - t * cg.C;
    gt_ky = t / cg.KW;
    gt_kx = t - gt_ky * cg.KW;
  }
  for (int k0 = kbeg; k0 < kend; k0 += GK) {
    // stage: 1024 elements of each operand, 4 per thread along the operand's contiguous axis
    if constexpr (GM == G_CONV_A || GM == G_DCONV_A) {
      const int r = tid >> 2, kq = (tid & 3) * 4, gm = m0 + r, gk = k0 + kq;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gm < M && gk < kend) {
        const int cc = GM == G_CONV_A ? cg.C : cg.Co, t = gk / cc, c = gk - t * cc, ky = t / cg.KW, kx = t - ky * cg.KW;
        if constexpr (GM == G_CONV_A) {
          const int ih = gp_y * cg.st - cg.pad + ky, iw = gp_x * cg.st - cg.pad + kx;
          if (ih >= 0 && ih < cg.H && iw >= 0 && iw < cg.W) v = ld4(A + (((size_t)gp_n * cg.H + ih) * cg.W + iw) * cg.C + c);
        } else {
          const int ty = gp_y + cg.pad - ky, tx = gp_x + cg.pad - kx;
          if (ty >= 0 && tx >= 0 && ty % cg.st == 0 && tx % cg.st == 0) {
            const int oh = ty / cg.st, ow = tx / cg.st;
            if (oh < cg.Ho && ow < cg.Wo) v = ld4(A + (((size_t)gp_n * cg.Ho + oh) * cg.Wo + ow) * cg.Co + c);
          }
        }
      }
      As[r * GS + kq + 0] = v.x;
      As[r * GS + kq + 1] = v.y;
      As[r * GS + kq + 2] = v.z;
      As[r * GS + kq + 3] = v.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        int r, k;
        if (!TA) { r = tid >> 2; k = (tid & 3) * 4 + u; } else { k = tid >> 4; r = (tid & 15) * 4 + u; }
        const int gm = m0 + r, gk = k0 + k;
        As[r * GS + k] = (gm < M && gk < kend) ? (TA ? A[(size_t)gk * lda + gm] : A[(size_t)gm * lda + gk]) : 0.f;
      }
    }
    if constexpr (GM == G_CONV_B) {
      static_assert(!TB, "the wgrad gather stages B as [k][j]");
      const int kb = tid >> 4, cq = (tid & 15) * 4, gn = n0 + cq, gkb = k0 + kb;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gn < N && gkb < kend) {
        const int ow = gkb % cg.Wo, oh = (gkb / cg.Wo) % cg.Ho, n = gkb / (cg.Wo * cg.Ho);
        const int ih = oh * cg.st - cg.pad + gt_ky, iw = ow * cg.st - cg.pad + gt_kx;
        if (ih >= 0 && ih < cg.H && iw >= 0 && iw < cg.W) v = ld4(B + (((size_t)n * cg.H + ih) * cg.W + iw) * cg.C + gt_c);
      }
      Bs[(cq + 0) * GS + kb] = v.x;
      Bs[(cq + 1) * GS + kb] = v.y;
      Bs[(cq + 2) * GS + kb] = v.z;
      Bs[(cq + 3) * GS + kb] = v.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        int c, kb;
        if (TB) { c = tid >> 2; kb = (tid & 3) * 4 + u; } else { kb = tid >> 4; c = (tid & 15) * 4 + u; }
        const int gn = n0 + c, gkb = k0 + kb;
        Bs[c * GS + kb] = (gn < N && gkb < kend) ? (TB ? B[(size_t)gn * ldb + gkb] : B[(size_t)gkb * ldb + gn]) : 0.f;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GK; kk += 4) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[(wm * 32 + i * 16 + (lane & 15)) * GS + kk + (lane >> 4)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[(wn * 32 + j * 16 + (lane & 15)) * GS + kk + (lane >> 4)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 32 + j * 16 + (lane & 15);
      if (col >= N) continue;
      if (part) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + r;
          if (row < M) part[((size_t)blockIdx.z * M + row) * N + col] = acc[i][j][r];
        }
        continue;
      }
      const float bv = bias ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + r;
        if (row >= M) continue;
        float* p = C + (size_t)row * ldc + col;
        const float v = alpha * acc[i][j][r] + bv;
        *p = beta != 0.f ? v + beta * *p : v;
      }
    }
}

__global__ void splitk_reduce_kernel(int M, int N, int S, const float* __restrict__ part, float alpha, float beta,
                                     float* C, int ldc, const float* __restrict__ bias) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)M * N) return;
  const int row = (int)(e / N), col = (int)(e - (int64_t)row * N);
  float a = 0.f;
  for (int z = 0; z < S; ++z) a += part[(size_t)z * M * N + e];
  float* p = C + (size_t)row * ldc + col;
  const float v = alpha * a + (bias ? bias[col] : 0.f);
  *p = beta != 0.f ? v + beta * *p : v;
}

// Column sums in two fixed-order stages: block (x, y) sums rows y RS .. (y + 1) RS of 64 columns
// (4 row phases per block, LDS combine) into part[y][N]; colsum_final adds the row slices.
constexpr int RS = 128;
__global__ void colsum_partial_kernel(int M, int N, const float* __restrict__ X, int ldx, const float* __restrict__ X2,
                                      const float* __restrict__ mean, const float* __restrict__ rstd, float* part,
                                      float* part2) {
  __shared__ float red[2][4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
  const int r0 = blockIdx.y * RS, r1 = min(M, r0 + RS);
  float s = 0.f, s2 = 0.f;
  if (c < N)
    for (int r = r0 + ph; r < r1; r += 4) {
      const float v = X[(size_t)r * ldx + c];
      s += v;
      if (X2) s2 += v * (X2[(size_t)r * ldx + c] - mean[r]) * rstd[r];   // LayerNorm dgamma term
    }
  red[0][ph][threadIdx.x & 63] = s;
  red[1][ph][threadIdx.x & 63] = s2;
  __syncthreads();
  if (ph == 0 && c < N) {
    const int l = threadIdx.x;
    part[(size_t)blockIdx.y * N + c] = ((red[0][0][l] + red[0][1][l]) + red[0][2][l]) + red[0][3][l];
    if (part2) part2[(size_t)blockIdx.y * N + c] = ((red[1][0][l] + red[1][1][l]) + red[1][2][l]) + red[1][3][l];
  }
}
__global__ void colsum_final_kernel(int N, int S, const float* __restrict__ part, float* out, float beta) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int z = 0; z < S; ++z) s += part[(size_t)z * N + n];
  out[n] = beta != 0.f ? beta * out[n] + s : s;
}

// ------------------------------------------------------------------------------------------
// LayerNorm over rows of d (one wave per row, two-pass mean / variance in registers)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ void ln_fwd_kernel(int rows, int d, const float* __restrict__ x, const float* __restrict__ g,
                              const float* __restrict__ b, float eps, float* y, float* mean, float* rstd) {
  const int row = blockIdx.x * (TT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + (size_t)row * d;
  float s = 0.f;
  for (int c = lane; c < d; c += 64) s += xr[c];
  const float mu = wave_sum(s) / d;
  float q = 0.f;
  for (int c = lane; c < d; c += 64) {
    const float t = xr[c] - mu;
    q += t * t;
  }
  const float rs = 1.0f / sqrtf(wave_sum(q) / d + eps);
  for (int c = lane; c < d; c += 64) y[(size_t)row * d + c] = (xr[c] - mu) * rs * g[c] + b[c];
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// dx = rstd (gdy - mean(gdy) - xhat mean(gdy xhat)), gdy = dy * gamma
__global__ void ln_bwd_kernel(int rows, int d, const float* __restrict__ x, const float* __restrict__ g,
                              const float* __restrict__ mean, const float* __restrict__ rstd,
                              const float* __restrict__ dy, float* dx) {
  const int row = blockIdx.x * (TT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float mu = mean[row], rs = rstd[row];
  const float* xr = x + (size_t)row * d;
  const float* dr = dy + (size_t)row * d;
  float s1 = 0.f, s2 = 0.f;
  for (int c = lane; c < d; c += 64) {
    const float gd = dr[c] * g[c], xh = (xr[c] - mu) * rs;
    s1 += gd;
    s2 += gd * xh;
  }
  const float m1 = wave_sum(s1) / d, m2 = wave_sum(s2) / d;
  for (int c = lane; c < d; c += 64) {
    const float gd = dr[c] * g[c], xh = (xr[c] - mu) * rs;
    dx[(size_t)row * d + c] = rs * (gd - m1 - xh * m2);
  }
}

// ------------------------------------------------------------------------------------------
// SpatialDepthWiseConv along frames: y[n][i][h dk + c] = b[c] + w[c][0] x[i-1] + w[c][1] x[i]
// + w[c][2] x[i+1] (zeros outside the clip), transformer.py:19-44
// ------------------------------------------------------------------------------------------
__global__ void seqconv_fwd_kernel(int n, int L, int H, int dk, const float* __restrict__ x, int ldx,
                                   const float* __restrict__ w, const float* __restrict__ b, float* y, int ldy) {
  const int64_t total = (int64_t)n * L * H * dk;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int ch = (int)(e % (H * dk)), c = ch % dk;
  const int64_t ri = e / (H * dk);
  const int i = (int)(ri % L);
  const float* xp = x + ri * ldx + ch;
  const float p0 = i > 0 ? xp[-(int64_t)ldx] : 0.f, p2 = i + 1 < L ? xp[ldx] : 0.f;
  y[ri * ldy + ch] = fmaf(w[c * 3 + 2], p2, fmaf(w[c * 3 + 1], xp[0], fmaf(w[c * 3 + 0], p0, b[c])));
}

// dx[i] = w0 dy[i+1] + w1 dy[i] + w2 dy[i-1]
__global__ void seqconv_bwd_kernel(int n, int L, int H, int dk, const float* __restrict__ dy, int lddy,
                                   const float* __restrict__ w, float* dx, int lddx) {
  const int64_t total = (int64_t)n * L * H * dk;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int ch = (int)(e % (H * dk)), c = ch % dk;
  const int64_t ri = e / (H * dk);
  const int i = (int)(ri % L);
  const float* gp = dy + ri * lddy + ch;
  const float n1 = i + 1 < L ? gp[lddy] : 0.f, p1 = i > 0 ? gp[-(int64_t)lddy] : 0.f;
  dx[ri * lddx + ch] = w[c * 3 + 0] * n1 + w[c * 3 + 1] * gp[0] + w[c * 3 + 2] * p1;
}

// dw[c][k] = sum over clips, frames, heads of dy[i] x[i + k - 1]; db[c] = sum dy.  One block per
// channel c, a fixed per-thread order and an LDS tree: deterministic.
__global__ void seqconv_param_grad_kernel(int n, int L, int H, int dk, const float* __restrict__ x, int ldx,
                                          const float* __restrict__ dy, int lddy, float* dw, float* db) {
  __shared__ float red[4][TT];
  const int c = blockIdx.x, tid = threadIdx.x;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t items = (int64_t)n * L * H;
  for (int64_t it = tid; it < items; it += TT) {
    const int h = (int)(it % H);
    const int64_t ri = it / H;
    const int i = (int)(ri % L);
    const int ch = h * dk + c;
    const float g = dy[ri * lddy + ch];
    const float* xp = x + ri * ldx + ch;
    s[0] += g * (i > 0 ? xp[-(int64_t)ldx] : 0.f);
    s[1] += g * xp[0];
    s[2] += g * (i + 1 < L ? xp[ldx] : 0.f);
    s[3] += g;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) red[q][tid] = s[q];
  __syncthreads();
  for (int o = TT / 2; o > 0; o >>= 1) {
    if (tid < o)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[q][tid] += red[q][tid + o];
    __syncthreads();
  }
  if (tid == 0) {
    dw[c * 3 + 0] = red[0][0];
    dw[c * 3 + 1] = red[1][0];
    dw[c * 3 + 2] = red[2][0];
    db[c] = red[3][0];
  }
}

// ------------------------------------------------------------------------------------------
// Attention core per (clip, head): O = softmax(Q K^T scale) V (transformer.py:104-118; no mask).
// Q / K / V / O rows of head h are columns h dk .. of their row-major token matrices.  The head's
// operands sit in LDS as [rows][dk] images, P (and dS in backward) as an Lq x Lk image; the
// launcher checks that they fit (att_lds_bytes <= 160 KiB).
// ------------------------------------------------------------------------------------------
constexpr int ATT_MAX_L = 256;

__host__ __device__ inline size_t att_lds_bytes(int Lq, int Lk, int dk, bool bwd) {
  return sizeof(float) * ((size_t)(bwd ? 2 * Lq + 2 * Lk : Lq + 2 * Lk) * dk + (size_t)Lq * Lk + (bwd ? Lq : 0));
}

__device__ __forceinline__ void stage_head(float* dst, const float* src, int rows, int ld, int h, int dk) {
  for (int e = threadIdx.x; e < rows * dk; e += blockDim.x) {
    const int r = e / dk, c = e - r * dk;
    dst[r * dk + c] = src[(size_t)r * ld + h * dk + c];
  }
}

// P[i][j] = softmax_j(Q_i . K_j scale) (row stride Lk): one wave per row i
__device__ void softmax_rows(float* P, const float* Q, const float* Kh, int Lq, int Lk, int dk, float scale) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int i = wave; i < Lq; i += nw) {
    float mx = -INFINITY;
    for (int j = lane; j < Lk; j += 64) {
      float s = 0.f;
      for (int c = 0; c < dk; ++c) s += Q[i * dk + c] * Kh[j * dk + c];
      s *= scale;
      P[i * Lk + j] = s;
      mx = fmaxf(mx, s);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.f;
    for (int j = lane; j < Lk; j += 64) {
      const float e = expf(P[i * Lk + j] - mx);
      P[i * Lk + j] = e;
      sum += e;
    }
    const float inv = 1.0f / wave_sum(sum);
    for (int j = lane; j < Lk; j += 64) P[i * Lk + j] *= inv;
  }
}

__global__ void __launch_bounds__(TT) attn_fwd_kernel(int H, int Lq, int Lk, int dk, float scale, const float* q,
                                                      int ldq, const float* k, const float* v, int ldkv, float* o,
                                                      int ldo) {
  extern __shared__ float sm[];
  float *Qs = sm, *Ks = Qs + Lq * dk, *Vs = Ks + Lk * dk, *P = Vs + Lk * dk;
  const int h = blockIdx.x, b = blockIdx.y;
  stage_head(Qs, q + (size_t)b * Lq * ldq, Lq, ldq, h, dk);
  stage_head(Ks, k + (size_t)b * Lk * ldkv, Lk, ldkv, h, dk);
  stage_head(Vs, v + (size_t)b * Lk * ldkv, Lk, ldkv, h, dk);
  __syncthreads();
  softmax_rows(P, Qs, Ks, Lq, Lk, dk, scale);
  __syncthreads();
  for (int e = threadIdx.x; e < Lq * dk; e += blockDim.x) {
    const int i = e / dk, c = e - i * dk;
    float s = 0.f;
    for (int j = 0; j < Lk; ++j) s += P[i * Lk + j] * Vs[j * dk + c];
    o[((size_t)b * Lq + i) * ldo + h * dk + c] = s;
  }
}

// dV = P^T dO; dP = dO V^T; dS = P (dP - rowsum(P dP)); dQ = scale dS K; dK = scale dS^T Q
__global__ void __launch_bounds__(TT) attn_bwd_kernel(int H, int Lq, int Lk, int dk, float scale, const float* q,
                                                      int ldq, const float* k, const float* v, int ldkv,
                                                      const float* dout, int ldo, float* dq, float* dkk, float* dv) {
  extern __shared__ float sm[];
  float *Qs = sm, *Ks = Qs + Lq * dk, *Vs = Ks + Lk * dk, *dO = Vs + Lk * dk, *P = dO + Lq * dk, *Dr = P + Lq * Lk;
  const int h = blockIdx.x, b = blockIdx.y;
  stage_head(Qs, q + (size_t)b * Lq * ldq, Lq, ldq, h, dk);
  stage_head(Ks, k + (size_t)b * Lk * ldkv, Lk, ldkv, h, dk);
  stage_head(Vs, v + (size_t)b * Lk * ldkv, Lk, ldkv, h, dk);
  stage_head(dO, dout + (size_t)b * Lq * ldo, Lq, ldo, h, dk);
  __syncthreads();
  softmax_rows(P, Qs, Ks, Lq, Lk, dk, scale);
  __syncthreads();
  // dV (before P is overwritten by dS)
  for (int e = threadIdx.x; e < Lk * dk; e += blockDim.x) {
    const int j = e / dk, c = e - j * dk;
    float s = 0.f;
    for (int i = 0; i < Lq; ++i) s += P[i * Lk + j] * dO[i * dk + c];
    dv[((size_t)b * Lk + j) * ldkv + h * dk + c] = s;
  }
  // D_i = sum_j P_ij dP_ij, one wave per row; then dS in place of P
  {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int i = wave; i < Lq; i += nw) {
      float s = 0.f;
      for (int j = lane; j < Lk; j += 64) {
        float dp = 0.f;
        for (int c = 0; c < dk; ++c) dp += dO[i * dk + c] * Vs[j * dk + c];
        s += P[i * Lk + j] * dp;
      }
      s = wave_sum(s);
      if (lane == 0) Dr[i] = s;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < Lq * Lk; e += blockDim.x) {
    const int i = e / Lk, j = e - i * Lk;
    float dp = 0.f;
    for (int c = 0; c < dk; ++c) dp += dO[i * dk + c] * Vs[j * dk + c];
    P[i * Lk + j] = P[i * Lk + j] * (dp - Dr[i]);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < Lq * dk; e += blockDim.x) {
    const int i = e / dk, c = e - i * dk;
    float s = 0.f;
    for (int j = 0; j < Lk; ++j) s += P[i * Lk + j] * Ks[j * dk + c];
    dq[((size_t)b * Lq + i) * ldq + h * dk + c] = scale * s;
  }
  for (int e = threadIdx.x; e < Lk * dk; e += blockDim.x) {
    const int j = e / dk, c = e - j * dk;
    float s = 0.f;
    for (int i = 0; i < Lq; ++i) s += P[i * Lk + j] * Qs[i * dk + c];
    dkk[((size_t)b * Lk + j) * ldkv + h * dk + c] = scale * s;
  }
}

// ------------------------------------------------------------------------------------------
// elementwise
// ------------------------------------------------------------------------------------------
__global__ void ew_kernel(int op, int64_t n, const float* __restrict__ a, const float* __restrict__ b, float* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = a[i];
  float r;
  switch (op) {
    case GGD_EW_RELU2: { const float t = fmaxf(x, 0.f); r = t * t; break; }
    case GGD_EW_RELU2_BWD: r = b[i] * 2.f * fmaxf(x, 0.f); break;
    case GGD_EW_SILU: r = x / (1.f + expf(-x)); break;
    case GGD_EW_SILU_BWD: { const float s = 1.f / (1.f + expf(-x)); r = b[i] * (s + x * s * (1.f - s)); break; }
    case GGD_EW_RELU: r = fmaxf(x, 0.f); break;
    case GGD_EW_RELU_BWD: r = x > 0.f ? b[i] : 0.f; break;
    case GGD_EW_SIGMOID: r = 1.f / (1.f + expf(-x)); break;
    case GGD_EW_SIGMOID_BWD: r = b[i] * x * (1.f - x); break;   // a: the sigmoid OUTPUT
    default: r = x + b[i]; break;  // GGD_EW_ADD
  }
  out[i] = r;
}

// x_t = ca[clip] x0 + cb[clip] noise (gaussian_diffusion.py:188-205 q_sample, per-clip coefficients)
__global__ void qsample_kernel(int64_t n, int per_clip, const float* __restrict__ x0, const float* __restrict__ noise,
                               const float* __restrict__ ca, const float* __restrict__ cb, float* xt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int clip = (int)(i / per_clip);
  xt[i] = ca[clip] * x0[i] + cb[clip] * noise[i];
}

// mse[clip] = mean over the clip's elements of (eps - noise)^2 (mean_flat, gaussian_diffusion.py:553-558);
// d_eps = grad_scale * 2 (eps - noise) / per_clip.  One block per clip, fixed reduction order.
__global__ void mse_kernel(int per_clip, const float* __restrict__ eps, const float* __restrict__ noise, float* mse,
                           float* d_eps, float grad_scale) {
  __shared__ float red[TT];
  const int clip = blockIdx.x, tid = threadIdx.x;
  const size_t base = (size_t)clip * per_clip;
  float s = 0.f;
  for (int e = tid; e < per_clip; e += TT) {
    const float dlt = eps[base + e] - noise[base + e];
    s += dlt * dlt;
    if (d_eps) d_eps[base + e] = grad_scale * 2.f * dlt / (float)per_clip;
  }
  red[tid] = s;
  __syncthreads();
  for (int o = TT / 2; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) mse[clip] = red[0] / (float)per_clip;
}

// sum of squares in two fixed-shape stages (deterministic): SUMSQ_BLOCKS partials, then one block
constexpr int SUMSQ_BLOCKS = 256;
__global__ void sumsq_partial_kernel(int64_t n, const float* __restrict__ x, float* part) {
  __shared__ float red[TT];
  const int tid = threadIdx.x;
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * TT + tid; i < n; i += (int64_t)SUMSQ_BLOCKS * TT) s += x[i] * x[i];
  red[tid] = s;
  __syncthreads();
  for (int o = TT / 2; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) part[blockIdx.x] = red[0];
}
__global__ void sumsq_final_kernel(const float* __restrict__ part, float* out) {
  __shared__ float red[SUMSQ_BLOCKS];
  const int tid = threadIdx.x;
  red[tid] = part[tid];
  __syncthreads();
  for (int o = SUMSQ_BLOCKS / 2; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) out[0] = red[0];
}

// torch.optim.AdamW (single-tensor path) in its operation order:
//   p *= 1 - lr wd; m = lerp(m, g, 1 - b1); v = b2 v + (1 - b2) g g;
//   p -= (lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps)
__global__ void adamw_kernel(int64_t n, float* p, const float* __restrict__ g, float* m, float* v, float lr, float b1,
                             float b2, float eps, float wd, float bc1, float bc2_sqrt, float gscale) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float gr = g[i] * gscale;
  float pv = p[i] * (1.f - lr * wd);
  const float mv = m[i] + (1.f - b1) * (gr - m[i]);
  const float vv = v[i] * b2 + (1.f - b2) * gr * gr;
  const float denom = sqrtf(vv) / bc2_sqrt + eps;
  pv = pv - (lr / bc1) * (mv / denom);
  p[i] = pv;
  m[i] = mv;
  v[i] = vv;
}

__global__ void scale_kernel(int64_t n, float* x, float s) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] *= s;
}

// clip_grad_norm_'s coefficient, then clip_grad_value_'s clamp (trainer.py:233-236), in place
__global__ void scale_clamp_kernel(int64_t n, float* x, float s, float lim) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = fminf(fmaxf(x[i] * s, -lim), lim);
}

// ------------------------------------------------------------------------------------------
// speech-encoder training ops, NHWC activations (rows = pixels (n, h, w), channels innermost)
// ------------------------------------------------------------------------------------------
// im2col: col[(n, oh, ow)][(ky, kx, c)] = x[n][oh s - pad + ky][ow s - pad + kx][c], 0 outside
__global__ void im2col_kernel(const float* __restrict__ x, int N, int H, int W, int C, int KH, int KW, int st, int pad,
                              int Ho, int Wo, float* __restrict__ col) {
  const int64_t total = (int64_t)N * Ho * Wo * KH * KW * C;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int c = (int)(e % C);
  int64_t t = e / C;
  const int kx = (int)(t % KW);
  t /= KW;
  const int ky = (int)(t % KH);
  const int64_t p = t / KH;
  const int ow = (int)(p % Wo), oh = (int)((p / Wo) % Ho), n = (int)(p / ((int64_t)Wo * Ho));
  const int ih = oh * st - pad + ky, iw = ow * st - pad + kx;
  col[e] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? x[(((int64_t)n * H + ih) * W + iw) * C + c] : 0.f;
}

// col2im as a gather: dx[n][ih][iw][c] = sum of the col entries that im2col copied from it
__global__ void col2im_kernel(const float* __restrict__ dcol, int N, int H, int W, int C, int KH, int KW, int st,
                              int pad, int Ho, int Wo, float* __restrict__ dx) {
  const int64_t total = (int64_t)N * H * W * C;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int c = (int)(e % C);
  const int64_t q = e / C;
  const int iw = (int)(q % W), ih = (int)((q / W) % H), n = (int)(q / ((int64_t)W * H));
  float s = 0.f;
  for (int ky = 0; ky < KH; ++ky) {
    const int ty = ih + pad - ky;
    if (ty < 0 || ty % st) continue;
    const int oh = ty / st;
    if (oh >= Ho) continue;
    for (int kx = 0; kx < KW; ++kx) {
      const int tx = iw + pad - kx;
      if (tx < 0 || tx % st) continue;
      const int ow = tx / st;
      if (ow >= Wo) continue;
      s += dcol[((((int64_t)n * Ho + oh) * Wo + ow) * KH * KW + ky * KW + kx) * C + c];
    }
  }
  dx[e] = s;
}

// per-channel column statistics over P rows of C channels, two fixed-order stages (RS-row slices):
//   mode 0: sum x;  mode 1: sum (x - mean[c])^2;  mode 2: sum dy and sum dy (x - mean[c]) rstd[c]
__global__ void chan_partial_kernel(int P, int C, int mode, const float* __restrict__ X, const float* __restrict__ DY,
                                    const float* __restrict__ mean, const float* __restrict__ rstd, float* part,
                                    float* part2, int rs) {
  __shared__ float red[2][4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rs, r1 = min(P, r0 + rs);
  float s = 0.f, s2 = 0.f;
  if (c < C) {
    const float mu = mode ? mean[c] : 0.f, rs = mode == 2 ? rstd[c] : 0.f;
    for (int r = r0 + ph; r < r1; r += 4) {
      const float v = X[(size_t)r * C + c];
      if (mode == 0) {
        s += v;
      } else if (mode == 1) {
        s += (v - mu) * (v - mu);
      } else {
        const float g = DY[(size_t)r * C + c];
        s += g;
        s2 += g * (v - mu) * rs;
      }
    }
  }
  red[0][ph][threadIdx.x & 63] = s;
  red[1][ph][threadIdx.x & 63] = s2;
  __syncthreads();
  if (ph == 0 && c < C) {
    const int l = threadIdx.x;
    part[(size_t)blockIdx.y * C + c] = ((red[0][0][l] + red[0][1][l]) + red[0][2][l]) + red[0][3][l];
    if (mode == 2) part2[(size_t)blockIdx.y * C + c] = ((red[1][0][l] + red[1][1][l]) + red[1][2][l]) + red[1][3][l];
  }
}
// out[c] = scale sum_z part[z][c] (S <= 256): one block per channel, one slice per thread, LDS
// tree in a fixed order; also rstd and the unbiased variance when asked (mode-1 partials)
__global__ void __launch_bounds__(256) chan_final_kernel(int C, int S, const float* __restrict__ part, float scale,
                                                         float* out, float* rstd, float* var_unbiased, float eps,
                                                         float unbias) {
  __shared__ float red[256];
  const int c = blockIdx.x, z = threadIdx.x;
  red[z] = z < S ? part[(size_t)z * C + c] : 0.f;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (z < o) red[z] += red[z + o];
    __syncthreads();
  }
  if (z) return;
  const float s = red[0] * scale;
  out[c] = s;
  if (rstd) rstd[c] = 1.0f / sqrtf(s + eps);
  if (var_unbiased) var_unbiased[c] = s * unbias;
}
// y = (x - mean) rstd g + b per channel
__global__ void bn_apply_kernel(int64_t n, int C, const float* __restrict__ x, const float* __restrict__ mean,
                                const float* __restrict__ rstd, const float* __restrict__ g, const float* __restrict__ b,
                                float* y) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int c = (int)(e % C);
  y[e] = (x[e] - mean[c]) * rstd[c] * g[c] + b[c];
}
// dx = g rstd (dy - dbeta / P - xhat dgamma / P)
__global__ void bn_bwd_apply_kernel(int64_t n, int C, int P, const float* __restrict__ x, const float* __restrict__ dy,
                                    const float* __restrict__ mean, const float* __restrict__ rstd,
                                    const float* __restrict__ g, const float* __restrict__ dbeta,
                                    const float* __restrict__ dgamma, float* dx) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int c = (int)(e % C);
  const float xh = (x[e] - mean[c]) * rstd[c];
  dx[e] = g[c] * rstd[c] * (dy[e] - dbeta[c] / P - xh * dgamma[c] / P);
}

// per-image channel sums: part[z][n][c] = sum over pixel slice z of X[n][p][c] (Y: X Y); block
// (channel block, image, slice), 4 pixel phases per block; img_chan_final adds the slices x scale
__global__ void img_chan_sum_kernel(int HW, int C, int ps, const float* __restrict__ X, const float* __restrict__ Y,
                                    float* part) {
  __shared__ float red[4][64];
  const int n = blockIdx.y, z = blockIdx.z, c = blockIdx.x * 64 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
  const int p0 = z * ps, p1 = min(HW, p0 + ps);
  float s = 0.f;
  if (c < C)
    for (int p = p0 + ph; p < p1; p += 4) {
      const size_t i = ((size_t)n * HW + p) * C + c;
      s += Y ? X[i] * Y[i] : X[i];
    }
  red[ph][threadIdx.x & 63] = s;
  __syncthreads();
  if (ph == 0 && c < C) {
    const int l = threadIdx.x;
    part[((size_t)z * gridDim.y + n) * C + c] = ((red[0][l] + red[1][l]) + red[2][l]) + red[3][l];
  }
}
__global__ void img_chan_final_kernel(int NC, int S, const float* __restrict__ part, float scale, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NC) return;
  float s = 0.f;
  for (int z = 0; z < S; ++z) s += part[(size_t)z * NC + i];
  out[i] = s * scale;
}
// out[n][p][c] = X[n][p][c] s[n][c] (+ add[n][c] when add is set)
__global__ void chan_scale_kernel(int64_t total, int HW, int C, const float* __restrict__ X, const float* __restrict__ s,
                                  const float* __restrict__ add, float* out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int c = (int)(e % C);
  const int64_t n = e / ((int64_t)HW * C);
  const float v = X ? X[e] * s[n * C + c] : 0.f;
  out[e] = add ? v + add[n * C + c] : v;
}

// PixelShuffle(r) on NHWC (torch.nn.PixelShuffle channel order c r^2 + i r + j):
// out[n][h r + i][w r + j][c] = in[n][h][w][c r^2 + i r + j]; dir 1 moves gradients back
__global__ void shuffle_kernel(int N, int H, int W, int C, int r, const float* __restrict__ src, float* __restrict__ dst,
                               int dir) {
  const int64_t total = (int64_t)N * H * r * W * r * C;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int c = (int)(e % C);
  const int64_t q = e / C;
  const int wo = (int)(q % (W * r)), ho = (int)((q / (W * r)) % (H * r)), n = (int)(q / ((int64_t)W * r * H * r));
  const int h = ho / r, i = ho - h * r, w = wo / r, j = wo - w * r;
  const int64_t in_i = (((int64_t)n * H + h) * W + w) * (C * r * r) + c * r * r + i * r + j;
  if (dir == 0) dst[e] = src[in_i];
  else dst[in_i] = src[e];
}

// head flatten (ResNetSE34V2.py:161-165): rows (n, w), features c H + h from NHWC x[n][h][w][c];
// dir 1 moves gradients back
__global__ void head_flat_kernel(int N, int H, int W, int C, const float* __restrict__ src, float* __restrict__ dst,
                                 int dir) {
  const int64_t total = (int64_t)N * H * W * C;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int c = (int)(e % C);
  const int64_t q = e / C;
  const int w = (int)(q % W), h = (int)((q / W) % H), n = (int)(q / ((int64_t)W * H));
  const int64_t row_i = ((int64_t)n * W + w) * (C * H) + c * H + h;
  if (dir == 0) dst[row_i] = src[e];
  else dst[e] = src[row_i];
}

inline unsigned blocks_for(int64_t n, int per = TT) { return (unsigned)((n + per - 1) / per); }

// grow-only workspace per device for split-K slices and reduction partials.  The training ops
// of one device are issued on one stream (training.py uses torch's current stream), so the
// consumers of a buffer run before the next op overwrites it; growing it frees the old one with
// hipFree, which waits for the device.  Not thread-safe: one host thread drives a device.
constexpr int WS_DEVICES = 64;
float* g_ws[WS_DEVICES] = {};
size_t g_ws_bytes[WS_DEVICES] = {};
float* workspace(size_t bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= WS_DEVICES) return nullptr;
  if (bytes <= g_ws_bytes[dev]) return g_ws[dev];
  if (g_ws[dev]) (void)hipFree(g_ws[dev]);
  g_ws[dev] = nullptr;
  g_ws_bytes[dev] = 0;
  if (hipMalloc((void**)&g_ws[dev], bytes) != hipSuccess) return nullptr;
  g_ws_bytes[dev] = bytes;
  return g_ws[dev];
}

// row slices of the per-channel reductions: at most 256 (the final stage loops over them), each
// at least RS rows
int chan_slices(int P) { return std::max(1, std::min(256, (P + RS - 1) / RS)); }

// column sums of X (and the LayerNorm dgamma sums when X2 is set) into out / out2
int colsums(int M, int N, const float* X, int ldx, const float* X2, const float* mean, const float* rstd, float* out,
            float* out2, float beta, hipStream_t s) {
  const int S = (M + RS - 1) / RS;
  float* ws = workspace(sizeof(float) * (size_t)S * N * 2);
  if (!ws) return -3;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((N + 63) / 64, S), dim3(256), 0, s, M, N, X, ldx, X2, mean, rstd, ws,
                     X2 ? ws + (size_t)S * N : nullptr);
  hipLaunchKernelGGL(colsum_final_kernel, dim3(blocks_for(N)), dim3(TT), 0, s, N, S, ws, out, beta);
  if (X2) hipLaunchKernelGGL(colsum_final_kernel, dim3(blocks_for(N)), dim3(TT), 0, s, N, S, ws + (size_t)S * N, out2, 0.f);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
inline int rc(hipError_t e) { return e == hipSuccess ? 0 : -3; }  // GGD_ERR_HIP

bool att_lds_ready = false;

int tgemm_launch(int ta, int tb, int gm, int M, int N, int K, float alpha, const float* A, int lda, const float* B,
                 int ldb, float beta, float* C, int ldc, const float* bias, ConvGeo cg, hipStream_t s);

}  // namespace

extern "C" {

int ggd_tr_gemm(int ta, int tb, int M, int N, int K, float alpha, const float* A, int lda, const float* B, int ldb,
                float beta, float* C, int ldc, const float* bias, void* stream) {
  if (M < 0 || N < 0 || K < 0 || !A || !B || !C) return -1;
  if (M == 0 || N == 0) return 0;
  return tgemm_launch(ta, tb, G_PLAIN, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, bias, ConvGeo{}, (hipStream_t)stream);
}

}  // extern "C"

namespace {
int tgemm_launch(int ta, int tb, int gm, int M, int N, int K, float alpha, const float* A, int lda, const float* B,
                 int ldb, float beta, float* C, int ldc, const float* bias, ConvGeo cg, hipStream_t s) {
  // few output tiles over a long K (the weight gradients dW = dY^T X, K = clips x frames): split
  // K so that the launch covers the chip, then add the slices in a fixed order
  const int tiles = ((N + GT - 1) / GT) * ((M + GT - 1) / GT);
  int S = 1;
  if (tiles < 256 && K >= 8 * GT) S = std::min((K + 255) / 256, (512 + tiles - 1) / tiles);
  const int kchunk = S > 1 ? (((K + S - 1) / S + GK - 1) / GK) * GK : K;
  if (S > 1) S = (K + kchunk - 1) / kchunk;
  float* part = nullptr;
  if (S > 1) {
    part = workspace(sizeof(float) * (size_t)S * M * N);
    if (!part) return -3;
  }
  const dim3 grid((N + GT - 1) / GT, (M + GT - 1) / GT, S), blk(256);
#define GGD_TGEMM(a_, b_, g_)                                                                              \
  hipLaunchKernelGGL((tgemm_kernel<a_, b_, g_>), grid, blk, 0, s, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, bias, \
                     kchunk, part, cg)
  if (gm == G_CONV_A) GGD_TGEMM(false, true, G_CONV_A);          // x (gathered) . W^T
  else if (gm == G_DCONV_A) GGD_TGEMM(false, false, G_DCONV_A);  // dy (gathered) . W'
  else if (gm == G_CONV_B) GGD_TGEMM(true, false, G_CONV_B);     // dy^T . x (gathered)
  else if (!ta && tb) GGD_TGEMM(false, true, G_PLAIN);
  else if (!ta && !tb) GGD_TGEMM(false, false, G_PLAIN);
  else if (ta && !tb) GGD_TGEMM(true, false, G_PLAIN);
  else GGD_TGEMM(true, true, G_PLAIN);
#undef GGD_TGEMM
  if (S > 1)
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks_for((int64_t)M * N)), dim3(TT), 0, s, M, N, S, part, alpha, beta,
                       C, ldc, bias);
  return rc(hipGetLastError());
}

// output size of a conv, or -2 (unsupported shape)
int conv_geo(int N, int H, int W, int C, int Co, int KH, int KW, int stride, int pad, ConvGeo& g) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || Co <= 0 || KH <= 0 || KW <= 0 || stride <= 0 || pad < 0) return -1;
  g = ConvGeo{H, W, C, KH, KW, stride, pad, (H + 2 * pad - KH) / stride + 1, (W + 2 * pad - KW) / stride + 1, Co};
  return g.Ho > 0 && g.Wo > 0 ? 0 : -2;
}
}  // namespace

extern "C" {

int ggd_tr_conv_fwd(int N, int H, int W, int C, int Co, int KH, int KW, int stride, int pad, const float* x,
                    const float* wp, const float* bias, float* y, void* stream) {
  ConvGeo g;
  const int e = conv_geo(N, H, W, C, Co, KH, KW, stride, pad, g);
  if (e) return e;
  if (!x || !wp || !y) return -1;
  if (C % 4) return -2;
  const int P = N * g.Ho * g.Wo, K = KH * KW * C;
  return tgemm_launch(0, 1, G_CONV_A, P, Co, K, 1.f, x, 0, wp, K, 0.f, y, Co, bias, g, (hipStream_t)stream);
}

int ggd_tr_conv_dgrad(int N, int H, int W, int C, int Co, int KH, int KW, int stride, int pad, const float* dy,
                      const float* wt, float* dx, void* stream) {
  ConvGeo g;
  const int e = conv_geo(N, H, W, C, Co, KH, KW, stride, pad, g);
  if (e) return e;
  if (!dy || !wt || !dx) return -1;
  if (Co % 4) return -2;
  return tgemm_launch(0, 0, G_DCONV_A, N * H * W, C, KH * KW * Co, 1.f, dy, 0, wt, C, 0.f, dx, C, nullptr, g,
                      (hipStream_t)stream);
}

int ggd_tr_conv_wgrad(int N, int H, int W, int C, int Co, int KH, int KW, int stride, int pad, const float* dy,
                      const float* x, float beta, float* dwp, void* stream) {
  ConvGeo g;
  const int e = conv_geo(N, H, W, C, Co, KH, KW, stride, pad, g);
  if (e) return e;
  if (!dy || !x || !dwp) return -1;
  if (C % 4) return -2;
  const int P = N * g.Ho * g.Wo, K = KH * KW * C;
  return tgemm_launch(1, 0, G_CONV_B, Co, K, P, 1.f, dy, Co, x, 0, beta, dwp, K, nullptr, g, (hipStream_t)stream);
}

int ggd_tr_colsum(int M, int N, const float* X, int ldx, float* out, float beta, void* stream) {
  if (M <= 0 || N <= 0 || !X || !out) return -1;
  return colsums(M, N, X, ldx, nullptr, nullptr, nullptr, out, nullptr, beta, (hipStream_t)stream);
}

int ggd_tr_layernorm_fwd(int rows, int d, const float* x, const float* g, const float* b, float eps, float* y,
                         float* mean, float* rstd, void* stream) {
  if (rows <= 0 || d <= 0 || !x || !g || !b || !y || !mean || !rstd) return -1;
  hipLaunchKernelGGL(ln_fwd_kernel, dim3(blocks_for(rows, TT / 64)), dim3(TT), 0, (hipStream_t)stream, rows, d, x, g, b,
                     eps, y, mean, rstd);
  return rc(hipGetLastError());
}

int ggd_tr_layernorm_bwd(int rows, int d, const float* x, const float* g, const float* mean, const float* rstd,
                         const float* dy, float* dx, float* dg, float* db, void* stream) {
  if (rows <= 0 || d <= 0 || !x || !g || !mean || !rstd || !dy || !dx) return -1;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(blocks_for(rows, TT / 64)), dim3(TT), 0, s, rows, d, x, g, mean, rstd, dy, dx);
  if (hipGetLastError() != hipSuccess) return -3;
  if (dg && db) return colsums(rows, d, dy, d, x, mean, rstd, db, dg, 0.f, s);   // db = sum dy, dg = sum dy xhat
  return 0;
}

int ggd_tr_seqconv_fwd(int n, int L, int H, int dk, const float* x, int ldx, const float* w, const float* b, float* y,
                       int ldy, void* stream) {
  if (n <= 0 || L <= 0 || H <= 0 || dk <= 0 || !x || !w || !b || !y) return -1;
  const int64_t total = (int64_t)n * L * H * dk;
  hipLaunchKernelGGL(seqconv_fwd_kernel, dim3(blocks_for(total)), dim3(TT), 0, (hipStream_t)stream, n, L, H, dk, x, ldx,
                     w, b, y, ldy);
  return rc(hipGetLastError());
}

int ggd_tr_seqconv_bwd(int n, int L, int H, int dk, const float* x, int ldx, const float* w, const float* dy, int lddy,
                       float* dx, int lddx, float* dw, float* db, void* stream) {
  if (n <= 0 || L <= 0 || H <= 0 || dk <= 0 || !x || !w || !dy || !dx) return -1;
  hipStream_t s = (hipStream_t)stream;
  const int64_t total = (int64_t)n * L * H * dk;
  hipLaunchKernelGGL(seqconv_bwd_kernel, dim3(blocks_for(total)), dim3(TT), 0, s, n, L, H, dk, dy, lddy, w, dx, lddx);
  if (dw && db) hipLaunchKernelGGL(seqconv_param_grad_kernel, dim3(dk), dim3(TT), 0, s, n, L, H, dk, x, ldx, dy, lddy, dw, db);
  return rc(hipGetLastError());
}

static void att_attrs() {
  if (att_lds_ready) return;
  (void)hipFuncSetAttribute((const void*)attn_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)attn_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipGetLastError();
  att_lds_ready = true;
}

int ggd_tr_attention_fwd(int n, int H, int Lq, int Lk, int dk, float scale, const float* q, int ldq, const float* k,
                         const float* v, int ldkv, float* o, int ldo, void* stream) {
  if (n <= 0 || H <= 0 || Lq <= 0 || Lq > ATT_MAX_L || Lk <= 0 || Lk > ATT_MAX_L || dk <= 0 || !q || !k || !v || !o ||
      att_lds_bytes(Lq, Lk, dk, false) > 160 * 1024)
    return -2;
  att_attrs();
  hipLaunchKernelGGL(attn_fwd_kernel, dim3(H, n), dim3(TT), att_lds_bytes(Lq, Lk, dk, false), (hipStream_t)stream, H, Lq, Lk, dk, scale, q, ldq,
                     k, v, ldkv, o, ldo);
  return rc(hipGetLastError());
}

int ggd_tr_attention_bwd(int n, int H, int Lq, int Lk, int dk, float scale, const float* q, int ldq, const float* k,
                         const float* v, int ldkv, const float* dout, int ldo, float* dq, float* dk_out, float* dv,
                         void* stream) {
  if (n <= 0 || H <= 0 || Lq <= 0 || Lq > ATT_MAX_L || Lk <= 0 || Lk > ATT_MAX_L || dk <= 0 || !q || !k || !v || !dout ||
      !dq || !dk_out || !dv || att_lds_bytes(Lq, Lk, dk, true) > 160 * 1024)
    return -2;
  att_attrs();
  hipLaunchKernelGGL(attn_bwd_kernel, dim3(H, n), dim3(TT), att_lds_bytes(Lq, Lk, dk, true), (hipStream_t)stream, H, Lq, Lk, dk, scale, q, ldq,
                     k, v, ldkv, dout, ldo, dq, dk_out, dv);
  return rc(hipGetLastError());
}

int ggd_tr_elementwise(int op, int64_t n, const float* a, const float* b, float* out, void* stream) {
  if (n < 0 || !a || !out || op < 0 || op > GGD_EW_SIGMOID_BWD) return -1;
  if ((op == GGD_EW_RELU2_BWD || op == GGD_EW_SILU_BWD || op == GGD_EW_ADD || op == GGD_EW_RELU_BWD ||
       op == GGD_EW_SIGMOID_BWD) && !b) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(ew_kernel, dim3(blocks_for(n)), dim3(TT), 0, (hipStream_t)stream, op, n, a, b, out);
  return rc(hipGetLastError());
}

int ggd_tr_q_sample(int n_clips, int per_clip, const float* x0, const float* noise, const float* ca, const float* cb,
                    float* xt, void* stream) {
  if (n_clips <= 0 || per_clip <= 0 || !x0 || !noise || !ca || !cb || !xt) return -1;
  const int64_t n = (int64_t)n_clips * per_clip;
  hipLaunchKernelGGL(qsample_kernel, dim3(blocks_for(n)), dim3(TT), 0, (hipStream_t)stream, n, per_clip, x0, noise, ca,
                     cb, xt);
  return rc(hipGetLastError());
}

int ggd_tr_mse(int n_clips, int per_clip, const float* eps, const float* noise, float* mse, float* d_eps,
               float grad_scale, void* stream) {
  if (n_clips <= 0 || per_clip <= 0 || !eps || !noise || !mse) return -1;
  hipLaunchKernelGGL(mse_kernel, dim3(n_clips), dim3(TT), 0, (hipStream_t)stream, per_clip, eps, noise, mse, d_eps,
                     grad_scale);
  return rc(hipGetLastError());
}

int ggd_tr_sumsq(int64_t n, const float* x, float* partial, float* out, void* stream) {
  if (n < 0 || !x || !partial || !out) return -1;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(SUMSQ_BLOCKS), dim3(TT), 0, s, n, x, partial);
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(SUMSQ_BLOCKS), 0, s, partial, out);
  return rc(hipGetLastError());
}

int ggd_tr_adamw(int64_t n, float* p, const float* g, float* m, float* v, float lr, float beta1, float beta2, float eps,
                 float weight_decay, int64_t step, float grad_scale, void* stream) {
  if (n < 0 || !p || !g || !m || !v || step < 1) return -1;
  if (n == 0) return 0;
  const float bc1 = (float)(1.0 - std::pow((double)beta1, (double)step));
  const float bc2 = (float)(1.0 - std::pow((double)beta2, (double)step));
  hipLaunchKernelGGL(adamw_kernel, dim3(blocks_for(n)), dim3(TT), 0, (hipStream_t)stream, n, p, g, m, v, lr, beta1, beta2,
                     eps, weight_decay, bc1, std::sqrt(bc2), grad_scale);
  return rc(hipGetLastError());
}

int ggd_tr_scale(int64_t n, float* x, float s, void* stream) {
  if (n < 0 || !x) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(scale_kernel, dim3(blocks_for(n)), dim3(TT), 0, (hipStream_t)stream, n, x, s);
  return rc(hipGetLastError());
}

int ggd_tr_scale_clamp(int64_t n, float* x, float s, float clip_value, void* stream) {
  if (n < 0 || !x || !(clip_value >= 0.f)) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(scale_clamp_kernel, dim3(blocks_for(n)), dim3(TT), 0, (hipStream_t)stream, n, x, s, clip_value);
  return rc(hipGetLastError());
}

int ggd_tr_sumsq_blocks(void) { return SUMSQ_BLOCKS; }

int ggd_tr_im2col(int N, int H, int W, int C, int KH, int KW, int stride, int pad, const float* x, float* col,
                  void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || KH <= 0 || KW <= 0 || stride <= 0 || pad < 0 || !x || !col) return -1;
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  if (Ho <= 0 || Wo <= 0) return -2;
  const int64_t total = (int64_t)N * Ho * Wo * KH * KW * C;
  hipLaunchKernelGGL(im2col_kernel, dim3(blocks_for(total)), dim3(TT), 0, (hipStream_t)stream, x, N, H, W, C, KH, KW,
                     stride, pad, Ho, Wo, col);
  return rc(hipGetLastError());
}

int ggd_tr_col2im(int N, int H, int W, int C, int KH, int KW, int stride, int pad, const float* dcol, float* dx,
                  void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || KH <= 0 || KW <= 0 || stride <= 0 || pad < 0 || !dcol || !dx) return -1;
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  if (Ho <= 0 || Wo <= 0) return -2;
  const int64_t total = (int64_t)N * H * W * C;
  hipLaunchKernelGGL(col2im_kernel, dim3(blocks_for(total)), dim3(TT), 0, (hipStream_t)stream, dcol, N, H, W, C, KH, KW,
                     stride, pad, Ho, Wo, dx);
  return rc(hipGetLastError());
}

int ggd_tr_batchnorm_fwd(int P, int C, const float* x, const float* g, const float* b, float eps, float* y, float* mean,
                         float* rstd, float* var_unbiased, void* stream) {
  if (P <= 1 || C <= 0 || !x || !g || !b || !y || !mean || !rstd) return -1;
  hipStream_t s = (hipStream_t)stream;
  const int S = chan_slices(P), rs = (P + S - 1) / S;
  float* ws = workspace(sizeof(float) * ((size_t)S * C + C));
  if (!ws) return -3;
  float* var = ws + (size_t)S * C;
  const dim3 gp((C + 63) / 64, S);
  hipLaunchKernelGGL(chan_partial_kernel, gp, dim3(256), 0, s, P, C, 0, x, nullptr, nullptr, nullptr, ws, nullptr, rs);
  hipLaunchKernelGGL(chan_final_kernel, dim3(C), dim3(256), 0, s, C, S, ws, 1.0f / P, mean, nullptr, nullptr,
                     0.f, 0.f);
  hipLaunchKernelGGL(chan_partial_kernel, gp, dim3(256), 0, s, P, C, 1, x, nullptr, mean, nullptr, ws, nullptr, rs);
  hipLaunchKernelGGL(chan_final_kernel, dim3(C), dim3(256), 0, s, C, S, ws, 1.0f / P, var, rstd, var_unbiased,
                     eps, (float)P / (float)(P - 1));
  const int64_t n = (int64_t)P * C;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(blocks_for(n)), dim3(TT), 0, s, n, C, x, mean, rstd, g, b, y);
  return rc(hipGetLastError());
}

int ggd_tr_batchnorm_bwd(int P, int C, const float* x, const float* g, const float* mean, const float* rstd,
                         const float* dy, float* dx, float* dg, float* db, void* stream) {
  if (P <= 1 || C <= 0 || !x || !g || !mean || !rstd || !dy || !dx || !dg || !db) return -1;
  hipStream_t s = (hipStream_t)stream;
  const int S = chan_slices(P), rs = (P + S - 1) / S;
  float* ws = workspace(sizeof(float) * (size_t)S * C * 2);
  if (!ws) return -3;
  hipLaunchKernelGGL(chan_partial_kernel, dim3((C + 63) / 64, S), dim3(256), 0, s, P, C, 2, x, dy, mean, rstd, ws,
                     ws + (size_t)S * C, rs);
  hipLaunchKernelGGL(chan_final_kernel, dim3(C), dim3(256), 0, s, C, S, ws, 1.0f, db, nullptr, nullptr, 0.f, 0.f);
  hipLaunchKernelGGL(chan_final_kernel, dim3(C), dim3(256), 0, s, C, S, ws + (size_t)S * C, 1.0f, dg, nullptr,
                     nullptr, 0.f, 0.f);
  const int64_t n = (int64_t)P * C;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(blocks_for(n)), dim3(TT), 0, s, n, C, P, x, dy, mean, rstd, g, db, dg, dx);
  return rc(hipGetLastError());
}

int ggd_tr_image_channel_sum(int N, int HW, int C, const float* x, const float* y, float scale, float* out,
                             void* stream) {
  if (N <= 0 || HW <= 0 || C <= 0 || !x || !out) return -1;
  hipStream_t s = (hipStream_t)stream;
  const int S = std::max(1, std::min(64, HW / 256)), ps = (HW + S - 1) / S;
  float* ws = workspace(sizeof(float) * (size_t)S * N * C);
  if (!ws) return -3;
  hipLaunchKernelGGL(img_chan_sum_kernel, dim3((C + 63) / 64, N, S), dim3(256), 0, s, HW, C, ps, x, y, ws);
  hipLaunchKernelGGL(img_chan_final_kernel, dim3(blocks_for((int64_t)N * C)), dim3(TT), 0, s, N * C, S, ws, scale, out);
  return rc(hipGetLastError());
}

int ggd_tr_channel_scale(int N, int HW, int C, const float* x, const float* s, const float* add, float* out,
                         void* stream) {
  if (N <= 0 || HW <= 0 || C <= 0 || (!x && !add) || (x && !s) || !out) return -1;
  const int64_t total = (int64_t)N * HW * C;
  hipLaunchKernelGGL(chan_scale_kernel, dim3(blocks_for(total)), dim3(TT), 0, (hipStream_t)stream, total, HW, C, x, s,
                     add, out);
  return rc(hipGetLastError());
}

int ggd_tr_pixel_shuffle(int N, int H, int W, int C, int r, const float* src, float* dst, int backward, void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || r <= 0 || !src || !dst) return -1;
  const int64_t total = (int64_t)N * H * r * W * r * C;
  hipLaunchKernelGGL(shuffle_kernel, dim3(blocks_for(total)), dim3(TT), 0, (hipStream_t)stream, N, H, W, C, r, src, dst,
                     backward ? 1 : 0);
  return rc(hipGetLastError());
}

int ggd_tr_head_flatten(int N, int H, int W, int C, const float* src, float* dst, int backward, void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || !src || !dst) return -1;
  const int64_t total = (int64_t)N * H * W * C;
  hipLaunchKernelGGL(head_flat_kernel, dim3(blocks_for(total)), dim3(TT), 0, (hipStream_t)stream, N, H, W, C, src, dst,
                     backward ? 1 : 0);
  return rc(hipGetLastError());
}

}  // extern "C"
