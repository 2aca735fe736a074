/* ggd_train.h -- C ABI of the training path's HIP kernels (libggd.so, csrc/ggd_train.hip).
 *
 * The reference trains with PyTorch autograd in fp32 (models/trainer.py:131-248
 * Trainer._compute_loss / _train_step), so its "interface" for this path is the set of torch
 * ops its modules call; each entry below replaces one of them, forward and backward, on plain
 * device pointers (f32, row-major, leading dimensions in elements) and a HIP stream.  The host
 * mirror (…_amd/training.py) wraps them in torch.autograd.Function objects, so the chain rule
 * itself is torch's and every arithmetic step is one of these kernels.
 *
 * Return: 0 ok, -1 bad argument, -2 unsupported shape, -3 HIP launch failure.
 */
#ifndef GGD_TRAIN_H
#define GGD_TRAIN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* C[M][N] = alpha opA opB + beta C (+ bias[n]); opA[m][k] = ta ? A[k lda + m] : A[m lda + k],
 * opB[k][n] = tb ? B[n ldb + k] : B[k ldb + n].  Replaces nn.Linear's F.linear (ta 0, tb 1;
 * models/modules/transformer.py:51,73, models/nn.py:189-190,213, model.py:100) and its
 * autograd backward: dX = dY W (ta 0, tb 0), dW = dY^T X (ta 1, tb 0). */
int ggd_tr_gemm(int ta, int tb, int M, int N, int K, float alpha, const float* A, int lda, const float* B, int ldb,
                float beta, float* C, int ldc, const float* bias, void* stream);
/* out[n] = beta out[n] + sum_m X[m][n]: nn.Linear bias gradient. */
int ggd_tr_colsum(int M, int N, const float* X, int ldx, float* out, float beta, void* stream);

/* nn.LayerNorm([d]) (models/nn.py:141-147,212): y = (x - mean) rstd gamma + beta, mean / rstd
 * saved per row; backward gives dx and (when dg, db are non-null) dgamma, dbeta. */
int ggd_tr_layernorm_fwd(int rows, int d, const float* x, const float* g, const float* b, float eps, float* y,
                         float* mean, float* rstd, void* stream);
int ggd_tr_layernorm_bwd(int rows, int d, const float* x, const float* g, const float* mean, const float* rstd,
                         const float* dy, float* dx, float* dg, float* db, void* stream);

/* SpatialDepthWiseConv (models/modules/transformer.py:19-44): a 3-tap conv along the frames of
 * each clip, one filter per d_k channel shared by all heads; x / y are [n clips][L][H dk]
 * row-major token matrices (leading dimensions ldx / ldy); w [dk][3], b [dk].  Backward gives dx
 * and (when dw, db are non-null) the filter gradients. */
int ggd_tr_seqconv_fwd(int n, int L, int H, int dk, const float* x, int ldx, const float* w, const float* b, float* y,
                       int ldy, void* stream);
int ggd_tr_seqconv_bwd(int n, int L, int H, int dk, const float* x, int ldx, const float* w, const float* dy, int lddy,
                       float* dx, int lddx, float* dw, float* db, void* stream);

/* MultiHeadAttention core (models/modules/transformer.py:104-118, no mask, dropout 0):
 * O = softmax_j(Q K^T scale) V per clip and head; q / o [n][Lq][H dk], k / v [n][Lk][H dk].
 * Backward recomputes P and gives dQ, dK, dV (same layouts).  Lq, Lk <= 256 with the head's
 * images inside 160 KiB of LDS (-2 otherwise). */
int ggd_tr_attention_fwd(int n, int H, int Lq, int Lk, int dk, float scale, const float* q, int ldq, const float* k,
                         const float* v, int ldkv, float* o, int ldo, void* stream);
int ggd_tr_attention_bwd(int n, int H, int Lq, int Lk, int dk, float scale, const float* q, int ldq, const float* k,
                         const float* v, int ldkv, const float* dout, int ldo, float* dq, float* dk_out, float* dv,
                         void* stream);

/* Elementwise ops: SquaredReLU (transformer.py:8-16), SiLU (nn.py:46, model.py:137-141). */
enum {
  GGD_EW_RELU2 = 0,      /* out = relu(a)^2 */
  GGD_EW_RELU2_BWD = 1,  /* out = b 2 relu(a)        (a: pre-activation, b: upstream gradient) */
  GGD_EW_SILU = 2,       /* out = a sigmoid(a) */
  GGD_EW_SILU_BWD = 3,   /* out = b (s + a s (1 - s)), s = sigmoid(a) */
  GGD_EW_ADD = 4,        /* out = a + b */
  GGD_EW_RELU = 5,       /* out = relu(a)                (ResNetSE34V2.py:119, ResNetBlocks.py:24,34) */
  GGD_EW_RELU_BWD = 6,   /* out = a > 0 ? b : 0           (a: pre-activation) */
  GGD_EW_SIGMOID = 7,    /* out = sigmoid(a)              (SELayer, ResNetBlocks.py:88) */
  GGD_EW_SIGMOID_BWD = 8 /* out = b a (1 - a)             (a: the sigmoid OUTPUT) */
};
int ggd_tr_elementwise(int op, int64_t n, const float* a, const float* b, float* out, void* stream);

/* GaussianDiffusion.q_sample (gaussian_diffusion.py:188-205) with per-clip coefficients
 * ca = sqrt(abar_t), cb = sqrt(1 - abar_t): xt = ca x0 + cb noise over per_clip elements each. */
int ggd_tr_q_sample(int n_clips, int per_clip, const float* x0, const float* noise, const float* ca, const float* cb,
                    float* xt, void* stream);
/* training_losses' mse (gaussian_diffusion.py:553-558, mean_flat): mse[clip] = mean (eps - noise)^2;
 * d_eps (nullable) = grad_scale 2 (eps - noise) / per_clip. */
int ggd_tr_mse(int n_clips, int per_clip, const float* eps, const float* noise, float* mse, float* d_eps,
               float grad_scale, void* stream);

/* sum of x^2 in two fixed-shape stages (partial holds ggd_tr_sumsq_blocks() floats): the grad
 * norm of trainer.py compute_grad_norm / clip_grad_norm_. */
int ggd_tr_sumsq(int64_t n, const float* x, float* partial, float* out, void* stream);
int ggd_tr_sumsq_blocks(void);
/* torch.optim.AdamW step (model_creation.py:176-178) over a flat parameter buffer, in torch's
 * operation order; grad_scale multiplies g first (clip_grad_norm_'s coefficient). */
int ggd_tr_adamw(int64_t n, float* p, const float* g, float* m, float* v, float lr, float beta1, float beta2, float eps,
                 float weight_decay, int64_t step, float grad_scale, void* stream);
/* x *= s (clip_grad_norm_ applied in place). */
int ggd_tr_scale(int64_t n, float* x, float s, void* stream);
/* x = clamp(x s, -clip_value, clip_value): clip_grad_norm_'s coefficient followed by
 * clip_grad_value_ (models/trainer.py:233-236), in place. */
int ggd_tr_scale_clamp(int64_t n, float* x, float s, float clip_value, void* stream);

/* ---- speech-encoder training (HA2G SE-ResNet34, ha2g/model/ResNetSE34V2.py:118-188,
 * ResNetBlocks.py:7-96) on NHWC activations: rows = pixels (n, h, w), channels innermost ---- */

/* nn.Conv2d (ha2g/model/ResNetBlocks.py:21-37, ResNetSE34V2.py:127-188) as implicit GEMMs on NHWC
 * images (no im2col copy; the conv operand is gathered while the GEMM stages it):
 *   fwd:   y[(n, oh, ow)][co] = sum_(ky, kx, c) x[n][oh s - pad + ky][ow s - pad + kx][c] wp[co][(ky, kx, c)] + bias
 *   dgrad: dx[(n, ih, iw)][c] = sum_(ky, kx, co) dy[n][(ih + pad - ky) / s][(iw + pad - kx) / s][co] wt[(ky, kx, co)][c]
 *          (exact divisions in range only)
 *   wgrad: dwp[co][(ky, kx, c)] = sum_(n, oh, ow) dy[(n, oh, ow)][co] x[...] + beta dwp
 * wp = the filter as [Co][KH][KW][C], wt = as [KH][KW][Co][C].  C (fwd, wgrad) / Co (dgrad) must be
 * a multiple of 4 (-2 otherwise: conv1's single input channel runs im2col + ggd_tr_gemm). */
int ggd_tr_conv_fwd(int N, int H, int W, int C, int Co, int KH, int KW, int stride, int pad, const float* x,
                    const float* wp, const float* bias, float* y, void* stream);
int ggd_tr_conv_dgrad(int N, int H, int W, int C, int Co, int KH, int KW, int stride, int pad, const float* dy,
                      const float* wt, float* dx, void* stream);
int ggd_tr_conv_wgrad(int N, int H, int W, int C, int Co, int KH, int KW, int stride, int pad, const float* dy,
                      const float* x, float beta, float* dwp, void* stream);
/* nn.Conv2d as im2col + ggd_tr_gemm (shapes the implicit GEMMs do not take): col[(n, oh, ow)][(ky, kx, c)]
 * (zeros outside the image); col2im is its adjoint (a gather: each input pixel sums the entries copied
 * from it). */
int ggd_tr_im2col(int N, int H, int W, int C, int KH, int KW, int stride, int pad, const float* x, float* col,
                  void* stream);
int ggd_tr_col2im(int N, int H, int W, int C, int KH, int KW, int stride, int pad, const float* dcol, float* dx,
                  void* stream);
/* nn.BatchNorm2d in train mode over P = N H W rows (batch statistics, biased variance in the
 * normalisation, eps); var_unbiased (nullable) receives the variance for the running-stat
 * update.  Backward gives dx, dgamma, dbeta. */
int ggd_tr_batchnorm_fwd(int P, int C, const float* x, const float* g, const float* b, float eps, float* y, float* mean,
                         float* rstd, float* var_unbiased, void* stream);
int ggd_tr_batchnorm_bwd(int P, int C, const float* x, const float* g, const float* mean, const float* rstd,
                         const float* dy, float* dx, float* dg, float* db, void* stream);
/* SELayer pieces (ResNetBlocks.py:81-96): out[n][c] = scale sum_p x[n][p][c] (y[n][p][c]);
 * channel_scale: out[n][p][c] = x[n][p][c] s[n][c] (+ add[n][c]; x null: add broadcast only). */
int ggd_tr_image_channel_sum(int N, int HW, int C, const float* x, const float* y, float scale, float* out,
                             void* stream);
int ggd_tr_channel_scale(int N, int HW, int C, const float* x, const float* s, const float* add, float* out,
                         void* stream);
/* nn.PixelShuffle(r) (ResNetSE34V2.py:169,179) on NHWC: src [N][H][W][C r^2] -> dst [N][H r][W r][C];
 * backward = 1 moves dst-shaped gradients back to the src shape. */
int ggd_tr_pixel_shuffle(int N, int H, int W, int C, int r, const float* src, float* dst, int backward, void* stream);
/* head flatten (ResNetSE34V2.py:161-165): NHWC [N][H][W][C] -> rows (n, w) x features (c H + h). */
int ggd_tr_head_flatten(int N, int H, int W, int C, const float* src, float* dst, int backward, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GGD_TRAIN_H */
