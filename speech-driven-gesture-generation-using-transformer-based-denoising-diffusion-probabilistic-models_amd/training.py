"""Training path: loss, backward, AdamW and the gradient all-reduce.

Mirrors the reference's training step (models/trainer.py:131-248):
  Trainer._compute_loss: x_start = poses^T, noise ~ N(0, 1), t ~ UniformSampler (resample.py:60-68),
      diffusion.training_losses (gaussian_diffusion.py:531-569) -> mse per clip -> mean, plus the
      configured speed losses on pred_x_start (speed_loss / speed_l1_loss / speed_constraint_loss,
      trainer.py:172-193; speed_losses below)
  Trainer._train_step: zero_grad, backward, compute_grad_norm (trainer.py:341-349), optional
      clip_grad_norm_ / clip_grad_value_, optimizer.step (AdamW, model_creation.py:176-178),
      lr_scheduler.step (lr_scheduler.py: ConstantLR / NoamLR "noamxf" / NoamDecayLR "noam")
  DDP (trainer.py:83, utils/pytorch_ddp.py:18): rank 0's parameters and buffers broadcast once at
      construction (broadcast_parameters), its BatchNorm buffers again before every forward
      (broadcast_buffers=True, DDP's default), gradients averaged over ranks by an all-reduce.

Every arithmetic op of the decoder's forward and backward is a hand-written HIP kernel behind
include/ggd_train.h (csrc/ggd_train.hip), wrapped here in torch.autograd.Function objects: torch
contributes the chain rule (with its gradient-accumulation adds where one tensor feeds several
ops) and a few copies (transposes, concatenations, padding).  Parameters live in ONE flat f32 buffer (each parameter a view of it), gradients in a
second flat buffer (each parameter's .grad a view; autograd accumulates into it in place), so
the all-reduce is one RCCL call per bucket and AdamW is one HIP launch over the whole model.

Scope: the one-way decoder under the s2g_v2 model (the beat-ours configuration: step encoder,
blend layer, decoder), the default model (memory = the step token and the three speech levels
concatenated, model.py:41-73) and the inpaint model (the default model plus the seed-pose
projection MLP, model.py:120-166, trained with the trainer's seed poses and masks,
trainer.py:139-146), and -- by default (train_encoder=True, as the reference) -- the HA2G speech
encoder, whose SE-ResNet trains with BatchNorm in train mode (batch statistics, running-stat
updates).  train_encoder=False freezes the encoder: it then runs as the HIP inference encoder
(eval mode) and its weights pass through state_dict() unchanged.  TrainableModel.eval() switches
the trained encoder to its running statistics (the reference's model.eval(), trainer.py:252).
"""
import ctypes
import math

import numpy as np
import torch as th
import torch.nn.functional as F

from . import native
from .weights import parameter_shapes

EW_RELU2, EW_RELU2_BWD, EW_SILU, EW_SILU_BWD, EW_ADD = 0, 1, 2, 3, 4   # include/ggd_train.h
EW_RELU, EW_RELU_BWD, EW_SIGMOID, EW_SIGMOID_BWD = 5, 6, 7, 8


def _lib():
    return native.load()


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _s(t):
    return ctypes.c_void_p(th.cuda.current_stream(t.device).cuda_stream)


def _ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed (ggd_train status {rc})")


def gemm(ta, tb, M, N, K, A, lda, B, ldb, C, ldc, alpha=1.0, beta=0.0, bias=None):
    _ok(_lib().ggd_tr_gemm(ta, tb, M, N, K, alpha, _p(A), lda, _p(B), ldb, beta, _p(C), ldc, _p(bias), _s(C)), "gemm")


# ------------------------------------------------------------------------------------------
# autograd Functions over the HIP kernels
# ------------------------------------------------------------------------------------------
_DIRECT_GRAD = [0]   # > 0 inside direct_grad_accumulation()


class direct_grad_accumulation:
    """Context manager: inside it the Linear weight / bias gradients of leaf parameters whose .grad
    exists (TrainableModel's views of the flat gradient buffer) are accumulated straight into that
    .grad (beta = 1) and returned to autograd as None.  Only Trainer.step's own loss.backward() runs
    inside it: there every such gradient is meant for .grad.  Outside it (torch.autograd.grad,
    backward(inputs=...), parameter hooks) the gradients go through autograd as usual."""

    def __enter__(self):
        _DIRECT_GRAD[0] += 1
        return self

    def __exit__(self, *exc):
        _DIRECT_GRAD[0] -= 1
        return False


def _grad_slot(p):
    """The .grad a weight-gradient kernel may accumulate into directly (beta = 1), sparing
    AccumulateGrad's separate add: inside direct_grad_accumulation() only, a leaf parameter whose
    .grad already exists as a contiguous f32 tensor.  None: return the gradient to autograd as usual."""
    if not _DIRECT_GRAD[0] or p is None or not p.is_leaf or not p.requires_grad or th.is_grad_enabled():
        return None
    g = p.grad
    if g is None or not g.is_contiguous() or g.dtype != th.float32 or g.shape != p.shape:
        return None
    return g


class _Linear(th.autograd.Function):
    """nn.Linear (F.linear): y = x W^T + b; dX = dY W, dW = dY^T X, db = colsum dY."""

    @staticmethod
    def forward(ctx, x, w, b):
        M, K = x.shape
        N = w.shape[0]
        y = x.new_empty(M, N)
        gemm(0, 1, M, N, K, x, K, w, K, y, N, bias=b)
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        ctx.b = b
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        M, K = x.shape
        N = w.shape[0]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = x.new_empty(M, K)
            gemm(0, 0, M, K, N, dy, N, w, K, dx, K)
        if ctx.needs_input_grad[1]:
            g = _grad_slot(w)
            if g is not None:   # accumulate into the parameter's .grad (the flat gradient buffer)
                gemm(1, 0, N, K, M, dy, N, x, K, g, K, beta=1.0)
            else:
                dw = w.new_empty(N, K)
                gemm(1, 0, N, K, M, dy, N, x, K, dw, K)
        if ctx.has_b and ctx.needs_input_grad[2]:
            b = ctx.b
            g = _grad_slot(b)
            if g is not None:
                _ok(_lib().ggd_tr_colsum(M, N, _p(dy), N, _p(g), 1.0, _s(dy)), "colsum")
            else:
                db = w.new_empty(N)
                _ok(_lib().ggd_tr_colsum(M, N, _p(dy), N, _p(db), 0.0, _s(dy)), "colsum")
        return dx, dw, db


def linear(x, w, b=None):
    shape = x.shape
    y = _Linear.apply(x.reshape(-1, shape[-1]).contiguous(), w, b)
    return y.reshape(*shape[:-1], w.shape[0])


class _LayerNorm(th.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, eps):
        rows, d = x.shape
        y = th.empty_like(x)
        mean = x.new_empty(rows)
        rstd = x.new_empty(rows)
        _ok(_lib().ggd_tr_layernorm_fwd(rows, d, _p(x), _p(g), _p(b), eps, _p(y), _p(mean), _p(rstd), _s(x)), "ln fwd")
        ctx.save_for_backward(x, g, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, g, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous()
        rows, d = x.shape
        dx = th.empty_like(x)
        dg = th.empty_like(g)
        db = th.empty_like(g)
        _ok(_lib().ggd_tr_layernorm_bwd(rows, d, _p(x), _p(g), _p(mean), _p(rstd), _p(dy), _p(dx), _p(dg), _p(db),
                                        _s(x)), "ln bwd")
        return dx, dg, db, None


def layer_norm(x, g, b, eps=1e-5):
    shape = x.shape
    return _LayerNorm.apply(x.reshape(-1, shape[-1]).contiguous(), g, b, eps).reshape(shape)


class _SeqConv(th.autograd.Function):
    """SpatialDepthWiseConv over frames of (n, L, H dk) token matrices."""

    @staticmethod
    def forward(ctx, x, w, b, heads):
        n, L, W = x.shape
        dk = W // heads
        y = th.empty_like(x)
        w3 = w.reshape(dk, 3)
        _ok(_lib().ggd_tr_seqconv_fwd(n, L, heads, dk, _p(x), W, _p(w3), _p(b), _p(y), W, _s(x)), "conv fwd")
        ctx.save_for_backward(x, w)
        ctx.heads = heads
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        n, L, W = x.shape
        H = ctx.heads
        dk = W // H
        dx = th.empty_like(x)
        dw = th.empty_like(w)
        db = w.new_empty(dk)
        _ok(_lib().ggd_tr_seqconv_bwd(n, L, H, dk, _p(x), W, _p(w.reshape(dk, 3)), _p(dy), W, _p(dx), W, _p(dw), _p(db),
                                      _s(x)), "conv bwd")
        return dx, dw, db, None


class _Attention(th.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, heads, scale):
        n, Lq, W = q.shape
        Lk = k.shape[1]
        dk = W // heads
        o = th.empty_like(q)
        _ok(_lib().ggd_tr_attention_fwd(n, heads, Lq, Lk, dk, scale, _p(q), W, _p(k), _p(v), W, _p(o), W, _s(q)),
            "attention fwd")
        ctx.save_for_backward(q, k, v)
        ctx.heads, ctx.scale = heads, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v = ctx.saved_tensors
        do = do.contiguous()
        n, Lq, W = q.shape
        Lk = k.shape[1]
        H = ctx.heads
        dq, dk_, dv = th.empty_like(q), th.empty_like(k), th.empty_like(v)
        _ok(_lib().ggd_tr_attention_bwd(n, H, Lq, Lk, W // H, ctx.scale, _p(q), W, _p(k), _p(v), W, _p(do), W, _p(dq),
                                        _p(dk_), _p(dv), _s(q)), "attention bwd")
        return dq, dk_, dv, None, None


def _ew(op, a, b=None):
    out = th.empty_like(a)
    _ok(_lib().ggd_tr_elementwise(op, a.numel(), _p(a), _p(b), _p(out), _s(a)), "elementwise")
    return out


class _Act(th.autograd.Function):
    @staticmethod
    def forward(ctx, x, fwd_op, bwd_op):
        x = x.contiguous()
        ctx.save_for_backward(x)
        ctx.bwd_op = bwd_op
        return _ew(fwd_op, x)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return _ew(ctx.bwd_op, x, dy.contiguous()), None, None


def squared_relu(x):
    """SquaredReLU (transformer.py:8-16)."""
    return _Act.apply(x, EW_RELU2, EW_RELU2_BWD)


def silu(x):
    return _Act.apply(x, EW_SILU, EW_SILU_BWD)


class _Add(th.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        return _ew(EW_ADD, a.contiguous(), b.contiguous())

    @staticmethod
    def backward(ctx, dy):
        return dy, dy


def add(a, b):
    return _Add.apply(a, b)


def relu(x):
    return _Act.apply(x, EW_RELU, EW_RELU_BWD)


class _Sigmoid(th.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = _ew(EW_SIGMOID, x.contiguous())
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return _ew(EW_SIGMOID_BWD, y, dy.contiguous())


# ------------------------------------------------------------------------------------------
# speech-encoder ops on NHWC activations (N, H, W, C): H = mel axis, W = frames
# ------------------------------------------------------------------------------------------
class _Conv2d(th.autograd.Function):
    """nn.Conv2d on NHWC images.  Input channels a multiple of 4 (every tower / head conv): implicit GEMMs
    (ggd_tr_conv_fwd / _dgrad / _wgrad) gather the conv operand from the image while staging it -- no
    im2col copy; db = colsum dY.  conv1 (one input channel): im2col + GEMM, dW = dY^T col, dcol = dY W,
    dX = col2im(dcol), col recomputed in backward (memory)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad):
        x = x.contiguous()
        N, H, W, C = x.shape
        Co, Ci, KH, KW = w.shape
        assert Ci == C
        Ho, Wo = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
        K, P = KH * KW * C, N * Ho * Wo
        wp = w.permute(0, 2, 3, 1).contiguous().reshape(Co, K)
        lib = _lib()
        y = x.new_empty(P, Co)
        implicit = C % 4 == 0 and Co % 4 == 0
        if implicit:
            _ok(lib.ggd_tr_conv_fwd(N, H, W, C, Co, KH, KW, stride, pad, _p(x), _p(wp), _p(b), _p(y), _s(x)),
                "conv fwd")
        else:
            col = x.new_empty(P, K)
            _ok(lib.ggd_tr_im2col(N, H, W, C, KH, KW, stride, pad, _p(x), _p(col), _s(x)), "im2col")
            gemm(0, 1, P, Co, K, col, K, wp, K, y, Co, bias=b)
        ctx.save_for_backward(x, w if implicit else wp)
        ctx.geo = (N, H, W, C, Co, KH, KW, stride, pad, Ho, Wo, b is not None, implicit)
        return y.view(N, Ho, Wo, Co)

    @staticmethod
    def backward(ctx, dy):
        x, wq = ctx.saved_tensors
        N, H, W, C, Co, KH, KW, stride, pad, Ho, Wo, has_b, implicit = ctx.geo
        K, P = KH * KW * C, N * Ho * Wo
        dy = dy.contiguous().view(P, Co)
        lib = _lib()
        dwp = x.new_empty(Co, K)
        dx = None
        if implicit:
            _ok(lib.ggd_tr_conv_wgrad(N, H, W, C, Co, KH, KW, stride, pad, _p(dy), _p(x), 0.0, _p(dwp), _s(dy)),
                "conv wgrad")
            if ctx.needs_input_grad[0]:
                wt = wq.permute(2, 3, 0, 1).contiguous()            # [KH][KW][Co][C]
                dx = th.empty_like(x)
                _ok(lib.ggd_tr_conv_dgrad(N, H, W, C, Co, KH, KW, stride, pad, _p(dy), _p(wt), _p(dx), _s(dy)),
                    "conv dgrad")
        else:
            col = x.new_empty(P, K)
            _ok(lib.ggd_tr_im2col(N, H, W, C, KH, KW, stride, pad, _p(x), _p(col), _s(x)), "im2col")
            gemm(1, 0, Co, K, P, dy, Co, col, K, dwp, K)
            if ctx.needs_input_grad[0]:
                dcol = col  # reuse the buffer
                gemm(0, 0, P, K, Co, dy, Co, wq, K, dcol, K)
                dx = th.empty_like(x)
                _ok(lib.ggd_tr_col2im(N, H, W, C, KH, KW, stride, pad, _p(dcol), _p(dx), _s(x)), "col2im")
        dw = dwp.view(Co, KH, KW, C).permute(0, 3, 1, 2).contiguous()
        db = None
        if has_b:
            db = x.new_empty(Co)
            _ok(lib.ggd_tr_colsum(P, Co, _p(dy), Co, _p(db), 0.0, _s(dy)), "colsum")
        return dx, dw, db, None, None


class _BatchNorm2d(th.autograd.Function):
    """nn.BatchNorm2d in train mode (batch statistics over N H W, eps 1e-5); `stats` receives the
    batch mean and unbiased variance for the running-stat update."""

    @staticmethod
    def forward(ctx, x, g, b, stats):
        N, H, W, C = x.shape
        P = N * H * W
        y = th.empty_like(x)
        mean, rstd, var_u = x.new_empty(C), x.new_empty(C), x.new_empty(C)
        _ok(_lib().ggd_tr_batchnorm_fwd(P, C, _p(x), _p(g), _p(b), 1e-5, _p(y), _p(mean), _p(rstd), _p(var_u), _s(x)),
            "bn fwd")
        stats.append((mean, var_u))
        ctx.save_for_backward(x, g, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, g, mean, rstd = ctx.saved_tensors
        N, H, W, C = x.shape
        dx, dg, db = th.empty_like(x), th.empty_like(g), th.empty_like(g)
        _ok(_lib().ggd_tr_batchnorm_bwd(N * H * W, C, _p(x), _p(g), _p(mean), _p(rstd), _p(dy.contiguous()), _p(dx),
                                        _p(dg), _p(db), _s(x)), "bn bwd")
        return dx, dg, db, None


class _ChanMean(th.autograd.Function):
    """AdaptiveAvgPool2d(1): (N, H, W, C) -> (N, C)."""

    @staticmethod
    def forward(ctx, x):
        N, H, W, C = x.shape
        out = x.new_empty(N, C)
        _ok(_lib().ggd_tr_image_channel_sum(N, H * W, C, _p(x), None, 1.0 / (H * W), _p(out), _s(x)), "pool")
        ctx.shape = x.shape
        return out

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.shape
        lib = _lib()
        d = dy.contiguous().clone()
        _ok(lib.ggd_tr_scale(d.numel(), _p(d), 1.0 / (H * W), _s(d)), "scale")
        dx = d.new_empty(N, H, W, C)
        _ok(lib.ggd_tr_channel_scale(N, H * W, C, None, None, _p(d), _p(dx), _s(d)), "broadcast")
        return dx


class _ChanScale(th.autograd.Function):
    """SELayer's x * y[:, :, None, None] on NHWC: (N, H, W, C) x (N, C)."""

    @staticmethod
    def forward(ctx, x, sc):
        N, H, W, C = x.shape
        out = th.empty_like(x)
        _ok(_lib().ggd_tr_channel_scale(N, H * W, C, _p(x), _p(sc), None, _p(out), _s(x)), "chan scale")
        ctx.save_for_backward(x, sc)
        return out

    @staticmethod
    def backward(ctx, dy):
        x, sc = ctx.saved_tensors
        N, H, W, C = x.shape
        dy = dy.contiguous()
        lib = _lib()
        dx = th.empty_like(x)
        _ok(lib.ggd_tr_channel_scale(N, H * W, C, _p(dy), _p(sc), None, _p(dx), _s(x)), "chan scale bwd")
        ds = sc.new_empty(N, C)
        _ok(lib.ggd_tr_image_channel_sum(N, H * W, C, _p(dy), _p(x), 1.0, _p(ds), _s(x)), "chan scale ds")
        return dx, ds


class _PixelShuffle(th.autograd.Function):
    @staticmethod
    def forward(ctx, x, r):
        N, H, W, Cr = x.shape
        C = Cr // (r * r)
        y = x.new_empty(N, H * r, W * r, C)
        _ok(_lib().ggd_tr_pixel_shuffle(N, H, W, C, r, _p(x), _p(y), 0, _s(x)), "shuffle")
        ctx.geo = (N, H, W, C, r)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C, r = ctx.geo
        dx = dy.new_empty(N, H, W, C * r * r)
        _ok(_lib().ggd_tr_pixel_shuffle(N, H, W, C, r, _p(dy.contiguous()), _p(dx), 1, _s(dy)), "shuffle bwd")
        return dx, None


class _HeadFlatten(th.autograd.Function):
    """NHWC (N, H, W, C) -> (N, W, C H): the reference's feat.reshape(N, -1, W).transpose(1, 2)."""

    @staticmethod
    def forward(ctx, x):
        N, H, W, C = x.shape
        y = x.new_empty(N, W, C * H)
        _ok(_lib().ggd_tr_head_flatten(N, H, W, C, _p(x), _p(y), 0, _s(x)), "flatten")
        ctx.geo = (N, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.geo
        dx = dy.new_empty(N, H, W, C)
        _ok(_lib().ggd_tr_head_flatten(N, H, W, C, _p(dy.contiguous()), _p(dx), 1, _s(dy)), "flatten bwd")
        return dx


# ------------------------------------------------------------------------------------------
# the trainable model
# ------------------------------------------------------------------------------------------
def positional_table(d, max_len):
    """PositionalEncoding table (transformer.py:157-166), [max_len][d]."""
    pos = th.arange(0, max_len, dtype=th.float32)[:, None]
    freq = th.exp(th.arange(0, d, 2, dtype=th.float32) * -(math.log(10000.0) / d))
    tab = th.zeros(max_len, d)
    tab[:, 0::2] = th.sin(pos * freq)
    tab[:, 1::2] = th.cos(pos * freq)
    return tab


def step_embedding(t, dim, max_period=10000):
    """diffusion_step_embedding (nn.py:17-35): [cos | sin] of t f_k, f_k = exp(-ln(1e4) k / (dim / 2))."""
    half = dim // 2
    freqs = th.exp(-math.log(max_period) * th.arange(0, half, dtype=th.float32, device=t.device) / half)
    arg = t[:, None].float() * freqs[None]
    return th.cat([th.cos(arg), th.sin(arg)], dim=-1)


_ENC_BUFFERS = (".running_mean", ".running_var", ".num_batches_tracked", "wav2spec.0.flipped_filter",
                "wav2spec.1.spectrogram.window", "wav2spec.1.mel_scale.fb")


def _trainable(arch, train_encoder=False):
    """Parameter names the training path updates (reference state_dict order): the decoder, step
    encoder and blend layer, plus the speech encoder's parameters when it is trained (its BN running
    statistics and front-end constants are buffers, never parameters)."""
    shapes = parameter_shapes(arch)
    out = []
    for k, (shape, init) in shapes.items():
        if init == "int0" or k.endswith(_ENC_BUFFERS):
            continue
        if k.startswith("speech_encoder.") and not train_encoder:
            continue
        out.append((k, shape))
    return out


class TrainableModel:
    """The denoiser (models/model.py:41-166) -- s2g_v2, default or inpaint model, one-way
    (nn.py:177-228) or two-way (nn.py:381-447) decoder -- with its trainable parameters in one flat
    f32 device buffer under the reference's state_dict names."""

    def __init__(self, arch, sd, device="cuda", train_encoder=False, pose_seed_len=None):
        if arch["type"] not in ("s2g_v2", "default", "inpaint") or \
                arch["decoder"] not in ("oneway_cross_attention", "cross_attention"):
            raise ValueError("the training path covers the one-way and two-way decoders under the s2g_v2, default "
                             "and inpaint models")
        if arch["type"] == "inpaint" and pose_seed_len is None:
            raise ValueError("the inpaint model trains with its pose_seed_len (Model.Generate.pose_seed_len, "
                             "model_creation.py:141)")
        self.arch = arch
        self.pose_seed_len = pose_seed_len   # Speech2GestureModelInpaint.pose_seed_len (model.py:134)
        self.device = th.device(device)
        if self.device.type != "cuda":
            raise ValueError("the training path runs on a GPU device only (no CPU fallback)")
        self.train_encoder = bool(train_encoder)
        names = _trainable(arch, self.train_encoder)
        total = sum(int(np.prod(s)) for _, s in names)
        self.flat = th.zeros(total, device=self.device)
        self.flat_grad = th.zeros(total, device=self.device)
        self.params = {}
        off = 0
        for k, shape in names:
            n = int(np.prod(shape))
            p = th.nn.Parameter(self.flat[off:off + n].view(shape))
            p.grad = self.flat_grad[off:off + n].view(shape)
            self.params[k] = p
            off += n
        self._pe = {}
        self._enc_sd = {k: v.detach().cpu().clone() for k, v in sd.items() if k.startswith("speech_encoder.")}
        self._encoder = None
        self._frontend = None
        self.training = True
        # BatchNorm running statistics of the trained encoder (buffers, updated in train mode)
        self.buffers = {k: v.detach().to(self.device).clone() for k, v in sd.items()
                        if k.startswith("speech_encoder.") and k.endswith(_ENC_BUFFERS[:3])} if self.train_encoder else {}
        self.load_state_dict(sd)

    # -- mode (nn.Module.train / eval) ---------------------------------------------------------
    def train(self, mode=True):
        """Train mode: the trained encoder's BatchNorms use batch statistics and update their
        running statistics.  Eval mode (model.eval(), trainer.py:252): the encoder runs with the
        running statistics and updates nothing."""
        self.training = bool(mode)
        if self.train_encoder:
            self._encoder = None  # an eval-mode encoder is rebuilt from the current (trained) weights
        return self

    def eval(self):
        return self.train(False)

    def _encoder_state(self):
        """The speech encoder's entries of state_dict(): trained parameters and running statistics
        when the encoder trains, the frozen weights otherwise; the front-end constants always."""
        sd = {}
        for k, v in self._enc_sd.items():
            if k in self.params:
                v = self.params[k].detach()
            elif k in self.buffers:
                v = self.buffers[k]
            sd[k] = v
        return sd

    def speech_encoder(self):
        """The HA2G encoder as the HIP inference encoder (f32, eval mode: BatchNorm on running
        statistics) on this model's CURRENT encoder weights."""
        if self._encoder is None:
            from .encoder import SpeechEncoder
            self._encoder = SpeechEncoder(self._encoder_state(), self.device, dtype="f32", d_model=self.arch["d_model"])
        return self._encoder

    def _frontend_encoder(self):
        """A HIP encoder context kept only for its parameter-free front end (pre-emphasis, STFT, mel,
        InstanceNorm: the wav2spec.* constants, which never train), built once: the trained
        encoder's weights change every step, and rebuilding a context per step to reach the front
        end cost a full weight upload per training step."""
        if self._frontend is None:
            from .encoder import SpeechEncoder
            self._frontend = SpeechEncoder(self._enc_sd, self.device, dtype="f32", d_model=self.arch["d_model"])
        return self._frontend

    # -- state ---------------------------------------------------------------------------------
    def load_state_dict(self, sd, strict=False):
        """Reference state_dict keys; with strict, every key of state_dict() must be present."""
        want = self.state_dict_keys()
        missing = [k for k in want if k not in sd]
        if strict and missing:
            raise RuntimeError(f"missing keys {missing[:5]}")
        with th.no_grad():
            for k, p in self.params.items():
                if k in sd:
                    p.copy_(sd[k].to(p.device, th.float32).reshape(p.shape))
            for k, b in self.buffers.items():
                if k in sd:
                    b.copy_(sd[k].to(b.device, b.dtype).reshape(b.shape))
            for k in self._enc_sd:
                if k in sd and k not in self.params and k not in self.buffers:
                    self._enc_sd[k] = sd[k].detach().cpu().clone()
        self._encoder = None
        self._frontend = None
        return missing

    def state_dict_keys(self):
        return [k for k in parameter_shapes(self.arch) if k in self.params or k in self._enc_sd]

    def state_dict(self):
        """The reference module tree's full state_dict (model.module.state_dict(), trainer.py:202),
        in its key order: parameters, BatchNorm buffers and the front-end constants
        (wav2spec.*: pre-emphasis filter, Hann window, mel filterbank); the frozen encoder's
        weights when train_encoder is False.  Loads into create_model(...)[0] with strict=True."""
        enc = self._encoder_state()
        out = {}
        for k in parameter_shapes(self.arch):
            if k in self.params:
                out[k] = self.params[k].detach().clone()
            elif k in enc:
                out[k] = enc[k].clone()
        return out

    def named_parameters(self):
        return iter(self.params.items())

    def parameters(self):
        return iter(self.params.values())

    def zero_grad(self):
        self.flat_grad.zero_()

    def _pe_rows(self, n, L):
        key = (n, L)
        if key not in self._pe:
            tab = positional_table(self.arch["d_model"], L).to(self.device)
            self._pe[key] = tab[None].expand(n, L, -1).contiguous()
        return self._pe[key]

    # -- forward (model.py:81-117 + nn.py:216-228), token-major (N, L, d) ----------------------
    def _mdha(self, pre, q_in, kv_in):
        P, H = self.params, self.arch["heads"]
        d = self.arch["d_model"]

        def heads(x, w):
            y = linear(x, P[f"{pre}.{w}.0.linear.weight"], P[f"{pre}.{w}.0.linear.bias"])
            return _SeqConv.apply(y.contiguous(), P[f"{pre}.{w}.1.conv.weight"], P[f"{pre}.{w}.1.conv.bias"], H)

        q, k, v = heads(q_in, "query"), heads(kv_in, "key"), heads(kv_in, "value")
        o = _Attention.apply(q, k, v, H, 1.0 / math.sqrt(d // H))
        return linear(o, P[f"{pre}.output.weight"], P[f"{pre}.output.bias"])

    # -- the HA2G encoder in train mode (ResNetSE34V2.py:118-188), NHWC ---------------------------
    def _bn(self, name, x):
        if not self.training:
            raise RuntimeError("encode() builds the train-mode graph; in eval mode the model encodes with "
                               "speech_encoder() (running statistics)")
        self._encoder = None     # the weights / statistics the cached eval encoder holds are changing
        stats = []
        y = _BatchNorm2d.apply(x, self.params[name + ".weight"], self.params[name + ".bias"], stats)
        mean, var_u = stats[0]
        with th.no_grad():   # nn.BatchNorm2d momentum 0.1 running-stat update
            self.buffers[name + ".running_mean"].mul_(0.9).add_(0.1 * mean)
            self.buffers[name + ".running_var"].mul_(0.9).add_(0.1 * var_u)
            self.buffers[name + ".num_batches_tracked"].add_(1)
        return y

    def _conv(self, name, x, stride=1, pad=0):
        return _Conv2d.apply(x, self.params[name + ".weight"], self.params.get(name + ".bias"), stride, pad)

    def _se_block(self, name, x, stride):
        """SEBasicBlock (ResNetBlocks.py:21-37): conv, ReLU, BN, conv, BN, SE, + residual, ReLU."""
        P = self.params
        out = self._bn(name + ".bn1", relu(self._conv(name + ".conv1", x, stride, 1)))
        out = self._bn(name + ".bn2", self._conv(name + ".conv2", out, 1, 1))
        y = relu(linear(_ChanMean.apply(out), P[name + ".se.fc.0.weight"], P[name + ".se.fc.0.bias"]))
        y = _Sigmoid.apply(linear(y, P[name + ".se.fc.2.weight"], P[name + ".se.fc.2.bias"]))
        out = _ChanScale.apply(out, y)
        if (name + ".downsample.0.weight") in P:
            res = self._bn(name + ".downsample.1", self._conv(name + ".downsample.0", x, stride, 0))
        else:
            res = x
        return relu(add(out, res))

    def encode(self, wav=None, img=None):
        """HA2GSpeechEncoder.forward (speech_encoder.py:37-61) with the SE-ResNet in train mode:
        (z_low, z_mid, z_high) with the autograd graph to the encoder's parameters.  img: the
        front end's InstanceNorm'd mel image (N, 128, F) when already computed."""
        P = self.params
        if img is None:
            img = self._frontend_encoder().frontend(wav)              # (N, 128, F), parameter-free
        r = "speech_encoder.wav_encoder.feat_extractor."
        x = img[..., None]                                           # NHWC, C = 1
        x = self._bn(r + "bn1", relu(self._conv(r + "conv1", x, 1, 1)))
        feats = []
        for li, (nblk, stride) in enumerate(zip((3, 4, 6, 3), (1, 2, 2, 2))):
            for bi in range(nblk):
                x = self._se_block(r + f"layer{li + 1}.{bi}", x, stride if bi == 0 else 1)
            feats.append(x)
        proj_w, proj_b = P["speech_encoder.wav_proj_layer.weight"], P["speech_encoder.wav_proj_layer.bias"]
        out = []
        for feat, hn, shuf in ((feats[1], "low", 1), (feats[2], "mid", 2), (feats[3], "high", 4)):
            if shuf > 1:
                feat = _PixelShuffle.apply(feat.contiguous(), shuf)
            h = self._bn(r + "bn_" + hn, relu(self._conv(r + "conv_" + hn, feat, 1, 0)))
            h = linear(_HeadFlatten.apply(h.contiguous()), P[r + f"fc_{hn}.weight"], P[r + f"fc_{hn}.bias"])
            out.append(linear(h, proj_w, proj_b))
        return tuple(out)

    def _ffn(self, q, sfx, h):
        """h + FeedForward(LayerNorm(h)) with SquaredReLU (transformer.py:129-154); sfx "" or "_mem"."""
        P = self.params
        u = layer_norm(h, P[q + f"norm_ff{sfx}.weight"], P[q + f"norm_ff{sfx}.bias"])
        f = squared_relu(linear(u, P[q + f"feed_forward{sfx}.layer1.weight"], P[q + f"feed_forward{sfx}.layer1.bias"]))
        return add(h, linear(f, P[q + f"feed_forward{sfx}.layer2.weight"], P[q + f"feed_forward{sfx}.layer2.bias"]))

    def _twoway(self, x, m):
        """CrossAttention.forward (nn.py:428-447) over embedded poses x (N, L, d) and memory m (N, Tm, d):
        one positional encoding over the joint sequence [x; m] (nn.py:438-442); per layer
        (CrossAttentionLayer, nn.py:381-418) self-attention of x and of m, attention over the joint
        sequence, then the feed-forward of x -- and of m except in the last layer.  The joint
        sequence is a concatenation of the two streams' token rows (data movement); every op on it
        runs on the HIP kernels with its backward."""
        P, a = self.params, self.arch
        N, L, _ = x.shape
        Tm = m.shape[1]
        pe = self._pe_rows(N, L + Tm)
        x = add(x, pe[:, :L].contiguous())
        m = add(m, pe[:, L:].contiguous())
        for i in range(a["n_layers"]):
            q = f"pose_decoder.layers.{i}."
            u = layer_norm(x, P[q + "norm_self_attn.weight"], P[q + "norm_self_attn.bias"])
            x = add(x, self._mdha(q + "self_attn", u, u))
            u = layer_norm(m, P[q + "norm_self_attn_mem.weight"], P[q + "norm_self_attn_mem.bias"])
            m = add(m, self._mdha(q + "self_attn_mem", u, u))
            h = th.cat([x, m], dim=1)
            u = layer_norm(h, P[q + "norm_cross_attn.weight"], P[q + "norm_cross_attn.bias"])
            h = add(h, self._mdha(q + "cross_attn", u, u))
            x, m = h[:, :L].contiguous(), h[:, L:].contiguous()
            x = self._ffn(q, "", x)
            if (q + "feed_forward_mem.layer1.weight") in P:
                m = self._ffn(q, "_mem", m)
        return x

    def __call__(self, x_t, t, z=None, wav=None, inpaint_pose=None, inpaint_mask=None):
        """x_t (N, C, L), t (N,) int64 original timesteps -> eps (N, C, L).  Speech: z = (z_low, z_mid,
        z_high) tokens (N, T_i, d) from the frozen encoder, or wav (N, T_wav) encoded here (through the
        trained encoder in train mode when train_encoder, else the HIP eval-mode encoder on the
        current weights -- no gradient reaches the encoder in eval mode).  The inpaint model also
        takes inpaint_pose (L, N, C) and inpaint_mask (L, N, 1), the reference's model kwargs."""
        if z is None:
            z = self.encode(wav) if (self.train_encoder and self.training) else self.speech_encoder()(wav)
        P, a = self.params, self.arch
        d = a["d_model"]
        N, C, L = x_t.shape
        e = step_embedding(t.to(self.device), d)
        s = linear(silu(linear(e, P["diffusion_step_encoder.proj.0.weight"], P["diffusion_step_encoder.proj.0.bias"])),
                   P["diffusion_step_encoder.proj.2.weight"], P["diffusion_step_encoder.proj.2.bias"])
        if a["type"] == "s2g_v2":
            # memory: [step token; blend(left-padded levels)] (model.py:91-106)
            longest = max(zi.shape[1] for zi in z)
            zz = th.cat([F.pad(zi, (0, 0, longest - zi.shape[1], 0)) for zi in z], dim=-1)
            sp = linear(zz, P["blend_layer.weight"], P["blend_layer.bias"])
            mem = th.cat([s[:, None], sp], dim=1)
        else:
            # default / inpaint: memory = [step token; z_low; z_mid; z_high] along time (model.py:44-67)
            mem = th.cat([s[:, None]] + [zi for zi in z], dim=1)
        Tm = mem.shape[1]
        pre = "pose_decoder."
        if a["decoder"] == "oneway_cross_attention":   # positions restart at 0 for the memory (nn.py:222-223)
            m = add(linear(mem, P[pre + "emb_mem.weight"], P[pre + "emb_mem.bias"]), self._pe_rows(N, Tm))
        x_in = x_t.transpose(1, 2).contiguous()                                      # (N, L, C)
        if a["type"] == "inpaint":
            # Speech2GestureModelInpaint.myforward (model.py:152-166): x + proj([pose * mask, mask]); the
            # batch's seed poses and mask are data (no parameters): their product and concatenation are
            # plain device tensor ops, the proj MLP runs on the HIP kernels with its gradients
            if inpaint_pose is None or inpaint_mask is None:
                raise TypeError("Speech2GestureModelInpaint.myforward() needs inpaint_pose and inpaint_mask")
            assert tuple(inpaint_pose.shape) == (L, N, C) and tuple(inpaint_mask.shape) == (L, N, 1)
            pose = inpaint_pose.to(self.device, th.float32).transpose(0, 1)
            mask = inpaint_mask.to(self.device, th.float32).transpose(0, 1)
            xi = th.cat([pose * mask, mask], dim=-1).contiguous()                    # (N, L, C + 1)
            u = silu(linear(xi, P["proj.0.weight"], P["proj.0.bias"]))
            u = silu(linear(u, P["proj.2.weight"], P["proj.2.bias"]))
            x_in = add(x_in, linear(u, P["proj.4.weight"], P["proj.4.bias"]))       # Dropout p = 0 (configs)
        if a["decoder"] == "cross_attention":
            h = self._twoway(linear(x_in, P[pre + "emb_x.weight"], P[pre + "emb_x.bias"]),
                             linear(mem, P[pre + "emb_mem.weight"], P[pre + "emb_mem.bias"]))
        else:
            h = add(linear(x_in, P[pre + "emb_x.weight"], P[pre + "emb_x.bias"]), self._pe_rows(N, L))
            for i in range(a["n_layers"]):
                q = pre + f"layers.{i}."
                u = layer_norm(h, P[q + "norm_self_attn.weight"], P[q + "norm_self_attn.bias"])
                h = add(h, self._mdha(q + "self_attn", u, u))
                u = layer_norm(h, P[q + "norm_cross_attn.weight"], P[q + "norm_cross_attn.bias"])
                h = add(h, self._mdha(q + "cross_attn", u, m))
                h = self._ffn(q, "", h)
        u = layer_norm(h, P[pre + "out_layers.0.weight"], P[pre + "out_layers.0.bias"])
        y = linear(u, P[pre + "out_layers.1.weight"], P[pre + "out_layers.1.bias"])
        return y.transpose(1, 2)


# ------------------------------------------------------------------------------------------
# loss (gaussian_diffusion.py:531-569)
# ------------------------------------------------------------------------------------------
class _DiffusionMSE(th.autograd.Function):
    @staticmethod
    def forward(ctx, eps, noise):
        eps = eps.contiguous()
        n = eps.shape[0]
        per = eps[0].numel()
        mse = eps.new_empty(n)
        d = th.empty_like(eps)
        _ok(_lib().ggd_tr_mse(n, per, _p(eps), _p(noise), _p(mse), _p(d), 1.0, _s(eps)), "mse")
        ctx.save_for_backward(d)
        return mse

    @staticmethod
    def backward(ctx, dmse):
        (d,) = ctx.saved_tensors
        n = d.shape[0]
        out = th.empty_like(d)
        zero = d.new_zeros(n)  # out = dmse[clip] d (the q_sample kernel with coefficients (dmse, 0))
        _ok(_lib().ggd_tr_q_sample(n, d[0].numel(), _p(d), _p(d), _p(dmse.contiguous()), _p(zero), _p(out), _s(d)),
            "mse bwd")
        return out, None


def q_sample(diffusion, x_start, t, noise):
    """gaussian_diffusion.py:188-205 with the fp64 tables cast to f32 per clip (_extract_into_tensor)."""
    idx = t.cpu().numpy()
    ca = th.from_numpy(diffusion.sqrt_alphas_cumprod[idx]).float().to(x_start.device)
    cb = th.from_numpy(diffusion.sqrt_one_minus_alphas_cumprod[idx]).float().to(x_start.device)
    xt = th.empty_like(x_start)
    n = x_start.shape[0]
    _ok(_lib().ggd_tr_q_sample(n, x_start[0].numel(), _p(x_start), _p(noise), _p(ca), _p(cb), _p(xt), _s(xt)),
        "q_sample")
    return xt


def training_losses(diffusion, model, x_start, t, model_kwargs, noise=None):
    """GaussianDiffusion.training_losses (gaussian_diffusion.py:531-569): returns mse (N,), eps and
    pred_x_start with the autograd graph to the parameters (the reference's speed losses,
    trainer.py:172-193, differentiate through pred_x_start), x_t and model_mean (detached)."""
    x_start = x_start.contiguous().float()
    if noise is None:
        noise = th.randn_like(x_start)
    noise = noise.contiguous().float()
    x_t = q_sample(diffusion, x_start, t, noise)
    eps = model(x_t, t, z=model_kwargs.get("speech_tokens"), wav=model_kwargs.get("wav"),
                inpaint_pose=model_kwargs.get("inpaint_pose"), inpaint_mask=model_kwargs.get("inpaint_mask"))
    assert eps.shape == noise.shape == x_start.shape
    mse = _DiffusionMSE.apply(eps, noise)
    idx = t.cpu().numpy()
    ext = lambda arr: th.from_numpy(arr[idx]).float().to(x_t.device).reshape(-1, 1, 1)
    # _predict_xstart_from_eps (gaussian_diffusion.py:287-292), on the graph
    x0 = ext(diffusion.sqrt_recip_alphas_cumprod) * x_t - ext(diffusion.sqrt_recipm1_alphas_cumprod) * eps
    with th.no_grad():
        mean = ext(diffusion.posterior_mean_coef1) * x0.detach() + ext(diffusion.posterior_mean_coef2) * x_t
    return {"mse": mse, "eps": eps, "x_t": x_t, "pred_x_start": x0, "model_mean": mean}


def wasserstein_distance_1d(xs, ys, eps=1e-12):
    """trainer.py:310-322: the 2-Wasserstein distance between the Gaussians fitted to xs and ys
    (unbiased variances), floored at sqrt(eps)."""
    assert xs.dim() == 1 and ys.dim() == 1, "must be 1-dimensional"
    mu1, var1, mu2, var2 = xs.mean(), xs.var(), ys.mean(), ys.var()
    dist_quad = (mu1 - mu2) ** 2 + (var1 + var2 - 2 * th.sqrt(var1.sqrt() * var2 * var1.sqrt()))
    if th.any(th.isnan(dist_quad)):
        raise ValueError("[Error] Nan value in loss")
    return th.maximum(dist_quad, th.zeros_like(dist_quad).fill_(eps)).sqrt()


SPEED_LOSSES = ("speed_loss", "speed_l1_loss", "speed_constraint_loss")


def speed_losses(x_start, pred_x_start, loss_params):
    """The extra loss terms of Trainer._compute_loss (trainer.py:172-196) on (N, C, T) poses:
    {term name: loss}, and their weighted sum.  An unknown name raises ValueError, as there."""
    terms, total = {}, 0.0
    for name, weight in (loss_params or {}).items():
        if name == "speed_constraint_loss":
            loss = th.abs(th.diff(pred_x_start, dim=2)).mean()
            terms["speed_constraint"] = loss
        elif name in ("speed_loss", "speed_l1_loss"):
            speed = th.abs(th.diff(x_start, dim=2)).mean([0, 1])            # (T-1,)
            speed_pred = th.abs(th.diff(pred_x_start, dim=2)).mean([0, 1])  # (T-1,)
            if name == "speed_loss":
                loss = wasserstein_distance_1d(speed, speed_pred)
                terms["speed"] = loss
            else:
                loss = F.smooth_l1_loss(speed_pred, speed)
                terms["speed_l1"] = loss
        else:
            raise ValueError(f"Unsupported loss: {name}")
        total = total + weight * loss
    return terms, total


# ------------------------------------------------------------------------------------------
# optimizer, schedules, sampler
# ------------------------------------------------------------------------------------------
class AdamW:
    """torch.optim.AdamW (betas 0.9 / 0.999, eps 1e-8, model_creation.py:176-178) over the flat
    parameter buffer: ONE HIP launch per step."""

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        self.model = model
        self.lr, self.betas, self.eps = float(lr), betas, float(eps)
        self.weight_decay = 0.0 if weight_decay is None else float(weight_decay)
        self.param_groups = [{"lr": self.lr, "initial_lr": self.lr}]
        self.exp_avg = th.zeros_like(model.flat)
        self.exp_avg_sq = th.zeros_like(model.flat)
        self.step_count = 0

    def zero_grad(self):
        self.model.zero_grad()

    def step(self, grad_scale=1.0):
        self.step_count += 1
        f = self.model.flat
        _ok(_lib().ggd_tr_adamw(f.numel(), _p(f), _p(self.model.flat_grad), _p(self.exp_avg), _p(self.exp_avg_sq),
                                float(self.param_groups[0]["lr"]), self.betas[0], self.betas[1], self.eps,
                                self.weight_decay, self.step_count, float(grad_scale), _s(f)), "adamw")

    def _views(self, flat):
        """(index, view of `flat`) per parameter, in the model's parameter order (the reference
        module tree's model.parameters() order: its state_dict order without the buffers)."""
        off = 0
        for i, p in enumerate(self.model.params.values()):
            n = p.numel()
            yield i, flat[off:off + n].view(p.shape)
            off += n

    def state_dict(self):
        """torch.optim.AdamW's layout ({'state': {i: {step, exp_avg, exp_avg_sq}}, 'param_groups'}),
        so the reference Trainer (trainer.py:203, 218) and this one read each other's checkpoints."""
        state = {}
        if self.step_count > 0:
            sq = dict(self._views(self.exp_avg_sq))
            for i, m in self._views(self.exp_avg):
                state[i] = {"step": th.tensor(float(self.step_count)), "exp_avg": m.clone(), "exp_avg_sq": sq[i].clone()}
        g = dict(self.param_groups[0])
        g.update({"betas": tuple(self.betas), "eps": self.eps, "weight_decay": self.weight_decay, "amsgrad": False,
                  "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
                  "params": list(range(len(self.model.params)))})
        return {"state": state, "param_groups": [g]}

    def load_state_dict(self, st):
        """torch.optim's layout (above), or this class's round-2 flat layout {step, exp_avg, exp_avg_sq}."""
        if "state" in st:
            n = len(self.model.params)
            if len(st["param_groups"]) != 1 or len(st["param_groups"][0]["params"]) != n:
                raise ValueError("optimizer state: expected one parameter group over %d parameters" % n)
            order = st["param_groups"][0]["params"]
            state = st["state"]
            self.step_count = 0
            with th.no_grad():
                for i, (j, m) in zip(order, self._views(self.exp_avg)):
                    s = state.get(i)
                    if s is None:
                        m.zero_()
                        continue
                    m.copy_(s["exp_avg"].reshape(m.shape))
                    self.step_count = int(float(s["step"]))
                for i, (j, v) in zip(order, self._views(self.exp_avg_sq)):
                    s = state.get(i)
                    v.copy_(s["exp_avg_sq"].reshape(v.shape)) if s is not None else v.zero_()
        else:
            self.step_count = int(st["step"])
            self.exp_avg.copy_(st["exp_avg"])
            self.exp_avg_sq.copy_(st["exp_avg_sq"])
        g = st["param_groups"][0]
        self.param_groups = [{"lr": float(g["lr"]), "initial_lr": float(g.get("initial_lr", g["lr"]))}]
        # torch.optim.Optimizer.load_state_dict (trainer.py:218) restores every group hyperparameter
        if "betas" in g:
            self.betas = tuple(float(b) for b in g["betas"])
        if "eps" in g:
            self.eps = float(g["eps"])
        if "weight_decay" in g:
            self.weight_decay = float(g["weight_decay"])


def parse_steps(s):
    """utils/string_parser.py parse_steps, as written: base * (number of 'k') * 1000, e.g. '4k' -> 4000,
    '200k' -> 200000, '100kk' -> 200000 (the reference's code, not its docstring)."""
    s = str(s)
    nk = s.count("k")
    base = int(s.strip("k"))
    return base if nk == 0 else base * nk * 1000


class LRScheduler:
    """lr_scheduler.py: ConstantLR ('const'), NoamLR ('noamxf'), NoamDecayLR ('noam'), with
    _LRScheduler's step counting (last_epoch starts at 0 and get_lr runs at construction)."""

    def __init__(self, optimizer, params=None):
        self.opt = optimizer
        self.type = (params or {}).get("type", "const")
        if self.type not in ("const", "noam", "noamxf"):
            raise ValueError("Unsupport lr_scheduler type.")
        self.warmup = float(parse_steps(params["warmup_steps"])) if self.type != "const" else 0.0
        self.d_model = float(params["d_model"]) if self.type == "noamxf" else 0.0
        self.base_lr = optimizer.param_groups[0]["initial_lr"]
        self.last_epoch = 0
        self._apply()

    def get_lr(self):
        if self.type == "const":
            return self.base_lr
        if self.type == "noamxf":
            cur = self.last_epoch + 1
            return self.base_lr * self.d_model ** -0.5 * min(cur ** -0.5, cur * self.warmup ** -1.5)
        # NoamDecayLR as create_lr_scheduler builds it (model_creation.py:23): no `minimum` floor
        last = max(1, self.last_epoch)
        return self.base_lr * self.warmup ** 0.5 * min(last ** -0.5, last * self.warmup ** -1.5)

    def _apply(self):
        self.opt.param_groups[0]["lr"] = self.get_lr()

    def step(self):
        self.last_epoch += 1
        self._apply()

    def get_last_lr(self):
        return [self.opt.param_groups[0]["lr"]]

    def state_dict(self):
        return {"last_epoch": self.last_epoch}

    def load_state_dict(self, st):
        self.last_epoch = int(st["last_epoch"])
        self._apply()


class UniformSampler:
    """resample.py:60-68 + ScheduleSampler.sample (:37-58): uniform t, unit weights."""

    def __init__(self, diffusion):
        self.num_timesteps = diffusion.num_timesteps

    def sample(self, batch_size, device, rng=np.random):
        idx = rng.choice(self.num_timesteps, size=(batch_size,))
        return th.from_numpy(idx).long().to(device), th.ones(batch_size, device=device)


# ------------------------------------------------------------------------------------------
# gradient all-reduce (DDP in kind) and the train step
# ------------------------------------------------------------------------------------------
BUCKET_ELEMS = 8 << 20   # 32 MiB of f32 per all-reduce: a handful of large collectives over xGMI


def allreduce_gradients(flat_grad, group=None):
    """Average the flat gradient over the ranks of `group` (DDP's averaging, trainer.py:83):
    bucketed all_reduce (RCCL over xGMI on GPUs, gloo on CPU)."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return flat_grad
    world = dist.get_world_size(group)
    if world == 1:
        return flat_grad
    for o in range(0, flat_grad.numel(), BUCKET_ELEMS):
        b = flat_grad[o:o + BUCKET_ELEMS]
        dist.all_reduce(b, group=group)
    flat_grad.div_(world)
    return flat_grad


def _dist_world(group=None):
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return 1
    return dist.get_world_size(group)


def broadcast_parameters(model, src=0, group=None):
    """DDP's construction-time synchronisation (DistributedDataParallel(model), trainer.py:83):
    every rank takes rank `src`'s parameters and buffers.  The parameters are ONE flat buffer
    (model.flat), so that is bucketed broadcasts of it, then one per buffer (BN statistics)."""
    import torch.distributed as dist
    if _dist_world(group) == 1:
        return model
    with th.no_grad():
        for o in range(0, model.flat.numel(), BUCKET_ELEMS):
            dist.broadcast(model.flat[o:o + BUCKET_ELEMS], src, group=group)
        broadcast_buffers(model, src, group)
    return model


def broadcast_buffers(model, src=0, group=None):
    """DDP's per-forward buffer broadcast (broadcast_buffers=True, its default): the BatchNorm
    running statistics of rank `src` overwrite every other rank's before the forward."""
    import torch.distributed as dist
    if _dist_world(group) == 1:
        return model
    bufs = getattr(model, "buffers", {}) or {}
    with th.no_grad():
        for k in sorted(bufs):
            dist.broadcast(bufs[k], src, group=group)
    if bufs and hasattr(model, "_encoder"):
        model._encoder = None
    return model


def grad_norm(model):
    """compute_grad_norm (trainer.py:341-349): the 2-norm of all gradients (HIP reduction)."""
    g = model.flat_grad
    lib = _lib()
    part = g.new_empty(lib.ggd_tr_sumsq_blocks())
    out = g.new_empty(1)
    _ok(lib.ggd_tr_sumsq(g.numel(), _p(g), _p(part), _p(out), _s(g)), "sumsq")
    return float(out.item()) ** 0.5


class Trainer:
    """The reference Trainer's step (trainer.py:131-248) on one rank.  With world > 1 (the caller
    initialises torch.distributed, backend 'nccl' = RCCL on ROCm) it behaves as the reference's
    DDP wrapper (trainer.py:83): rank 0's parameters and buffers are broadcast at construction,
    its BN buffers again before every forward, and gradients are averaged by allreduce_gradients."""

    def __init__(self, model, diffusion, speech_encoder, lr=1e-3, weight_decay=None, scheduler_params=None,
                 grad_norm_clip_value=None, grad_clip_value=None, loss_params=None, seed=0):
        for name in (loss_params or {}):
            if name not in SPEED_LOSSES:
                raise ValueError(f"Unsupported loss: {name}")
        self.loss_params = dict(loss_params or {})
        broadcast_parameters(model)
        self.model = model
        self.diffusion = diffusion
        self.encoder = speech_encoder if speech_encoder is not None else (lambda wav: model.speech_encoder()(wav))
        self.optimizer = AdamW(model, lr=lr, weight_decay=weight_decay)
        self.lr_scheduler = LRScheduler(self.optimizer, scheduler_params)
        self.schedule_sampler = UniformSampler(diffusion)
        self.grad_norm_clip_value = grad_norm_clip_value
        self.grad_clip_value = grad_clip_value
        self.rng = np.random.RandomState(seed)
        self.train_step = 0

    def _compute_loss(self, batch, noise=None, t=None):
        poses = batch["pose"].to(self.model.device)          # (N, T, C)
        z = batch.get("speech_tokens")
        kw = {"speech_tokens": z}
        if z is None and self.model.train_encoder:
            kw = {"wav": batch["wav"]}                       # encoded with grad (train-mode SE-ResNet)
        elif z is None:
            kw = {"speech_tokens": self.encoder(batch["wav"])}   # frozen HA2G encoder (eval mode)
        if self.model.arch["type"] == "inpaint":
            # trainer.py:139-146: the seed poses (the clip's first pose_seed_len frames) and their mask
            inpaint_poses = poses.clone()
            inpaint_masks = th.ones_like(inpaint_poses)[:, :, 0:1]          # (N, T, 1)
            inpaint_masks[:, self.model.pose_seed_len:] = 0
            kw["inpaint_pose"] = inpaint_poses.transpose(0, 1)              # (T, N, C)
            kw["inpaint_mask"] = inpaint_masks.transpose(0, 1)              # (T, N, 1)
        x_start = poses.transpose(1, 2)
        if noise is None:
            noise = th.randn_like(x_start)
        if t is None:
            t, _ = self.schedule_sampler.sample(poses.shape[0], self.model.device, self.rng)
        out = training_losses(self.diffusion, self.model, x_start, t, kw, noise=noise)
        denoise = out["mse"].mean()
        terms, extra = speed_losses(x_start, out["pred_x_start"], self.loss_params)
        return {"loss": denoise + extra, "denoise": denoise, **terms}

    def step(self, batch, noise=None, t=None):
        """zero_grad -> (buffer broadcast) -> loss -> backward -> all-reduce -> grad norm ->
        clip_grad_norm_ -> clip_grad_value_ -> AdamW -> lr step."""
        self.model.train()
        self.optimizer.zero_grad()
        broadcast_buffers(self.model)
        terms = self._compute_loss(batch, noise=noise, t=t)
        with direct_grad_accumulation():
            terms["loss"].backward()
        allreduce_gradients(self.model.flat_grad)
        gn = grad_norm(self.model)
        scale = 1.0
        if self.grad_norm_clip_value is not None:   # clip_grad_norm_: coef = max_norm / (norm + 1e-6), <= 1
            scale = min(1.0, float(self.grad_norm_clip_value) / (gn + 1e-6))
        if self.grad_clip_value is not None:        # clip_grad_value_ on the clipped gradients, in place
            g = self.model.flat_grad
            _ok(_lib().ggd_tr_scale_clamp(g.numel(), _p(g), float(scale), float(self.grad_clip_value), _s(g)),
                "clip_grad_value_")
            scale = 1.0
        self.optimizer.step(grad_scale=scale)
        self.lr_scheduler.step()
        self.train_step += 1
        return {"loss": float(terms["loss"].item()), "grad_norm": gn, "lr": self.lr_scheduler.get_last_lr()[0]}

    # -- checkpoints in the reference's dict layout (trainer.py:200-224) ------------------------
    def checkpoint(self):
        return {"model_state_dict": self.model.state_dict(), "optimizer_state_dict": self.optimizer.state_dict(),
                "lr_scheduler_state_dict": self.lr_scheduler.state_dict(), "train_step": self.train_step}

    def load_checkpoint(self, ck):
        self.model.load_state_dict(ck["model_state_dict"])
        self.optimizer.load_state_dict(ck["optimizer_state_dict"])
        self.lr_scheduler.load_state_dict(ck["lr_scheduler_state_dict"])
        self.train_step = int(ck["train_step"])
