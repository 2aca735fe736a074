"""HIP-backed denoiser with the reference model protocol.

Drop-in for ``Speech2GestureModel`` / ``Speech2GestureModelV2`` (models/model.py:19-117):

    eps = model(x_t (N, C, L) f32, t (N,) int64 original timesteps, wav=(N, T_wav))

Behind the call: the speech encoder (encoder.py) runs once per distinct ``wav``
tensor and its memory is installed in the libggd context; the decoder forward
(step token, emb + PE, n_layers x {self-attn, cross-attn, FFN}, out projection)
runs as hand-written gfx950 kernels through ``ggd_denoise``.  There is no CPU
or eager-PyTorch fallback for the decoder.
"""
import ctypes
import weakref

import numpy as np
import torch as th

from . import native
from .encoder import SpeechEncoder, speech_len
from .weights import arch_from_config, parameter_shapes

# "fp8": bf16 activations, OCP e4m3 per-step decoder weights with per-channel scales (GGD_FP8W)
_DTYPES = {"bf16": native.BF16, "f32": native.F32, "fp32": native.F32, "fp8": native.FP8W}


_LIVE = weakref.WeakSet()   # every open context (sync_all)


def sync_all():
    """ggd_sync on every open context: waits for their streams and raises the error of any
    persistent loop that failed after a non-blocking ggd_sample returned."""
    for c in list(_LIVE):
        c.sync()


class _Ctx:
    """One libggd context (fixed L, Ts, max_batch)."""

    def __init__(self, lib, device_index, desc, sd):
        self.lib = lib
        self.desc = desc
        self.h = ctypes.c_void_p()
        rc = lib.ggd_create(device_index, ctypes.byref(desc), ctypes.byref(self.h))
        if rc != 0:
            msg = lib.ggd_last_error(self.h).decode() if self.h else "ggd_create failed"
            lib.ggd_destroy(self.h)
            self.h = None
            if rc == native.GGD_ERR_UNSUPPORTED:
                raise ValueError(msg)
            raise native.GgdError(msg)
        for name, v in sd.items():
            if not v.is_floating_point():
                continue
            a = v.detach().to("cpu", th.float32).contiguous()
            native.check(self.h, lib.ggd_load_weight(self.h, name.encode(), ctypes.c_void_p(a.data_ptr()),
                                                     a.numel()), f"load {name}")
        native.check(self.h, lib.ggd_finalize_weights(self.h), "finalize weights")
        self.schedule_key = None
        self.memory_key = None
        _LIVE.add(self)

    def sync(self):
        """Wait for the context's work; raise if an earlier non-blocking loop failed (ggd_sync)."""
        if self.h:
            native.check(self.h, self.lib.ggd_sync(self.h), "sync")

    def set_schedule(self, betas, timestep_map):
        key = (np.asarray(betas, np.float64).tobytes(), tuple(int(t) for t in timestep_map))
        if key == self.schedule_key:
            return
        b = np.ascontiguousarray(betas, dtype=np.float64)
        tm = np.ascontiguousarray(timestep_map, dtype=np.int64)
        native.check(self.h, self.lib.ggd_set_schedule(self.h, b.ctypes.data, len(b), tm.ctypes.data),
                     "set schedule")
        self.schedule_key = key

    def close(self):
        if self.h:
            self.lib.ggd_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _stream_ptr(device):
    return ctypes.c_void_p(th.cuda.current_stream(device).cuda_stream)


class Speech2GestureModel:
    """HIP sampler model for Model.type in {'s2g_v2', 'default', 'inpaint'} (model_creation.py:133-161)."""

    def __init__(self, d_pose, model_params, dtype="bf16", device="cuda"):
        self.arch = arch_from_config(model_params, d_pose)
        if self.arch["type"] not in ("s2g_v2", "default", "inpaint"):
            raise ValueError(f"Unsupported model_type {self.arch['type']}")
        self.diffusion_steps = int(model_params["Diffusion"]["diffusion_steps"])
        self.dtype = dtype
        self.device = th.device(device)
        self._sd = None
        self._ctx = {}
        self._encoder = None
        self._mem_cache = None
        self._pending = {}      # wav identity -> (speech tokens, ready event) from prefetch_speech
        self._side = None       # HIP stream the prefetched encoder runs on
        self.training = False

    # -- torch.nn.Module-like surface used by the reference callers -------------------------
    def to(self, device):
        device = th.device(device)
        if device.type != "cuda":
            raise ValueError("the HIP sampler runs on a GPU device only (no CPU fallback)")
        if device != self.device:
            self._release()
            self.device = device
        return self

    def eval(self):
        self.training = False
        return self

    def train(self, mode=True):
        if mode:
            raise ValueError("the HIP sampler model is inference-only: train through "
                             "create_model(..., is_training=True) -> training.TrainableModel")
        return self

    def state_dict(self):
        return dict(self._sd) if self._sd is not None else {}

    def sync(self):
        """Wait for this model's contexts; raise if a non-blocking sampling loop failed (ggd_sync)."""
        for c in list(self._ctx.values()):
            c.sync()

    def load_state_dict(self, sd, strict=True):
        """Accepts the reference's model_state_dict (models/model.py module tree key names)."""
        want = parameter_shapes(self.arch)
        missing = [k for k in want if k not in sd]
        unexpected = [k for k in sd if k not in want]
        if strict and (missing or unexpected):
            raise RuntimeError(f"Error(s) in loading state_dict: missing {missing[:5]}, unexpected {unexpected[:5]}")
        for k, (shape, _) in want.items():
            if k in sd and tuple(sd[k].shape) != tuple(shape):
                raise RuntimeError(f"size mismatch for {k}: {tuple(sd[k].shape)} vs {tuple(shape)}")
        self._sd = {k: v.detach().cpu() for k, v in sd.items()}
        self._release()
        return missing, unexpected

    def parameters(self):
        for v in (self._sd or {}).values():
            if v.is_floating_point():
                yield v

    # -- internals --------------------------------------------------------------------------
    def _release(self):
        for c in self._ctx.values():
            c.close()
        self._ctx = {}
        self._encoder = None
        self._mem_cache = None
        self._pending = {}

    def encoder(self):
        if self._encoder is None:
            if self._sd is None:
                raise RuntimeError("load_state_dict() before use")
            self._encoder = SpeechEncoder(self._sd, self.device, dtype=self.dtype, d_model=self.arch["d_model"])
        return self._encoder

    def context(self, L, Ts, n):
        key = (L, Ts)
        c = self._ctx.get(key)
        if c is not None and c.desc.max_batch >= n:
            return c
        if c is not None:
            c.close()
        if self._sd is None:
            raise RuntimeError("load_state_dict() before use")
        a = self.arch
        desc = native.Desc(
            model_type={"s2g_v2": native.MODEL_S2G_V2, "default": native.MODEL_DEFAULT,
                        "inpaint": native.MODEL_INPAINT}[a["type"]],
            decoder_type=native.DEC_ONEWAY if a["decoder"] == "oneway_cross_attention" else native.DEC_TWOWAY,
            d_model=a["d_model"], heads=a["heads"], n_layers=a["n_layers"], d_pose=a["d_pose"],
            seq_len=L, speech_len=Ts, max_batch=max(n, 1), dtype=_DTYPES[self.dtype],
            diffusion_steps=self.diffusion_steps)
        with th.cuda.device(self.device):
            c = _Ctx(native.load(), self.device.index or 0, desc, self._sd)
        self._ctx[key] = c
        return c

    @staticmethod
    def _wav_key(wav):
        return (wav.data_ptr(), tuple(wav.shape), wav._version)

    def prefetch_speech(self, wav):
        """Start the speech encoder for a LATER sampling call's batch on a side HIP stream.

        The encoder (4.8 GFLOP per clip) and a reverse loop whose workgroups do not fill the
        chip (psk: one workgroup per clip) can then run at once: issue ``prefetch_speech(wav_next)``
        before the current batch's loop; the call that later samples ``wav_next`` waits on the
        encoder's event instead of encoding again.  The side stream starts after the work
        already queued on the current stream (so ``wav`` is complete), never the other way round.
        Pass the same device tensor to both calls: a host tensor is copied anew by each call and
        is not recognised (it is then encoded again; at most 8 unconsumed prefetches are kept).
        """
        wav = wav.to(self.device, th.float32)
        if self._side is None:
            self._side = th.cuda.Stream(self.device)
        cur = th.cuda.current_stream(self.device)
        self._side.wait_stream(cur)
        with th.cuda.stream(self._side):
            tok = self.encoder().memory(wav, self.arch["type"])
            ev = th.cuda.Event()
            ev.record(self._side)
        wav.record_stream(self._side)
        # the entry holds ``wav`` itself: while it is pending, no other tensor can be allocated at
        # its address, so a key match always means the same tensor (not a reused block)
        self._pending[self._wav_key(wav)] = (tok, ev, wav)
        while len(self._pending) > 8:  # prefetched but never sampled (e.g. a host wav copied twice)
            self._pending.pop(next(iter(self._pending)))

    def prepare(self, wav, L):
        """Encode ``wav`` once (cached per device tensor identity/version) and install the memory.

        The cache key is the device tensor's address, shape and version; the cache entry keeps
        that tensor alive, so while it is cached no other tensor can be allocated at the same
        address and a key match means the same, unmodified tensor.  A host ``wav`` is copied to
        the device by each call, so each call encodes it afresh (a per-step caller passes the
        device copy; GaussianSpacedDiffusion._loop does).
        """
        wav = wav.to(self.device, th.float32)
        n = wav.shape[0]
        Ts = speech_len(self.arch["type"], wav.shape[1])
        ctx = self.context(L, Ts, n)
        key = (wav.data_ptr(), tuple(wav.shape), wav._version, L, id(ctx))
        if self._mem_cache is not None and self._mem_cache[0] == key and ctx.memory_key == key:
            return ctx, n
        pending = self._pending.pop(self._wav_key(wav), None)
        if pending is not None:  # encoded by prefetch_speech on the side stream
            tok, ev, _ = pending
            cur = th.cuda.current_stream(self.device)
            cur.wait_event(ev)
            tok.record_stream(cur)
        else:
            if self._side is not None:  # the encoder's buffers may still be in use by a prefetch
                th.cuda.current_stream(self.device).wait_stream(self._side)
            tok = self.encoder().memory(wav, self.arch["type"])
        assert tok.shape[1] == Ts, (tok.shape, Ts)
        native.check(ctx.h, ctx.lib.ggd_set_memory(ctx.h, ctypes.c_void_p(tok.data_ptr()), n, Ts, tok.shape[2],
                                                   _stream_ptr(self.device)), "set memory")
        ctx.memory_key = key
        self._mem_cache = (key, tok, wav)  # tok: alive until the ctx has consumed it; wav: pins the key
        return ctx, n

    def condition(self, ctx, n, L, inpaint_pose=None, inpaint_mask=None):
        """Speech2GestureModelInpaint (models/model.py:152-166): install proj([pose*mask, mask]) for the
        next calls.  inpaint_pose (L, N, C), inpaint_mask (L, N, 1) as the reference's model_kwargs."""
        if self.arch["type"] != "inpaint":
            if inpaint_pose is not None or inpaint_mask is not None:
                raise ValueError(f"unsupported model kwargs ['inpaint_mask', 'inpaint_pose'] for type {self.arch['type']}")
            return
        if inpaint_pose is None or inpaint_mask is None:
            raise TypeError("Speech2GestureModelInpaint.myforward() needs inpaint_pose and inpaint_mask")
        C = self.arch["d_pose"]
        assert tuple(inpaint_pose.shape) == (L, n, C), f"inpaint_pose must be (L, N, C), got {tuple(inpaint_pose.shape)}"
        assert tuple(inpaint_mask.shape) == (L, n, 1), f"inpaint_mask must be (L, N, 1), got {tuple(inpaint_mask.shape)}"
        pose = inpaint_pose.to(self.device, th.float32).transpose(0, 1).contiguous()
        mask = inpaint_mask.to(self.device, th.float32).reshape(L, n).transpose(0, 1).contiguous()
        native.check(ctx.h, ctx.lib.ggd_set_inpaint(ctx.h, ctypes.c_void_p(pose.data_ptr()),
                                                    ctypes.c_void_p(mask.data_ptr()), n, _stream_ptr(self.device)),
                     "set inpaint")

    @th.no_grad()
    def __call__(self, x_t, t, wav=None, inpaint_pose=None, inpaint_mask=None, **kwargs):
        """eps = model(x_t, t, wav=...[, inpaint_pose, inpaint_mask])  (models/model.py:12-15, 152-166)."""
        if kwargs:
            raise ValueError(f"unsupported model kwargs {sorted(kwargs)}")
        assert wav is not None and wav.dim() == 2, "wav (N, T) is required"
        assert x_t.dim() == 3 and x_t.shape[1] == self.arch["d_pose"], f"x_t must be (N, C, L), got {tuple(x_t.shape)}"
        N, C, L = x_t.shape
        assert t.shape == (N,), f"t must be (N,), got {tuple(t.shape)}"
        ctx, n = self.prepare(wav, L)
        assert n == N, "wav batch differs from x_t batch"
        self.condition(ctx, n, L, inpaint_pose, inpaint_mask)
        x = x_t.to(self.device, th.float32).contiguous()
        tt = t.to(self.device, th.int32).contiguous()
        if int(tt.min()) < 0 or int(tt.max()) >= self.diffusion_steps:
            raise AssertionError("timestep out of range")
        eps = th.empty_like(x)
        native.check(ctx.h, ctx.lib.ggd_denoise(ctx.h, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(tt.data_ptr()),
                                                ctypes.c_void_p(eps.data_ptr()), N, _stream_ptr(self.device)),
                     "denoise")
        return eps
