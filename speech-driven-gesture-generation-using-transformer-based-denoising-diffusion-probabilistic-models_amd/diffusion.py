"""Gaussian diffusion sampler API, driving the fused HIP reverse loop.

Mirrors models/modules/gaussian_diffusion.py and respace.py:
  get_named_beta_schedule (:20-40), space_timesteps (respace.py:13-68),
  GaussianSpacedDiffusion(use_timesteps, betas, model_var_type) (respace.py:71-101),
  p_sample_loop (:331-366), ddim_sample_loop (:414-441).
The host keeps the fp64 schedule tables (needed for the API and for the C ABI);
the loop itself -- T' x (denoiser + posterior update) -- runs inside libggd as one
hipGraph replay per step (ggd_sample).

Noise: the reference draws th.randn for x_T and th.randn_like every step
(gaussian_diffusion.py:392,326,474).  Here ``noise`` (x_T) and ``step_noise``
((T', N, C, L), loop order) may be supplied; otherwise both come from the
counter-based stream keyed by (seed, global clip id, step) so multi-GPU runs are
bit-identical to single-GPU runs.
"""
import ctypes
import enum
import math

import numpy as np
import torch as th

from . import native


def get_named_beta_schedule(schedule_name, num_diffusion_timesteps):
    """gaussian_diffusion.py:20-40."""
    if schedule_name == "linear":
        scale = 1000 / num_diffusion_timesteps
        return np.linspace(scale * 0.0001, scale * 0.02, num_diffusion_timesteps, dtype=np.float64)
    if schedule_name == "squaredcos_cap_v2":
        f = lambda u: math.cos(u * math.pi / 2) ** 2
        return np.array([min(1 - f((i + 1) / num_diffusion_timesteps) / f(i / num_diffusion_timesteps), 0.999)
                         for i in range(num_diffusion_timesteps)])
    raise NotImplementedError(f"unknown beta schedule: {schedule_name}")


def space_timesteps(num_timesteps, section_counts):
    """respace.py:13-68 ("ddimN", "fast27", "path:<npy>", comma-separated section counts)."""
    if isinstance(section_counts, str):
        if section_counts.startswith("path:"):
            return set(int(s) for s in np.load(section_counts[len("path:"):], allow_pickle=False))
        if section_counts.startswith("ddim"):
            want = int(section_counts[len("ddim"):])
            for stride in range(1, num_timesteps):
                if len(range(0, num_timesteps, stride)) == want:
                    return set(range(0, num_timesteps, stride))
            raise ValueError(f"cannot create exactly {num_timesteps} steps with an integer stride")
        if section_counts == "fast27":
            steps = space_timesteps(num_timesteps, "10,10,3,2,2")
            steps.remove(num_timesteps - 1)
            steps.add(num_timesteps - 3)
            return steps
        section_counts = [int(x) for x in section_counts.split(",")]
    per, extra = divmod(num_timesteps, len(section_counts))
    start, steps = 0, []
    for i, count in enumerate(section_counts):
        size = per + (1 if i < extra else 0)
        if size < count:
            raise ValueError(f"cannot divide section of {size} steps into {count}")
        stride = 1 if count <= 1 else (size - 1) / (count - 1)
        cur = 0.0
        for _ in range(count):
            steps.append(start + round(cur))
            cur += stride
        start += size
    return set(steps)


class ModelVarType(enum.Enum):
    FIXED_SMALL = enum.auto()


class GaussianDiffusion:
    """Schedule tables of gaussian_diffusion.py:87-143 (fp64)."""

    def __init__(self, *, betas, model_var_type):
        if model_var_type != "fixed_small":
            raise ValueError(f"Unsupported model_var_type {model_var_type}")
        self.model_var_type = ModelVarType.FIXED_SMALL
        betas = np.array(betas, dtype=np.float64)
        assert betas.ndim == 1, "betas must be 1-D"
        assert (betas > 0).all() and (betas <= 1).all()
        self.betas = betas
        self.num_timesteps = int(betas.shape[0])
        self.alphas = 1.0 - betas
        self.alphas_cumprod = np.cumprod(self.alphas, axis=0)
        self.alphas_cumprod_prev = np.append(1.0, self.alphas_cumprod[:-1])
        self.alphas_cumprod_next = np.append(self.alphas_cumprod[1:], 0.0)
        self.sqrt_alphas_cumprod = np.sqrt(self.alphas_cumprod)
        self.sqrt_one_minus_alphas_cumprod = np.sqrt(1.0 - self.alphas_cumprod)
        self.log_one_minus_alphas_cumprod = np.log(1.0 - self.alphas_cumprod)
        self.sqrt_recip_alphas_cumprod = np.sqrt(1.0 / self.alphas_cumprod)
        self.sqrt_recipm1_alphas_cumprod = np.sqrt(1.0 / self.alphas_cumprod - 1.0)
        self.posterior_variance = betas * (1.0 - self.alphas_cumprod_prev) / (1.0 - self.alphas_cumprod)
        self.posterior_log_variance_clipped = np.log(np.append(self.posterior_variance[1], self.posterior_variance[1:]))
        self.posterior_mean_coef1 = betas * np.sqrt(self.alphas_cumprod_prev) / (1.0 - self.alphas_cumprod)
        self.posterior_mean_coef2 = (1.0 - self.alphas_cumprod_prev) * np.sqrt(self.alphas) / (1.0 - self.alphas_cumprod)
        self.timestep_map = list(range(self.num_timesteps))


class InpaintDenoise:
    """The generator's x0-replacement ``denoise_fn`` (generator.py:272-281) as data, so the fused
    HIP loop can apply it in its update epilogue.  Calling it evaluates the same formula."""

    def __init__(self, poses, masks, trans):
        self.poses = poses        # (N, L, C)
        self.masks = masks        # (N, L, 1)
        self.trans = trans        # (L,) f32 ramp (zeros when trans_factor is None)

    def __call__(self, x0):
        t = self.trans.view(1, -1, 1)
        y = x0.transpose(1, 2)
        y = (1 - t) * self.masks * self.poses + t * self.masks * y + (1 - self.masks) * y
        return y.transpose(1, 2)


_EXTRA_KEYS = ("mean", "variance", "log_variance", "eps", "pred_x_start", "raw_x_start")


class GaussianSpacedDiffusion(GaussianDiffusion):
    """respace.py:71-101: keeps the steps in ``use_timesteps``; the model sees original t."""

    def __init__(self, use_timesteps, **kwargs):
        self.use_timesteps = set(use_timesteps)
        self.original_num_steps = len(kwargs["betas"])
        base = GaussianDiffusion(**kwargs)
        last, new_betas, tmap = 1.0, [], []
        for i, ac in enumerate(base.alphas_cumprod):
            if i in self.use_timesteps:
                new_betas.append(1 - ac / last)
                last = ac
                tmap.append(i)
        kwargs["betas"] = np.array(new_betas)
        super().__init__(**kwargs)
        self.timestep_map = tmap

    # ------------------------------------------------------------------ sampling loops
    def p_sample_loop(self, model, shape, model_kwargs, noise=None, denoise_fn=None, device=None,
                      progress=False, **kw):
        """gaussian_diffusion.py:331-366 -> final step dict (incl. 'sample')."""
        return self._loop(native.DDPM, 0.0, model, shape, model_kwargs, noise, denoise_fn, device, **kw)

    def ddim_sample_loop(self, model, shape, noise=None, denoise_fn=None, model_kwargs=None, device=None,
                         progress=False, eta=0.0, **kw):
        """gaussian_diffusion.py:414-441 -> final step dict (incl. 'sample')."""
        return self._loop(native.DDIM, float(eta), model, shape, model_kwargs, noise, denoise_fn, device, **kw)

    def _loop(self, alg, eta, model, shape, model_kwargs, noise, denoise_fn, device, step_noise=None,
              seed=None, clip_offset=0, n_steps=None, use_graph=False, extras=True, prefetch_wav=None, sync=False):
        """sync=False (default): returns once the loop is issued on the device, like any PyTorch GPU
        op; a persistent loop's status words are checked by the next call or model.sync() / .sync_all().
        sync=True blocks, checks, and re-runs a loop that could not be co-resident on a route that
        needs no co-residency."""
        assert isinstance(shape, (tuple, list)) and len(shape) == 3, "shape must be (N, C, L)"
        model_kwargs = dict(model_kwargs or {})
        wav = model_kwargs.pop("wav", None)
        inp_pose, inp_mask = model_kwargs.pop("inpaint_pose", None), model_kwargs.pop("inpaint_mask", None)
        if model_kwargs:
            raise ValueError(f"unsupported model kwargs {sorted(model_kwargs)}")
        N, C, L = (int(s) for s in shape)
        dev = th.device(device) if device is not None else model.device
        if wav is not None:  # one device copy for the whole loop (the per-step path re-keys on it)
            wav = wav.to(model.device, th.float32)
        ctx, n = model.prepare(wav, L)
        assert n == N, "wav batch differs from shape[0]"
        model.condition(ctx, n, L, inp_pose, inp_mask)
        if prefetch_wav is not None:
            # the next batch's speech encoder starts once this batch's memory is installed and
            # runs beside this loop (Speech2GestureModel.prefetch_speech)
            model.prefetch_speech(prefetch_wav)
        ctx.set_schedule(self.betas, self.timestep_map)
        if seed is None:
            seed = int(th.randint(0, 2 ** 62, (1,)).item())
        x_T = None
        if noise is not None:
            assert tuple(noise.shape) == (N, C, L)
            x_T = noise.to(dev, th.float32).contiguous()
        T = self.num_timesteps
        steps = T if not n_steps else min(int(n_steps), T)
        zs = None
        if step_noise is not None:
            assert tuple(step_noise.shape[1:]) == (N, C, L) and step_noise.shape[0] >= steps
            zs = step_noise.to(dev, th.float32).contiguous()
        if denoise_fn is not None and not isinstance(denoise_fn, InpaintDenoise):
            return self._loop_per_step(alg, eta, model, ctx, wav, N, C, L, x_T, zs, denoise_fn, steps, dev, seed)
        inp_p = inp_m = trans = None
        if denoise_fn is not None:
            inp_p = denoise_fn.poses.to(dev, th.float32).contiguous()
            inp_m = denoise_fn.masks.to(dev, th.float32).reshape(N, L).contiguous()
            trans = denoise_fn.trans.to(dev, th.float32).reshape(L).contiguous()
        out = th.empty((N, C, L), device=dev, dtype=th.float32)
        ext = th.empty((6, N, C, L), device=dev, dtype=th.float32) if extras else None
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        a = native.SampleArgs(alg=alg, eta=eta, n=N, x_T=ptr(x_T), noise=ptr(zs), seed=seed,
                              clip_offset=int(clip_offset), inpaint_poses=ptr(inp_p), inpaint_masks=ptr(inp_m),
                              trans=ptr(trans), out=ptr(out), extras=ptr(ext), n_steps=steps,
                              use_graph=1 if use_graph else 0, sync=1 if sync else 0)
        native.check(ctx.h, ctx.lib.ggd_sample(ctx.h, ctypes.byref(a),
                                               ctypes.c_void_p(th.cuda.current_stream(dev).cuda_stream)), "sample")
        res = {"sample": out}
        if ext is not None:
            res.update({k: ext[i] for i, k in enumerate(_EXTRA_KEYS)})
        return res

    def _loop_per_step(self, alg, eta, model, ctx, wav, N, C, L, x_T, zs, denoise_fn, steps, dev, seed):
        """Arbitrary Python ``denoise_fn``: model + posterior kernels per step, the callable between them."""
        g = th.Generator(device=dev).manual_seed(seed)
        x = x_T if x_T is not None else th.randn((N, C, L), device=dev, generator=g)
        stream = lambda: ctypes.c_void_p(th.cuda.current_stream(dev).cuda_stream)
        out = None
        for k, i in enumerate(list(range(self.num_timesteps))[::-1][:steps]):
            t = th.full((N,), self.timestep_map[i], dtype=th.long, device=dev)
            eps = model(x, t, wav=wav)
            raw = th.empty_like(x)
            z = zs[k] if zs is not None else th.randn((N, C, L), device=dev, generator=g)
            native.check(ctx.h, ctx.lib.ggd_posterior_step(ctx.h, alg, eta, i, ctypes.c_void_p(x.data_ptr()),
                                                            ctypes.c_void_p(eps.data_ptr()), None,
                                                            ctypes.c_void_p(z.data_ptr()), None,
                                                            ctypes.c_void_p(raw.data_ptr()), N, stream()), "posterior")
            x0 = denoise_fn(raw.clone()).contiguous()
            xn = th.empty_like(x)
            native.check(ctx.h, ctx.lib.ggd_posterior_step(ctx.h, alg, eta, i, ctypes.c_void_p(x.data_ptr()),
                                                            ctypes.c_void_p(eps.data_ptr()), ctypes.c_void_p(x0.data_ptr()),
                                                            ctypes.c_void_p(z.data_ptr()), ctypes.c_void_p(xn.data_ptr()),
                                                            None, N, stream()), "posterior")
            var = float(self.posterior_variance[i])
            logv = float(self.posterior_log_variance_clipped[i])
            mean = (th.tensor(self.posterior_mean_coef1[i]).float() * x0
                    + th.tensor(self.posterior_mean_coef2[i]).float() * x)
            out = {"sample": xn, "mean": mean, "variance": th.full_like(x, var), "log_variance": th.full_like(x, logv),
                   "eps": eps, "pred_x_start": x0, "raw_x_start": raw}
            x = xn
        return out

    # ------------------------------------------------------------------ variational bound
    def _ext(self, arr, i, like):
        """_extract_into_tensor (gaussian_diffusion.py:681-694): fp64 table value -> f32 per clip."""
        return th.tensor(float(arr[i]), dtype=th.float32, device=like.device)

    def calc_bpd_loop(self, model, x_start, model_kwargs, noise=None, seed=None):
        """gaussian_diffusion.py:624-678 (bits per dim over every kept step t = T' - 1 .. 0, with the
        _vb_terms_bpd terms of :575-606 and the prior term of :608-622).  The model runs on the HIP
        denoiser (one ggd_denoise per t for the whole batch); the per-t noise is noise[k] for the
        k-th iteration when given ((T', N, C, L)), else drawn on the device in loop order."""
        x_start = x_start.float()
        dev = x_start.device
        N = x_start.shape[0]
        dims = list(range(1, x_start.dim()))
        g = th.Generator(device=dev).manual_seed(seed if seed is not None else 0) if noise is None else None
        log2 = math.log(2.0)
        vb, xmse, mse = [], [], []
        for k, i in enumerate(list(range(self.num_timesteps))[::-1]):
            z = noise[k].to(dev).float() if noise is not None else th.randn(x_start.shape, device=dev, generator=g)
            x_t = self._ext(self.sqrt_alphas_cumprod, i, x_start) * x_start + \
                self._ext(self.sqrt_one_minus_alphas_cumprod, i, x_start) * z
            t = th.full((N,), self.timestep_map[i], dtype=th.long, device=dev)
            eps = model(x_t, t, **model_kwargs).float()
            x0 = self._ext(self.sqrt_recip_alphas_cumprod, i, x_start) * x_t - \
                self._ext(self.sqrt_recipm1_alphas_cumprod, i, x_start) * eps
            c1, c2 = self._ext(self.posterior_mean_coef1, i, x_start), self._ext(self.posterior_mean_coef2, i, x_start)
            model_mean = c1 * x0 + c2 * x_t
            true_mean = c1 * x_start + c2 * x_t
            logv = self._ext(self.posterior_log_variance_clipped, i, x_start)
            if i == 0:   # decoder NLL: -log N(x_0; model mean, exp(logv)) (losses.py)
                c = (x_start - model_mean) * th.exp(-0.5 * logv)
                term = -((-c ** 2 / 2) - math.log(math.sqrt(2 * math.pi)))
            else:        # KL(q(x_{t-1} | x_t, x_0) || p(x_{t-1} | x_t)), equal fixed variances
                term = 0.5 * (-1.0 + logv - logv + th.exp(logv - logv) + (true_mean - model_mean) ** 2 * th.exp(-logv))
            vb.append(term.mean(dim=dims) / log2)
            xmse.append(((x0 - x_start) ** 2).mean(dim=dims))
            e2 = (self._ext(self.sqrt_recip_alphas_cumprod, i, x_start) * x_t - x0) / \
                self._ext(self.sqrt_recipm1_alphas_cumprod, i, x_start)
            mse.append(((e2 - z) ** 2).mean(dim=dims))
        vb, xmse, mse = th.stack(vb, 1), th.stack(xmse, 1), th.stack(mse, 1)
        last = self.num_timesteps - 1
        qm = self._ext(self.sqrt_alphas_cumprod, last, x_start) * x_start
        qlv = self._ext(self.log_one_minus_alphas_cumprod, last, x_start)
        prior = (0.5 * (-1.0 - qlv + th.exp(qlv) + qm ** 2)).mean(dim=dims) / log2
        return {"total_bpd": vb.sum(dim=1) + prior, "prior_bpd": prior, "vb": vb, "x_start_mse": xmse, "mse": mse}

