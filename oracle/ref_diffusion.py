"""Oracle: CPU restatement of the reference diffusion sampler and generator.

Test infrastructure only (see oracle/__init__.py).  Restates
  models/modules/gaussian_diffusion.py:20-143,207-329,331-529,681-694
  models/modules/respace.py:13-113
  models/generator.py:218-296 (generate_sample) and :80-195 (generate_sequence)
fp64 numpy schedule tables, fp32 torch tensor math, exactly the reference's
operation order (the HIP update kernel is checked bit-for-bit against it).
"""
import math

import numpy as np
import torch as th

from . import philox


# ----------------------------------------------------------------------------
# schedules
# ----------------------------------------------------------------------------

def named_betas(name, T):
    """get_named_beta_schedule: gaussian_diffusion.py:20-40 (+ betas_for_alpha_bar :43-60)."""
    if name == "linear":
        s = 1000 / T
        return np.linspace(s * 0.0001, s * 0.02, T, dtype=np.float64)
    if name == "squaredcos_cap_v2":
        f = lambda u: np.cos(u * np.pi / 2) ** 2
        return np.array([min(1 - f((i + 1) / T) / f(i / T), 0.999) for i in range(T)])
    raise NotImplementedError(name)


def spaced_steps(T, spec):
    """space_timesteps: respace.py:13-68 ('ddimN', 'fast27', 'a,b,c'; path: unsupported here)."""
    if isinstance(spec, str):
        if spec.startswith("ddim"):
            want = int(spec[4:])
            for stride in range(1, T):
                if len(range(0, T, stride)) == want:
                    return set(range(0, T, stride))
            raise ValueError(f"cannot create exactly {T} steps with an integer stride")
        if spec == "fast27":
            s = spaced_steps(T, "10,10,3,2,2")
            s.remove(T - 1)
            s.add(T - 3)
            return s
        spec = [int(v) for v in spec.split(",")]
    per, extra = divmod(T, len(spec))
    out, start = [], 0
    for i, cnt in enumerate(spec):
        size = per + (1 if i < extra else 0)
        if size < cnt:
            raise ValueError(f"cannot divide section of {size} steps into {cnt}")
        stride = 1 if cnt <= 1 else (size - 1) / (cnt - 1)
        cur = 0.0
        for _ in range(cnt):
            out.append(start + round(cur))
            cur += stride
        start += size
    return set(out)


class Schedule:
    """GaussianDiffusion.__init__ tables (gaussian_diffusion.py:87-143) on respaced betas (respace.py:80-93)."""

    def __init__(self, betas, use_timesteps=None):
        betas = np.asarray(betas, dtype=np.float64)
        if use_timesteps is not None:
            base_ac = np.cumprod(1.0 - betas)
            last, nb, tmap = 1.0, [], []
            for i, ac in enumerate(base_ac):
                if i in use_timesteps:
                    nb.append(1 - ac / last)
                    last = ac
                    tmap.append(i)
            betas = np.array(nb)
            self.timestep_map = tmap
        else:
            self.timestep_map = list(range(len(betas)))
        self.betas = betas
        self.num_timesteps = len(betas)
        a = 1.0 - betas
        self.alphas_cumprod = np.cumprod(a)
        self.alphas_cumprod_prev = np.append(1.0, self.alphas_cumprod[:-1])
        self.sqrt_recip_alphas_cumprod = np.sqrt(1.0 / self.alphas_cumprod)
        self.sqrt_recipm1_alphas_cumprod = np.sqrt(1.0 / self.alphas_cumprod - 1.0)
        self.posterior_variance = betas * (1.0 - self.alphas_cumprod_prev) / (1.0 - self.alphas_cumprod)
        self.posterior_log_variance_clipped = np.log(
            np.append(self.posterior_variance[1], self.posterior_variance[1:]))
        self.posterior_mean_coef1 = betas * np.sqrt(self.alphas_cumprod_prev) / (1.0 - self.alphas_cumprod)
        self.posterior_mean_coef2 = (1.0 - self.alphas_cumprod_prev) * np.sqrt(a) / (1.0 - self.alphas_cumprod)


def make_schedule(noise_schedule="linear", diffusion_steps=1000, respacing=""):
    """create_diffusion: models/model_creation.py:30-48 (respacing only at inference)."""
    betas = named_betas(noise_schedule, diffusion_steps)
    spec = respacing if respacing else [diffusion_steps]
    return Schedule(betas, spaced_steps(diffusion_steps, spec))


def _ext(arr, i, shape):
    """_extract_into_tensor: gaussian_diffusion.py:681-694 (fp64 table -> fp32, broadcast)."""
    v = th.from_numpy(np.asarray(arr))[i].float()
    while v.dim() < len(shape):
        v = v[..., None]
    return v + th.zeros(shape)


# ----------------------------------------------------------------------------
# noise providers
# ----------------------------------------------------------------------------

class TorchNoise:
    """Faithful reference order: x_T = th.randn(shape), then randn_like each step."""

    def __init__(self, seed):
        self.g = th.Generator().manual_seed(seed)

    def initial(self, shape):
        return th.randn(shape, generator=self.g)

    def step(self, i, shape):
        return th.randn(shape, generator=self.g)


class PhiloxNoise:
    """Counter-based stream keyed by global clip id (oracle/philox.py), as the HIP sampler draws it."""

    def __init__(self, seed, clip_ids):
        self.seed, self.clips = seed, np.asarray(clip_ids)

    def initial(self, shape):
        return th.from_numpy(philox.clip_noise(self.seed, self.clips, 0, philox.TAG_XT, shape[1], shape[2]))

    def step(self, i, shape):
        return th.from_numpy(philox.clip_noise(self.seed, self.clips, i, philox.TAG_STEP, shape[1], shape[2]))


class InjectedNoise:
    """Per-step noise supplied as a (T', N, C, L) tensor indexed by loop iteration."""

    def __init__(self, x_T, steps):
        self.x_T, self.steps, self.k = x_T, steps, 0

    def initial(self, shape):
        return self.x_T

    def step(self, i, shape):
        z = self.steps[self.k]
        self.k += 1
        return z


# ----------------------------------------------------------------------------
# reverse loops
# ----------------------------------------------------------------------------

def p_mean_variance(sch, model, x, i, model_kwargs, denoise_fn=None):
    """p_mean_variance: gaussian_diffusion.py:234-285 through _WrappedModel (respace.py:110-113)."""
    n = x.shape[0]
    it = th.full((n,), i, dtype=th.long)
    t_orig = th.tensor(sch.timestep_map, dtype=th.long)[it]
    eps = model(x, t_orig, **model_kwargs)
    var = _ext(sch.posterior_variance, it, x.shape)
    logvar = _ext(sch.posterior_log_variance_clipped, it, x.shape)
    # _predict_xstart_from_eps: :287-292
    x0 = _ext(sch.sqrt_recip_alphas_cumprod, it, x.shape) * x - _ext(sch.sqrt_recipm1_alphas_cumprod, it, x.shape) * eps
    raw = x0.clone()
    if denoise_fn is not None:
        x0 = denoise_fn(x0)
    # q_posterior_mean_variance: :207-232
    mean = _ext(sch.posterior_mean_coef1, it, x.shape) * x0 + _ext(sch.posterior_mean_coef2, it, x.shape) * x
    return {"mean": mean, "variance": var, "log_variance": logvar, "eps": eps,
            "pred_x_start": x0, "raw_x_start": raw}


def p_sample(sch, model, x, i, model_kwargs, noise, denoise_fn=None):
    """p_sample: gaussian_diffusion.py:300-329."""
    out = p_mean_variance(sch, model, x, i, model_kwargs, denoise_fn)
    z = noise.step(i, x.shape)
    nz = float(i != 0)
    out["sample"] = out["mean"] + nz * th.exp(0.5 * out["log_variance"]) * z
    return out


def ddim_sample(sch, model, x, i, model_kwargs, noise, denoise_fn=None, eta=0.0):
    """ddim_sample: gaussian_diffusion.py:443-484 (noise drawn even at eta = 0, :474)."""
    out = p_mean_variance(sch, model, x, i, model_kwargs, denoise_fn)
    n = x.shape[0]
    it = th.full((n,), i, dtype=th.long)
    # _predict_eps_from_xstart: :294-298
    eps = (_ext(sch.sqrt_recip_alphas_cumprod, it, x.shape) * x - out["pred_x_start"]) \
        / _ext(sch.sqrt_recipm1_alphas_cumprod, it, x.shape)
    ab = _ext(sch.alphas_cumprod, it, x.shape)
    abp = _ext(sch.alphas_cumprod_prev, it, x.shape)
    sigma = eta * th.sqrt((1 - abp) / (1 - ab)) * th.sqrt(1 - ab / abp)
    z = noise.step(i, x.shape)
    mean_pred = out["pred_x_start"] * th.sqrt(abp) + th.sqrt(1 - abp - sigma ** 2) * eps
    nz = float(i != 0)
    out["sample"] = mean_pred + nz * sigma * z
    return out


def sample_loop(sch, model, shape, model_kwargs, noise, alg="ddpm", denoise_fn=None, eta=0.0,
                x_T=None, n_steps=None, snapshots=()):
    """p_sample_loop(_progressive) :331-412 / ddim_sample_loop(_progressive) :414-529.

    ``n_steps`` truncates the loop after that many iterations (parity tests at
    reduced cost); the iterations run are exactly the reference's first ones.
    ``snapshots``: iteration counts after which x is recorded in out["snapshots"][k]
    (the drift curve of a long loop from one oracle run).
    """
    x = x_T if x_T is not None else noise.initial(shape)
    out = None
    snaps = {}
    idx = list(range(sch.num_timesteps))[::-1]
    if n_steps is not None:
        idx = idx[:n_steps]
    for k, i in enumerate(idx):
        with th.no_grad():
            if alg == "ddpm":
                out = p_sample(sch, model, x, i, model_kwargs, noise, denoise_fn)
            elif alg == "ddim":
                out = ddim_sample(sch, model, x, i, model_kwargs, noise, denoise_fn, eta)
            else:
                raise ValueError(f"Unsupported sample algorithm: {alg}")
        x = out["sample"]
        if k + 1 in snapshots:
            snaps[k + 1] = x.clone()
    if snapshots:
        out["snapshots"] = snaps
    return out


# ----------------------------------------------------------------------------
# generator (models/generator.py)
# ----------------------------------------------------------------------------

def trans_ramp(trans_factor, pose_seed_len, L):
    """Inpaint x0-replacement ramp: generator.py:258-268 (fp32 arange, then ones to length L)."""
    if trans_factor is None:
        return th.zeros(1, L, 1)
    r = th.arange(trans_factor, 1, (1 - trans_factor) / pose_seed_len)[None, :, None]
    return th.cat([r, th.ones((1, L - r.size(1), 1))], dim=1)


def make_denoise_fn(inpaint_poses, inpaint_masks, trans):
    """denoise_fn: generator.py:272-281.  poses (N,L,C), masks (N,L,1), trans (1,L,1) or scalar 0."""

    def fn(x0):
        y = x0.transpose(1, 2)
        y = (1 - trans) * inpaint_masks * inpaint_poses + trans * inpaint_masks * y + (1 - inpaint_masks) * y
        return y.transpose(1, 2)

    return fn


def generate_sample(sch, model, shape, wavs, noise, inpaint_poses=None, inpaint_masks=None,
                    sample_alg="ddim", trans_factor=None, pose_seed_len=None, x_T=None, n_steps=None):
    """Generator.generate_sample: generator.py:218-296 -> (N, L, C)."""
    denoise_fn = None
    if inpaint_poses is not None:
        if trans_factor is not None:
            trans = trans_ramp(trans_factor, pose_seed_len, shape[2])
        else:
            trans = 0
        denoise_fn = make_denoise_fn(inpaint_poses, inpaint_masks, trans)
    model_kwargs = {"wav": wavs}
    if getattr(model, "cfg", {}).get("type") == "inpaint":  # generator.py:244-249
        model_kwargs["inpaint_pose"] = inpaint_poses.transpose(0, 1)
        model_kwargs["inpaint_mask"] = inpaint_masks.transpose(0, 1)
    out = sample_loop(sch, model, shape, model_kwargs, noise, sample_alg, denoise_fn,
                      x_T=x_T, n_steps=n_steps)
    return out["sample"].transpose(1, 2)


def sequence_plan(n_wav, wav_sr, pose_fps, pose_window_len, pose_seed_len):
    """Window bookkeeping of generate_sequence: generator.py:109-115,128-130,171-174."""
    seq_len = n_wav // wav_sr * pose_fps
    stride = pose_window_len - pose_seed_len
    n_div = int(np.ceil(seq_len / stride))
    if (seq_len - pose_seed_len) % stride == 0:
        n_div -= 1
    win = int(wav_sr * pose_window_len / pose_fps)
    plan, ws, we, ps = [], 0, win, 0
    for _ in range(n_div):
        plan.append((ws, we))
        ws = int(ps / pose_fps * wav_sr)
        we = ws + win
        ps += stride
    return seq_len, plan


def combine_windows(samples, pose_seed_len, seq_len, smooth_trans):
    """Chunk combination with optional linear cross-fade: generator.py:177-191."""
    parts = []
    for i, x in enumerate(samples):
        if smooth_trans and i > 0:
            ratio = th.arange(0, 1, 1 / pose_seed_len)[:pose_seed_len].view(1, -1, 1)
            tr = x[:, :pose_seed_len] * ratio + samples[i - 1][:, -pose_seed_len:] * (1 - ratio)
            x = th.cat([tr, x[:, pose_seed_len:]], dim=1)
        parts.append(x[:, :-pose_seed_len] if i < len(samples) - 1 else x)
    return th.cat(parts, dim=1)[:, :seq_len]


def generate_sequence(sch, model, wav_seqs, wav_sr, pose_dim, pose_fps, pose_window_len, pose_seed_len,
                      make_noise, smooth_trans=True, trans_factor=None, init_poses=None, sample_alg="ddim",
                      n_steps=None):
    """Generator.generate_sequence: generator.py:80-195 for ONE batch (batch_size >= N).

    Window k samples wav[:, ws:we] (zero-padded past the end) with its first ``pose_seed_len``
    frames inpainted from window k-1's tail (window 0: from ``init_poses`` if given, else no
    inpainting); the windows are joined by combine_windows.  ``make_noise(k)`` gives window k's
    noise provider.  Where the reference would crash (init_poses None: ``init_poses.to`` at
    :105 and ``inpaint_poses[...]`` of a None at :148) this follows the evident intent: no
    seed poses for window 0, zeros elsewhere in the seed-pose buffer from window 1 on.
    """
    n, n_wav = wav_seqs.shape
    seq_len, plan = sequence_plan(n_wav, wav_sr, pose_fps, pose_window_len, pose_seed_len)
    samples, sample, inpaint_poses = [], None, None
    for k, (ws, we) in enumerate(plan):
        wavs = wav_seqs[:, ws:we]
        masks = th.ones((n, pose_window_len, 1))
        masks[:, pose_seed_len:] = 0
        if k == 0:
            if init_poses is None:
                inpaint_poses = masks = None
            else:
                inpaint_poses = th.zeros((n, pose_window_len, pose_dim))
                inpaint_poses[:, :pose_seed_len] = init_poses
        else:
            if inpaint_poses is None:
                inpaint_poses = th.zeros((n, pose_window_len, pose_dim))
            inpaint_poses[:, :pose_seed_len] = sample[:, -pose_seed_len:]
        if we > n_wav:
            wavs = th.cat([wavs, th.zeros((n, we - n_wav))], dim=1)
        sample = generate_sample(sch, model, (n, pose_dim, pose_window_len), wavs, make_noise(k),
                                 inpaint_poses, masks, sample_alg, trans_factor, pose_seed_len, n_steps=n_steps)
        samples.append(sample)
    return combine_windows(samples, pose_seed_len, seq_len, smooth_trans)


# ----------------------------------------------------------------------------
# variational bound in bits per dim: gaussian_diffusion.py:571-678 + losses.py
# ----------------------------------------------------------------------------

def normal_kl(mean1, logvar1, mean2, logvar2):
    """losses.py normal_kl."""
    logvar1 = logvar1 if isinstance(logvar1, th.Tensor) else th.tensor(logvar1)
    logvar2 = logvar2 if isinstance(logvar2, th.Tensor) else th.tensor(logvar2)
    return 0.5 * (-1.0 + logvar2 - logvar1 + th.exp(logvar1 - logvar2) + ((mean1 - mean2) ** 2) * th.exp(-logvar2))


def continuous_gaussian_log_likelihood(x, means, log_scales):
    """losses.py continuous_gaussian_log_likelihood (log N(x; mean, exp(log_scale)^2) in nats, no
    -log(scale) term, as the reference writes it)."""
    c = (x - means) * th.exp(-log_scales)
    return (-c ** 2 / 2) - th.log(th.sqrt(2 * th.tensor(math.pi)))


def mean_flat(x):
    return x.mean(dim=list(range(1, x.dim())))


def calc_bpd_loop(sch, model, x_start, model_kwargs, noises):
    """calc_bpd_loop (gaussian_diffusion.py:624-678) with the per-t noise given as noises[k] for the
    k-th iteration (t = T' - 1 - k), in place of th.randn_like."""
    n = x_start.shape[0]
    shape = x_start.shape
    vb, xmse, mse = [], [], []
    for k, i in enumerate(list(range(sch.num_timesteps))[::-1]):
        it = th.full((n,), i, dtype=th.long)
        noise = noises[k]
        ac = np.asarray(sch.alphas_cumprod)
        x_t = _ext(np.sqrt(ac), it, shape) * x_start + _ext(np.sqrt(1.0 - ac), it, shape) * noise
        # _vb_terms_bpd (:575-606)
        true_mean = (_ext(sch.posterior_mean_coef1, it, shape) * x_start
                     + _ext(sch.posterior_mean_coef2, it, shape) * x_t)
        true_logvar = _ext(sch.posterior_log_variance_clipped, it, shape)
        out = p_mean_variance(sch, model, x_t, i, model_kwargs)
        kl = mean_flat(normal_kl(true_mean, true_logvar, out["mean"], out["log_variance"])) / math.log(2.0)
        nll = -continuous_gaussian_log_likelihood(x_start, out["mean"], 0.5 * out["log_variance"])
        nll = mean_flat(nll) / math.log(2.0)
        vb.append(th.where(it == 0, nll, kl))
        xmse.append(mean_flat((out["pred_x_start"] - x_start) ** 2))
        # _predict_eps_from_xstart (:294-298)
        eps = ((_ext(sch.sqrt_recip_alphas_cumprod, it, shape) * x_t - out["pred_x_start"])
               / _ext(sch.sqrt_recipm1_alphas_cumprod, it, shape))
        mse.append(mean_flat((eps - noise) ** 2))
    vb, xmse, mse = th.stack(vb, 1), th.stack(xmse, 1), th.stack(mse, 1)
    # _prior_bpd (:608-622): q(x_T | x_0) against N(0, 1)
    last = th.full((n,), sch.num_timesteps - 1, dtype=th.long)
    ac = np.asarray(sch.alphas_cumprod)
    qm = _ext(np.sqrt(ac), last, shape) * x_start
    qlv = _ext(np.log(1.0 - ac), last, shape)
    prior = mean_flat(normal_kl(qm, qlv, th.zeros(()), th.zeros(()))) / math.log(2.0)
    return {"total_bpd": vb.sum(dim=1) + prior, "prior_bpd": prior, "vb": vb, "x_start_mse": xmse, "mse": mse}
