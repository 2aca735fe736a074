"""Generator: the reference's inference driver (models/generator.py) over the HIP sampler."""
import time
from typing import Tuple

import numpy as np
import torch as th

from .diffusion import InpaintDenoise


class Generator:
    def __init__(self, model, diffusion):
        self.model = model
        self.diffusion = diffusion

    def _choose_sample_func(self, sample_alg):
        """generator.py:34-45."""
        if sample_alg == "ddim":
            return self.diffusion.ddim_sample_loop
        if sample_alg == "ddpm":
            return self.diffusion.p_sample_loop
        raise ValueError(f"Unsupported sample algorithm: {sample_alg}")

    @th.no_grad()
    def gpu_warm_up_ddim(self, shape, model_kwargs, device, num_iteration=10):
        """generator.py:17-32."""
        for _ in range(num_iteration):
            self.diffusion.ddim_sample_loop(self.model, shape, model_kwargs=model_kwargs, device=device)

    @th.no_grad()
    def eval_infer_time_ddim(self, shape, model_kwargs, sample_alg="ddim", repetitions=10, device="cuda"):
        """generator.py:47-78: 10 warm-up loops, then ``repetitions`` timed loops -> (mean_ms, std_ms)."""
        sample_func = self._choose_sample_func(sample_alg)
        start = th.cuda.Event(enable_timing=True)
        end = th.cuda.Event(enable_timing=True)
        timings = np.zeros((repetitions, 1))
        self.gpu_warm_up_ddim(shape, model_kwargs, device)
        for rep in range(repetitions):
            start.record()
            sample_func(self.model, shape, model_kwargs=model_kwargs, device=device, progress=False)
            end.record()
            th.cuda.synchronize()
            timings[rep] = start.elapsed_time(end)
        return np.sum(timings) / repetitions, np.std(timings)

    @th.no_grad()
    def eval_bpd(self, poses, wavs, pose_seed_len=None, noise=None, seed=None):
        """generator.py:197-216: the variational bound of poses (N, T, C) given wavs (N, T_wav),
        diffusion.calc_bpd_loop on x_start = poses^T; the inpaint model conditions on the first
        pose_seed_len frames."""
        poses = poses.to(self.model.device, th.float32)
        model_kwargs = {"wav": wavs.to(self.model.device, th.float32)}
        if getattr(self.model, "arch", {}).get("type") == "inpaint":
            assert pose_seed_len is not None, "Provide pose_seed_len for inpaint model."
            masks = th.ones_like(poses)[:, :, :1]
            masks[:, pose_seed_len:] = 0
            model_kwargs["inpaint_pose"] = poses.clone().transpose(0, 1)
            model_kwargs["inpaint_mask"] = masks.transpose(0, 1)
        return self.diffusion.calc_bpd_loop(self.model, poses.transpose(1, 2), model_kwargs, noise=noise, seed=seed)

    @th.no_grad()
    def generate_sample(self, shape: Tuple[int], wavs: th.Tensor, noise: th.Tensor = None,
                        inpaint_poses: th.Tensor = None, inpaint_masks: th.Tensor = None,
                        sample_alg: str = "ddim", trans_factor: float = None, pose_seed_len: int = None,
                        return_dtype: str = "tensor", device: str = "cuda", progress: bool = True,
                        check_status: bool = True, **kw):
        """generator.py:218-296 -> (N, L, C).  The sampling loop is issued non-blocking; with
        check_status (default) the model's contexts are synced before the result is returned, so
        a persistent loop that failed on the device raises here instead of handing back x_T."""
        wavs = wavs.to(device)
        if inpaint_poses is not None:
            assert inpaint_masks is not None, "Provide inpaint_masks."
            inpaint_poses = inpaint_poses.to(device)
            inpaint_masks = inpaint_masks.to(device)
        assert len(wavs.shape) == 2, f"Wav dim should be (N,T). Got: {wavs.shape}"
        assert len(shape) == 3, f"Shape should be (N,C,T). Got: {shape}"
        sample_func = self._choose_sample_func(sample_alg)
        denoise_fn = None
        if inpaint_poses is not None:
            L = shape[2]
            if trans_factor is not None:
                assert 0 <= trans_factor <= 1
                assert pose_seed_len is not None, "Provide pose_seed_len when using trans_factor."
                ramp = th.arange(trans_factor, 1, (1 - trans_factor) / pose_seed_len, device=device)
                trans = th.cat([ramp, th.ones(L - ramp.numel(), device=device)])
            else:
                trans = th.zeros(L, device=device)
            denoise_fn = InpaintDenoise(inpaint_poses, inpaint_masks, trans)
        model_kwargs = {"wav": wavs}
        if self.model.arch["type"] == "inpaint":  # generator.py:244-249
            assert inpaint_poses is not None and len(inpaint_poses.shape) == 3
            assert len(inpaint_masks.shape) == 3 and inpaint_masks.size()[:2] == inpaint_poses.size()[:2]
            model_kwargs["inpaint_pose"] = inpaint_poses.transpose(0, 1)  # -> (T, N, C)
            model_kwargs["inpaint_mask"] = inpaint_masks.transpose(0, 1)  # -> (T, N, 1)
        out = sample_func(self.model, shape, noise=noise, denoise_fn=denoise_fn, model_kwargs=model_kwargs,
                          device=device, progress=progress, **kw)
        sample = out["sample"].transpose(1, 2)
        if check_status:
            self._check_status()
        return self.tensor2dtype(sample, return_dtype)

    def _check_status(self):
        """model.sync(): wait for the sampling contexts and raise the error of any loop that failed
        after its non-blocking ggd_sample returned (status words, ggd_sync)."""
        sync = getattr(self.model, "sync", None)
        if sync is not None:
            sync()

    @th.no_grad()
    def generate_batches(self, shape: Tuple[int], wav_batches, sample_alg: str = "ddim",
                         device: str = "cuda", **kw):
        """generate_sample over independent clip batches, back to back -> list of (N, L, C).

        Serving form of generator.py:218-296 for a queue of batches: batch k+1's speech encoder
        is issued on a side HIP stream (model.prefetch_speech) once batch k's speech memory is
        installed, so it runs beside batch k's reverse loop; outputs equal per-batch
        generate_sample calls.
        """
        wav_batches = [w.to(device) for w in wav_batches]
        outs = []
        for k, wav in enumerate(wav_batches):
            nxt = wav_batches[k + 1] if k + 1 < len(wav_batches) else None
            shp = (wav.shape[0],) + tuple(shape[1:])
            outs.append(self.generate_sample(shp, wav, sample_alg=sample_alg, device=device, progress=False,
                                             prefetch_wav=nxt, check_status=False, **kw))
        self._check_status()     # once, after every batch is issued (a failed loop raises here)
        return outs

    @th.no_grad()
    def generate_sequence(self, wav_seqs, wav_sr, pose_dim, pose_fps, pose_window_len, pose_seed_len,
                          return_dtype="tensor", smooth_trans=True, trans_factor=None, init_poses=None,
                          sample_alg="ddim", batch_size=64, device="cuda", progress=True, **kw):
        """generator.py:80-195: windowed autoregressive generation of whole sequences.

        Windows of ``pose_window_len`` frames advance by (window - seed) frames; each window's
        first ``pose_seed_len`` frames are inpainted from the previous window's tail.
        """
        assert len(wav_seqs.shape) == 2, "Provide batch dimension"
        if init_poses is not None:
            assert len(init_poses.shape) == 3, "Provide batch dimension"
            assert len(init_poses) == len(wav_seqs), "Init pose batch size does not meet wav_seqs."
            init_poses = init_poses.to(device)
        wav_seqs = wav_seqs.to(device)
        num_seq, wav_seq_len = wav_seqs.shape
        seq_len = wav_seq_len // wav_sr * pose_fps
        stride = pose_window_len - pose_seed_len
        num_div = int(np.ceil(seq_len / stride))
        if (seq_len - pose_seed_len) % stride == 0:
            num_div -= 1
        wav_win = int(wav_sr * pose_window_len / pose_fps)
        outs = []
        for b0 in range(0, num_seq, batch_size):
            wav_seq = wav_seqs[b0:b0 + batch_size]
            n = len(wav_seq)
            ws, we, ps = 0, wav_win, 0
            samples, sample, inpaint_poses = [], None, None
            for idx in range(num_div):
                wavs = wav_seq[:, ws:we]
                masks = th.ones((n, pose_window_len, 1), device=device)
                masks[:, pose_seed_len:] = 0
                if idx == 0:
                    if init_poses is None:
                        inpaint_poses = masks = None
                    else:
                        inpaint_poses = th.zeros((n, pose_window_len, pose_dim), device=device)
                        inpaint_poses[:, :pose_seed_len] = init_poses[b0:b0 + batch_size]
                else:
                    if inpaint_poses is None:
                        inpaint_poses = th.zeros((n, pose_window_len, pose_dim), device=device)
                    inpaint_poses[:, :pose_seed_len] = sample[:, -pose_seed_len:]
                if we > wav_seq_len:
                    wavs = th.cat([wavs, th.zeros((n, we - wav_seq_len), device=device)], dim=1)
                sample = self.generate_sample((n, pose_dim, pose_window_len), wavs, inpaint_poses=inpaint_poses,
                                              inpaint_masks=masks, sample_alg=sample_alg, trans_factor=trans_factor,
                                              pose_seed_len=pose_seed_len, device=device, progress=progress,
                                              check_status=False, **kw)
                samples.append(sample)
                ws = int(ps / pose_fps * wav_sr)
                we = ws + wav_win
                ps += stride
            parts = []
            for i, x in enumerate(samples):
                if smooth_trans and i > 0:
                    ratio = th.arange(0, 1, 1 / pose_seed_len, device=device)[:pose_seed_len].view(1, -1, 1)
                    tr = x[:, :pose_seed_len] * ratio + samples[i - 1][:, -pose_seed_len:] * (1 - ratio)
                    x = th.cat([tr, x[:, pose_seed_len:]], dim=1)
                parts.append(x[:, :-pose_seed_len] if i < len(samples) - 1 else x)
            outs.append(th.cat(parts, dim=1)[:, :seq_len])
        self._check_status()
        return self.tensor2dtype(th.cat(outs, dim=0), return_dtype)

    @staticmethod
    def tensor2dtype(x, dtype):
        """generator.py:298-309."""
        if dtype == "tensor":
            return x
        if dtype == "cpu_tensor":
            return x.cpu()
        if dtype == "array":
            return x.cpu().numpy()
        raise ValueError(f"Unsupported dtype: {dtype}")
