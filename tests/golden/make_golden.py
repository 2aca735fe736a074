"""Generate tests/golden/beat_c2_small.npz: golden vectors of the CPU oracle for the C2 model.

The reference cannot be run here (environment denial) and ships no fixtures, so
these vectors pin the ORACLE (this repo's fp32 restatement) against drift; the GPU parity tests
also compare the HIP path with them.  Inputs are fully determined by seeds:
  weights  init_state_dict(beat-ours arch, seed 0, perturb=True)  (torch CPU generator)
  wav      N(0, 0.1^2), torch.Generator seed 1, (2, 32000)
  x, t     N(0, 1) (2, 123, 40) from the same generator; t = [999, 417]
  noise    counter stream (oracle/philox.py), seed 3, global clips [0, 1]

Run:  python tests/golden/make_golden.py   (about 10 s on 8 cores)
"""
import os
import sys

import numpy as np
import torch as th

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402
from oracle import philox, ref_denoiser, ref_diffusion  # noqa: E402

OUT = os.path.join(HERE, "beat_c2_small.npz")
D_POSE, L, N = 123, 40, 2


def inputs():
    g = th.Generator().manual_seed(1)
    wav = th.randn(N, 32000, generator=g) * 0.1
    x = th.randn(N, D_POSE, L, generator=g)
    t = th.tensor([999, 417])
    return wav, x, t


def build(pkg):
    cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
    arch = pkg.arch_from_config(cfg.Model, D_POSE)
    sd = pkg.init_state_dict(arch, seed=0, perturb=True)
    om = ref_denoiser.OracleModel(sd, {k: arch[k] for k in ("type", "d_model", "decoder", "heads", "n_layers")},
                                  cache_speech=True)
    return arch, sd, om


def compute(om):
    wav, x, t = inputs()
    out = {"wav_head": wav[:, :256].numpy(), "x": x.numpy(), "t": t.numpy()}
    with th.no_grad():
        out["eps"] = om(x, t, wav=wav).numpy()
        sch = ref_diffusion.make_schedule("linear", 1000, "")
        for alg in ("ddpm", "ddim"):
            noise = ref_diffusion.PhiloxNoise(3, [0, 1])
            r = ref_diffusion.sample_loop(sch, om, (N, D_POSE, L), {"wav": wav}, noise, alg, n_steps=5)
            out[f"{alg}5_sample"] = r["sample"].numpy()
            out[f"{alg}5_pred_x_start"] = r["pred_x_start"].numpy()
    out["noise_xT_clip5"] = philox.clip_noise(3, [5], 0, philox.TAG_XT, D_POSE, L)[0, :4].copy()
    out["noise_step7_clips01"] = philox.clip_noise(3, [0, 1], 7, philox.TAG_STEP, D_POSE, L)[:, :2].copy()
    sch = ref_diffusion.make_schedule("linear", 1000, "")
    out["sched_coef1"] = np.asarray(sch.posterior_mean_coef1[[0, 1, 500, 999]])
    out["sched_logvar"] = np.asarray(sch.posterior_log_variance_clipped[[0, 1, 500, 999]])
    return out


if __name__ == "__main__":
    th.set_num_threads(min(8, os.cpu_count() or 1))
    pkg = ge.load_package()
    _, _, om = build(pkg)
    res = compute(om)
    np.savez_compressed(OUT, **{k: np.asarray(v) for k, v in res.items()})
    print("wrote", OUT, {k: np.asarray(v).shape for k, v in res.items()})
