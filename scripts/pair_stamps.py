"""Step-phase stamps of the per-clip loops (psk_kernel, one workgroup or a clip pair per clip) at the
C5 shape: workgroup 0's s_memtime at the PSTAMP points of iteration 0 (emb, SA/CA of the last layer,
all layers, step end), in microseconds from the step start."""
import os as _os
_os.environ["GGD_DIAG"] = "1"  # ggd_diag lives in libggd_diag.so only (native.py)
import ctypes
import os
import sys

import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
native = __import__(ge.PKG_NAME + ".native", fromlist=["x"])
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
NL = int(next((a.split("=")[1] for a in sys.argv[1:] if a.startswith("layers=")), 4))  # layers=N
if NL != 4:
    cfg.Model.Decoder["n_layers"] = NL
model, _, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
diffusion = pkg.create_diffusion(dict(cfg.Model.Diffusion.to_dict(), timestep_respacing="ddim50"), False)
B = int(next((a for a in sys.argv[1:] if a.isdigit()), 128))
wav = th.randn(B, 32000, device="cuda") * 0.1
ctx, _ = model.prepare(wav, 40)


def diag(what, vals, n_out=17):
    arr = (ctypes.c_int32 * len(vals))(*vals)
    res = (ctypes.c_double * n_out)()
    native.check(ctx.h, ctx.lib.ggd_diag(ctx.h, what, arr, len(vals), 1, ctypes.cast(res, ctypes.c_void_p)), "diag")
    return list(res)


names = ["emb", "L3 SA", "L3 CA", "layers", "step"]
# slots 6 .. 16 inside the last layer (ggd_persist.hip LSTAMP): after LN1, the SA out-projection's
# MFMAs and its partial exchange, LN2, the CA query GEMM, the CA out-projection + residual, LN3,
# the FFN chunks, the FFN partial exchange, the CA out-projection's MFMAs and its exchange
lnames = ["ln1", "sa-oproj", "sa-sum", "ln2", "caq", "ca-res", "ln3", "ffn", "ffsum", "ca-oproj", "ca-sum"]
for label, pair in (("clip pair", 2),) if NL != 4 else (("one workgroup per clip", 1), ("clip pair", 2)):
    diag(7, [0])            # the per-clip loops
    diag(14, [pair, 0])
    for rep in range(3):
        diag(8, [1])
        diffusion.ddim_sample_loop(model, (B, 123, 40), model_kwargs={"wav": wav}, seed=1, n_steps=3, extras=False)
        t = diag(8, [2])
        print(f"{label:24s} rep {rep}: " + "  ".join(f"{n} {t[i]:7.2f}" for i, n in enumerate(names)), flush=True)
        print(" " * 24 + "    last layer: " + "  ".join(f"{n} {t[5 + i]:7.2f}" for i, n in enumerate(lnames)), flush=True)
diag(14, [0, 0])
diag(7, [2])
