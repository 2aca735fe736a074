"""Per-phase time inside the persistent clip-group loop: body vs clip-group barrier (GPU box).

    python3 scripts/mega_stamps.py [layers=N]

The bf16 clip-group loop, the row-block decomposition (ggd_rows.hip mr_kernel; round 6 removed the
bf16 head / chunk loop).  layers=N: a decoder of N layers (same weights' first N layers)."""
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
dev = th.device("cuda:0")
HEADS = False
NL = int(next((a.split("=")[1] for a in sys.argv[1:] if a.startswith("layers=")), 4))
if NL != 4:
    cfg.Model.Decoder["n_layers"] = NL
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device=dev)
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
wav = th.randn(32, 32000, device=dev) * 0.1
ctx, _ = model.prepare(wav, 40)
print(f"{'head / chunk loop (mk_kernel)' if HEADS else 'row-block loop (mr_kernel)'}, {NL} layers", flush=True)


def diag(what, p, n_out=1):
    arr = (ctypes.c_int32 * len(p))(*p)
    out = (ctypes.c_double * max(n_out, 1))()
    native.check(ctx.h, ctx.lib.ggd_diag(ctx.h, what, arr, len(p), 1, ctypes.cast(out, ctypes.c_void_p)), "diag")
    return list(out)


diffusion.p_sample_loop(model, (32, 123, 40), model_kwargs={"wav": wav}, seed=1, extras=False, n_steps=5)
# bf16 loop: KA KB KC per layer (the FFN-down reduction runs inside the next phase) + KE
# (round 4: the last layer's KD runs inside KE's rows phase -- 16 barriers per step)
names = [f"L{li}{ph}" for li in range(NL) for ph in ("ABCD" if li < NL - 1 else "ABC")] + ["E"]
NB = len(names)
for rep in range(3):
    diag(10, [1])
    diffusion.p_sample_loop(model, (32, 123, 40), model_kwargs={"wav": wav}, seed=1, extras=False, n_steps=5)
    t = diag(10, [2], 2 * 17 * 2)
    for step in range(2):
        base = step * 2 * NB
        prev = t[base - 1] if step else 0.0
        cells = []
        tb = tw = 0.0
        for i, nm in enumerate(names):
            done, passed = t[base + 2 * i], t[base + 2 * i + 1]
            body, wait = done - prev, passed - done
            tb += body
            tw += wait
            cells.append(f"{nm} {body:5.2f}+{wait:4.2f}")
            prev = passed
        print(f"rep {rep} step {step}: body {tb:6.1f} us, barrier {tw:5.1f} us | " + "  ".join(cells), flush=True)
diag(10, [0])

# inside the phases of layer 1 (workgroup 0, last step) and KE
diag(11, [1])
diffusion.p_sample_loop(model, (32, 123, 40), model_kwargs={"wav": wav}, seed=1, extras=False, n_steps=3)
t = diag(11, [2], 80)
labels = {0: "KA ln|qkv+conv|-|attn", 1: "KB load|oproj|ln2|q+conv|fix|attn", 2: "KC load|oproj|ln3|ffn1|ffn2",
          3: "KD sum|-|store", 4: "KE ln+out|stage|upd"} if HEADS else \
    {0: "KA stage|qkv+conv|attn", 1: "KB stage|sa-oproj|ln2+fix|q+conv+ca|ca-oproj+ln3", 2: "KC stage|ffn1|ffn2",
     3: "KD sum+ln1", 4: "KE loads|sum|ln|eps|upd|emb+ln1"}
for j in range(5):
    v = [round(x, 2) for x in t[16 * j + 1:16 * j + 8] if x >= 0]
    print(f"{labels[j]:40s} {v}", flush=True)
diag(11, [0])
