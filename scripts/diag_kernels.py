"""Per-kernel latency table via ggd_diag (back-to-back launches, hipEvents on the ctx stream)."""
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
dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype=dtype, device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
wav = th.randn(32, 32000, device="cuda:0") * 0.1
ctx, n = model.prepare(wav, 40)
ctx.set_schedule(diffusion.betas, diffusion.timestep_map)
lib = ctx.lib


def stamps(which, n=32):
    arr = (ctypes.c_int32 * 2)(which, n)
    out = (ctypes.c_double * 16)()
    native.check(ctx.h, lib.ggd_diag(ctx.h, 6, arr, 2, 1, ctypes.cast(out, ctypes.c_void_p)), "diag stamps")
    return [round(v, 2) for v in out[:8] if v >= 0]


def diag(what, params, iters=200):
    arr = (ctypes.c_int32 * len(params))(*params)
    out = ctypes.c_double()
    native.check(ctx.h, lib.ggd_diag(ctx.h, what, arr, len(params), iters, ctypes.cast(ctypes.byref(out), ctypes.c_void_p)), "diag")
    return out.value


PRO = {"T": 0, "LN": 1, "F32": 2}
EPI = {"T": 0, "RELU2": 1, "F32": 2, "SILU": 3, "RESID": 4, "PE": 5}
rows = [
    ("qkv LN->T 1280x768x256", "LN", "T", 1280, 768, 256),
    ("ffn1 LN->RELU2 1280x1024x256", "LN", "RELU2", 1280, 1024, 256),
    ("ffn2 T->RESID 1280x256x1024", "T", "RESID", 1280, 256, 1024),
    ("oproj T->RESID 1280x256x256", "T", "RESID", 1280, 256, 256),
    ("qca LN->T 1280x256x256", "LN", "T", 1280, 256, 256),
    ("out LN->F32 1280x128x256", "LN", "F32", 1280, 128, 256),
    ("emb F32->PE 1280x256x256", "F32", "PE", 1280, 256, 256),
    ("T->T 1280x768x256 (bf16 A)", "T", "T", 1280, 768, 256),
    ("T->T 64x64x256 (1 WG)", "T", "T", 64, 64, 256),
    ("LN->T 64x64x256 (1 WG)", "LN", "T", 64, 64, 256),
    ("T->T 1280x64x256", "T", "T", 1280, 64, 256),
    ("T->T 64x768x256", "T", "T", 64, 768, 256),
]
print(f"dtype={dtype}")
for name, pro, epi, M, N, K in rows:
    res = []
    for mt in (32, 64):
        for nox in (0, 1):
            res.append(diag(0, [PRO[pro], EPI[epi], M, N, K, mt, nox]))
    print(f"{name:34s} mt32 xcd {res[0]:7.2f}  mt32 plain {res[1]:7.2f}  mt64 xcd {res[2]:7.2f}  mt64 plain {res[3]:7.2f} us")
for cross in (0, 1):
    for nn in (32, 8, 1):
        print(f"attention cross={cross} n={nn:2d}: {diag(1, [cross, nn]):7.2f} us")
print(f"step eager n=32: {diag(2, [32], 50):8.2f} us")
print(f"step graph n=32: {diag(3, [32], 200):8.2f} us")
print(f"step graph n=8 : {diag(3, [8], 200):8.2f} us")
print(f"step graph n=1 : {diag(3, [1], 200):8.2f} us")
for which, name in enumerate(["KA ln1+qkv+sa", "KB oproj+ln2+q+ca", "KC oproj+ln3+ffn1", "KD ffn2+resid", "KE out+upd+emb"]):
    print(f"fused {name:22s} n=32: {diag(4, [which, 32]):7.2f} us   n=1: {diag(4, [which, 1]):7.2f} us")
for which, name in enumerate(["KA: ln|gemm|conv|attn", "KB: load|oproj|ln2|qgemm+kv|conv|attn", "KC: load|oproj|ln3|ffn1", "KD: load|gemm|reduce", "KE: ln+out|stage|upd|emb"]):
    print(f"phases {name:40s}", stamps(which))
print("--- calibration ---")
print(f"empty launch 1 WG      : {diag(5, [0, 0, 1, 1]):7.2f} us")
print(f"empty launch 256 WG    : {diag(5, [0, 0, 256, 1]):7.2f} us")
print(f"empty launch 2048 WG   : {diag(5, [0, 0, 2048, 1]):7.2f} us")
print(f"shader clock           : {diag(5, [2, 2000000, 1, 1], 3):7.3f} GHz")
n_small = diag(5, [1, 2000, 1, 4], 3)
n_big = diag(5, [1, 2000, 1, 1024], 3)
print(f"dependent load, 4 MiB buffer   : {n_small * 1000 / 2000:7.1f} ns/load")
print(f"dependent load, 1 GiB buffer   : {n_big * 1000 / 2000:7.1f} ns/load")
print(f"bulk 64 KiB x 1 WG    : {diag(5, [3, 0, 1, 64]):7.2f} us")
print(f"bulk 64 KiB x 256 WG  : {diag(5, [3, 0, 256, 64]):7.2f} us")
print(f"bulk 16 KiB x 1 WG    : {diag(5, [4, 0, 1, 64]):7.2f} us")
print(f"bulk 16 KiB x 256 WG  : {diag(5, [4, 0, 256, 64]):7.2f} us")
print("--- clip-group hand-off (8 workgroups per group, sc1 stores / loads, atomic arrival) ---")
for kb in (4, 40):
    for blocks in (8, 256):
        r1 = diag(5, [5, 1 | (kb << 16), blocks, 64], 3)
        r100 = diag(5, [5, 101 | (kb << 16), blocks, 64], 3)
        print(f"{blocks:4d} WGs, {kb:3d} KiB per WG: {(r100 - r1) / 100:7.3f} us per round (launch+1 round {r1:7.2f} us)")
