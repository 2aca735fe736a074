"""Where a bench pass spends its time: encoder, memory install, sampling loop (GPU box)."""
import os as _os
_os.environ["GGD_DIAG"] = "1"  # ggd_diag lives in libggd_diag.so only (native.py)
import os
import sys
import time

import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
enc_mod = __import__(ge.PKG_NAME + ".encoder", fromlist=["x"])
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
dev = th.device("cuda:0")
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device=dev)
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
wavs = [th.randn(32, 32000, device=dev) * 0.1 for _ in range(6)]


def timed(fn, reps=5):
    fn()
    th.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    th.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


enc = model.encoder()
print(f"encoder 32 clips (CHUNK={enc.CHUNK})      : {timed(lambda: enc(wavs[0])):8.2f} ms", flush=True)
for ch in (16, 32):
    enc.CHUNK = ch
    print(f"encoder 32 clips (CHUNK={ch})     : {timed(lambda: enc(wavs[0])):8.2f} ms", flush=True)
enc.CHUNK = 8
# host-side issue time alone (no sync)
th.cuda.synchronize()
t0 = time.perf_counter()
enc(wavs[1])
t1 = time.perf_counter()
th.cuda.synchronize()
t2 = time.perf_counter()
print(f"encoder host issue {1e3 * (t1 - t0):.2f} ms, drain {1e3 * (t2 - t1):.2f} ms", flush=True)

k = [0]


def prep():
    k[0] += 1
    model.prepare(wavs[k[0] % 6], 40)


print(f"prepare (encoder + set_memory)      : {timed(prep):8.2f} ms", flush=True)
ctx, n = model.prepare(wavs[0], 40)
ctx.set_schedule(diffusion.betas, diffusion.timestep_map)
samp = lambda: diffusion.p_sample_loop(model, (32, 123, 40), model_kwargs={"wav": wavs[0]}, seed=7, extras=False)
print(f"p_sample_loop, memory cached        : {timed(samp, 3):8.2f} ms", flush=True)
th.cuda.synchronize()
t0 = time.perf_counter()
samp()
t1 = time.perf_counter()
th.cuda.synchronize()
t2 = time.perf_counter()
print(f"p_sample_loop host issue {1e3 * (t1 - t0):.2f} ms, drain {1e3 * (t2 - t1):.2f} ms", flush=True)
full = lambda: diffusion.p_sample_loop(model, (32, 123, 40), model_kwargs={"wav": wavs[(k.__setitem__(0, k[0] + 1) or k[0]) % 6]},
                                       seed=7, extras=False)
print(f"p_sample_loop, new wav each call    : {timed(full, 3):8.2f} ms", flush=True)

# slope / intercept of the sampling call in the number of denoise steps
for ns in (100, 500, 1000):
    f = lambda: diffusion.p_sample_loop(model, (32, 123, 40), model_kwargs={"wav": wavs[0]}, seed=7, extras=False,
                                        n_steps=ns)
    print(f"p_sample_loop n_steps={ns:4d}           : {timed(f, 3):8.2f} ms", flush=True)
native = __import__(ge.PKG_NAME + ".native", fromlist=["x"])
import ctypes  # noqa: E402
for what in (2, 3):
    for it in (200, 1000):
        arr = (ctypes.c_int32 * 1)(32)
        out = ctypes.c_double()
        th.cuda.synchronize()
        t0 = time.perf_counter()
        native.check(ctx.h, ctx.lib.ggd_diag(ctx.h, what, arr, 1, it, ctypes.cast(ctypes.byref(out), ctypes.c_void_p)),
                     "diag")
        th.cuda.synchronize()
        wall = (time.perf_counter() - t0) / it * 1e6
        print(f"diag {'graph' if what == 3 else 'eager'} step, {it} iters: events {out.value:8.2f} us, wall {wall:8.2f} us",
              flush=True)
f = lambda: diffusion.p_sample_loop(model, (32, 123, 40), model_kwargs={"wav": wavs[0]}, seed=7, extras=False,
                                    use_graph=False)
print(f"p_sample_loop eager launches        : {timed(f, 2):8.2f} ms", flush=True)

# the encoder captured as one graph per fixed chunk (static input / output buffers)
for ch in (8, 32):
    enc.CHUNK = ch
    xin = wavs[0][:ch].clone()
    try:
        s = th.cuda.Stream()
        s.wait_stream(th.cuda.current_stream())
        with th.cuda.stream(s), th.backends.cudnn.flags(enabled=True, benchmark=False, deterministic=True):
            for _ in range(2):
                ref = enc._encode(xin)
        th.cuda.current_stream().wait_stream(s)
        g = th.cuda.CUDAGraph()
        with th.cuda.graph(g), th.backends.cudnn.flags(enabled=True, benchmark=False, deterministic=True):
            outs = enc._encode(xin)
        g.replay()
        th.cuda.synchronize()
        same = all(bool(th.equal(a, b)) for a, b in zip(ref, outs))
        print(f"encoder graph CHUNK={ch}: capture ok, replay == eager: {same}, "
              f"replay x{32 // ch}: {timed(lambda: [g.replay() for _ in range(32 // ch)]):8.2f} ms", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"encoder graph CHUNK={ch}: capture failed: {type(e).__name__}: {str(e)[:200]}", flush=True)
