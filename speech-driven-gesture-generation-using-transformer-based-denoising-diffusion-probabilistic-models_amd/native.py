"""ctypes binding of libggd.so -- the C ABI in include/ggd.h.

The library is built in-tree (``build()``; ``__graft_entry__.build()`` calls it) so
the ``.so`` travels with the repository snapshot to the GPU box.  There is no
fallback: if the library is missing, ``load()`` raises.

``libggd_diag.so`` is the same library built with -DGGD_DIAG plus ggd_diag.hip: it adds the
``ggd_diag`` microbenchmarks / phase stamps used by scripts/ (``GGD_DIAG=1`` loads it instead).
The product library never exports them.
"""
import ctypes
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
PRODUCT_LIB = os.path.join(PKG_DIR, "libggd.so")
DIAG_LIB = os.path.join(PKG_DIR, "libggd_diag.so")
LIB_PATH = DIAG_LIB if os.environ.get("GGD_DIAG") == "1" else PRODUCT_LIB
# A/B experiments (scripts/ab.sh): another build of the same library, same ABI
if os.environ.get("GGD_LIB"):
    LIB_PATH = os.path.abspath(os.environ["GGD_LIB"])
SOURCES = ["ggd_kernels.hip", "ggd_fused.hip", "ggd_mega.hip", "ggd_rows.hip", "ggd_persist.hip", "ggd_encoder.hip", "ggd_train.hip", "ggd_chain.hip", "ggd_attn.hip", "ggd_long.hip",
           "ggd_api.hip"]
DIAG_SOURCES = ["ggd_diag.hip"]   # + ggd_api.hip again with -DGGD_DIAG
HEADERS = ["ggd_kernels.h", "ggd_common.h", "ggd_chainlib.h", "ggd_fusedlib.h", "ggd_phases.h", "ggd_megasync.h", os.path.join("..", "..", "include", "ggd.h"),
           os.path.join("..", "..", "include", "ggd_train.h")]

GGD_OK, GGD_IGNORED = 0, 1
GGD_ERR_ARG, GGD_ERR_UNSUPPORTED, GGD_ERR_HIP, GGD_ERR_STATE, GGD_ERR_NAME = -1, -2, -3, -4, -5
MODEL_S2G_V2, MODEL_DEFAULT, MODEL_INPAINT = 0, 1, 2
DEC_ONEWAY, DEC_TWOWAY = 0, 1
F32, BF16, FP8W = 0, 1, 2   # ggd_dtype (include/ggd.h)
DDPM, DDIM = 0, 1
MEM_BLEND, MEM_CONCAT = 0, 1   # ggd_enc_run_memory layouts

EXPORTS = [
    "ggd_create", "ggd_destroy", "ggd_last_error", "ggd_load_weight", "ggd_finalize_weights",
    "ggd_set_schedule", "ggd_set_memory", "ggd_set_inpaint", "ggd_denoise", "ggd_posterior_step", "ggd_sample",
    "ggd_sync",
    "ggd_set_profiling", "ggd_kernel_time", "ggd_profile_kind", "ggd_set_route", "ggd_route_info", "ggd_version",
    "ggd_mx_linear", "ggd_mx_layernorm", "ggd_mx_ffn_up",
    "ggd_enc_create", "ggd_enc_destroy", "ggd_enc_last_error", "ggd_enc_load_weight", "ggd_enc_finalize",
    "ggd_enc_lengths", "ggd_enc_run", "ggd_enc_run_memory",
    # training path (include/ggd_train.h)
    "ggd_tr_gemm", "ggd_tr_colsum", "ggd_tr_layernorm_fwd", "ggd_tr_layernorm_bwd", "ggd_tr_seqconv_fwd",
    "ggd_tr_seqconv_bwd", "ggd_tr_attention_fwd", "ggd_tr_attention_bwd", "ggd_tr_elementwise", "ggd_tr_q_sample",
    "ggd_tr_mse", "ggd_tr_sumsq", "ggd_tr_sumsq_blocks", "ggd_tr_adamw", "ggd_tr_scale", "ggd_tr_scale_clamp",
    "ggd_tr_conv_fwd", "ggd_tr_conv_dgrad", "ggd_tr_conv_wgrad", "ggd_tr_im2col", "ggd_tr_col2im", "ggd_tr_batchnorm_fwd", "ggd_tr_batchnorm_bwd", "ggd_tr_image_channel_sum",
    "ggd_tr_channel_scale", "ggd_tr_pixel_shuffle", "ggd_tr_head_flatten", "ggd_enc_frontend",
]


class Desc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "model_type", "decoder_type", "d_model", "heads", "n_layers", "d_pose", "seq_len",
        "speech_len", "max_batch", "dtype", "diffusion_steps")]


class SampleArgs(ctypes.Structure):
    _fields_ = [
        ("alg", ctypes.c_int32), ("eta", ctypes.c_float), ("n", ctypes.c_int32),
        ("x_T", ctypes.c_void_p), ("noise", ctypes.c_void_p), ("seed", ctypes.c_uint64),
        ("clip_offset", ctypes.c_int64), ("inpaint_poses", ctypes.c_void_p),
        ("inpaint_masks", ctypes.c_void_p), ("trans", ctypes.c_void_p), ("out", ctypes.c_void_p),
        ("extras", ctypes.c_void_p), ("n_steps", ctypes.c_int32), ("use_graph", ctypes.c_int32),
        ("sync", ctypes.c_int32),
    ]


def _deps(path, seen=None):
    """The file and every local header it includes, transitively (#include "...")."""
    import re
    seen = set() if seen is None else seen
    path = os.path.normpath(path)
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    with open(path) as f:
        for inc in re.findall(r'^\s*#include\s+"([^"]+)"', f.read(), re.M):
            _deps(os.path.join(os.path.dirname(path), inc), seen)
    return seen


def _sources():
    return [os.path.join(CSRC, s) for s in SOURCES + DIAG_SOURCES] + [os.path.join(CSRC, h) for h in HEADERS]


def is_stale():
    for lib in (PRODUCT_LIB, DIAG_LIB):
        if not os.path.exists(lib):
            return True
        t = os.path.getmtime(lib)
        if any(os.path.getmtime(p) > t for p in _sources()):
            return True
    return False


def build(force=False, verbose=False):
    """Compile libggd.so for gfx950 with hipcc (cross-compiles without a GPU)."""
    if not force and not is_stale():
        return LIB_PATH
    # -fno-slp-vectorize: no packed-f32 (v_pk_*_f32) code from the SLP vectorizer.  Beside MFMAs it
    # costs issue slots (MI355X_MICROARCH.md, filler prices), and with it hipcc 7.2 clobbered a live
    # register of psk_kernel (the per-thread pose state) around the one-pass LayerNorm.
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-fno-slp-vectorize", "-Wno-unused-value", "-Wno-unused-result"]
    os.makedirs(os.path.join(PKG_DIR, "build"), exist_ok=True)
    units = [(src, src.replace(".hip", ".o"), []) for src in SOURCES + DIAG_SOURCES]
    units.append(("ggd_api.hip", "ggd_api_diag.o", ["-DGGD_DIAG"]))
    procs = []
    for src, obj_name, extra in units:  # one hipcc per translation unit, in parallel
        obj = os.path.join(PKG_DIR, "build", obj_name)
        dep_t = max(os.path.getmtime(f) for f in _deps(os.path.join(CSRC, src)))
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > dep_t:
            continue  # object newer than its source and every header it includes
        cmd = ["hipcc"] + flags + extra + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd, cwd=CSRC))
    if any(p.wait() != 0 for p in procs):
        raise RuntimeError("hipcc failed")
    obj = lambda n: os.path.join(PKG_DIR, "build", n)
    product = [obj(s.replace(".hip", ".o")) for s in SOURCES]
    diag = [o for o in product if not o.endswith("ggd_api.o")] + [obj("ggd_api_diag.o"), obj("ggd_diag.o")]
    for lib, objs in ((PRODUCT_LIB, product), (DIAG_LIB, diag)):
        cmd = ["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", lib + ".tmp"]
        subprocess.run(cmd, check=True, cwd=CSRC)
        os.replace(lib + ".tmp", lib)
    return PRODUCT_LIB


_lib = None


def load():
    """Load libggd.so (after torch, so both share torch's HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  -- torch's libamdhip64 must be the one the library binds to
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libggd.so not built at {LIB_PATH}; run __graft_entry__.build() "
                          "(the HIP path has no fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    P, I32, I64, F, VP = ctypes.POINTER, ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p
    CTX = ctypes.c_void_p
    sig = {
        "ggd_create": (ctypes.c_int, [ctypes.c_int, P(Desc), P(CTX)]),
        "ggd_destroy": (ctypes.c_int, [CTX]),
        "ggd_last_error": (ctypes.c_char_p, [CTX]),
        "ggd_load_weight": (ctypes.c_int, [CTX, ctypes.c_char_p, VP, I64]),
        "ggd_finalize_weights": (ctypes.c_int, [CTX]),
        "ggd_set_schedule": (ctypes.c_int, [CTX, VP, I32, VP]),
        "ggd_set_memory": (ctypes.c_int, [CTX, VP, I32, I32, I32, VP]),
        "ggd_set_inpaint": (ctypes.c_int, [CTX, VP, VP, I32, VP]),
        "ggd_denoise": (ctypes.c_int, [CTX, VP, VP, VP, I32, VP]),
        "ggd_posterior_step": (ctypes.c_int, [CTX, I32, F, I32, VP, VP, VP, VP, VP, VP, I32, VP]),
        "ggd_sample": (ctypes.c_int, [CTX, P(SampleArgs), VP]),
        "ggd_sync": (ctypes.c_int, [CTX]),
        "ggd_set_profiling": (ctypes.c_int, [CTX, I32]),
        "ggd_kernel_time": (ctypes.c_int, [CTX, I32, P(ctypes.c_double), P(I64)]),
        "ggd_profile_kind": (ctypes.c_int, [CTX]),
        "ggd_set_route": (ctypes.c_int, [CTX, I32, I32]),
        "ggd_route_info": (ctypes.c_int, [CTX, I32, VP]),
        "ggd_version": (ctypes.c_char_p, []),
        "ggd_mx_linear": (ctypes.c_int, [I32, I32, I32, VP, VP, VP, VP, VP, VP]),
        "ggd_mx_layernorm": (ctypes.c_int, [VP, VP, VP, VP, VP, VP]),
        "ggd_mx_ffn_up": (ctypes.c_int, [VP, VP, VP, VP, VP, VP, VP, VP]),
        "ggd_enc_create": (ctypes.c_int, [ctypes.c_int, I32, I32, I32, I32, P(CTX)]),
        "ggd_enc_destroy": (ctypes.c_int, [CTX]),
        "ggd_enc_last_error": (ctypes.c_char_p, [CTX]),
        "ggd_enc_load_weight": (ctypes.c_int, [CTX, ctypes.c_char_p, VP, I64]),
        "ggd_enc_finalize": (ctypes.c_int, [CTX]),
        "ggd_enc_lengths": (ctypes.c_int, [CTX, P(I32), P(I32), P(I32)]),
        "ggd_enc_run": (ctypes.c_int, [CTX, VP, I32, VP, VP, VP, VP]),
        "ggd_enc_run_memory": (ctypes.c_int, [CTX, VP, I32, I32, VP, VP]),
        "ggd_tr_gemm": (ctypes.c_int, [I32, I32, I32, I32, I32, F, VP, I32, VP, I32, F, VP, I32, VP, VP]),
        "ggd_tr_colsum": (ctypes.c_int, [I32, I32, VP, I32, VP, F, VP]),
        "ggd_tr_layernorm_fwd": (ctypes.c_int, [I32, I32, VP, VP, VP, F, VP, VP, VP, VP]),
        "ggd_tr_layernorm_bwd": (ctypes.c_int, [I32, I32, VP, VP, VP, VP, VP, VP, VP, VP, VP]),
        "ggd_tr_seqconv_fwd": (ctypes.c_int, [I32, I32, I32, I32, VP, I32, VP, VP, VP, I32, VP]),
        "ggd_tr_seqconv_bwd": (ctypes.c_int, [I32, I32, I32, I32, VP, I32, VP, VP, I32, VP, I32, VP, VP, VP]),
        "ggd_tr_attention_fwd": (ctypes.c_int, [I32, I32, I32, I32, I32, F, VP, I32, VP, VP, I32, VP, I32, VP]),
        "ggd_tr_attention_bwd": (ctypes.c_int, [I32, I32, I32, I32, I32, F, VP, I32, VP, VP, I32, VP, I32, VP, VP,
                                                VP, VP]),
        "ggd_tr_elementwise": (ctypes.c_int, [I32, I64, VP, VP, VP, VP]),
        "ggd_tr_q_sample": (ctypes.c_int, [I32, I32, VP, VP, VP, VP, VP, VP]),
        "ggd_tr_mse": (ctypes.c_int, [I32, I32, VP, VP, VP, VP, F, VP]),
        "ggd_tr_sumsq": (ctypes.c_int, [I64, VP, VP, VP, VP]),
        "ggd_tr_sumsq_blocks": (ctypes.c_int, []),
        "ggd_tr_adamw": (ctypes.c_int, [I64, VP, VP, VP, VP, F, F, F, F, F, I64, F, VP]),
        "ggd_tr_scale": (ctypes.c_int, [I64, VP, F, VP]),
        "ggd_tr_scale_clamp": (ctypes.c_int, [I64, VP, F, F, VP]),
        "ggd_tr_conv_fwd": (ctypes.c_int, [I32] * 9 + [VP, VP, VP, VP, VP]),
        "ggd_tr_conv_dgrad": (ctypes.c_int, [I32] * 9 + [VP, VP, VP, VP]),
        "ggd_tr_conv_wgrad": (ctypes.c_int, [I32] * 9 + [VP, VP, F, VP, VP]),
        "ggd_tr_im2col": (ctypes.c_int, [I32, I32, I32, I32, I32, I32, I32, I32, VP, VP, VP]),
        "ggd_tr_col2im": (ctypes.c_int, [I32, I32, I32, I32, I32, I32, I32, I32, VP, VP, VP]),
        "ggd_tr_batchnorm_fwd": (ctypes.c_int, [I32, I32, VP, VP, VP, F, VP, VP, VP, VP, VP]),
        "ggd_tr_batchnorm_bwd": (ctypes.c_int, [I32, I32, VP, VP, VP, VP, VP, VP, VP, VP, VP]),
        "ggd_tr_image_channel_sum": (ctypes.c_int, [I32, I32, I32, VP, VP, F, VP, VP]),
        "ggd_tr_channel_scale": (ctypes.c_int, [I32, I32, I32, VP, VP, VP, VP, VP]),
        "ggd_tr_pixel_shuffle": (ctypes.c_int, [I32, I32, I32, I32, I32, VP, VP, I32, VP]),
        "ggd_tr_head_flatten": (ctypes.c_int, [I32, I32, I32, I32, VP, VP, I32, VP]),
        "ggd_enc_frontend": (ctypes.c_int, [CTX, VP, I32, VP, VP]),
    }
    if LIB_PATH == DIAG_LIB or hasattr(lib, "ggd_diag"):  # (also a GGD_LIB diag variant, scripts/build_variant.sh)
        sig["ggd_diag"] = (ctypes.c_int, [CTX, I32, VP, I32, I32, VP])
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class GgdError(RuntimeError):
    pass


def check(ctx, code, what, last_error="ggd_last_error"):
    """Map a ggd_status to the reference's exception types."""
    if code >= 0:
        return code
    msg = getattr(load(), last_error)(ctx)
    msg = msg.decode() if msg else ""
    text = f"{what}: {msg}"
    if code == GGD_ERR_UNSUPPORTED:
        raise ValueError(text)
    if code in (GGD_ERR_ARG, GGD_ERR_NAME):
        raise AssertionError(text)
    raise GgdError(text)
