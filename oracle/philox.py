"""Oracle: numpy restatement of the sampler's counter-based Gaussian noise stream.

Test infrastructure only.  The reference draws ``th.randn`` / ``th.randn_like``
(models/generator.py:285, models/modules/gaussian_diffusion.py:326,474); a
multi-GPU sampler cannot reproduce torch's global RNG order, so the HIP path
(and this oracle) key every draw by (seed, global clip id, step, stream tag)
instead -- BASELINE.md "Value distributions and seeds".

Generator: Philox4x32-10 (Salmon et al., SC'11) -> Box-Muller.
  counter = (e // 4, clip, step, tag), key = (seed_lo, seed_hi)
  element e of a clip is its flat index in the reference (C, L) layout.
  4 uint32 outputs u0..u3 -> two Box-Muller pairs:
      r = sqrt(-2 ln((u0 + 1) * 2^-32)),  th = 2 pi (u1 * 2^-32)
      z[e%4 == 0] = r cos th, z[1] = r sin th, (u2, u3) likewise for z[2], z[3].
All float math is float32, in the same order as csrc/ggd_kernels.hip:philox_normal.
"""
import numpy as np

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = np.uint32(0x9E3779B9)
_W1 = np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)

TAG_STEP = 0
TAG_XT = 1


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32 with 10 rounds; all arguments uint32 arrays/scalars."""
    c0 = np.asarray(c0, dtype=np.uint32).copy()
    c1 = np.broadcast_to(np.asarray(c1, dtype=np.uint32), c0.shape).copy()
    c2 = np.broadcast_to(np.asarray(c2, dtype=np.uint32), c0.shape).copy()
    c3 = np.broadcast_to(np.asarray(c3, dtype=np.uint32), c0.shape).copy()
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    for _ in range(10):
        p0 = c0.astype(np.uint64) * _M0
        p1 = c2.astype(np.uint64) * _M1
        hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
        lo0 = (p0 & _MASK).astype(np.uint32)
        hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
        lo1 = (p1 & _MASK).astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = np.uint32((int(k0) + int(_W0)) & 0xFFFFFFFF)
        k1 = np.uint32((int(k1) + int(_W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def normal_block(seed, clips, step, tag, n_elem):
    """Gaussian draws for ``clips`` (global ids) x ``n_elem`` elements -> float32 (len(clips), n_elem)."""
    clips = np.asarray(clips, dtype=np.uint32)
    e = np.arange(n_elem, dtype=np.uint32)
    grp = (e // 4)[None, :].repeat(len(clips), 0)
    cl = clips[:, None].repeat(n_elem, 1)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    u = philox4x32_10(grp, cl, np.uint32(step & 0xFFFFFFFF), np.uint32(tag),
                      seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    sel = (e % 4)[None, :]
    inv = np.float32(2.3283064365386963e-10)  # 2^-32
    two_pi = np.float32(6.283185307179586)
    a = np.where(sel < 2, u[0], u[2]).astype(np.float32)
    b = np.where(sel < 2, u[1], u[3]).astype(np.float32)
    ua = (a + np.float32(1.0)) * inv
    ub = b * inv
    r = np.sqrt(np.float32(-2.0) * np.log(ua).astype(np.float32)).astype(np.float32)
    th_ = (two_pi * ub).astype(np.float32)
    z = np.where(sel % 2 == 0, r * np.cos(th_).astype(np.float32), r * np.sin(th_).astype(np.float32))
    return z.astype(np.float32)


def clip_noise(seed, clip_ids, step, tag, C, L):
    """Noise in the reference (N, C, L) layout for the given global clip ids."""
    z = normal_block(seed, clip_ids, step, tag, C * L)
    return z.reshape(len(clip_ids), C, L)
