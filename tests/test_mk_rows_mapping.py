"""Index math of the clip-group loop's KE rows phase (csrc/ggd_phases.h ker_phase), restated on
the CPU: workgroup p owns frames [p L / 8, (p + 1) L / 8); thread t takes channel t % 128 and the
(t / 128)-th Philox quad (4 consecutive elements of the reference's (C, L) order,
oracle/philox.py) that starts at or before the channel's first frame of the block, and updates the
elements of the quad that are that channel's frames of the block.  Every element of every clip
must be updated exactly once, by a thread whose quad holds it at the right position, for every L
the loop serves (1..64) and C <= 128; and for L % 4 == 0 all lanes of a wave hold the same frame
(the coalesced x stores).
"""
import pytest

FT = 512


def thread_quad(t, C, cmap):
    """(channel, k-th quad) of thread t, or None: GGD_MK_CMAP = 1 (channel t % 128) or 0 (t / 3)."""
    if cmap:
        uc, k = t & 127, t >> 7
        return (uc, k) if uc < C and t < 3 * 128 else None
    uc, k = t // 3, t % 3
    return (uc, k) if uc < C else None


def ke_rows_cover(L, C, cmap=1):
    seen = {}
    for p in range(8):
        r0 = p * L // 8
        R = (p + 1) * L // 8 - r0
        for t in range(FT):
            tq = thread_quad(t, C, cmap)
            if tq is None:
                continue
            uc, k = tq
            qi = ((uc * L + r0) >> 2) + k
            for u in range(4):
                e = 4 * qi + u
                lr = e - uc * L
                if r0 <= lr < r0 + R:
                    key = (uc, lr)
                    assert key not in seen, (L, C, key, seen.get(key), (p, t, u))
                    seen[key] = (p, t, u, e)
    return seen


@pytest.mark.parametrize("cmap", [0, 1])
@pytest.mark.parametrize("C", [123, 128, 1, 7])
def test_every_element_updated_once(C, cmap):
    for L in range(1, 65):
        seen = ke_rows_cover(L, C, cmap)
        assert len(seen) == L * C, (L, C)
        for (c, l), (p, t, u, e) in seen.items():
            assert e == c * L + l                       # the quad position is the reference's element
            assert p * L // 8 <= l < (p + 1) * L // 8   # the block that owns the frame


def test_lanes_of_a_wave_share_a_frame_when_L_is_a_multiple_of_4():
    for L in range(4, 65, 4):
        for p in range(8):
            r0 = p * L // 8
            for w in range(6):           # waves holding quads (threads < 384)
                for u in range(4):
                    frames = {4 * (((uc * L + r0) >> 2) + ((64 * w + lane) >> 7)) + u - uc * L
                              for lane in range(64) for uc in [(64 * w + lane) & 127] if uc < 123}
                    assert len(frames) == 1, (L, p, w, u, frames)
