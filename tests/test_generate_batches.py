"""Generator.generate_batches host plumbing (CPU, fake sampler): batch k's loop receives batch
k+1's wav as ``prefetch_wav`` and the outputs come back in order, one per batch."""
import torch as th

import __graft_entry__ as ge


class _FakeModel:
    arch = {"type": "s2g_v2"}


class _FakeDiffusion:
    def __init__(self):
        self.calls = []

    def ddim_sample_loop(self, model, shape, noise=None, denoise_fn=None, model_kwargs=None, device=None,
                         progress=False, prefetch_wav=None, **kw):
        self.calls.append((model_kwargs["wav"], prefetch_wav, tuple(shape)))
        n, c, length = shape
        return {"sample": th.full((n, c, length), float(len(self.calls)))}


def test_generate_batches_prefetches_next_batch():
    pkg = ge.load_package()
    diff = _FakeDiffusion()
    gen = pkg.Generator(_FakeModel(), diff)
    wavs = [th.randn(n, 320) for n in (3, 2, 4)]
    outs = gen.generate_batches((0, 5, 7), wavs, sample_alg="ddim", device="cpu")
    assert [o.shape for o in outs] == [(3, 7, 5), (2, 7, 5), (4, 7, 5)]
    assert [float(o[0, 0, 0]) for o in outs] == [1.0, 2.0, 3.0]
    assert th.equal(diff.calls[0][1], wavs[1]) and th.equal(diff.calls[1][1], wavs[2])
    assert diff.calls[2][1] is None
    assert [c[2] for c in diff.calls] == [(3, 5, 7), (2, 5, 7), (4, 5, 7)]


class _SyncModel(_FakeModel):
    def __init__(self):
        self.syncs = 0

    def sync(self):
        self.syncs += 1


def test_generator_checks_loop_status_before_returning():
    """ADVICE: the sampling loop is non-blocking, so the Generator entry points sync the model
    (ggd_sync raises a failed loop's error) before handing results back: once per
    generate_sample, once per generate_batches call."""
    pkg = ge.load_package()
    m = _SyncModel()
    gen = pkg.Generator(m, _FakeDiffusion())
    gen.generate_sample((2, 5, 7), th.randn(2, 320), sample_alg="ddim", device="cpu", progress=False)
    assert m.syncs == 1
    gen.generate_batches((0, 5, 7), [th.randn(n, 320) for n in (3, 2)], sample_alg="ddim", device="cpu")
    assert m.syncs == 2
