"""Host logic of the training path (no GPU): the gradient all-reduce over gloo (world 2, as DDP
averages, trainer.py:83 / utils/pytorch_ddp.py:18), the learning-rate schedules
(models/lr_scheduler.py) and the uniform timestep sampler (models/modules/resample.py:60-68)."""
import importlib
import os
import socket

import numpy as np
import pytest
import torch as th
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import ROOT  # noqa: F401  (puts the repo on sys.path)


def _training():
    import __graft_entry__ as ge
    return importlib.import_module(ge.PKG_NAME + ".training")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _grad_of(rank, n):
    return th.arange(n, dtype=th.float32) * (rank + 1) + rank


def _worker(rank, world, port, n, bucket, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = _training()
        tr.BUCKET_ELEMS = bucket
        g = _grad_of(rank, n)
        out = tr.allreduce_gradients(g)
        q.put((rank, out.clone(), out.data_ptr() == g.data_ptr()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allreduce_gradients_averages_over_ranks(world):
    n, bucket = 1000, 384     # three buckets, the last one ragged
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, bucket, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = sum(_grad_of(r, n) for r in range(world)) / world
    for rank, out, in_place in res:
        assert in_place, rank          # the flat gradient buffer is reduced in place (bucket views)
        assert th.allclose(out, want, rtol=0, atol=1e-4), rank


def test_allreduce_is_identity_without_a_process_group():
    g = th.arange(10, dtype=th.float32)
    assert th.equal(_training().allreduce_gradients(g.clone()), g)


class _Opt:
    def __init__(self, lr):
        self.param_groups = [{"lr": lr, "initial_lr": lr}]


def test_lr_schedules_follow_lr_scheduler_py():
    tr = _training()
    # NoamLR ('noamxf'): base d^-0.5 min(s^-0.5, s w^-1.5), s = last_epoch + 1
    o = _Opt(1.0)
    s = tr.LRScheduler(o, {"type": "noamxf", "warmup_steps": "4k", "d_model": 256})
    for step in range(1, 6):
        assert o.param_groups[0]["lr"] == pytest.approx(256 ** -0.5 * min(step ** -0.5, step * 4000 ** -1.5))
        s.step()
    # NoamDecayLR ('noam'): base w^0.5 min(e^-0.5, e w^-1.5), e = max(1, last_epoch)
    o = _Opt(2.0)
    s = tr.LRScheduler(o, {"type": "noam", "warmup_steps": "10"})
    seen = []
    for _ in range(25):
        seen.append(o.param_groups[0]["lr"])
        s.step()
    want = [2.0 * 10 ** 0.5 * min(max(1, e) ** -0.5, max(1, e) * 10 ** -1.5) for e in range(25)]
    assert np.allclose(seen, want)
    # ConstantLR
    o = _Opt(0.3)
    s = tr.LRScheduler(o, None)
    s.step()
    assert o.param_groups[0]["lr"] == 0.3
    with pytest.raises(ValueError):
        tr.LRScheduler(_Opt(1.0), {"type": "cosine"})
    assert tr.parse_steps("200k") == 200000 and tr.parse_steps("40") == 40


def test_uniform_sampler_draws_every_step_with_unit_weights():
    tr = _training()

    class D:
        num_timesteps = 50

    t, w = tr.UniformSampler(D()).sample(4000, "cpu", np.random.RandomState(0))
    assert t.dtype == th.int64 and int(t.min()) == 0 and int(t.max()) == 49
    assert len(th.unique(t)) == 50 and th.equal(w, th.ones(4000))
