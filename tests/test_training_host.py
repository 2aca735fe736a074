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


# ------------------------------------------------------------------------------------------
# DDP semantics (trainer.py:83): construction-time broadcast of rank 0's parameters / buffers,
# and the averaged gradient of per-rank half batches == the gradient of the union batch
# ------------------------------------------------------------------------------------------
class _FlatModel:
    """What broadcast_parameters touches on a TrainableModel: the flat parameter buffer and the
    BatchNorm buffers (CPU tensors here; the same calls move device tensors over RCCL)."""

    def __init__(self, rank, n):
        g = th.Generator().manual_seed(100 + rank)
        self.flat = th.randn(n, generator=g)
        self.buffers = {"a.running_mean": th.randn(7, generator=g), "a.num_batches_tracked": th.tensor(rank + 3)}


def _bcast_worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = _training()
        tr.BUCKET_ELEMS = 300
        m = _FlatModel(rank, n)
        tr.broadcast_parameters(m)
        q.put((rank, m.flat.numpy().copy(), {k: v.numpy().copy() for k, v in m.buffers.items()}))  # by value
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


def test_broadcast_parameters_takes_rank0_state():
    n = 1000
    res = _spawn(_bcast_worker, 2, n)
    want = _FlatModel(0, n)
    assert not th.equal(_FlatModel(1, n).flat, want.flat)     # rank 1 started elsewhere
    for rank, flat, bufs in res:
        assert th.equal(th.from_numpy(flat), want.flat), rank
        for k, v in want.buffers.items():
            assert th.equal(th.from_numpy(bufs[k]), v), (rank, k)


def _decoder_grad(clips):
    """Flat gradient (training._trainable order, encoder frozen) of the mean per-clip diffusion MSE
    over `clips` of a fixed synthetic batch, by torch autograd through the CPU oracle
    (gaussian_diffusion.py:531-569 on oracle/ref_denoiser.denoise, speech tokens given)."""
    import __graft_entry__ as ge
    from oracle import ref_denoiser
    from tests.conftest import oracle_cfg
    pkg = ge.load_package()
    tr = _training()
    cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
    arch = pkg.arch_from_config(cfg.Model, 123)
    sd = pkg.init_state_dict(arch, seed=0, perturb=True)
    names = [k for k, _ in tr._trainable(arch, False)]
    for k in names:
        sd[k] = sd[k].float().clone().requires_grad_(True)
    g = th.Generator().manual_seed(11)
    n, L = 4, 40
    x0 = th.randn(n, 123, L, generator=g)
    noise = th.randn(n, 123, L, generator=g)
    t = th.tensor([999, 421, 77, 3])
    z = tuple(th.randn(n, Ti, 256, generator=g) * 0.3 for Ti in (31, 30, 30))
    diffusion = pkg.create_diffusion(cfg.Model.Diffusion.to_dict(), True)
    idx = t.numpy()
    ca = th.from_numpy(diffusion.sqrt_alphas_cumprod[idx]).float().reshape(-1, 1, 1)
    cb = th.from_numpy(diffusion.sqrt_one_minus_alphas_cumprod[idx]).float().reshape(-1, 1, 1)
    sel = th.tensor(clips)
    x_t = (ca * x0 + cb * noise)[sel]
    speech = ref_denoiser.speech_memory(sd, oracle_cfg(arch), tuple(a[sel] for a in z))
    eps = ref_denoiser.denoise(sd, oracle_cfg(arch), x_t, t[sel], speech=speech)
    loss = ((eps - noise[sel]) ** 2).mean(dim=(1, 2)).mean()
    loss.backward()
    return th.cat([sd[k].grad.reshape(-1) for k in names])


def _grad_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    th.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = _decoder_grad([2 * rank, 2 * rank + 1])
        out = _training().allreduce_gradients(g)
        q.put((rank, out.numpy().copy()))   # by value: the worker exits before the parent reads
    finally:
        dist.destroy_process_group()


def test_ddp_average_of_half_batches_equals_union_batch_gradient():
    res = _spawn(_grad_worker, 2)
    want = _decoder_grad([0, 1, 2, 3])
    scale = want.abs().max().item()
    for rank, got in res:
        err = (th.from_numpy(got) - want).abs().max().item()
        assert err <= 1e-5 * scale, (rank, err, scale)
    assert (res[0][1] == res[1][1]).all()       # every rank holds the same averaged gradient


def test_parse_steps_follows_string_parser_code():
    tr = _training()
    assert tr.parse_steps("100") == 100 and tr.parse_steps("500k") == 500000
    assert tr.parse_steps("100kk") == 200000    # string_parser.py: base * count('k') * 1000


def test_noam_decay_has_no_floor():
    """create_lr_scheduler builds NoamDecayLR without `minimum` (model_creation.py:23)."""
    tr = _training()
    o = _Opt(1.0)
    s = tr.LRScheduler(o, {"type": "noam", "warmup_steps": "10", "minimum": 0.5})
    for _ in range(1000):
        s.step()
    assert o.param_groups[0]["lr"] == pytest.approx(10 ** 0.5 * 1000 ** -0.5)


def test_speed_losses_follow_trainer_py():
    """trainer.py:172-193 and wasserstein_distance_1d (trainer.py:310-322), checked against the
    closed forms in float64 numpy; gradients reach pred_x_start; unknown names raise."""
    tr = _training()
    g = th.Generator().manual_seed(4)
    x = th.randn(3, 5, 12, generator=g, dtype=th.float64)
    p = (x + 0.3 * th.randn(3, 5, 12, generator=g, dtype=th.float64)).requires_grad_(True)
    params = {"speed_loss": 0.5, "speed_l1_loss": 2.0, "speed_constraint_loss": 0.25}
    terms, total = tr.speed_losses(x, p, params)
    xn, pn = x.numpy(), p.detach().numpy()
    sp, sq = np.abs(np.diff(xn, axis=2)).mean((0, 1)), np.abs(np.diff(pn, axis=2)).mean((0, 1))
    v1, v2 = sp.var(ddof=1), sq.var(ddof=1)
    w2 = np.sqrt(max((sp.mean() - sq.mean()) ** 2 + v1 + v2 - 2 * np.sqrt(np.sqrt(v1) * v2 * np.sqrt(v1)), 1e-12))
    d = sq - sp
    l1 = np.where(np.abs(d) < 1.0, 0.5 * d * d, np.abs(d) - 0.5).mean()
    sc = np.abs(np.diff(pn, axis=2)).mean()
    assert abs(terms["speed"].item() - w2) <= 1e-12
    assert abs(terms["speed_l1"].item() - l1) <= 1e-12
    assert abs(terms["speed_constraint"].item() - sc) <= 1e-12
    assert abs(total.item() - (0.5 * w2 + 2.0 * l1 + 0.25 * sc)) <= 1e-12
    total.backward()
    assert p.grad is not None and p.grad.abs().sum().item() > 0
    with pytest.raises(ValueError, match="Unsupported loss"):
        tr.speed_losses(x, p, {"foot_contact_loss": 1.0})
    # no extra losses: nothing added
    terms, total = tr.speed_losses(x, p, None)
    assert terms == {} and total == 0.0


def test_adamw_load_state_dict_restores_group_hyperparameters():
    """torch.optim.Optimizer.load_state_dict (trainer.py:218) restores lr, betas, eps and
    weight_decay of the saved group; a resumed run then steps with the checkpoint's values."""
    import types
    tr = _training()
    params = {"a": th.zeros(3, 2), "b": th.zeros(4)}
    model = types.SimpleNamespace(flat=th.zeros(10), params=params)
    saved = tr.AdamW(model, lr=2e-4, betas=(0.8, 0.95), eps=1e-6, weight_decay=0.05)
    st = saved.state_dict()
    opt = tr.AdamW(model, lr=1e-3)
    opt.load_state_dict(st)
    assert opt.param_groups[0]["lr"] == pytest.approx(2e-4)
    assert opt.betas == (0.8, 0.95) and opt.eps == 1e-6 and opt.weight_decay == 0.05
    # the same checkpoint restored into torch's AdamW carries the same hyperparameters
    ref = th.optim.AdamW([th.nn.Parameter(th.zeros(3, 2)), th.nn.Parameter(th.zeros(4))], lr=1e-3)
    ref.load_state_dict(st)
    g = ref.param_groups[0]
    assert tuple(g["betas"]) == opt.betas and g["eps"] == opt.eps and g["weight_decay"] == opt.weight_decay


def test_grad_slot_only_for_existing_leaf_grads():
    """training._grad_slot: a weight-gradient kernel accumulates (beta = 1) into .grad only for a
    leaf parameter whose contiguous f32 .grad already exists (the flat gradient buffer's views),
    and only outside create_graph backward; everything else goes back to autograd."""
    tr = _training()
    flat = th.zeros(12)
    p = th.nn.Parameter(flat[:6].view(2, 3).clone())
    with th.no_grad():
        assert tr._grad_slot(p) is None                   # no .grad yet: autograd creates it
        p.grad = flat[6:].view(2, 3)
        assert tr._grad_slot(p) is None                   # outside Trainer.step's backward: autograd
        with tr.direct_grad_accumulation():
            assert tr._grad_slot(p).data_ptr() == flat[6:].data_ptr()
            assert tr._grad_slot(p * 2) is None           # not a leaf
            assert tr._grad_slot(None) is None
            q = th.nn.Parameter(th.zeros(3, 2))
            q.grad = th.zeros(2, 3).t()                   # non-contiguous .grad
            assert tr._grad_slot(q) is None
        assert tr._grad_slot(p) is None
    with tr.direct_grad_accumulation():
        assert tr._grad_slot(p) is None                    # grad mode on (create_graph backward)
