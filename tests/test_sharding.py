"""Multi-rank sharding of the clip batch over gloo on CPU, world size 2 and 3.

The sampler is the CPU oracle (2 DDPM steps of the beat-ours architecture) with the counter-based
noise keyed by GLOBAL clip id (oracle/ref_diffusion.PhiloxNoise), as the HIP sampler draws it: the
gathered result must equal the single-rank result bit for bit, in global clip order, for balanced
and ragged shards.  Each clip is sampled on its own, so its arithmetic does not depend on how
many clips share its shard.
"""
import os
import socket

import numpy as np
import pytest
import torch as th
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import ROOT  # noqa: F401  (puts the repo on sys.path)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


_ORACLE = {}


def oracle_sample(wav_shard, clip_offset, n_steps=2, seed=11):
    """(n_local, C, L) poses of the clips [clip_offset, clip_offset + n_local): oracle DDPM steps."""
    from oracle import ref_denoiser, ref_diffusion
    import __graft_entry__ as ge
    if not _ORACLE:
        pkg = ge.load_package()
        cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
        arch = pkg.arch_from_config(cfg.Model, 123)
        sd = pkg.init_state_dict(arch, seed=0, bounded=True)
        _ORACLE["om"] = ref_denoiser.OracleModel(
            sd, {k: arch[k] for k in ("type", "d_model", "decoder", "heads", "n_layers")}, cache_speech=True)
        _ORACLE["sch"] = ref_diffusion.make_schedule("linear", 1000, "")
    outs = []
    for j in range(wav_shard.shape[0]):
        noise = ref_diffusion.PhiloxNoise(seed, np.array([clip_offset + j]))
        outs.append(ref_diffusion.sample_loop(_ORACLE["sch"], _ORACLE["om"], (1, 123, 40), {"wav": wav_shard[j:j + 1]},
                                              noise, "ddpm", n_steps=n_steps)["sample"])
    return th.cat(outs)


def _wavs(n_total):
    return th.randn(n_total, 32000, generator=th.Generator().manual_seed(5)) * 0.1


def _worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import __graft_entry__ as ge
        sharding = __import__(ge.PKG_NAME + ".sharding", fromlist=["x"])
        th.set_num_threads(1)
        out = sharding.sample_sharded(oracle_sample, _wavs(n_total), n_total, rank, world, th.device("cpu"))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def single_rank():
    import __graft_entry__ as ge
    sharding = __import__(ge.PKG_NAME + ".sharding", fromlist=["x"])
    nt = th.get_num_threads()
    th.set_num_threads(1)  # as the workers: the CPU GEMMs' blocking depends on the thread count
    try:
        return sharding.sample_sharded(oracle_sample, _wavs(5), 5, 0, 1, th.device("cpu"))
    finally:
        th.set_num_threads(nt)


@pytest.mark.parametrize("world,n_total", [(2, 4), (2, 5), (3, 5)])
def test_sharded_gather_matches_single_rank(single_rank, world, n_total):
    want = single_rank[:n_total]  # wav rows and noise depend on the global clip id only
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert th.equal(results[r], want), r


def test_shard_ranges_cover_batch():
    import __graft_entry__ as ge
    sharding = __import__(ge.PKG_NAME + ".sharding", fromlist=["x"])
    for n in (1, 7, 32, 256):
        for world in (1, 2, 3, 8):
            spans = [sharding.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1
