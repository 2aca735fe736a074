"""Multi-rank sharding of the clip batch over gloo on CPU, world size 2 and 3.

The sample function stands in for the HIP sampler: a deterministic function of the global clip
id (as the counter-keyed noise makes the real sampler), so the gathered result must equal the
single-rank result exactly, in global clip order, for balanced and ragged shards.
"""
import os
import socket

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


def fake_sample(wav_shard, clip_offset):
    """(n_local, C, L) output that depends only on (global clip id, that clip's wav)."""
    n = wav_shard.shape[0]
    ids = th.arange(clip_offset, clip_offset + n, dtype=th.float32)
    return (ids[:, None, None] * 1000.0 + wav_shard[:, None, :6].sum(-1, keepdim=True)).expand(n, 5, 6).contiguous()


def _worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import __graft_entry__ as ge
        sharding = __import__(ge.PKG_NAME + ".sharding", fromlist=["x"])
        g = th.Generator().manual_seed(5)
        wavs = th.randn(n_total, 32, generator=g)
        out = sharding.sample_sharded(fake_sample, wavs, n_total, rank, world, th.device("cpu"))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total", [(2, 8), (2, 7), (3, 8)])
def test_sharded_gather_matches_single_rank(world, n_total):
    import __graft_entry__ as ge
    sharding = __import__(ge.PKG_NAME + ".sharding", fromlist=["x"])
    g = th.Generator().manual_seed(5)
    wavs = th.randn(n_total, 32, generator=g)
    want = sharding.sample_sharded(fake_sample, wavs, n_total, 0, 1, th.device("cpu"))
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
