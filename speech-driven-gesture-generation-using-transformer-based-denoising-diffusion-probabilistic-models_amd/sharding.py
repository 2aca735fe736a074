"""Batch-sharded sampling over ranks (one process per GPU, torch.distributed over RCCL).

Clips are independent units (no cross-batch op in eval: BN uses running stats,
InstanceNorm and attention are per clip), so rank r of G samples clips
[r*N/G, (r+1)*N/G) with zero per-step communication; the counter-based noise is
keyed by GLOBAL clip id, so 1/2/4/8-GPU outputs are bit-identical.  The only
collective is one all-gather of the final poses.  The
reference's only distributed code is training DDP (utils/pytorch_ddp.py:18,
models/trainer.py:83); this replaces it in kind for inference.
"""
import torch as th
import torch.distributed as dist


def shard_range(n_total, rank, world):
    """Contiguous, balanced [start, stop) of the clips owned by ``rank``."""
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def sample_sharded(sample_fn, wavs, n_total, rank, world, device, stats=None):
    """Run ``sample_fn(wav_shard, clip_offset) -> (n_local, ...)`` on this rank's clips and
    all-gather the results in global clip order on every rank.

    ``stats`` (a dict, optional) receives the all-gather's payload bytes and its timing: on a GPU a
    pair of events on the current stream around the collective (``gather_events``: the stream waits
    for RCCL there, so the span also holds the wait for the slowest rank), on CPU ``gather_ms``."""
    import time
    start, stop = shard_range(n_total, rank, world)
    local = sample_fn(wavs[start:stop], start).contiguous()
    if world == 1:
        return local
    counts = [shard_range(n_total, r, world) for r in range(world)]
    sizes = [b - a for a, b in counts]
    maxn = max(sizes)
    pad = th.zeros((maxn,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    gathered = th.empty((world * maxn,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if stats is None:
        dist.all_gather_into_tensor(gathered, pad)
    elif gathered.is_cuda:
        e0, e1 = th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)
        e0.record()
        dist.all_gather_into_tensor(gathered, pad)
        e1.record()
        stats["gather_events"] = (e0, e1)
    else:
        t0 = time.perf_counter()
        dist.all_gather_into_tensor(gathered, pad)
        stats["gather_ms"] = (time.perf_counter() - t0) * 1e3
    if stats is not None:
        stats["gather_bytes"] = gathered.numel() * gathered.element_size()
        stats["gather_bytes_per_rank"] = pad.numel() * pad.element_size()
    parts = [gathered[r * maxn: r * maxn + sizes[r]] for r in range(world)]
    return th.cat(parts, dim=0)
