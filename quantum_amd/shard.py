"""Multi-GPU sharding of packet batches.

Packets are independent GCM instances, so the path shards with no data-path collective: one process
per GPU owns a disjoint subset of packets (and the keys they use).  The only cross-rank traffic is
the benchmark's barrier and max-over-ranks timing, done here through torch.distributed (RCCL on
GPUs, gloo in the CPU tests).

Mirrors the reference's own parallelism: quantum runs NumWorkers independent per-queue workers
(main.go:72-75, worker/outgoing.go:83-93); here the unit of independence is a GPU.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = 0x9E3779B97F4A7C15


def key_shard(key_idx, world: int) -> np.ndarray:
    """GPU that owns a packet with this key index: hash(key_idx) mod G.

    Keeping each peer's packets on one GPU keeps that GPU's key table to ~keys/G entries and keeps
    a flow's packets in order on one device."""
    k = np.asarray(key_idx, dtype=np.uint64)
    h = (k * np.uint64(_GOLDEN)) >> np.uint64(32)
    return (h % np.uint64(world)).astype(np.int64)


def packet_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of a single-key batch: sizes differ by at most one packet."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def partition_by_key(key_idx, world: int) -> list[np.ndarray]:
    """Packet indices per GPU for a keyed batch (stable order within each GPU)."""
    owner = key_shard(key_idx, world)
    return [np.nonzero(owner == g)[0] for g in range(world)]


def reduce_step_time(elapsed_s: float, ok: bool, dist=None, device=None) -> tuple[float, bool]:
    """Max elapsed time and AND of the per-rank status over all ranks (the bench contract)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return elapsed_s, ok
    import torch

    t = torch.tensor([elapsed_s, 0.0 if ok else 1.0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0].item()), t[1].item() == 0.0
