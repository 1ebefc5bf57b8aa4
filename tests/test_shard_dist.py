"""CPU: multi-GPU sharding logic and the cross-rank reduction, world_size 2 over gloo."""
import os
import socket

import numpy as np
import pytest

from quantum_amd import shard


def test_packet_range_covers_disjointly():
    for n in (0, 1, 7, 1 << 20, (1 << 20) + 3):
        for world in (1, 2, 3, 8):
            spans = [shard.packet_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and b >= a
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.packet_range(10, 2, 2)


def test_key_partition_is_a_function_of_key():
    rng = np.random.default_rng(1)
    keys = rng.integers(0, 1024, size=100_000)
    parts = shard.partition_by_key(keys, 8)
    allidx = np.sort(np.concatenate(parts))
    assert np.array_equal(allidx, np.arange(len(keys)))
    for g, idx in enumerate(parts):
        assert np.all(shard.key_shard(keys[idx], 8) == g)  # every packet of a key on one GPU
    per_gpu_keys = [len(np.unique(keys[idx])) for idx in parts]
    assert sum(per_gpu_keys) == len(np.unique(keys))  # key tables are disjoint
    assert min(len(p) for p in parts) > 0.5 * len(keys) / 8  # not degenerate


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard.packet_range(1000, world, rank)
        t, ok = shard.reduce_step_time(0.5 + rank, rank != 1 or True, dist)
        t2, ok2 = shard.reduce_step_time(1.0, rank == 0, dist)  # rank 1 reports failure
        per = shard.gather_rank_stats([rank, 0.25 * (rank + 1), hi - lo], dist)
        dist.barrier()
        q.put((rank, lo, hi, t, ok, t2, ok2, per))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_reduction():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, lo0, hi0, t0, ok0, t20, ok20, p0), (r1, lo1, hi1, t1, ok1, t21, ok21, p1) = res
    assert (lo0, hi0, lo1, hi1) == (0, 500, 500, 1000)
    assert t0 == t1 == 1.5 and ok0 and ok1  # max over ranks, all ok
    assert t20 == t21 == 1.0 and not ok20 and not ok21  # one failing rank fails the step
    assert p0 == p1 == [[0.0, 0.25, 500.0], [1.0, 0.5, 500.0]]  # every rank's own figures, in rank order
    assert shard.gather_rank_stats([1, 2]) == [[1.0, 2.0]]  # no process group: this rank only
