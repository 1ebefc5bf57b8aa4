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


def gather_rank_stats(values, dist=None, device=None) -> list[list[float]]:
    """Every rank's scalar measurements (its own step time, kernel times, packets), in rank order --
    the per-GPU figures of a multi-GPU line.  One small all_gather after the
    timed region; without a process group, [values]."""
    vals = [float(v) for v in values]
    if dist is None or not dist.is_initialized():
        return [vals]
    import torch

    t = torch.tensor(vals, dtype=torch.float64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[float(x) for x in o.cpu().tolist()] for o in out]


class Group:
    """Several GPUs behind one process (qgcm_group_*, include/qgcm.h): quantum is one process
    (main.go:29-114) whose workers all call one Encryption plugin, so its drop-in drives every GPU of a
    node from that process.  Keyed host batches are split by key_shard over the member contexts (one
    host thread and stream set per member, no collective); results land in the caller's slots."""

    def __init__(self, devices, max_keys: int = 4096):
        import ctypes as C

        from . import _lib

        devs = (C.c_int * len(devices))(*devices)
        err = C.create_string_buffer(_lib.ERRLEN)
        h = _lib.lib().qgcm_group_create(devs, len(devices), max_keys, err, _lib.ERRLEN)
        if not h:
            raise _lib.QgcmError(f"qgcm_group_create({list(devices)}): {err.value.decode()}")
        self.handle, self.devices, self.max_keys = h, list(devices), max_keys
        self._views = []  # weak references to the member contexts handed out

    def member(self, m: int):
        """Member m's device context (borrowed: the group owns it) for device batches on it.  The view
        keeps the group alive; closing the group invalidates it (its handle becomes None)."""
        import weakref

        from . import _lib
        from .crypto import Context

        if not self.handle:
            raise _lib.QgcmError("group is closed")
        h = _lib.lib().qgcm_group_ctx(self.handle, m)
        if not h:
            raise _lib.QgcmError(f"no member {m}")
        c = Context.borrowed(h, self.devices[m], self.max_keys, owner=self)
        self._views.append(weakref.ref(c))
        return c

    def shard(self, key_idx: int) -> int:
        from . import _lib

        return _lib.check(_lib.lib().qgcm_group_shard(self.handle, key_idx), "qgcm_group_shard")

    def member_cpus(self, m: int) -> int:
        """CPUs member m's host thread is pinned to (its GPU's NUMA-local CPUs; 0 = not pinned)."""
        from . import _lib

        return _lib.check(_lib.lib().qgcm_group_member_cpus(self.handle, m), "qgcm_group_member_cpus")

    def last_path(self, m: int) -> str:
        """How member m moved its records in the last seal_host / open_host call: "copy" (host gather and
        scatter through pinned staging), "zerocopy" (its GPU gathers over PCIe), "dma" (whole runs of
        adjacent records, one DMA each way) or "direct" (a worker-sized batch of 16-B-aligned records in a
        pinned arena, sealed in place over PCIe by one workgroup per packet)."""
        from . import _lib

        code = _lib.check(_lib.lib().qgcm_group_last_path(self.handle, m), "qgcm_group_last_path")
        return ("copy", "zerocopy", "dma", "direct")[code]

    def order(self, key_idx) -> tuple[np.ndarray, np.ndarray]:
        """qgcm_group_order: the input indices member by member (stable) and each member's count -- the
        layout in which a keyed batch takes the DMA-run path."""
        from . import _lib

        k = np.ascontiguousarray(key_idx, dtype=np.uint32)
        order = np.empty(len(k), np.uint32)
        counts = np.empty(len(self.devices), np.uint32)
        _lib.check(_lib.lib().qgcm_group_order(self.handle, k.ctypes.data, len(k), order.ctypes.data,
                                               counts.ctypes.data), "qgcm_group_order")
        return order, counts

    def last_zerocopy(self) -> bool:
        """True if the last seal_host / open_host call ran the zero-copy path (pinned arena)."""
        from . import _lib

        return _lib.check(_lib.lib().qgcm_group_last_zerocopy(self.handle), "qgcm_group_last_zerocopy") == 1

    def set_keys(self, first: int, keys: bytes) -> None:
        from . import _lib

        _lib.check(_lib.lib().qgcm_group_set_keys(self.handle, first, len(keys) // 32, keys), "qgcm_group_set_keys")

    def _run(self, seal: bool, arena_ptr: int, descs, n: int, nonces_ptr, aad_len: int, status_ptr) -> int:
        from . import _lib

        L = _lib.lib()
        d = descs.ctypes.data if hasattr(descs, "ctypes") else descs
        rc = (L.qgcm_group_seal_host(self.handle, arena_ptr, d, n, nonces_ptr, aad_len, status_ptr) if seal else
              L.qgcm_group_open_host(self.handle, arena_ptr, d, n, aad_len, status_ptr))
        return _lib.check(rc, "qgcm_group_seal_host" if seal else "qgcm_group_open_host")

    def seal_host(self, arena_ptr: int, descs, n: int, nonces_ptr=None, aad_len: int = 4, status_ptr=None) -> int:
        """descs: numpy structured/uint8 array of qgcm_desc records (host).  Returns failed packets."""
        return self._run(True, arena_ptr, descs, n, nonces_ptr, aad_len, status_ptr)

    def open_host(self, arena_ptr: int, descs, n: int, aad_len: int = 4, status_ptr=None) -> int:
        return self._run(False, arena_ptr, descs, n, None, aad_len, status_ptr)

    def close(self) -> None:
        from . import _lib

        if self.handle:
            for ref in self._views:  # borrowed member contexts must not outlive the members
                c = ref()
                if c is not None:
                    c.handle = None
                    c._owner = None
            self._views = []
            _lib.lib().qgcm_group_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def host_descs(offsets, lengths, keys) -> np.ndarray:
    """qgcm_desc records {u64 offset, u32 len, u32 key_idx} as a host numpy array."""
    dt = np.dtype([("offset", "<u8"), ("len", "<u4"), ("key_idx", "<u4")])
    d = np.zeros(len(offsets), dtype=dt)
    d["offset"], d["len"], d["key_idx"] = offsets, lengths, keys
    return d
