"""Secondary BASELINE configs (bench.py measures the headline config 2):

  config3  2^20 packets, lengths ~ U{64..9000}, 1024 per-peer keys derived as common/mapping.go:90-99
           (X25519 twice + PBKDF2-HMAC-SHA512 x10000), key_idx ~ U[0,1024), AAD = the peer IP;
           device-resident descriptor batches (qgcm_seal_batch / qgcm_open_batch).
  e2e      config 2 from HOST memory: pinned staging + H2D + kernels + D2H (qgcm_seal_host /
           qgcm_open_host), the PCIe-inclusive rate DESIGN.md reports (never bench.py's value).
  config5  compression + encryption chain on 2^20 x 1350 B host packets (compressible mix: each
           packet's first half seeded random bytes, second half a repeated 48-B HTTP request line):
           snappy (host C++ codec, `threads` workers) -> seal, then open -> uncompress, pipelined
           with PCIe copies and the device (qgcm_compress_seal_host / qgcm_open_uncompress_host).

  config4_shard  one GPU's 8 x 2^20-packet shard of config 4 (64 x 2^20 x 1350 B over 8 GPUs).
  group_e2e      keyed host batches through the one-process multi-GPU dispatcher (qgcm_group_*):
                 2^20 x 1350 B, 64 keys, G member contexts (on the 1-GPU box all on device 0), pinned
                 host arena; the PCIe-inclusive rate of quantum's single process.

Prints one JSON line per config.  Usage: python tools/bench_configs.py [config3] [e2e] [config4_shard] ...
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from quantum_amd import _lib, batch  # noqa: E402
from quantum_amd.crypto import Context, derive_key  # noqa: E402


def config3(reps: int = 5) -> dict:
    """Config 3 on the parity-checked workload (quantum_amd/workloads.py), as bench.py's extra_configs."""
    import bench

    return dict(bench.extra_config3(reps=reps, verify=False), config="config3")


def e2e(reps: int = 3, pinned: bool = True) -> dict:
    """Config 2 from host memory through qgcm_seal_host/qgcm_open_host (pipelined chunks)."""
    if pinned:
        import bench

        return dict(bench.extra_e2e(derive_key(b"AES256Key-32Characters1234567890", bytes(range(32))), reps),
                    config="e2e_config2_host_memory", host_memory="pinned")
    N, L = 1 << 20, 1350
    stride = batch.slot_stride(L, align=64)
    ctx = Context(device=0, max_keys=4)
    ctx.set_key(0, derive_key(b"AES256Key-32Characters1234567890", bytes(range(32))))
    L_ = _lib.lib()
    dev = torch.zeros(N * stride, dtype=torch.uint8, device="cuda")
    non_d = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(dev, stride, N, L, 0x0100630a, 0x5EED0001, non_d, 0x5EED0002)
    host = bytearray(dev.cpu().numpy().tobytes())
    nonces = bytearray(non_d.cpu().numpy().tobytes())
    a_ptr, ka = batch.host_ptr(host)
    n_ptr, kn = batch.host_ptr(nonces)
    rc = 0
    ts, to = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        rc |= L_.qgcm_seal_host(ctx.handle, a_ptr, stride, N, L, 0, n_ptr, 4, None)
        t1 = time.perf_counter()
        rc |= L_.qgcm_open_host(ctx.handle, a_ptr, stride, N, L + 28, 0, 4, None)
        t2 = time.perf_counter()
        ts.append(t1 - t0)
        to.append(t2 - t1)
    s, o = float(np.median(ts)), float(np.median(to))
    del ka, kn
    ctx.close()
    return {"config": "e2e_config2_host_memory", "host_memory": "pageable", "packets": N, "payload_len": L,
            "value": round(2 * N * L / (s + o) / 2**30, 2), "unit": "GiB/s", "seal_s": round(s, 4),
            "open_s": round(o, 4), "status_ok": rc == 0}


def config5(reps: int = 3, threads: int = 16) -> dict:
    import bench

    return dict(bench.extra_config5(derive_key(b"AES256Key-32Characters1234567890", bytes(range(32))), threads,
                                    reps), config="config5_snappy_then_gcm_host")


def config4_shard(reps: int = 5, world: int = 8, rank: int = 0) -> dict:
    """One GPU's shard of config 4: 64 x 2^20 x 1350 B packets split over `world` GPUs by the
    contiguous single-key partition (quantum_amd.shard.packet_range), i.e. 8 x 2^20 packets
    (11.8 GB of slots) resident on this GPU.  The 8-GPU aggregate is the driver's N=8 bench run;
    this measures the per-GPU rate at config 4's per-GPU size, against which its efficiency is read.
    Parity at this size: sealed -> opened round trip of every packet (status) plus a spot check of
    the first 4096 slots against a 4096-packet reference batch sealed separately."""
    from quantum_amd import shard

    total, L = 64 << 20, 1350
    lo, hi = shard.packet_range(total, world, rank)
    N = hi - lo
    stride = batch.slot_stride(L, align=64)
    ctx = Context(device=0, max_keys=4)
    key = derive_key(b"AES256Key-32Characters1234567890", bytes(range(32)))
    ctx.set_key(0, key)
    alloc = torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda")
    arena = alloc[60:]
    nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
    status = torch.zeros(N, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(arena, stride, N, L, 0x0100630a, 0x5EED0001 + rank, nonces, 0x5EED0002 + rank)
    head = arena[:4096 * stride].clone()
    batch.seal_uniform(ctx, head, stride, 4096, L, 0, nonces[:12 * 4096])
    ts, to = [], []
    ok = True
    for r in range(reps + 1):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        batch.seal_uniform(ctx, arena, stride, N, L, 0, nonces)
        e[1].record()
        if r == 0:
            ok &= bool(torch.equal(arena[:4096 * stride], head))
        batch.open_uniform(ctx, arena, stride, N, L + 28, 0, status=status)
        e[2].record()
        torch.cuda.synchronize()
        ok &= int(status.sum()) == N
        if r > 0:
            ts.append(e[0].elapsed_time(e[1]))
            to.append(e[1].elapsed_time(e[2]))
    s, o = float(np.median(ts)), float(np.median(to))
    ctx.close()
    return {"config": "config4_per_gpu_shard", "world": world, "rank": rank, "packets_total": total,
            "packets_this_gpu": N, "payload_len": L, "slot_stride": stride,
            "arena_GB": round(N * stride / 1e9, 2), "value": round(2 * N * L / ((s + o) * 1e-3) / 2**30, 2),
            "unit": "GiB/s (this GPU)", "seal_ms": round(s, 3), "open_ms": round(o, 3), "status_ok": ok}


def group_e2e(G: int = 1, reps: int = 3) -> dict:
    from quantum_amd import shard

    N, L, NK = 1 << 20, 1350, 64
    stride = batch.slot_stride(L, align=64)
    rng = np.random.default_rng(0x5EED0006)
    grp = shard.Group([0] * G, max_keys=NK)
    grp.set_keys(0, rng.bytes(32 * NK))
    L_ = _lib.lib()
    a_ptr, n_ptr = L_.qgcm_host_alloc(N * stride), L_.qgcm_host_alloc(12 * N)
    host = np.frombuffer((C.c_uint8 * (N * stride)).from_address(a_ptr), np.uint8)
    nonces = np.frombuffer((C.c_uint8 * (12 * N)).from_address(n_ptr), np.uint8)
    host[:] = np.frombuffer(rng.bytes(N * stride), np.uint8)
    nonces[:] = np.frombuffer(rng.bytes(12 * N), np.uint8)
    offs = np.arange(N, dtype=np.int64) * stride
    kidx = rng.integers(0, NK, size=N)
    d_seal = shard.host_descs(offs, np.full(N, L), kidx)
    d_open = shard.host_descs(offs, np.full(N, L + 28), kidx)
    status = np.zeros(N, np.uint8)
    plain = host[:4096 * stride].copy()
    bad = grp.seal_host(a_ptr, d_seal, N, n_ptr, 4, status.ctypes.data)
    bad += grp.open_host(a_ptr, d_open, N, 4, status.ctypes.data)
    ok = bad == 0 and bool(np.array_equal(host[:4096 * stride].reshape(4096, stride)[:, :4 + L],
                                          plain.reshape(4096, stride)[:, :4 + L]))
    ts, to = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        bad += grp.seal_host(a_ptr, d_seal, N, n_ptr, 4, None)
        t1 = time.perf_counter()
        bad += grp.open_host(a_ptr, d_open, N, 4, None)
        t2 = time.perf_counter()
        ts.append(t1 - t0)
        to.append(t2 - t1)
    s, o = float(np.median(ts)), float(np.median(to))
    cpus = [grp.member_cpus(m) for m in range(G)]
    zc = grp.last_zerocopy()
    grp.close()
    del host, nonces
    L_.qgcm_host_free(a_ptr)
    L_.qgcm_host_free(n_ptr)
    return {"config": "group_e2e_keyed_host", "members": G, "devices": [0] * G, "packets": N, "payload_len": L,
            "keys": NK, "value": round(2 * N * L / (s + o) / 2**30, 2), "unit": "GiB/s", "seal_s": round(s, 4),
            "open_s": round(o, 4), "member_cpus": cpus, "zerocopy": zc,
            "copy_threads": int(os.environ.get("QGCM_GROUP_THREADS", "4")), "status_ok": ok and bad == 0}


if __name__ == "__main__":
    which = sys.argv[1:] or ["config3", "e2e", "e2e_pageable", "config5", "config4_shard"]
    runs = {"config3": config3, "e2e": e2e, "e2e_pageable": lambda: e2e(pinned=False), "config5": config5,
            "config4_shard": config4_shard, "group_e2e": group_e2e, "group_e2e2": lambda: group_e2e(2)}
    for w in which:
        print(json.dumps(runs[w]()), flush=True)
