"""Config 5 (bench.extra_config5's workload, host packets, copies included) under the chain's codec
split knobs, one process: QGCM_CHAIN_DEV_AHEAD (seal), QGCM_CHAIN_DEV_BACKLOG (open), QGCM_CHAIN_SLOTS
and QGCM_CHAIN_CHUNK_MB are read at qgcm_create, so each setting gets a context of its own, timed in
turn, interleaved over `rounds`.

    python3 tools/exp_chain_policy.py [rounds] [chunks|slots]   (chunk size x codec threads, or chunks in
    flight x chunk size)
"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import bench  # noqa: E402
from quantum_amd import _lib, batch  # noqa: E402
from quantum_amd.crypto import Context  # noqa: E402


def main() -> None:
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    N, L, stride = 1 << 20, 1350, 1472
    key = bench.derive_key(bench.SECRET, bench.SALT)
    Lb = _lib.lib()
    a_ptr, n_ptr = Lb.qgcm_host_alloc(N * stride), Lb.qgcm_host_alloc(12 * N)
    host = np.frombuffer((C.c_uint8 * (N * stride)).from_address(a_ptr), np.uint8).reshape(N, stride)
    nons = np.frombuffer((C.c_uint8 * (12 * N)).from_address(n_ptr), np.uint8)
    host[:] = __import__("quantum_amd.workloads", fromlist=["W"]).config5_packets(N, L, stride)
    nons[:] = np.random.default_rng(1).integers(0, 256, 12 * N, dtype=np.uint8)
    plain = host[:, :4 + L].copy()
    lens = np.full(N, L, np.uint32)
    # (name, codec mode, QGCM_CHAIN_DEV_AHEAD, QGCM_CHAIN_DEV_BACKLOG, QGCM_CHAIN_CHUNK_MB, codec threads)
    slots = {}
    if len(sys.argv) > 2 and sys.argv[2] == "chunks":
        settings = [(f"c{mb}t{t}", 1, "2", "", str(mb), t) for mb in (16, 32, 64) for t in (14, 15, 16)]
    elif len(sys.argv) > 2 and sys.argv[2] == "slots":  # chunks in flight (QGCM_CHAIN_SLOTS) x chunk size
        settings = []
        for ns in (3, 4, 6, 8):
            for mb in (16, 32):
                settings.append((f"s{ns}c{mb}", 1, "2", "", str(mb), 16))
                slots[f"s{ns}c{mb}"] = str(ns)
        settings.append(("host_s6c16", 0, "2", "", "16", 16))
        slots["host_s6c16"] = "6"
    else:
        settings = [("host", 0, "2", "0", "32", 16), ("device", 2, "2", "", "32", 16),
                    ("ahead1", 1, "1", "999999", "32", 16),
                    ("ahead2", 1, "2", "999999", "32", 16), ("ahead3", 1, "3", "999999", "32", 16),
                    ("ahead4", 1, "4", "999999", "32", 16), ("back0", 1, "2", "0", "32", 16),
                    ("back45", 1, "2", "45", "32", 16), ("back90", 1, "2", "90", "32", 16),
                    ("back180", 1, "2", "180", "32", 16)]
    res = {name: {"seal": [], "open": [], "dev": []} for name, *_ in settings}
    for _ in range(rounds):
        for name, mode, ahead, back, mb, threads in settings:
            os.environ["QGCM_CHAIN_DEV_AHEAD"], os.environ["QGCM_CHAIN_CHUNK_MB"] = ahead, mb
            os.environ["QGCM_CHAIN_SLOTS"] = slots.get(name, "3")
            if back:
                os.environ["QGCM_CHAIN_DEV_BACKLOG"] = back
            else:
                os.environ.pop("QGCM_CHAIN_DEV_BACKLOG", None)
            ctx = Context(device=0, max_keys=4)
            ctx.set_key(0, key)
            batch.chain_codec(ctx, mode)
            c0 = ctx.launch_counts()
            lens[:] = L
            t0 = time.perf_counter()
            bad = batch.compress_seal_host(ctx, a_ptr, stride, N, lens, 0, n_ptr, threads=threads)
            t1 = time.perf_counter()
            bad += batch.open_uncompress_host(ctx, a_ptr, stride, N, lens, 0, threads=threads)
            t2 = time.perf_counter()
            c1 = ctx.launch_counts()
            assert bad == 0 and np.array_equal(host[:, :4 + L], plain), name
            res[name]["seal"].append(t1 - t0)
            res[name]["open"].append(t2 - t1)
            res[name]["dev"].append((c1["snappy_enc"] - c0["snappy_enc"], c1["snappy_dec"] - c0["snappy_dec"]))
            ctx.close()
    for name, r in res.items():
        s, o = float(np.median(r["seal"])), float(np.median(r["open"]))
        print(json.dumps({"setting": name, "value": round(2 * N * L / (s + o) / 2**30, 2),
                          "seal_ms": round(1e3 * s, 2), "open_ms": round(1e3 * o, 2), "device_chunks": r["dev"]}))


if __name__ == "__main__":
    main()
