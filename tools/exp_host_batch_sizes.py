"""Worker-sized host batches: qgcm_seal_host + qgcm_open_host round trips on a pinned arena of n
Payload.Raw slots (1350 B, 1472-B stride), and the same through a one-member group
(qgcm_group_seal_host / open_host), for n from one recvmmsg batch (64) up to 2^18: median microseconds
per seal+open pair and the payload rate, so a batched worker can pick its batch size.

    python3 tools/exp_host_batch_sizes.py [reps] [sizes, comma-separated]
"""
import ctypes as C
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from quantum_amd import _lib, shard  # noqa: E402
from quantum_amd.crypto import Context  # noqa: E402


def main() -> None:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    L, stride, nmax = 1350, 1472, 1 << 18
    key = bytes(range(32))
    ctx = Context(device=0, max_keys=2)
    ctx.set_key(0, key)
    grp = shard.Group([0], max_keys=2)
    grp.set_keys(0, key)
    Lb = _lib.lib()
    a_ptr, n_ptr = Lb.qgcm_host_alloc(nmax * stride), Lb.qgcm_host_alloc(12 * nmax)
    host = np.frombuffer((C.c_uint8 * (nmax * stride)).from_address(a_ptr), np.uint8)
    host[:] = np.random.default_rng(1).integers(0, 256, host.size, dtype=np.uint8)
    Lb.qgcm_random_nonces(n_ptr, nmax)
    sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [64, 256, 1024, 4096, 16384, 65536, nmax]
    for n in sizes:
        d_seal = shard.host_descs(np.arange(n, dtype=np.uint64) * stride, np.full(n, L, np.uint32),
                                  np.zeros(n, np.uint32))
        d_open = shard.host_descs(np.arange(n, dtype=np.uint64) * stride, np.full(n, L + 28, np.uint32),
                                  np.zeros(n, np.uint32))
        for path in ("host", "group"):
            ts = []
            for r in range(reps + 3):
                t0 = time.perf_counter()
                if path == "host":
                    bad = Lb.qgcm_seal_host(ctx.handle, a_ptr, stride, n, L, 0, n_ptr, 4, None)
                    bad += Lb.qgcm_open_host(ctx.handle, a_ptr, stride, n, L + 28, 0, 4, None)
                else:
                    bad = grp.seal_host(a_ptr, d_seal, n, n_ptr, 4)
                    bad += grp.open_host(a_ptr, d_open, n, 4)
                if r >= 3:
                    ts.append(time.perf_counter() - t0)
                assert bad == 0, (path, n, bad)
            us = statistics.median(ts) * 1e6
            print(json.dumps({"path": path, "packets": n, "pair_us": round(us, 1),
                              "GiB_s": round(2 * n * L / (us * 1e-6) / 2**30, 2),
                              "member_path": grp.last_path(0) if path == "group" else "seal_host"}), flush=True)
    Lb.qgcm_host_free(a_ptr)
    Lb.qgcm_host_free(n_ptr)
    grp.close()
    ctx.close()


if __name__ == "__main__":
    main()
