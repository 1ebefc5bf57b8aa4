"""Small keyed batches: qgcm_group_seal_host / open_host (one member, pinned arena, 64 keys, 1350 B)
with the worklist built in one workgroup (QGCM_SMALL_WORKLIST=1, the default up to 4096 packets) or by
the multi-launch radix-sort path (0), alternating in one process: median microseconds per seal+open pair.
The knob is read at qgcm_group_create, so each setting has a group of its own, created after the
environment variable is set (as tests/test_gpu_fuzz.py's fuzz_ctxs does).

    python3 tools/exp_small_worklist.py [reps]
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


def main() -> None:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    L, stride, nmax = 1350, 1472, 4096
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 256, 64 * 32, dtype=np.uint8).tobytes()
    grps = {}
    for small in ("1", "0"):
        os.environ["QGCM_SMALL_WORKLIST"] = small
        grps[small] = shard.Group([0], max_keys=64)
        grps[small].set_keys(0, keys)
    os.environ.pop("QGCM_SMALL_WORKLIST", None)
    Lb = _lib.lib()
    a_ptr, n_ptr = Lb.qgcm_host_alloc(nmax * stride), Lb.qgcm_host_alloc(12 * nmax)
    host = np.frombuffer((C.c_uint8 * (nmax * stride)).from_address(a_ptr), np.uint8)
    host[:] = rng.integers(0, 256, host.size, dtype=np.uint8)
    Lb.qgcm_random_nonces(n_ptr, nmax)
    for n in (64, 256, 1024, 4096):
        kidx = rng.integers(0, 64, n).astype(np.uint32)
        offs = np.arange(n, dtype=np.uint64) * stride
        d_seal = shard.host_descs(offs, np.full(n, L, np.uint32), kidx)
        d_open = shard.host_descs(offs, np.full(n, L + 28, np.uint32), kidx)
        res = {"1": [], "0": []}
        for r in range(reps + 3):
            for small, grp in grps.items():
                t0 = time.perf_counter()
                bad = grp.seal_host(a_ptr, d_seal, n, n_ptr, 4) + grp.open_host(a_ptr, d_open, n, 4)
                if r >= 3:
                    res[small].append(time.perf_counter() - t0)
                assert bad == 0
        print(json.dumps({"packets": n, "pair_us_small": round(statistics.median(res["1"]) * 1e6, 1),
                          "pair_us_multilaunch": round(statistics.median(res["0"]) * 1e6, 1)}), flush=True)
    Lb.qgcm_host_free(a_ptr)
    Lb.qgcm_host_free(n_ptr)
    for grp in grps.values():
        grp.close()


if __name__ == "__main__":
    main()
