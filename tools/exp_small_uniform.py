"""Latency of small device-resident uniform batches (qgcm_seal_uniform / qgcm_open_uniform, 1350 B)
through the latency kernel (the default up to 256 packets; QGCM_ONE_UNIFORM_MAX raises the cut-off
here) and through the quad batch kernel (QGCM_VARIANT=12 forces it), in one process: one JSON line per batch size with the median microseconds per call."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from quantum_amd import batch  # noqa: E402
from quantum_amd.crypto import Context  # noqa: E402

L = 1350
key = bytes(range(32))
ctxs = {}
os.environ["QGCM_ONE_UNIFORM_MAX"] = "1000000"  # measure the latency kernel past its default cut-off
for name, env in (("one_kernel", None), ("quad", "12")):
    if env:
        os.environ["QGCM_VARIANT"] = env
    c = Context(device=0, max_keys=2)
    c.set_key(0, key)
    ctxs[name] = c
    os.environ.pop("QGCM_VARIANT", None)
os.environ.pop("QGCM_ONE_UNIFORM_MAX")
stride = batch.slot_stride(L)
for n in (1, 16, 64, 256, 512, 1024, 2048, 4096, 8192):
    arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(arena, stride, n, L, 0x0100630a, 1, nonces, 2)
    out = {"n": n, "len": L}
    for name, c in ctxs.items():
        ts = []
        for _ in range(200):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            batch.seal_uniform(c, arena, stride, n, L, 0, nonces)
            batch.open_uniform(c, arena, stride, n, L + 28, 0)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name + "_us_seal_open"] = round(statistics.median(ts) * 1e6, 1)
    print(json.dumps(out), flush=True)
