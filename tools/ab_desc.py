"""A/B the descriptor-batch kernel variants on the config-3 workload in ONE process, interleaved.

Each variant is its own qgcm context (QGCM_DESC_VARIANT is read at qgcm_create) with the same 1024
keys.  Correctness: every variant's sealed arena must equal the first variant's byte for byte.
Usage: python tools/ab_desc.py 7,10,8 [rounds]; an entry v:cN runs variant v with QGCM_DESC_CHUNK=N
(packets per sorted chunk), e.g. 7,7:c131072,7:c262144.  AB_KEYS=k draws key indices from k keys
(default 1024), AB_LEN=L gives every packet length L (default U{64..9000}), AB_ALIGN=A aligns every slot
to A bytes (default 4), AB_SHUFFLE=1 lists the descriptors in a random order,
AB_KEYSORTED=1 lays the slots out in (key, length descending) order.
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from quantum_amd import batch  # noqa: E402
from quantum_amd.crypto import Context  # noqa: E402

variants = (sys.argv[1] if len(sys.argv) > 1 else "7,10").split(",")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
N = 1 << 20
NUSE = int(os.environ.get("AB_KEYS", 1024))
NK = max(1024, NUSE)
FIXED_LEN = int(os.environ.get("AB_LEN", 0))
rng = np.random.default_rng(0x5EED0003)
keys = rng.bytes(32 * NK)
ctxs = {}
for v in variants:
    os.environ["QGCM_DESC_VARIANT"] = v.split(":")[0]
    os.environ["QGCM_DESC_CHUNK"] = v.split(":c")[1] if ":c" in v else "0"
    c = Context(device=0, max_keys=NK)
    c.set_keys(0, keys)
    ctxs[v] = c
lens = rng.integers(64, 9001, size=N, dtype=np.int64)
kidx = rng.integers(0, NUSE, size=N, dtype=np.int64)
if FIXED_LEN:
    lens[:] = FIXED_LEN
if int(os.environ.get("AB_KEYSORTED", 0)):  # lay the slots out in (key, length descending) order
    o = np.lexsort((-lens, kidx))
    lens, kidx = lens[o], kidx[o]
ALIGN = int(os.environ.get("AB_ALIGN", 4))  # slot alignment in bytes (4 = packed, as config 3)
slot = (4 + lens + 28 + ALIGN - 1) & ~(ALIGN - 1)
offs = np.zeros(N, dtype=np.int64)
offs[1:] = np.cumsum(slot)[:-1]
total = int(offs[-1] + slot[-1])
plain = torch.randint(0, 256, (total + 64,), dtype=torch.uint8, device="cuda")
arena = plain.clone()
nonces = torch.randint(0, 256, (12 * N,), dtype=torch.uint8, device="cuda")
status = torch.zeros(N, dtype=torch.uint8, device="cuda")
# AB_SHUFFLE=1: the descriptors in a random order (same slots): a tile then gathers scattered slots
order = np.random.default_rng(7).permutation(N) if int(os.environ.get("AB_SHUFFLE", 0)) else np.arange(N)
d_seal = batch.make_descs(offs[order], lens[order], kidx[order], "cuda")
d_open = batch.make_descs(offs[order], lens[order] + 28, kidx[order], "cuda")
ref = None
for v, c in ctxs.items():
    arena.copy_(plain)
    batch.seal_batch(c, arena, d_seal, N, nonces, status=status)
    ok = int(status.sum()) == N
    if ref is None:
        ref = arena.clone()
    same = bool(torch.equal(arena, ref))
    batch.open_batch(c, arena, d_open, N, status=status)
    rt = int(status.sum()) == N and bool(torch.equal(arena[:64], plain[:64]))
    print(f"variant {v}: status_ok={ok} same_as_first={same} roundtrip_ok={rt}", flush=True)
payload = int(lens.sum())
res = {v: ([], []) for v in variants}
for r in range(rounds + 1):
    for v, c in ctxs.items():
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        batch.seal_batch(c, arena, d_seal, N, nonces, status=status)
        e[1].record()
        batch.open_batch(c, arena, d_open, N, status=status)
        e[2].record()
        torch.cuda.synchronize()
        if r > 0:
            res[v][0].append(e[0].elapsed_time(e[1]))
            res[v][1].append(e[1].elapsed_time(e[2]))
for v in variants:
    s, o = statistics.median(res[v][0]), statistics.median(res[v][1])
    print(f"variant {v}: seal {s:.3f} ms  open {o:.3f} ms  -> {2 * payload / ((s + o) * 1e-3) / 2**30:.1f} GiB/s",
          flush=True)
