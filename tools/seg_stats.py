"""Per-workgroup statistics of the segmented descriptor kernel (variant 14) from a side build with
-DQGCM_SEG_STATS: phases, tiles, span, idle/busy wave time, table fills, and the end of each CU (both
its workgroups done) by XCC.
Usage: python tools/seg_stats.py path/to/libqgcm_stats.so   (AB_KEYS / AB_LEN as tools/ab_desc.py)
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from quantum_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
from quantum_amd import batch  # noqa: E402
from quantum_amd.crypto import Context  # noqa: E402

N, NK = 1 << 20, 1024
NUSE = int(os.environ.get("AB_KEYS", NK))
FIXED_LEN = int(os.environ.get("AB_LEN", 0))
rng = np.random.default_rng(0x5EED0003)
keys = rng.bytes(32 * NK)
os.environ["QGCM_DESC_VARIANT"] = "14"
ctx = Context(device=0, max_keys=NK)
ctx.set_keys(0, keys)
lens = rng.integers(64, 9001, size=N, dtype=np.int64)
kidx = rng.integers(0, NUSE, size=N, dtype=np.int64)
if FIXED_LEN:
    lens[:] = FIXED_LEN
slot = (4 + lens + 28 + 3) & ~3
offs = np.zeros(N, dtype=np.int64)
offs[1:] = np.cumsum(slot)[:-1]
arena = torch.randint(0, 256, (int(offs[-1] + slot[-1]) + 64,), dtype=torch.uint8, device="cuda")
nonces = torch.randint(0, 256, (12 * N,), dtype=torch.uint8, device="cuda")
d_seal = batch.make_descs(offs, lens, kidx, "cuda")
d_open = batch.make_descs(offs, lens + 28, kidx, "cuda")
L = _lib.lib()
L.qgcm_debug_seg_stats.argtypes = [C.c_void_p, C.c_int, C.c_int]
buf = np.zeros(4096 * 16, dtype=np.uint64)
for it in range(6):
    seal = it % 2 == 0
    L.qgcm_debug_seg_stats(buf.ctypes.data, buf.size, 1)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    if seal:
        batch.seal_batch(ctx, arena, d_seal, N, nonces)
    else:
        batch.open_batch(ctx, arena, d_open, N)
    e[1].record()
    torch.cuda.synchronize()
    L.qgcm_debug_seg_stats(buf.ctypes.data, buf.size, 0)
    st = buf.reshape(-1, 16).astype(np.int64)
    st = st[st[:, 2] > 0]
    span = (st[:, 3] - st[:, 2]) / 100.0  # us (100 MHz)
    t0 = st[:, 2].min()
    print(f"iter {it}: {'seal' if seal else 'open'} {e[0].elapsed_time(e[1]):.3f} ms, {len(st)} WGs, kernel span "
          f"{(st[:, 3].max() - t0) / 100:.0f} us; WG start spread {(st[:, 2].max() - t0) / 100:.0f} us; "
          f"WG span min/med/max {span.min():.0f}/{np.median(span):.0f}/{span.max():.0f} us")
    idle, busy = st[:, 4].sum(), st[:, 5].sum()
    print(f"  phases/WG min/med/max {st[:, 0].min()}/{int(np.median(st[:, 0]))}/{st[:, 0].max()}, "
          f"tiles/WG min/med/max "
          f"{st[:, 1].min()}/{int(np.median(st[:, 1]))}/{st[:, 1].max()}; wave idle {idle / (idle + busy):.3f} of wave "
          f"time; wave-0 run search {st[:, 7].sum() / 100 / len(st):.1f} us/WG", flush=True)
    homes = st[:, 6]
    print(f"  home runs: {len(np.unique(homes))} distinct, first 8 {homes[:8].tolist()}, max {homes.max()}")
    ends = np.sort((st[:, 3] - t0) / 100)
    print("  WG end times (us) deciles:", [int(x) for x in np.quantile(ends, [0, .1, .25, .5, .75, .9, 1])])
    xcc = st[:, 8] & 0xF
    cu = (xcc << 8) | ((st[:, 9] >> 8) & 0xFF)
    keys, inv = np.unique(cu, return_inverse=True)
    cend = np.array([st[inv == c, 3].max() for c in range(len(keys))]) - t0
    cx = np.array([xcc[inv == c][0] for c in range(len(keys))])
    print(f"  CUs {len(keys)}: CU idle at the end {float((cend.max() - cend).mean() / cend.max()):.4f} of the span; "
          "mean CU end per XCC (us):", [round(float(cend[cx == x].mean()) / 100) for x in np.unique(cx)],
          "tiles per XCC:", [int(st[xcc == x, 1].sum()) for x in np.unique(xcc)], flush=True)
