"""Per-launch fixed cost of the quad kernel (LDS table fill + ramp): seal time of uniform batches of
1, 2, 3, 4 full passes of the persistent grid (2^17 packets per pass: 512 workgroups x 16 waves x 16
packets), median of interleaved repeats; fixed cost = intercept of time vs passes."""
import os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from quantum_amd import batch
from quantum_amd.crypto import Context, derive_key

L = 1350
stride = batch.slot_stride(L, align=64)
ctx = Context(0, 4)
ctx.set_key(0, derive_key(b"AES256Key-32Characters1234567890", bytes(range(32))))
N = 4 << 17
alloc = torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda")
arena = alloc[60:]
nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
batch.fill_uniform(arena, stride, N, L, 0x0100630a, 0x5EED0001, nonces, 0x5EED0002)
res = {p: [] for p in (1, 2, 3, 4)}
for r in range(12):
    for p in res:
        n = p << 17
        for _ in range(3):
            batch.seal_uniform(ctx, arena, stride, n, L, 0, nonces)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            batch.seal_uniform(ctx, arena, stride, n, L, 0, nonces)
        e1.record()
        torch.cuda.synchronize()
        if r:
            res[p].append(e0.elapsed_time(e1) / 5 * 1e3)
xs, ys = list(res), [statistics.median(v) for v in res.values()]
mx, my = statistics.mean(xs), statistics.mean(ys)
slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
for x, y in zip(xs, ys):
    print(f"passes {x}: {y:.1f} us per seal launch", flush=True)
print(f"per pass {slope:.1f} us, fixed per launch {my - slope * mx:.1f} us", flush=True)
