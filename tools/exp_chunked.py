"""One 8 x 2^20-packet seal/open launch vs the same batch as eight 2^20-packet launches, interleaved in
one process (is the config-4 per-GPU gap the kernel's length or its size?).  Prints GiB/s and the
clock each form ran at (GRBM-free: from the time per packet against the 2^20-packet form)."""
import os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from quantum_amd import batch
from quantum_amd.crypto import Context, derive_key

N, L, C = int(sys.argv[2]) << 20 if len(sys.argv) > 2 else 8 << 20, 1350, int(sys.argv[1]) if len(sys.argv) > 1 else 8
stride = batch.slot_stride(L, align=64)
ctx = Context(0, 4)
ctx.set_key(0, derive_key(b"AES256Key-32Characters1234567890", bytes(range(32))))
alloc = torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda")
arena = alloc[60:]
nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
batch.fill_uniform(arena, stride, N, L, 0x0100630a, 0x5EED0001, nonces, 0x5EED0002)
n = N // C


def one():
    batch.seal_uniform(ctx, arena, stride, N, L, 0, nonces)
    batch.open_uniform(ctx, arena, stride, N, L + 28, 0)


def chunked():
    for c in range(C):
        a = arena[c * n * stride:(c + 1) * n * stride]
        batch.seal_uniform(ctx, a, stride, n, L, 0, nonces[12 * c * n:12 * (c + 1) * n])
    for c in range(C):
        a = arena[c * n * stride:(c + 1) * n * stride]
        batch.open_uniform(ctx, a, stride, n, L + 28, 0)


res = {"one": [], "chunked": []}
for r in range(8):
    for name, f in (("one", one), ("chunked", chunked)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(2):
            f()  # back to back, as a sustained load
        e0.record(); f(); f(); e1.record(); torch.cuda.synchronize()
        if r:
            res[name].append(e0.elapsed_time(e1) / 2)
for name, v in res.items():
    ms = statistics.median(v)
    print(f"{name:8s} ({C} chunks)" if name == "chunked" else f"{name:8s}", f"{ms:.2f} ms per seal+open  ->",
          f"{2 * N * L / (ms * 1e-3) / 2**30:.1f} GiB/s", flush=True)
