"""Does the launch pattern change config 2's speed?  Event records between launches, seal/open
alternation and the size of the allocation the arena lives in, in one process: none does (within
~1%).  (Written when a 64 M-packet batch looked ~12% faster per byte; that batch's synthetic fill had
stopped at 2^32 work items, leaving zero payloads and nonces -- fixed)
  alt     bench.py's step (seal, open) with three events per step
  noev    the same launches with one event pair around all steps
  runs    R seals back to back, then R opens
  big     'alt' on a config-2 arena carved from a --big-gb allocation
Usage: python tools/exp_batchsize.py [--steps 200] [--big-gb 90]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from quantum_amd import batch  # noqa: E402
from quantum_amd.crypto import Context, derive_key  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--steps", type=int, default=200)
p.add_argument("--big-gb", type=float, default=90.0)
args = p.parse_args()
N, L = 1 << 20, 1350
stride = batch.slot_stride(L, align=64)
ctx = Context(device=0, max_keys=4)
ctx.set_key(0, derive_key(b"AES256Key-32Characters1234567890", bytes(range(32))))
stream = torch.cuda.current_stream()
nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
status = torch.zeros(N, dtype=torch.uint8, device="cuda")


def make_arena(base: torch.Tensor) -> torch.Tensor:
    a = base[60:60 + N * stride]
    batch.fill_uniform(a, stride, N, L, 0x0100630A, 0x5EED0001, nonces, 0x5EED0002)
    return a


def seal(a):
    batch.seal_uniform(ctx, a, stride, N, L, 0, nonces, status=None, stream=stream)


def open_(a):
    batch.open_uniform(ctx, a, stride, N, L + 28, 0, status=status, stream=stream)


def gibs(ms_total: float, steps: int) -> float:
    return 2 * N * L * steps / (ms_total * 1e-3) / 2**30


def settle(a, ms=500):
    t = time.perf_counter()
    k = 0
    while (time.perf_counter() - t) * 1e3 < ms:
        seal(a)
        open_(a)
        k += 1
        if k % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()


def mode_alt(a):
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    for e in evs:
        e[0].record(stream)
        seal(a)
        e[1].record(stream)
        open_(a)
        e[2].record(stream)
    torch.cuda.synchronize()
    return gibs(sum(e[0].elapsed_time(e[2]) for e in evs), args.steps)


def mode_noev(a):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        seal(a)
        open_(a)
    e1.record(stream)
    torch.cuda.synchronize()
    return gibs(e0.elapsed_time(e1), args.steps)


def mode_runs(a):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        seal(a)
    for _ in range(args.steps):
        open_(a)
    e1.record(stream)
    torch.cuda.synchronize()
    return gibs(e0.elapsed_time(e1), args.steps)


small = make_arena(torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda"))
settle(small)
for rnd in range(2):
    print(f"round {rnd}: alt {mode_alt(small):.1f}  noev {mode_noev(small):.1f}  runs {mode_runs(small):.1f} GiB/s",
          flush=True)
# rotating: step k seals and opens arena k % R (a region is revisited only after R - 1 others)
rot = [make_arena(torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda")) for _ in range(16)]
for R in (1, 2, 4, 16):
    settle(rot[0])
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
    for k, e in enumerate(evs):
        e[0].record(stream)
        seal(rot[k % R])
        open_(rot[k % R])
        e[1].record(stream)
    torch.cuda.synchronize()
    print(f"rotating over {R} arenas: {gibs(sum(e[0].elapsed_time(e[1]) for e in evs), args.steps):.1f} GiB/s", flush=True)
# seal of arena k, then open of arena k-8 (a region is opened long after it was sealed)
evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
for k, e in enumerate(evs):
    e[0].record(stream)
    seal(rot[k % 16])
    open_(rot[(k + 8) % 16])
    e[1].record(stream)
torch.cuda.synchronize()
print(f"seal k, open k-8 of 16: {gibs(sum(e[0].elapsed_time(e[1]) for e in evs), args.steps):.1f} GiB/s (opens fail: "
      "those arenas were not sealed with these nonces; the work is the same)", flush=True)
del rot
big_alloc = torch.empty(int(args.big_gb * 1e9), dtype=torch.uint8, device="cuda")
for where in ("start", "end"):
    off = 0 if where == "start" else big_alloc.numel() - (N * stride + 64)
    big = make_arena(big_alloc[off:])
    settle(big)
    print(f"arena at the {where} of a {args.big_gb:.0f} GB allocation: alt {mode_alt(big):.1f}  "
          f"noev {mode_noev(big):.1f}  runs {mode_runs(big):.1f} GiB/s", flush=True)
settle(small)
print(f"small again: alt {mode_alt(small):.1f} GiB/s", flush=True)
