"""Config 2 (2^20 x 1350 B, seal + open per step) on arenas from different allocations, interleaved in
one process: does where the arena lives change the kernel's speed?  (It does not: 853-856 GiB/s for
all but the physically contiguous allocation, 844.  Batches past ~12.6 M slots had looked ~13% faster
only because the synthetic fill then stopped at 2^32 work items and left zero payloads and nonces;
DESIGN.md 4.1.)
  torch        torch.zeros (the caching allocator -> hipMalloc), as bench.py
  hipMalloc    hipMalloc of exactly the arena
  contiguous   hipExtMallocWithFlags(hipDeviceMallocContiguous)
  big@0 / big@14G   offset 0 / 14 GB of one 16-GB torch allocation
Usage: python tools/exp_alloc.py [--rounds 3]
"""
import argparse
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from quantum_amd import _lib, batch  # noqa: E402
from quantum_amd.crypto import Context, derive_key  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rounds", type=int, default=3)
p.add_argument("--steps", type=int, default=100)
args = p.parse_args()
N, L = 1 << 20, 1350
stride = batch.slot_stride(L, align=64)
SIZE = N * stride + 64
hip = C.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
ctx = Context(device=0, max_keys=4)
ctx.set_key(0, derive_key(b"AES256Key-32Characters1234567890", bytes(range(32))))
stream = torch.cuda.current_stream()
lib = _lib.lib()
nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
status = torch.zeros(N, dtype=torch.uint8, device="cuda")


def raw(flags=None) -> int:
    ptr = C.c_void_p()
    rc = hip.hipMalloc(C.byref(ptr), SIZE) if flags is None else hip.hipExtMallocWithFlags(C.byref(ptr), SIZE, flags)
    assert rc == 0, f"hip alloc rc={rc}"
    return ptr.value


keep = []
t_small = torch.zeros(SIZE, dtype=torch.uint8, device="cuda")
big = torch.zeros(16 << 30, dtype=torch.uint8, device="cuda")
keep += [t_small, big]
arenas = {"torch": t_small.data_ptr(), "hipMalloc": raw(), "contiguous": raw(0x4),
          "big@0": big.data_ptr(), "big@14G": big.data_ptr() + (14 << 30)}
for name, ptr in arenas.items():
    lib.qgcm_fill_uniform(C.c_void_p(ptr + 60), stride, N, L, 0x0100630A, 0x5EED0001, C.c_void_p(nonces.data_ptr()),
                          0x5EED0002, C.c_void_p(stream.cuda_stream))
h = stream.cuda_stream


def steps(ptr: int, k: int) -> float:
    a = C.c_void_p(ptr + 60)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(k):
        assert lib.qgcm_seal_uniform(ctx.handle, a, stride, N, L, 0, C.c_void_p(nonces.data_ptr()), 4, None,
                                     C.c_void_p(h)) == 0
        assert lib.qgcm_open_uniform(ctx.handle, a, stride, N, L + 28, 0, 4, C.c_void_p(status.data_ptr()),
                                     C.c_void_p(h)) == 0
    e1.record(stream)
    torch.cuda.synchronize()
    assert int(status.sum()) == N
    return 2 * N * L * k / (e0.elapsed_time(e1) * 1e-3) / 2**30


t = time.perf_counter()
while time.perf_counter() - t < 1.0:
    steps(arenas["torch"], 8)
for r in range(args.rounds):
    print(f"round {r}: " + "  ".join(f"{n} {steps(ptr, args.steps):.1f}" for n, ptr in arenas.items()) + " GiB/s",
          flush=True)
