"""A/B whole builds of libqgcm on the config-5 chain (snappy -> seal, open -> uncompress over 2^20 x
1350 B pinned host slots) in ONE process, interleaved rounds: the chain is host-CPU sensitive and
boxes differ, so only same-process comparisons mean anything.  Every build must restore the input.
Usage: python tools/ab_libs_chain.py lib1.so lib2.so [...] [--rounds R] [--threads T]
"""
import ctypes as C
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402, F401  (shares its HIP runtime with the libraries)

from quantum_amd import _lib  # noqa: E402


def opt(name, default):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


rounds, threads = opt("--rounds", 3), opt("--threads", 16)
paths = [a for a in sys.argv[1:] if a.endswith(".so")]
N, L, stride = 1 << 20, 1350, 1472
libs = {}
for path in paths:
    lib = C.CDLL(os.path.abspath(path))
    _lib._bind(lib)
    err = C.create_string_buffer(_lib.ERRLEN)
    ctx = lib.qgcm_create(0, 4, err, _lib.ERRLEN)
    assert ctx, err.value
    key = C.create_string_buffer(32)
    assert lib.qgcm_derive_key(b"AES256Key-32Characters1234567890", 32, bytes(range(32)), 32, key) == 0
    assert lib.qgcm_set_key(ctx, 0, key.raw) == 0
    a_ptr, n_ptr = lib.qgcm_host_alloc(N * stride), lib.qgcm_host_alloc(12 * N)
    libs[path] = (lib, ctx, a_ptr, n_ptr)

rng = np.random.default_rng(0x5EED0005)
plain = np.zeros((N, stride), np.uint8)
plain[:, :4] = np.frombuffer(bytes([10, 99, 0, 1]), np.uint8)
half = L // 2
plain[:, 4:4 + half] = rng.integers(0, 256, (N, half), dtype=np.uint8)
line = np.frombuffer(b"GET /quantum/v1/peers HTTP/1.1\r\nHost: 10.99.0.1\r\n", np.uint8)
plain[:, 4 + half:4 + L] = np.tile(line, (L - half) // len(line) + 1)[:L - half]
nonce_bytes = rng.integers(0, 256, 12 * N, dtype=np.uint8)
res = {p: ([], []) for p in libs}
for r in range(rounds + 1):
    for path, (lib, ctx, a_ptr, n_ptr) in libs.items():
        host = np.frombuffer((C.c_uint8 * (N * stride)).from_address(a_ptr), np.uint8).reshape(N, stride)
        np.frombuffer((C.c_uint8 * (12 * N)).from_address(n_ptr), np.uint8)[:] = nonce_bytes
        host[:] = plain
        lens = np.full(N, L, np.uint32)
        t0 = time.perf_counter()
        b1 = lib.qgcm_compress_seal_host(ctx, a_ptr, stride, N, lens.ctypes.data, 0, n_ptr, 4, threads, None)
        t1 = time.perf_counter()
        b2 = lib.qgcm_open_uncompress_host(ctx, a_ptr, stride, N, lens.ctypes.data, 0, 4, threads, None)
        t2 = time.perf_counter()
        ok = b1 == 0 and b2 == 0 and bool((lens == L).all()) and np.array_equal(host[:, :4 + L], plain[:, :4 + L])
        if r == 0:
            print(f"{path}: round trip ok={ok}", flush=True)
        else:
            res[path][0].append(t1 - t0)
            res[path][1].append(t2 - t1)
for path in libs:
    s, o = statistics.median(res[path][0]), statistics.median(res[path][1])
    print(f"{path}: compress+seal {s * 1e3:.1f} ms  open+uncompress {o * 1e3:.1f} ms  -> "
          f"{2 * N * L / (s + o) / 2**30:.2f} GiB/s", flush=True)
