"""Deterministic snappy test inputs (shared by tests/golden/make_snappy_golden.py, tests/test_snappy.py
and the GPU codec tests): every case is regenerated from its name, so the golden file holds only the
expected outputs (libsnappy 1.1.8's bytes, see oracle/snappy_oracle.py)."""
from __future__ import annotations

import numpy as np

from quantum_amd.workloads import stream_bytes

LINE = b"GET /quantum/v1/peers HTTP/1.1\r\nHost: 10.99.0.1\r\n"  # bench.py extra_config5's line
WORDS = [b"GET ", b"/index.html", b" HTTP/1.1\r\n", b"Host: 10.99.0.1\r\n", b"\x00\x00", b"quantum "]
LENGTHS = [0, 1, 2, 3, 4, 5, 15, 16, 17, 18, 19, 20, 31, 32, 33, 59, 60, 61, 63, 64, 65, 67, 68, 69, 127, 128,
           255, 256, 257, 1349, 1350, 1351, 1433, 2047, 2048, 2049, 4096, 9000, 16384, 16385, 65535, 65536,
           65537, 70000, 140000]
KINDS = ["zeros", "random", "line", "half", "words", "runs"]


def make(kind: str, n: int, seed: int = 0) -> bytes:
    """Input of `n` bytes: zeros, splitmix64 bytes, a repeated HTTP line, config 5's packet (first half
    random, second half the line), a word salad with back-references, or byte runs."""
    s = 0x5EED5A00 + 131 * seed + n
    if kind == "zeros":
        return bytes(n)
    if kind == "random":
        return stream_bytes(s, 0, n)
    if kind == "line":
        return (LINE * (n // len(LINE) + 1))[:n]
    if kind == "half":
        h = n // 2
        return stream_bytes(s, 0, h) + (LINE * (n // len(LINE) + 1))[:n - h]
    r = np.frombuffer(stream_bytes(s, 0, 8 * (n + 8)), dtype="<u8")
    out = bytearray()
    k = 0
    while len(out) < n:
        v = int(r[k % len(r)])
        k += 1
        if kind == "runs":
            out += bytes([v & 0xFF]) * (1 + (v >> 8) % 90)
        elif v % 10 < 4:
            out += WORDS[(v >> 8) % len(WORDS)]
        elif v % 10 < 7 and out:
            a = (v >> 8) % len(out)
            out += out[a:a + 1 + (v >> 32) % 80]
        else:
            out += stream_bytes(s + k, 0, 1 + (v >> 8) % 40)
    return bytes(out[:n])


def cases() -> list[tuple[str, int]]:
    return [(k, n) for k in KINDS for n in LENGTHS]
