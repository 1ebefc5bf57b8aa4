"""CPU baseline scaling on the GPU box's host: OpenSSL AES-256-GCM seal+open of 1350-B packets with
crypto/aes.go semantics, at 1..T threads, with the per-packet getrandom nonce (mode 0, the reference)
and with counter nonces (mode 1), to see what limits the all-thread figure bench.py reports."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402

key, L = bytes(range(32)), 1350
for mode in (0, 1):
    for t in [1, 2, 4, 8, 16, 32]:
        n = 150000
        wall = O.ossl_cpu_baseline(key, t, n, L, mode)
        print(json.dumps({"mode": ["getrandom", "counter"][mode], "threads": t, "packets_per_thread": n,
                          "wall_s": round(wall, 3), "GiBps": round(2 * t * n * L / wall / 2**30, 3)}), flush=True)
