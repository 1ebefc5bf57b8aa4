"""Per-call latency of the drop-in per-packet path (qgcm_seal_one / qgcm_open_one, the form
crypto/aes.go:41-62 Encrypt/Decrypt take behind plugin/encryption.go:16-40 Apply).
Prints one JSON line per payload length: median / p90 microseconds per seal and per open call,
and checks every round trip.  Run under rocprofv3 --kernel-trace --stats to split kernel time
from the launch + synchronize overhead."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from quantum_amd import crypto  # noqa: E402


def main() -> None:
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    key = crypto.derive_key(b"AES256Key-32Characters1234567890", bytes(range(32)))
    aes = crypto.AES(key)
    aad = bytes([10, 99, 0, 1])
    for L in (64, 1350, 9000):
        plain = bytes((i * 131 + 7) & 255 for i in range(L))
        ts, to = [], []
        for _ in range(calls):
            buf = bytearray(plain + bytes(28))
            t0 = time.perf_counter()
            n, err = aes.Encrypt(buf, L, aad)
            t1 = time.perf_counter()
            assert err is None and n == L + 28
            m, err = aes.Decrypt(buf, aad)
            t2 = time.perf_counter()
            assert err is None and m == L and bytes(buf[:L]) == plain
            ts.append(t1 - t0)
            to.append(t2 - t1)
        ts.sort()
        to.sort()
        print(json.dumps({"len": L, "calls": calls,
                          "seal_us_median": round(ts[len(ts) // 2] * 1e6, 1),
                          "seal_us_p90": round(ts[int(len(ts) * 0.9)] * 1e6, 1),
                          "open_us_median": round(to[len(to) // 2] * 1e6, 1),
                          "open_us_p90": round(to[int(len(to) * 0.9)] * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
