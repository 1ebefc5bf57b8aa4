"""Writes tests/golden/config5_digest.json: BASELINE config 5 (the compression + encryption chain) at its
stated workload, 2^20 x 1350 B packets in 1472-B Payload.Raw slots (quantum_amd/workloads.py config5_*).

Outgoing, the chain runs plugin/compression.go:44-51 (snappy.Encode, copied into Raw[4:], Length
updated) and then plugin/encryption.go:24-30 (crypto/aes.go:41-52 Encrypt on the compressed packet),
in the order main.go:50-51 sorts them.  The expected bytes come from two independent implementations:
  * snappy: libsnappy 1.1.8 (/opt/conda/lib/libsnappy.so.1, in this image), cross-checked on a sample
    of packets against oracle/snappy_oracle.py (the plain-Python restatement of golang/snappy's
    block encoder, which golang/snappy is not in the reference to pin -- SURVEY.md s8c);
  * seal: OpenSSL 3 EVP aes-256-gcm with crypto/aes.go framing (oracle/ossl_check.c), its first
    packets cross-checked against the plain-C restatement (oracle/gcm_oracle.c).
A slot's bytes past its sealed record keep what compression.go's copy left there (the original
packet's tail), so the digest covers whole slots.

    python3 tests/golden/make_config5_golden.py
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from oracle import snappy_oracle as SO  # noqa: E402
from quantum_amd import workloads as W  # noqa: E402

TEST_SECRET = b"AES256Key-32Characters1234567890"
TEST_SALT = bytes(range(32))


def sha_chunks(a: np.ndarray) -> str:
    h = hashlib.sha256()
    flat = a.reshape(-1)
    for i in range(0, flat.size, 1 << 28):
        h.update(memoryview(flat[i:i + (1 << 28)]))
    return h.hexdigest()


def libsnappy():
    lib = C.CDLL("/opt/conda/lib/libsnappy.so.1")
    lib.snappy_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.POINTER(C.c_size_t)]
    lib.snappy_max_compressed_length.argtypes = [C.c_size_t]
    lib.snappy_max_compressed_length.restype = C.c_size_t
    return lib


def main() -> None:
    t0 = time.time()
    N, L, S = W.C5_N, W.C5_LEN, W.C5_STRIDE
    key = O.ossl_pbkdf2_sha512(TEST_SECRET, TEST_SALT)
    slots = W.config5_packets(N, L, S)
    plain_sha = sha_chunks(slots)
    nonces = W.config5_nonces(N)
    lib = libsnappy()
    cap = lib.snappy_max_compressed_length(L)
    buf = C.create_string_buffer(cap)
    m = C.c_size_t()
    clens = np.zeros(N, np.uint32)
    base = slots.ctypes.data
    for i in range(N):
        m.value = cap
        assert lib.snappy_compress(base + i * S + 4, L, buf, C.byref(m)) == 0
        c = m.value
        assert c + 28 <= S - 4, "compressed packet leaves no room for tag and nonce"
        C.memmove(base + i * S + 4, buf, c)
        clens[i] = c
    # the restatement of golang/snappy's encoder agrees with libsnappy on a sample of packets
    plain = W.config5_packets(64, L, S)  # the first 64 packets (same seeded stream)
    sample = list(range(64))
    for i in sample:
        want = SO.encode(bytes(plain[i, 4:4 + L]))
        assert bytes(slots[i, 4:4 + clens[i]]) == want, f"libsnappy != restatement at packet {i}"
    compressed_sha = sha_chunks(slots)
    offs = (np.arange(N, dtype=np.uint64) * np.uint64(S)).astype(np.uint64)
    kidx = np.zeros(N, np.uint32)
    check = 4096
    ref = slots[:check].copy()
    flat = slots.reshape(-1)
    O.ossl_seal_descs(key, flat, offs, clens, kidx, nonces, 4, os.cpu_count() or 1)
    O.aesgo_seal_descs(key, ref.reshape(-1), offs[:check].copy(), clens[:check].copy(), kidx[:check].copy(),
                       nonces, 4, 1)
    assert np.array_equal(ref, slots[:check]), "restatement != openssl on the config-5 prefix"
    sealed_sha = sha_chunks(slots)
    sealed_lens = clens + np.uint32(28)
    out = dict(n=N, len=L, stride=S, key=key.hex(), aad=W.AAD_WORD.to_bytes(4, "little").hex(),
               seed_payload=W.C5_SEED_PAYLOAD, seed_nonce=W.C5_SEED_NONCE,
               snappy="libsnappy 1.1.8 snappy_compress; oracle/snappy_oracle.py on packets 0..63",
               seal="OpenSSL 3 EVP aes-256-gcm, crypto/aes.go framing; oracle/gcm_oracle.c on packets 0..4095",
               sha256_plain=plain_sha, sha256_compressed=compressed_sha, sha256_sealed=sealed_sha,
               sha256_sealed_lens=hashlib.sha256(sealed_lens.astype("<u4").tobytes()).hexdigest(),
               sealed_bytes=int(sealed_lens.sum()), compressed_min=int(clens.min()), compressed_max=int(clens.max()),
               first_sealed_lens=[int(x) for x in sealed_lens[:8]])
    with open(os.path.join(HERE, "config5_digest.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(f"config5 golden written in {time.time() - t0:.1f} s: sealed/plain {out['sealed_bytes'] / (N * L):.4f}")


if __name__ == "__main__":
    main()
