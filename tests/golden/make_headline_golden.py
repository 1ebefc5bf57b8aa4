"""Golden digests of bench.py's headline layout (BASELINE config 2 exactly as the driver times it).

bench.py seals and opens 2^20 x 1350-B packets in 1408-B Payload.Raw slots (the smallest 64-B multiple
that holds 4 + 1350 + 28 B) whose arena starts 60 B into a 64-B-aligned allocation, so every payload
(Raw[4:]) is 64-B aligned and the quad kernel moves whole 64-B granules.  The fill is
qgcm_fill_uniform's (AAD 0a630001, splitmix64 payloads / nonces from seeds 0x5EED0001 / 0x5EED0002,
zeroed gaps): the bytes depend only on the arena offset, not on where the allocation sits, so the
digests below pin the arena the bench hashes after its timed loop.

  sha256_plain   the filled arena (what every timed open returns to, apart from the tails)
  sha256_sealed  after one seal (crypto/aes.go:41-52: ct in place, tag at [4+L, 4+L+16), nonce after)
  sha256_opened  after seal then open: the plaintext back, tag || nonce left in each slot
                 (crypto/aes.go:60 opens data[:length]; Open never writes the tail)

The sealed arena is computed twice and asserted equal: by the C restatement (oracle/gcm_oracle.c,
FIPS-197 + SP 800-38D bit-serial GHASH + the crypto/aes.go framing) over EVERY packet, and by
OpenSSL 3 EVP aes-256-gcm (oracle/ossl_check.c).  Under a minute on 8 threads.

  python tests/golden/make_headline_golden.py   ->  tests/golden/headline_digest.json
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from oracle import oracle as O  # noqa: E402
import make_golden as G  # noqa: E402

N, L, STRIDE, ARENA_OFFSET = 1 << 20, 1350, 1408, 60


def sha(a: np.ndarray) -> str:
    return G.sha_chunks(a)


def main() -> None:
    threads = int(os.environ.get("THREADS", "8"))
    key = bytes.fromhex(json.load(open(os.path.join(HERE, "aesgo.json")))["key"])
    arena, nonces = G.batch_arena(N, L, STRIDE)
    plain_sha = sha(arena)
    offs = np.arange(N, dtype=np.uint64) * np.uint64(STRIDE)
    lens = np.full(N, L, dtype=np.uint32)
    kidx = np.zeros(N, dtype=np.uint32)
    t0 = time.time()
    ref = arena.copy()
    O.aesgo_seal_descs(key, ref, offs, lens, kidx, nonces, 4, threads)  # restatement, every packet
    t1 = time.time()
    O.ossl_seal_uniform(key, arena.ctypes.data, STRIDE, N, L, 4, nonces.ctypes.data)  # OpenSSL
    assert np.array_equal(ref, arena), "restatement != OpenSSL on the headline arena"
    del ref
    sealed_sha = sha(arena)
    opened, _ = G.batch_arena(N, L, STRIDE)
    view_o, view_s = opened.reshape(N, STRIDE), arena.reshape(N, STRIDE)
    view_o[:, 4 + L:4 + L + 28] = view_s[:, 4 + L:4 + L + 28]
    out = dict(n=N, len=L, stride=STRIDE, arena_offset_in_64B_allocation=ARENA_OFFSET, payload_align=64,
               aad=G.h(G.AAD), key_sha256=hashlib.sha256(key).hexdigest(),
               seed_payload=G.SEED_PAYLOAD, seed_nonce=G.SEED_NONCE,
               sha256_plain=plain_sha, sha256_sealed=sealed_sha, sha256_opened=sha(opened),
               oracle_checked_prefix=N, openssl_checked=N,
               note=f"restatement over all {N} packets in {t1 - t0:.0f} s on {threads} threads, equal to OpenSSL")
    json.dump(out, open(os.path.join(HERE, "headline_digest.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
