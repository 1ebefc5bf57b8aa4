"""Golden digests of every rank's arena prefix in bench.py's multi-GPU line (N = 2, 4, 8).

At N > 1 bench.py runs one process per GPU. Rank r fills its own arena exactly as the headline does
(stride 1408, arena 60 B into a 64-B-aligned allocation, AAD 0a630001) but from the seeds
0x5EED0001 + r (payloads) and 0x5EED0002 + r (nonces) (bench.py main, qgcm_fill_uniform). The bytes
of slot i depend only on i and the seeds, not on how many packets the rank holds. So one digest of
each rank's first P slots covers every N, and the config-4 shards (64 M / N packets each) as well as
the --packets runs of the one-device rehearsals.

For r = 0..7 and P in {2^20, 2^18, 2^16}:
  sealed   the first P slots after one seal (crypto/aes.go:41-52: ct in place, tag, nonce after it)
  opened   after seal then open: plaintext back, tag || nonce left in each slot's tail
           (crypto/aes.go:60 opens data[:length]; Open never writes the tail)

Each rank's 2^20 sealed slots are computed twice and asserted equal: by the C restatement
(oracle/gcm_oracle.c, FIPS-197 + SP 800-38D bit-serial GHASH + crypto/aes.go framing) over every
packet, and by OpenSSL 3 EVP aes-256-gcm (oracle/ossl_check.c). Rank 0 is also asserted equal to
headline_digest.json (the same seeds). About 4 minutes on 8 threads.

  python tests/golden/make_rank_golden.py   ->  tests/golden/rank_digest.json
"""
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

L, STRIDE, RANKS = 1350, 1408, 8
PREFIXES = (1 << 20, 1 << 18, 1 << 16)


def rank_arena(n: int, seed_payload: int, seed_nonce: int) -> tuple[np.ndarray, np.ndarray]:
    """qgcm_fill_uniform's layout from a rank's seeds (make_golden.batch_arena with other seeds)."""
    arena = np.zeros(n * STRIDE, dtype=np.uint8)
    view = arena.reshape(n, STRIDE)
    view[:, :4] = np.frombuffer(G.AAD, dtype=np.uint8)
    view[:, 4:4 + L] = np.frombuffer(O.stream_bytes(seed_payload, 0, n * L), dtype=np.uint8).reshape(n, L)
    nonces = np.frombuffer(O.stream_bytes(seed_nonce, 0, 12 * n), dtype=np.uint8).copy()
    return arena, nonces


def main() -> None:
    threads = int(os.environ.get("THREADS", "8"))
    key = bytes.fromhex(json.load(open(os.path.join(HERE, "aesgo.json")))["key"])
    head = json.load(open(os.path.join(HERE, "headline_digest.json")))
    n = max(PREFIXES)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(STRIDE)
    lens = np.full(n, L, dtype=np.uint32)
    kidx = np.zeros(n, dtype=np.uint32)
    ranks = []
    t0 = time.time()
    for r in range(RANKS):
        sp, sn = G.SEED_PAYLOAD + r, G.SEED_NONCE + r
        plain, nonces = rank_arena(n, sp, sn)
        ref = plain.copy()
        O.aesgo_seal_descs(key, ref, offs, lens, kidx, nonces, 4, threads)  # restatement, every packet
        sealed = plain.copy()
        O.ossl_seal_uniform(key, sealed.ctypes.data, STRIDE, n, L, 4, nonces.ctypes.data)  # OpenSSL
        assert np.array_equal(ref, sealed), f"restatement != OpenSSL on rank {r}"
        del ref
        opened = plain
        vo, vs = opened.reshape(n, STRIDE), sealed.reshape(n, STRIDE)
        vo[:, 4 + L:4 + L + 28] = vs[:, 4 + L:4 + L + 28]
        row = {"rank": r, "seed_payload": sp, "seed_nonce": sn, "prefixes": {}}
        for p in PREFIXES:
            row["prefixes"][str(p)] = {"sha256_sealed": G.sha_chunks(sealed[:p * STRIDE]),
                                       "sha256_opened": G.sha_chunks(opened[:p * STRIDE])}
        if r == 0:
            top = row["prefixes"][str(1 << 20)]
            assert (top["sha256_sealed"], top["sha256_opened"]) == (head["sha256_sealed"], head["sha256_opened"])
        ranks.append(row)
        print(f"rank {r}: {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    out = dict(len=L, stride=STRIDE, arena_offset_in_64B_allocation=60, aad=G.h(G.AAD),
               key_sha256=head["key_sha256"], prefixes=list(PREFIXES), ranks=ranks,
               note=(f"restatement over all {n} packets of each of {RANKS} ranks, equal to OpenSSL, "
                     f"{time.time() - t0:.0f} s on {threads} threads; rank 0 equals headline_digest.json"))
    json.dump(out, open(os.path.join(HERE, "rank_digest.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
