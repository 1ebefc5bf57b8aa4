"""tests/golden/rank_digest.json, the per-rank arena digests bench.py checks at N > 1 (CPU): rank 0's 2^20
prefix equals the headline golden (the same seeds), and the 2^16 prefixes of ranks 1 and 7 are recomputed
here from their seeds with OpenSSL, the first 256 packets also with the C restatement."""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from oracle import oracle as O  # noqa: E402


def _gold(name):
    return json.load(open(os.path.join(HERE, "golden", name)))


def test_rank0_equals_headline():
    rank, head = _gold("rank_digest.json"), _gold("headline_digest.json")
    r0 = rank["ranks"][0]
    assert (r0["seed_payload"], r0["seed_nonce"]) == (head["seed_payload"], head["seed_nonce"])
    top = r0["prefixes"][str(1 << 20)]
    assert top["sha256_sealed"] == head["sha256_sealed"] and top["sha256_opened"] == head["sha256_opened"]
    assert [r["rank"] for r in rank["ranks"]] == list(range(8))
    assert [r["seed_payload"] for r in rank["ranks"]] == [0x5EED0001 + r for r in range(8)]


def test_rank_prefixes_recomputed():
    import make_rank_golden as M

    gold = _gold("rank_digest.json")
    key = bytes.fromhex(_gold("aesgo.json")["key"])
    n, L, stride = 1 << 16, gold["len"], gold["stride"]
    for r in (1, 7):
        row = gold["ranks"][r]
        plain, nonces = M.rank_arena(n, row["seed_payload"], row["seed_nonce"])
        sealed = plain.copy()
        O.ossl_seal_uniform(key, sealed.ctypes.data, stride, n, L, 4, nonces.ctypes.data)
        ref = plain[:256 * stride].copy()
        O.lib().oracle_seal_uniform(key, ref.ctypes.data, stride, 256, L, 4, nonces.ctypes.data)
        assert np.array_equal(ref, sealed[:256 * stride])
        want = row["prefixes"][str(n)]
        assert hashlib.sha256(sealed.tobytes()).hexdigest() == want["sha256_sealed"]
        opened = plain.reshape(n, stride)
        opened[:, 4 + L:4 + L + 28] = sealed.reshape(n, stride)[:, 4 + L:4 + L + 28]
        assert hashlib.sha256(opened.tobytes()).hexdigest() == want["sha256_opened"]
