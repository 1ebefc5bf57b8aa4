"""quantum_amd/workloads.py (the config-3 definition bench.py measures) against the oracle's own
splitmix64 stream and the golden key-table digest -- CPU only (host key math, no GPU)."""
import hashlib

import numpy as np

from oracle import oracle as O
from quantum_amd import workloads as W


def test_stream_bytes_match_oracle():
    for seed, off, n in ((W.SEED_NONCE, 0, 100), (W.SEED_ARENA, 5, 77), (W.SEED_ME, 32, 32), (7, 8 * 1000 + 3, 1),
                         (W.SEED_PEERS, 64 * 1023 + 32, 32)):
        assert W.stream_bytes(seed, off, n) == O.stream_bytes(seed, off, n), (seed, off, n)


def test_nonces_and_lengths():
    n = 5000
    assert np.array_equal(W.nonces(n), np.frombuffer(O.stream_bytes(W.SEED_NONCE, 0, 12 * n), np.uint8))
    L = W.lengths(n)
    assert L[:len(W.FORCED)].tolist() == W.FORCED
    assert L.min() >= 64 and L.max() <= 9000
    k = W.key_indices(n)
    assert k.max() < W.NKEYS
    assert W.splitmix64(W.SEED_LEN, np.array([123], np.uint64))[0] == O.splitmix64_at(W.SEED_LEN, 123)


def test_peer_keys_match_golden(kdf):
    """The 1024 peer keys through the product's host key math equal the golden table digest."""
    assert hashlib.sha256(W.peer_keys()).hexdigest() == kdf["peers"]["sha256_of_1024_keys"]
