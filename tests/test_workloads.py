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


def test_config5_workload_and_host_codec_match_golden():
    """Config 5 at its stated size on the CPU: the workload definition hashes to the golden plaintext
    digest, and libqgcm's host snappy encoder (compression.go Outgoing on every slot) produces exactly
    libsnappy's compressed arena (tests/golden/config5_digest.json sha256_compressed)."""
    import ctypes as C
    import json
    import os

    from quantum_amd import _lib

    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "config5_digest.json")))
    slots = W.config5_packets()
    N, S = W.C5_N, W.C5_STRIDE

    def sha(a):
        h = hashlib.sha256()
        flat = a.reshape(-1)
        for i in range(0, flat.size, 1 << 28):
            h.update(memoryview(flat[i:i + (1 << 28)]))
        return h.hexdigest()

    assert sha(slots) == gold["sha256_plain"]
    lens = np.full(N, W.C5_LEN, np.uint32)
    assert _lib.lib().qgcm_snappy_compress_slots(slots.ctypes.data, S, N, lens.ctypes.data, 8) == 0
    assert int(lens.sum()) + 28 * N == gold["sealed_bytes"]
    assert sha(slots) == gold["sha256_compressed"]
