"""BASELINE config 3 for the golden generator (tests/golden/make_golden.py) and the GPU parity tests
(tests/test_gpu_config3.py) -- TEST INFRASTRUCTURE.

The workload itself is defined once in quantum_amd/workloads.py (bench.py measures the same one);
this module adds the oracle-side views: the peer inputs and nonces drawn through the oracle's own
splitmix64 stream (so the package's numpy stream is checked against the C restatement) and the whole
arena built on the host.
"""
from __future__ import annotations

import numpy as np

from quantum_amd.workloads import (AAD_WORD, CHUNK, FORCED, N, NKEYS, SEED_ARENA, SEED_KEY, SEED_LEN,  # noqa: F401
                                   SEED_ME, SEED_NONCE, SEED_PEERS, aad_of_key, key_indices, layout, lengths,
                                   put_aads, splitmix64, tail_index)
from quantum_amd import workloads as _W


def peer_inputs(O) -> tuple[bytes, bytes, list[bytes], list[bytes]]:
    """This node's private key and salt, and each peer's private key and salt (kdf.json recipe),
    from the oracle's stream; equal to quantum_amd.workloads.peer_inputs() (asserted here)."""
    me_priv = O.stream_bytes(SEED_ME, 0, 32)
    me_salt = O.stream_bytes(SEED_ME, 32, 32)
    privs = [O.stream_bytes(SEED_PEERS, 64 * i, 32) for i in range(NKEYS)]
    salts = [O.stream_bytes(SEED_PEERS, 64 * i + 32, 32) for i in range(NKEYS)]
    assert (me_priv, me_salt, privs, salts) == _W.peer_inputs()
    return me_priv, me_salt, privs, salts


def nonces(O, n: int = N) -> np.ndarray:
    out = np.frombuffer(O.stream_bytes(SEED_NONCE, 0, 12 * n), dtype=np.uint8).copy()
    assert np.array_equal(out, _W.nonces(n))
    return out


def host_arena(O, size: int, offs: np.ndarray, kidx: np.ndarray) -> np.ndarray:
    """The arena as the device builds it (qgcm_fill_uniform chunks, then the AADs), on the host."""
    chunks = size // CHUNK
    a = np.empty(size, dtype=np.uint8)
    v = a.reshape(chunks, CHUNK)
    v[:, :4] = np.frombuffer(AAD_WORD.to_bytes(4, "little"), dtype=np.uint8)
    stream = np.frombuffer(O.stream_bytes(SEED_ARENA, 0, chunks * (CHUNK - 4)), dtype=np.uint8)
    v[:, 4:] = stream.reshape(chunks, CHUNK - 4)
    del stream
    put_aads(a, offs, kidx)
    return a
