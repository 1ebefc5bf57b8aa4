"""BASELINE config 3 on the GPU: 2^20 packets of U{64..9000} B under 1024 per-peer keys
(common/mapping.go:90-99 key provenance, crypto/aes.go:41-62 per packet), through the descriptor
batch entry points qgcm_seal_batch / qgcm_open_batch -- the default segmented kernel (variant 14:
one 5-bit comb per workgroup, short keys through variant 13) and the per-wave sorted quad-tile kernel
alone (variant 13 for every tile).

* a 32768-packet prefix of the workload (every one of the 1024 keys, the counter-segment edge
  lengths 4064..4097 and 8160..8193, 9000 B) byte-for-byte against the C restatement, then open with
  a tampered sample (status 0 + zeroed plaintext, tag and nonce untouched; the rest authentic);
* the full 2^20-packet arena (4.75 GB of payload) against tests/golden/config3_digest.json: SHA-256
  before sealing (the device fill), after sealing, after opening.

The workload is defined in tests/config3_workload.py; keys are derived through the product's own
X25519 + PBKDF2 (libqgcm keymath) and checked against the golden digest of the same table.
"""
import hashlib
import os

import numpy as np
import pytest

import config3_workload as W
from oracle import oracle as O

pytestmark = pytest.mark.gpu

THREADS = 16  # the GPU box's CPU share


@pytest.fixture(scope="module")
def torch():
    import torch as T

    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


@pytest.fixture(scope="module")
def c3_keys(torch, kdf):
    """The 1024 peer keys through the product path: secret = X25519(me.priv, peer.pub), salt likewise,
    key = PBKDF2-HMAC-SHA512(secret, salt, 10000, 32) (qgcm_x25519*, qgcm_derive_keys)."""
    from quantum_amd.crypto import derive_keys, x25519, x25519_base

    me_priv, me_salt, privs, salts = W.peer_inputs(O)
    secrets = b"".join(x25519(me_priv, x25519_base(p)) for p in privs)
    salts_ = b"".join(x25519(me_salt, x25519_base(s)) for s in salts)
    keys = derive_keys(secrets, salts_)
    digest = hashlib.sha256(keys).hexdigest()
    assert digest == kdf["peers"]["sha256_of_1024_keys"]
    return keys


@pytest.fixture(scope="module")
def c3_ctxs(torch, c3_keys):
    from quantum_amd.crypto import Context

    out = {}
    old = os.environ.get("QGCM_DESC_VARIANT")
    try:
        for v in (13, 14):
            os.environ["QGCM_DESC_VARIANT"] = str(v)
            out[v] = Context(device=0, max_keys=W.NKEYS)
            out[v].set_keys(0, c3_keys)
    finally:
        if old is None:
            os.environ.pop("QGCM_DESC_VARIANT", None)
        else:
            os.environ["QGCM_DESC_VARIANT"] = old
    yield out
    for c in out.values():
        c.close()


def device_arena(torch, size: int, offs, kidx):
    """The config-3 arena built on the device (qgcm_fill_uniform over 1 MiB chunks, then the AADs)."""
    from quantum_amd import batch

    arena = torch.empty(size, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(arena, W.CHUNK, size // W.CHUNK, W.CHUNK - 4, W.AAD_WORD, W.SEED_ARENA, None, 0)
    W.put_aads(arena, offs, kidx)
    return arena


def sha_device(torch, t) -> str:
    h = hashlib.sha256()
    step = 1 << 28
    for i in range(0, t.numel(), step):
        h.update(memoryview(t[i:i + step].cpu().numpy()))
    return h.hexdigest()


@pytest.mark.parametrize("v", [13, 14])
def test_config3_prefix_vs_oracle(torch, c3_ctxs, c3_keys, v):
    from quantum_amd import batch

    ctx = c3_ctxs[v]
    n = 32768
    lens, kidx = W.lengths(n), W.key_indices(n)
    assert len(np.unique(kidx)) == W.NKEYS  # the batch touches every key of the table
    offs, size = W.layout(lens)
    nonces_h = W.nonces(O, n)
    arena = device_arena(torch, size, offs, kidx)
    plain = W.host_arena(O, size, offs, kidx)
    assert np.array_equal(arena.cpu().numpy(), plain)  # the device fill is the workload definition

    ref = plain.copy()
    O.aesgo_seal_descs(c3_keys, ref, offs, lens, kidx, nonces_h, 4, THREADS)
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    nonces = torch.from_numpy(nonces_h).cuda()
    batch.seal_batch(ctx, arena, batch.make_descs(offs, lens, kidx, "cuda"), n, nonces, status=status)
    assert int(status.sum()) == n
    got = arena.cpu().numpy()
    if not np.array_equal(got, ref):
        bad = [i for i in range(n) if not np.array_equal(got[offs[i]:offs[i] + 4 + lens[i] + 28],
                                                          ref[offs[i]:offs[i] + 4 + lens[i] + 28])]
        pytest.fail(f"variant {v}: {len(bad)} packets differ from the oracle, first {bad[:8]} "
                    f"(lengths {[int(lens[i]) for i in bad[:8]]})")

    # open: a tampered sample fails (plaintext zeroed, tag/nonce untouched), everything else round-trips
    rng = np.random.default_rng(0x5EED0035)
    bad = np.unique(rng.choice(n, 600, replace=False))
    tampered = ref.copy()
    for j, i in enumerate(bad):
        L = int(lens[i])
        where = j % 4  # ciphertext byte, tag byte, nonce byte, AAD byte
        pos = [4 + (j * 131) % max(L, 1) if L else 4 + L, 4 + L + (j % 16), 4 + L + 16 + (j % 12), j % 4][where]
        tampered[int(offs[i]) + pos] ^= 0x10
    arena.copy_(torch.from_numpy(tampered).cuda())
    batch.open_batch(ctx, arena, batch.make_descs(offs, lens + 28, kidx, "cuda"), n, status=status)
    st = status.cpu().numpy()
    want = np.ones(n, dtype=np.uint8)
    want[bad] = 0
    assert np.array_equal(st, want)
    exp = tampered.copy()
    ost = np.zeros(n, dtype=np.uint8)
    O.aesgo_open_descs(c3_keys, exp, offs, lens + 28, kidx, ost, 4, THREADS)
    assert np.array_equal(ost, want)  # the oracle agrees on which packets are authentic
    assert np.array_equal(arena.cpu().numpy(), exp)  # restored / zeroed bytes identical to the oracle's


@pytest.mark.parametrize("v", [13, 14])
def test_config3_full_arena_digest(torch, c3_ctxs, config3_digest, v):
    """All 2^20 packets (1024 keys, 4.75 GB of payload): digests before sealing, sealed and opened
    equal the golden ones (OpenSSL over the same workload, prefix cross-checked with the oracle)."""
    from quantum_amd import batch

    g = config3_digest
    ctx = c3_ctxs[v]
    lens, kidx = W.lengths(), W.key_indices()
    assert int(lens.sum()) == g["payload_bytes"]
    offs, size = W.layout(lens)
    assert size == g["arena_bytes"]
    arena = device_arena(torch, size, offs, kidx)
    assert sha_device(torch, arena) == g["sha256_plain"]
    nonces = torch.from_numpy(W.nonces(O)).cuda()
    status = torch.zeros(W.N, dtype=torch.uint8, device="cuda")
    batch.seal_batch(ctx, arena, batch.make_descs(offs, lens, kidx, "cuda"), W.N, nonces, status=status)
    assert int(status.sum()) == W.N
    assert sha_device(torch, arena) == g["sha256_sealed"]
    status.zero_()
    batch.open_batch(ctx, arena, batch.make_descs(offs, lens + 28, kidx, "cuda"), W.N, status=status)
    assert int(status.sum()) == W.N
    assert sha_device(torch, arena) == g["sha256_opened"]
    del arena
    torch.cuda.empty_cache()
