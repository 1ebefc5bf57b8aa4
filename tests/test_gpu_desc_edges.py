"""Descriptor-batch edge cases on the GPU (qgcm_seal_batch / qgcm_open_batch):

* a descriptor naming a key slot that was never set fails -- status 0, slot untouched -- in every
  descriptor kernel (the segmented kernel 14, the per-wave quad tiles 13), as Apply does for a peer whose
  Mapping.AES is nil (common/mapping.go:94-99; Go would dereference nil, plugin/encryption.go:23,31);
  the packets around it are sealed / opened bit-exact against the oracle;
* the largest key index a context accepts (QGCM_MAX_KEYS - 1 = 2^20 - 2 at max_keys = 2^20 - 1)
  with an empty payload (seal L = 0, open len = 28): its sort key is the closest a valid packet gets
  to the excluded marker and it must still be processed.
"""
import ctypes
import os
import random

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

QGCM_MAX_KEYS = (1 << 20) - 1


@pytest.fixture(scope="module")
def torch():
    import torch as T

    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


def make_ctx(max_keys: int, variant: int | None = None):
    from quantum_amd.crypto import Context

    old = os.environ.get("QGCM_DESC_VARIANT")
    try:
        if variant is not None:
            os.environ["QGCM_DESC_VARIANT"] = str(variant)
        return Context(device=0, max_keys=max_keys)
    finally:
        if old is None:
            os.environ.pop("QGCM_DESC_VARIANT", None)
        else:
            os.environ["QGCM_DESC_VARIANT"] = old


def packed(lens):
    offs, pos = [], 0
    for L in lens:
        offs.append(pos)
        pos += (4 + L + 28 + 3) & ~3
    return offs, pos + 64


@pytest.mark.parametrize("v", [13, 14])
def test_unset_key_slot_is_rejected(torch, v):
    from quantum_amd import batch

    ctx = make_ctx(64, v)
    rng = random.Random(0x0E5 + v)
    keys = {k: rng.randbytes(32) for k in (0, 1, 2, 3)}
    ctx.set_keys(0, b"".join(keys[k] for k in range(4)))
    n = 400
    # every 7th packet names an unset slot (5, 40 or 63: inside max_keys, never set)
    kidx = [rng.choice([5, 40, 63]) if i % 7 == 3 else rng.randrange(4) for i in range(n)]
    lens = [rng.choice([0, 1, 16, 17, 1350, 4081]) if i % 3 else rng.randint(0, 2000) for i in range(n)]
    offs, size = packed(lens)
    arena_h = np.frombuffer(rng.randbytes(size), dtype=np.uint8).copy()
    nonces_h = np.frombuffer(rng.randbytes(12 * n), dtype=np.uint8).copy()
    ref = arena_h.copy()
    unset = [k not in keys for k in kidx]
    for i, L in enumerate(lens):
        if unset[i]:
            continue
        buf = bytearray(ref[offs[i] + 4:offs[i] + 4 + L + 28].tobytes())
        O.aesgo_encrypt(keys[kidx[i]], buf, L, bytes(ref[offs[i]:offs[i] + 4]), bytes(nonces_h[12 * i:12 * i + 12]))
        ref[offs[i] + 4:offs[i] + 4 + L + 28] = np.frombuffer(bytes(buf), dtype=np.uint8)
    arena = torch.from_numpy(arena_h.copy()).cuda()
    status = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    batch.seal_batch(ctx, arena, batch.make_descs(offs, lens, kidx, "cuda"), n, torch.from_numpy(nonces_h).cuda(),
                     status=status)
    st = status.cpu().numpy()
    assert st.tolist() == [0 if u else 1 for u in unset]
    assert np.array_equal(arena.cpu().numpy(), ref)  # unset-key slots untouched, the rest == oracle
    # open the same batch: unset-key packets stay untouched again (never zeroed as auth failures)
    status.fill_(7)
    batch.open_batch(ctx, arena, batch.make_descs(offs, [L + 28 for L in lens], kidx, "cuda"), n, status=status)
    st = status.cpu().numpy()
    assert st.tolist() == [0 if u else 1 for u in unset]
    got = arena.cpu().numpy()
    for i, L in enumerate(lens):
        o = offs[i]
        if unset[i]:
            assert np.array_equal(got[o:o + 4 + L + 28], arena_h[o:o + 4 + L + 28])
        else:
            assert np.array_equal(got[o:o + 4 + L], arena_h[o:o + 4 + L])
    ctx.close()


def test_uniform_and_one_calls_reject_unset_key(torch):
    from quantum_amd import _lib, batch

    ctx = make_ctx(8)
    arena = torch.zeros(4 * 128, dtype=torch.uint8, device="cuda")
    with pytest.raises(_lib.QgcmError):
        batch.seal_uniform(ctx, arena, 128, 4, 64, 3)
    data = bytearray(64 + 28)
    buf = (ctypes.c_uint8 * len(data)).from_buffer(data)
    assert _lib.lib().qgcm_seal_one(ctx.handle, 3, ctypes.addressof(buf), 64, None, 0, None) == -1
    assert _lib.lib().qgcm_open_one(ctx.handle, 3, ctypes.addressof(buf), 64 + 28, None, 0) == -1
    del buf
    assert bytes(data) == bytes(64 + 28)
    ctx.close()


def test_largest_key_index_empty_payload(torch):
    """max_keys = QGCM_MAX_KEYS (the key tables take ~77 GB of the 288 GB HBM): key index
    QGCM_MAX_KEYS - 1 with L = 0 sorts at (2^20 - 2) << 12 | 4095, next to the all-ones excluded
    marker, and is sealed / opened like any other packet; a batch sharing it with key 0 stays exact."""
    from quantum_amd import batch

    ctx = make_ctx(QGCM_MAX_KEYS)
    rng = random.Random(0x0E6)
    top = QGCM_MAX_KEYS - 1
    k_top, k0 = rng.randbytes(32), rng.randbytes(32)
    ctx.set_key(top, k_top)
    ctx.set_key(0, k0)
    lens = [0, 0, 5, 1350, 0, 17]
    kidx = [top, 0, top, top, top, 0]
    n = len(lens)
    offs, size = packed(lens)
    arena_h = np.frombuffer(rng.randbytes(size), dtype=np.uint8).copy()
    nonces_h = np.frombuffer(rng.randbytes(12 * n), dtype=np.uint8).copy()
    ref = arena_h.copy()
    for i, L in enumerate(lens):
        buf = bytearray(ref[offs[i] + 4:offs[i] + 4 + L + 28].tobytes())
        key = k_top if kidx[i] == top else k0
        O.aesgo_encrypt(key, buf, L, bytes(ref[offs[i]:offs[i] + 4]), bytes(nonces_h[12 * i:12 * i + 12]))
        ref[offs[i] + 4:offs[i] + 4 + L + 28] = np.frombuffer(bytes(buf), dtype=np.uint8)
    arena = torch.from_numpy(arena_h.copy()).cuda()
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    batch.seal_batch(ctx, arena, batch.make_descs(offs, lens, kidx, "cuda"), n, torch.from_numpy(nonces_h).cuda(),
                     status=status)
    assert status.cpu().tolist() == [1] * n
    assert np.array_equal(arena.cpu().numpy(), ref)
    status.zero_()
    batch.open_batch(ctx, arena, batch.make_descs(offs, [L + 28 for L in lens], kidx, "cuda"), n, status=status)
    assert status.cpu().tolist() == [1] * n
    got = arena.cpu().numpy()
    for i, L in enumerate(lens):
        assert np.array_equal(got[offs[i]:offs[i] + 4 + L], arena_h[offs[i]:offs[i] + 4 + L])
    ctx.close()
    torch.cuda.empty_cache()


def test_launch_counts_name_the_kernels(torch):
    """qgcm_launch_counts: a single-key batch past 2048 packets runs the quad kernel, a small one the
    latency kernel, a keyed descriptor batch the segmented kernel plus the per-wave kernel."""
    from quantum_amd import batch
    from quantum_amd.crypto import Context

    ctx = Context(device=0, max_keys=64)
    try:
        rng = np.random.default_rng(5)
        ctx.set_keys(0, rng.bytes(32 * 64))
        L = 1350
        stride = batch.slot_stride(L)
        for n, kind in ((100, "one"), (5000, "quad")):
            before = ctx.launch_counts()
            arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
            batch.seal_uniform(ctx, arena, stride, n, L, 3, None)
            torch.cuda.synchronize()
            after = ctx.launch_counts()
            assert after[kind] - before[kind] == 1, (n, before, after)
        n = 20000
        kidx = np.concatenate([np.zeros(15000, np.int64), rng.integers(1, 64, n - 15000)])
        offs = np.arange(n, dtype=np.int64) * stride
        arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
        before = ctx.launch_counts()
        batch.seal_batch(ctx, arena, batch.make_descs(offs, np.full(n, L), kidx, "cuda"), n, None)
        torch.cuda.synchronize()
        after = ctx.launch_counts()
        assert after["segmented"] - before["segmented"] == 1 and after["per_wave"] - before["per_wave"] == 1
    finally:
        ctx.close()
