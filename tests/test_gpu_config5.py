"""GPU: BASELINE config 5 at its stated workload -- the compression + encryption chain on 2^20 x 1350 B
packets (plugin/compression.go:16-56 then plugin/encryption.go:16-40, in the order main.go:50-51 sorts
them), against tests/golden/config5_digest.json (libsnappy 1.1.8 + OpenSSL, cross-checked with the
restatements; tests/golden/make_config5_golden.py).

Bar: byte-exact.  The whole sealed arena (every 1472-B Payload.Raw slot, bytes past the record
included) and the sealed lengths hash to the golden digests
  * through the host-memory chain (qgcm_compress_seal_host, copies included) with the codec on the
    host workers, split between host and device, and on the device only;
  * through the device-resident chain (qgcm_snappy_compress_batch writing the seal descriptors, then
    qgcm_seal_batch);
and opening + uncompressing restores every slot to the plaintext arena (its golden digest)."""
import ctypes as C
import hashlib

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as T

    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


@pytest.fixture(scope="module")
def gold():
    return golden("config5_digest.json")


def _sha(a: np.ndarray) -> str:
    h = hashlib.sha256()
    flat = a.reshape(-1)
    for i in range(0, flat.size, 1 << 28):
        h.update(memoryview(flat[i:i + (1 << 28)]))
    return h.hexdigest()


def _lens_sha(lens) -> str:
    return hashlib.sha256(np.asarray(lens, dtype="<u4").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def c5(torch, gold):
    from quantum_amd import _lib, workloads as W
    from quantum_amd.crypto import Context, derive_key

    N, L, S = W.C5_N, W.C5_LEN, W.C5_STRIDE
    key = derive_key(b"AES256Key-32Characters1234567890", bytes(range(32)))
    assert key.hex() == gold["key"]
    ctx = Context(device=0, max_keys=4)
    ctx.set_key(0, key)
    plain = W.config5_packets(N, L, S)
    assert _sha(plain) == gold["sha256_plain"]
    nonces = W.config5_nonces(N)
    Lb = _lib.lib()
    a_ptr, n_ptr = Lb.qgcm_host_alloc(N * S), Lb.qgcm_host_alloc(12 * N)
    assert a_ptr and n_ptr
    host = np.frombuffer((C.c_uint8 * (N * S)).from_address(a_ptr), np.uint8).reshape(N, S)
    nons = np.frombuffer((C.c_uint8 * (12 * N)).from_address(n_ptr), np.uint8)
    nons[:] = nonces
    yield dict(ctx=ctx, plain=plain, nonces=nonces, host=host, a_ptr=a_ptr, n_ptr=n_ptr, N=N, L=L, S=S)
    del host, nons
    Lb.qgcm_host_free(a_ptr)
    Lb.qgcm_host_free(n_ptr)
    ctx.close()


@pytest.mark.parametrize("mode,name", [(0, "host"), (1, "split"), (2, "device")])
def test_config5_host_chain_full_size(c5, gold, mode, name):
    from quantum_amd import batch

    ctx, host, N, L, S = c5["ctx"], c5["host"], c5["N"], c5["L"], c5["S"]
    host[:] = c5["plain"]
    prev = batch.chain_codec(ctx, mode)
    try:
        lens = np.full(N, L, np.uint32)
        status = np.zeros(N, np.uint8)
        c0 = ctx.launch_counts()
        bad = batch.compress_seal_host(ctx, c5["a_ptr"], S, N, lens, 0, c5["n_ptr"], threads=16,
                                       status_ptr=status.ctypes.data)
        c1 = ctx.launch_counts()
        assert bad == 0 and bool((status == 1).all())
        assert int(lens.sum()) == gold["sealed_bytes"]
        assert _lens_sha(lens) == gold["sha256_sealed_lens"]
        assert _sha(host) == gold["sha256_sealed"], f"sealed arena differs from the golden digest (codec {name})"
        if mode == 2:  # every chunk's codec ran on the device
            assert c1["snappy_enc"] > c0["snappy_enc"]
        if mode == 0:
            assert c1["snappy_enc"] == c0["snappy_enc"]
        bad = batch.open_uncompress_host(ctx, c5["a_ptr"], S, N, lens, 0, threads=16, status_ptr=status.ctypes.data)
        assert bad == 0 and bool((status == 1).all()) and bool((lens == L).all())
        assert np.array_equal(host[:, :4 + L], c5["plain"][:, :4 + L])
    finally:
        batch.chain_codec(ctx, prev)


def test_config5_device_resident_chain_full_size(torch, c5, gold):
    """Device snappy -> seal on HBM-resident slots (extra_configs.config5_resident's path), then open ->
    device uncompress."""
    from quantum_amd import batch

    ctx, N, L, S = c5["ctx"], c5["N"], c5["L"], c5["S"]
    plain = torch.from_numpy(c5["plain"].reshape(-1)).cuda()
    arena = plain.clone()
    nonces = torch.from_numpy(c5["nonces"]).cuda()
    lens = torch.full((N,), L, dtype=torch.int32, device="cuda")
    descs = torch.empty(16 * N, dtype=torch.uint8, device="cuda")
    status = torch.zeros(N, dtype=torch.uint8, device="cuda")
    limit = S - 4 - 28
    batch.snappy_compress(ctx, arena, S, N, lens, S - 4, limit, status, descs_out=descs, key_idx=0)
    torch.cuda.synchronize()
    assert bool((status == 1).all())
    batch.seal_batch(ctx, arena, descs, N, nonces, status=status)
    torch.cuda.synchronize()
    assert bool((status == 1).all())
    sealed_lens = lens.cpu().numpy().astype(np.uint32) + 28
    assert _lens_sha(sealed_lens) == gold["sha256_sealed_lens"]
    assert _sha(arena.cpu().numpy()) == gold["sha256_sealed"]
    d = descs.view(torch.int32).view(N, 4)
    d[:, 2] += 28  # the receiver's descriptors carry the sealed lengths
    batch.open_batch(ctx, arena, descs, N, status=status)
    clen = lens.clone()
    batch.snappy_uncompress(ctx, arena, S, N, clen, limit, S - 4, status)
    torch.cuda.synchronize()
    assert bool((status == 1).all()) and bool((clen == L).all())
    assert torch.equal(arena.view(N, S)[:, :4 + L], plain.view(N, S)[:, :4 + L])
    del arena, plain
    torch.cuda.empty_cache()


def test_config5_host_chain_tampered_packets_device_decoder_matches_host(torch, gold):
    """Packets whose open fails are left to the caller by the decoder (status_in): 2^16 config-5 slots
    sealed by the chain, 1 in 61 of them tampered (a ciphertext, tag or nonce byte flipped), then opened
    and uncompressed with the codec on the host workers and, from the same sealed bytes, on the device
    (the group decoder by default).  Both must give the same arena, lengths and statuses; the untouched
    packets come back as plaintext, the tampered ones fail."""
    from quantum_amd import _lib, batch, workloads as W
    from quantum_amd.crypto import Context, derive_key

    N, L, S = 1 << 16, W.C5_LEN, W.C5_STRIDE
    key = derive_key(b"AES256Key-32Characters1234567890", bytes(range(32)))
    ctx = Context(device=0, max_keys=4)
    ctx.set_key(0, key)
    Lb = _lib.lib()
    a_ptr, n_ptr = Lb.qgcm_host_alloc(N * S), Lb.qgcm_host_alloc(12 * N)
    try:
        host = np.frombuffer((C.c_uint8 * (N * S)).from_address(a_ptr), np.uint8).reshape(N, S)
        nons = np.frombuffer((C.c_uint8 * (12 * N)).from_address(n_ptr), np.uint8)
        plain = W.config5_packets(N, L, S)
        host[:] = plain
        nons[:] = W.config5_nonces(N)
        lens = np.full(N, L, np.uint32)
        status = np.zeros(N, np.uint8)
        assert batch.compress_seal_host(ctx, a_ptr, S, N, lens, 0, n_ptr, threads=16,
                                        status_ptr=status.ctypes.data) == 0
        rng = np.random.default_rng(0x5EED0061)
        bad = np.arange(0, N, 61)
        for i in bad:  # a byte of the record [4, 4 + lens[i]): ciphertext, tag or nonce
            j = 4 + int(rng.integers(0, int(lens[i])))
            host[i, j] ^= 1 + int(rng.integers(0, 255))
        sealed, sealed_lens = host.copy(), lens.copy()
        out = {}
        for mode in (0, 2):
            host[:] = sealed
            lens[:] = sealed_lens
            status[:] = 0
            prev = batch.chain_codec(ctx, mode)
            try:
                failed = batch.open_uncompress_host(ctx, a_ptr, S, N, lens, 0, threads=16,
                                                    status_ptr=status.ctypes.data)
            finally:
                batch.chain_codec(ctx, prev)
            out[mode] = (failed, host.copy(), lens.copy(), status.copy())
        f0, h0, l0, s0 = out[0]
        f2, h2, l2, s2 = out[2]
        assert f0 == f2 == len(bad)
        assert np.array_equal(s0, s2) and not s0[bad].any() and int(s0.sum()) == N - len(bad)
        assert np.array_equal(l0, l2)
        assert np.array_equal(h0, h2), "device decoder output differs from the host codec's"
        good = np.setdiff1d(np.arange(N), bad)
        assert np.array_equal(h0[good, :4 + L], plain[good, :4 + L]) and bool((l0[good] == L).all())
    finally:
        Lb.qgcm_host_free(a_ptr)
        Lb.qgcm_host_free(n_ptr)
        ctx.close()
