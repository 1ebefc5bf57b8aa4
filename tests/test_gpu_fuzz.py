"""Seeded random descriptor batches on the GPU against the oracle (crypto/aes.go:41-62 per packet,
common/mapping.go:90-99 per-peer keys).

Each case draws a batch shape the fixed tests do not: a skewed key mix (a few keys with runs long
enough for the segmented kernel's shared-table path, many with a handful of packets for its
per-wave pass), lengths from 0 to 9000 B with the counter-segment edges, slots packed at 4-B
alignment with random gaps, AAD of 0 or 4 bytes, and invalid packets mixed in (unset key slots,
key indices past max_keys, opens shorter than 28 B) that must come back status 0 with their slot
untouched.  Seal is compared byte for byte with the C restatement; then a tampered sample is
opened (status 0 and zeroed plaintext for the tampered, the rest authentic).  Every case runs
through the default descriptor kernel (variant 14 + 13) and the per-wave kernel alone (variant 13).
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

MAX_KEYS = 4096
SET_KEYS = 3000  # slots [0, 3000) hold keys; [3000, 4096) were never set


@pytest.fixture(scope="module")
def torch():
    import torch as T

    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


@pytest.fixture(scope="module")
def fuzz_keys():
    return np.random.default_rng(0x5EED00F0).bytes(32 * MAX_KEYS)


@pytest.fixture(scope="module")
def fuzz_ctxs(torch, fuzz_keys):
    """One context per (kernel variant, QGCM_SMALL_WORKLIST): both knobs are read at qgcm_create."""
    from quantum_amd.crypto import Context

    out = {}
    saved = {k: os.environ.get(k) for k in ("QGCM_DESC_VARIANT", "QGCM_SMALL_WORKLIST")}
    try:
        for v in (None, 13):
            for small in ("1", "0"):
                if v is None:
                    os.environ.pop("QGCM_DESC_VARIANT", None)
                else:
                    os.environ["QGCM_DESC_VARIANT"] = str(v)
                os.environ["QGCM_SMALL_WORKLIST"] = small
                c = Context(device=0, max_keys=MAX_KEYS)
                c.set_keys(0, fuzz_keys[:32 * SET_KEYS])
                out[("default" if v is None else v, small)] = c
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    yield out
    for c in out.values():
        c.close()


SIZES = (1, 17, 700, 3000, 9000, 24000, 16000, 5000, 768, 4096)  # 768: the smallest batch a key can fill a run in; 4096: the largest one-workgroup worklist


def draw_case(case: int):
    rng = np.random.default_rng(0xF0220000 + case)
    n = SIZES[case % len(SIZES)]
    # skewed key mix: a few hot keys (long runs) and a long tail
    hot = rng.integers(0, SET_KEYS, size=int(rng.integers(1, 4)))
    tail = rng.integers(0, SET_KEYS, size=n)
    kidx = np.where(rng.random(n) < rng.uniform(0.2, 0.9), hot[rng.integers(0, len(hot), size=n)], tail)
    kidx = kidx.astype(np.uint32)
    lens = rng.integers(0, 9001, size=n).astype(np.uint32)
    edges = np.array([0, 1, 15, 16, 17, 1350, 4064, 4079, 4080, 4081, 4096, 8191, 8192, 9000], dtype=np.uint32)
    pick = rng.random(n) < 0.2
    lens[pick] = edges[rng.integers(0, len(edges), size=int(pick.sum()))]
    # invalid packets: an unset key slot or a key index past max_keys
    bad_key = rng.random(n) < 0.02
    kidx[bad_key] = np.where(rng.random(int(bad_key.sum())) < 0.5,
                             rng.integers(SET_KEYS, MAX_KEYS, size=int(bad_key.sum())),
                             MAX_KEYS + rng.integers(0, 1000, size=int(bad_key.sum()))).astype(np.uint32)
    gap = rng.integers(0, 5, size=n).astype(np.int64) * 4
    slot = ((4 + lens.astype(np.int64) + 28 + 3) & ~3) + gap
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(slot)[:-1].astype(np.uint64)
    size = int(offs[-1]) + int(slot[-1]) + 64
    aad_len = int(rng.choice([0, 4]))
    return rng, n, kidx, lens, offs, slot, size, aad_len, ~bad_key


@pytest.mark.parametrize("small", ["1", "0"])
@pytest.mark.parametrize("variant", ["default", 13])
@pytest.mark.parametrize("seed", range(len(SIZES)))
def test_descriptor_fuzz_vs_oracle(torch, fuzz_ctxs, fuzz_keys, variant, seed, small):
    """small: QGCM_SMALL_WORKLIST -- batches of up to 4096 packets build their worklist in one workgroup
    ("1", the default) or through the multi-launch radix-sort path ("0"); larger batches always take
    the latter."""
    from quantum_amd import batch

    ctx = fuzz_ctxs[(variant, small)]
    rng, n, kidx, lens, offs, slot, size, aad_len, valid = draw_case(seed)
    plain = np.frombuffer(rng.bytes(size), dtype=np.uint8).copy()
    nonces = np.frombuffer(rng.bytes(12 * n), dtype=np.uint8).copy()

    # expected seal: the oracle on the valid packets; invalid slots stay as they were
    ref = plain.copy()
    vi = np.nonzero(valid)[0]
    if len(vi):
        O.aesgo_seal_descs(fuzz_keys, ref, np.ascontiguousarray(offs[vi]), np.ascontiguousarray(lens[vi]),
                           np.ascontiguousarray(kidx[vi]), np.ascontiguousarray(nonces.reshape(n, 12)[vi]).reshape(-1),
                           aad_len, 8)
    arena = torch.from_numpy(plain.copy()).cuda()
    # statuses start as junk: the call itself must clear those of packets it leaves out
    status = torch.full((n,), 0x5A, dtype=torch.uint8, device="cuda")
    batch.seal_batch(ctx, arena, batch.make_descs(offs, lens, kidx, "cuda"), n, torch.from_numpy(nonces).cuda(),
                     aad_len=aad_len, status=status)
    st = status.cpu().numpy()
    assert np.array_equal(st, valid.astype(np.uint8)), f"seal status: {int((st != valid).sum())} packets differ"
    got = arena.cpu().numpy()
    if not np.array_equal(got, ref):
        bad = [int(i) for i in range(n) if not np.array_equal(got[offs[i]:offs[i] + slot[i]], ref[offs[i]:offs[i] + slot[i]])]
        pytest.fail(f"seed {seed}: {len(bad)} of {n} slots differ, first {bad[:5]} keys {kidx[bad[:5]].tolist()} "
                    f"lengths {lens[bad[:5]].tolist()}")

    # open: tamper a sample (a ciphertext, tag or nonce byte), and shorten a few descriptors below 28
    tampered = ref.copy()
    tam = np.zeros(n, dtype=bool)
    for i in rng.choice(n, size=max(1, n // 50), replace=False):
        L = int(lens[i])
        pos = int(offs[i]) + 4 + int(rng.integers(0, L + 28))
        tampered[pos] ^= 1 << int(rng.integers(0, 8))
        tam[i] = True
    olens = lens.astype(np.int64) + 28
    short = rng.random(n) < 0.01
    olens[short] = rng.integers(0, 28, size=int(short.sum()))
    olens = olens.astype(np.uint32)
    ok = valid & ~short
    exp = tampered.copy()
    ost = np.zeros(n, dtype=np.uint8)
    oi = np.nonzero(ok)[0]
    if len(oi):
        sub = np.zeros(len(oi), dtype=np.uint8)
        O.aesgo_open_descs(fuzz_keys, exp, np.ascontiguousarray(offs[oi]), np.ascontiguousarray(olens[oi]),
                           np.ascontiguousarray(kidx[oi]), sub, aad_len, 8)
        ost[oi] = sub
    assert not np.any(ost[ok & ~tam] == 0), "oracle rejected an untampered packet"
    arena.copy_(torch.from_numpy(tampered).cuda())
    status.fill_(0x5A)
    batch.open_batch(ctx, arena, batch.make_descs(offs, olens, kidx, "cuda"), n, aad_len=aad_len, status=status)
    assert np.array_equal(status.cpu().numpy(), ost)
    assert np.array_equal(arena.cpu().numpy(), exp)


def test_descriptor_batch_4m_packets(torch, fuzz_ctxs, fuzz_keys):
    """One descriptor batch of 2^22 packets (64 keys, U{64..2000} B, 4.4 GB of slots): the worklist
    sort, the run table and the per-run tile queues at four times config 3's packet count.  A sample
    of 4096 packets is compared with the oracle after sealing; after opening every packet must
    authenticate and the sampled payloads must be back to their plaintext."""
    from quantum_amd import batch

    ctx = fuzz_ctxs[("default", "1")]
    n = 1 << 22
    rng = np.random.default_rng(0xF0224000)
    kidx = rng.integers(0, 64, size=n).astype(np.uint32)
    lens = rng.integers(64, 2001, size=n).astype(np.uint32)
    slot = (4 + lens.astype(np.int64) + 28 + 3) & ~3
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(slot)[:-1].astype(np.uint64)
    size = int(offs[-1]) + int(slot[-1]) + 64
    arena = torch.randint(0, 256, (size,), dtype=torch.uint8, device="cuda")
    nonces = torch.randint(0, 256, (12 * n,), dtype=torch.uint8, device="cuda")

    sample = np.sort(rng.choice(n, size=4096, replace=False))
    plain = {int(i): arena[int(offs[i]):int(offs[i]) + int(slot[i])].cpu().numpy().copy() for i in sample}
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    batch.seal_batch(ctx, arena, batch.make_descs(offs, lens, kidx, "cuda"), n, nonces, status=status)
    assert bool(status.bool().all())
    nz = nonces.cpu().numpy()
    for i in sample:
        i = int(i)
        L = int(lens[i])
        buf = plain[i].copy()
        O.aesgo_seal_descs(fuzz_keys, buf, np.zeros(1, dtype=np.uint64), np.array([L], dtype=np.uint32),
                           np.array([kidx[i]], dtype=np.uint32), np.ascontiguousarray(nz[12 * i:12 * i + 12]), 4, 1)
        got = arena[int(offs[i]):int(offs[i]) + int(slot[i])].cpu().numpy()
        assert np.array_equal(got[:4 + L + 28], buf[:4 + L + 28]), f"packet {i} (key {kidx[i]}, {L} B)"
    batch.open_batch(ctx, arena, batch.make_descs(offs, lens + 28, kidx, "cuda"), n, status=status)
    assert bool(status.bool().all())
    for i in sample:
        i = int(i)
        L = int(lens[i])
        got = arena[int(offs[i]):int(offs[i]) + 4 + L].cpu().numpy()
        assert np.array_equal(got, plain[i][:4 + L])
    del arena, nonces, status
    torch.cuda.empty_cache()


@pytest.mark.parametrize("small", ["1", "0"])
@pytest.mark.parametrize("n", [752, 753, 760, 767, 768, 769])
def test_single_key_run_threshold(torch, fuzz_ctxs, fuzz_keys, n, small):
    """A key becomes a segmented-kernel run at kSegMinTiles = 48 tiles, i.e. 753 packets (ceil(n / 16)
    = 48).  Batches of 753..767 packets of ONE key are a run, so the segmented kernel must launch for
    them (it was skipped below 768 packets, leaving the key's packets unsealed with status 0).  Both
    worklist builds (one workgroup, small = "1"; multi-launch radix sort, "0"); 4-B-aligned packed slots
    so the one-workgroup-per-packet path does not take them; seal against the oracle, open back."""
    from quantum_amd import batch

    ctx = fuzz_ctxs[("default", small)]
    rng = np.random.default_rng(0xF0230000 + n)
    kidx = np.full(n, 17, dtype=np.uint32)
    lens = rng.integers(0, 1500, size=n).astype(np.uint32)
    slot = (4 + lens.astype(np.int64) + 28 + 3) & ~3
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(slot)[:-1].astype(np.uint64)
    offs += 4  # 4 mod 16: never the one-workgroup-per-packet path
    size = int(offs[-1]) + int(slot[-1]) + 64
    plain = np.frombuffer(rng.bytes(size), dtype=np.uint8).copy()
    nonces = np.frombuffer(rng.bytes(12 * n), dtype=np.uint8).copy()
    ref = plain.copy()
    O.aesgo_seal_descs(fuzz_keys, ref, offs, lens, kidx, nonces, 4, 8)
    arena = torch.from_numpy(plain.copy()).cuda()
    status = torch.full((n,), 0x5A, dtype=torch.uint8, device="cuda")
    batch.seal_batch(ctx, arena, batch.make_descs(offs, lens, kidx, "cuda"), n, torch.from_numpy(nonces).cuda(),
                     aad_len=4, status=status)
    assert bool((status == 1).all()), f"{int((status != 1).sum())} packets unsealed"
    assert np.array_equal(arena.cpu().numpy(), ref)
    batch.open_batch(ctx, arena, batch.make_descs(offs, lens + 28, kidx, "cuda"), n, aad_len=4, status=status)
    assert bool((status == 1).all())
    got = arena.cpu().numpy()
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        assert np.array_equal(got[o:o + 4 + L], plain[o:o + 4 + L]), i
