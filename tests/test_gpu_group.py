"""Several device contexts behind one process (qgcm_group_*, SURVEY.md s8e, main.go:72-75) and BASELINE
config 4's per-GPU shard.

* G = 2 and G = 3 member contexts on device 0 (the 1-GPU box stands in for a node's GPUs): a keyed
  host batch is split by hash(key_idx) mod G (quantum_amd.shard.key_shard), each member runs its
  packets on its own thread and streams, and every slot comes back in place bit-exact with the
  oracle; keys live only on their owning member; tamper -> status 0 + zeroed plaintext; a key that no
  member holds -> status 0, slot untouched.
* One GPU's full config-4 shard: 8 x 2^20 packets x 1350 B (11.8 GB of slots resident), its first
  2^20 slots equal to the committed config-2 digest, every packet authentic after the open and its
  payload restored.
"""
import ctypes as C
import hashlib
import random

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

AAD = bytes([10, 99, 0, 1])
DESC_ONE_MAX = 8192  # gcm_internal.h kDescOneMax
DIRECT_MAX = 65536  # gcm_internal.h kDirectMax


@pytest.fixture(scope="module")
def torch():
    import torch as T

    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


def host_buffer(nbytes: int, pinned: bool):
    from quantum_amd import _lib

    if pinned:
        ptr = _lib.lib().qgcm_host_alloc(nbytes)
        assert ptr
        arr = np.frombuffer((C.c_uint8 * nbytes).from_address(ptr), dtype=np.uint8)
        return arr, ptr, lambda: _lib.lib().qgcm_host_free(ptr)
    arr = np.zeros(nbytes, dtype=np.uint8)
    return arr, arr.ctypes.data, lambda: None


@pytest.mark.parametrize("G,pinned,threads,zc,dma,grouped", [
    (2, True, "4", "1", "0", False), (3, False, "7", "1", "0", False), (1, True, "1", "1", "0", False),
    (2, True, "3", "0", "0", False),
    (1, True, "4", "1", "1", False), (2, True, "4", "1", "1", True), (3, False, "4", "1", "1", True),
    (2, True, "4", "1", "1", False)])
def test_group_keyed_host_batch_vs_oracle(torch, G, pinned, threads, zc, dma, grouped, monkeypatch):
    """threads: QGCM_GROUP_THREADS, the gather/scatter copy threads per member; zc: QGCM_GROUP_ZEROCOPY
    (pinned arenas take the GPU gather/scatter path unless it is 0; pageable ones always the copy path);
    dma: QGCM_GROUP_DMA -- a member whose packets form long runs of adjacent records (one member, or the
    batch laid out member by member in qgcm_group_order's order: `grouped`) copies whole runs by DMA;
    interleaved members fall back to the paths above."""
    from quantum_amd import shard

    monkeypatch.setenv("QGCM_GROUP_THREADS", threads)
    monkeypatch.setenv("QGCM_GROUP_ZEROCOPY", zc)
    monkeypatch.setenv("QGCM_GROUP_DMA", dma)
    grp = shard.Group([0] * G, max_keys=256)
    try:
        rng = random.Random(0x6A0 + G)
        nkeys = 40
        keys = [rng.randbytes(32) for _ in range(nkeys)]
        grp.set_keys(0, b"".join(keys))
        assert [grp.shard(k) for k in range(256)] == shard.key_shard(np.arange(256), G).tolist()
        owners = shard.key_shard(np.arange(nkeys), G)
        assert len(set(owners.tolist())) == G  # every member owns some of the peers
        n = 3000
        kidx = [200 if i % 97 == 5 else rng.randrange(nkeys) for i in range(n)]  # key 200: no member has it
        lens = [rng.choice([0, 1, 15, 16, 17, 1350, 1433, 4081]) if i % 4 else rng.randint(0, 3000) for i in range(n)]
        if grouped:  # the batch assembled member by member (qgcm_group_order)
            order, counts = grp.order(kidx)
            assert counts.tolist() == [int((shard.key_shard(np.array(kidx), G) == m).sum()) for m in range(G)]
            assert np.array_equal(np.concatenate(shard.partition_by_key(kidx, G)), order)
            kidx = [kidx[i] for i in order]
            lens = [lens[i] for i in order]
        want_path = "dma" if dma == "1" and (G == 1 or grouped) else ("zerocopy" if pinned and zc == "1" else "copy")
        offs, pos = [], 0
        for i, L in enumerate(lens):  # 4-B and 16-B aligned slots mixed
            offs.append(pos)
            pos += (4 + L + 28 + 15) & ~15 if i % 2 else (4 + L + 28 + 3) & ~3
        arena, aptr, free = host_buffer(pos + 64, pinned)
        try:
            arena[:] = np.frombuffer(rng.randbytes(pos + 64), dtype=np.uint8)
            for i in range(n):
                arena[offs[i]:offs[i] + 4] = np.frombuffer(AAD, dtype=np.uint8)
            plain = arena.copy()
            nonces, _, free_n = host_buffer(12 * n, pinned)  # pinned nonces keep the seal zero-copy too
            nonces[:] = np.frombuffer(rng.randbytes(12 * n), dtype=np.uint8)
            ref = plain.copy()
            for i, L in enumerate(lens):
                if kidx[i] >= nkeys:
                    continue
                buf = bytearray(ref[offs[i] + 4:offs[i] + 4 + L + 28].tobytes())
                O.aesgo_encrypt(keys[kidx[i]], buf, L, AAD, bytes(nonces[12 * i:12 * i + 12]))
                ref[offs[i] + 4:offs[i] + 4 + L + 28] = np.frombuffer(bytes(buf), dtype=np.uint8)
            descs = shard.host_descs(offs, lens, kidx)
            status = np.full(n, 7, dtype=np.uint8)
            unset = sum(k >= nkeys for k in kidx)
            bad = grp.seal_host(aptr, descs, n, nonces.ctypes.data, 4, status.ctypes.data)
            assert [grp.last_path(m) for m in range(G)] == [want_path] * G
            assert grp.last_zerocopy() == (want_path == "zerocopy")
            assert bad == unset
            assert status.tolist() == [0 if k >= nkeys else 1 for k in kidx]
            assert np.array_equal(arena, ref)  # every slot in place, input order kept

            tampered = set(rng.sample([i for i in range(n) if kidx[i] < nkeys], 40))
            for i in tampered:
                arena[offs[i] + 4 + lens[i] + rng.randrange(28)] ^= 0x04
            before = arena.copy()
            d_open = shard.host_descs(offs, [L + 28 for L in lens], kidx)
            status[:] = 7
            bad = grp.open_host(aptr, d_open, n, 4, status.ctypes.data)
            assert [grp.last_path(m) for m in range(G)] == [want_path] * G
            assert bad == unset + len(tampered)
            for i, L in enumerate(lens):
                o = offs[i]
                if kidx[i] >= nkeys:
                    assert status[i] == 0 and np.array_equal(arena[o:o + 4 + L + 28], before[o:o + 4 + L + 28])
                elif i in tampered:
                    assert status[i] == 0 and not arena[o + 4:o + 4 + L].any()
                    assert np.array_equal(arena[o + 4 + L:o + 4 + L + 28], before[o + 4 + L:o + 4 + L + 28])
                else:
                    assert status[i] == 1 and np.array_equal(arena[o:o + 4 + L], plain[o:o + 4 + L])
            del nonces
            free_n()
        finally:
            free()
    finally:
        grp.close()


@pytest.mark.parametrize("shift,slots", [(0, "3"), (68, "3"), (0, "2"), (0, "16")])
def test_group_dma_runs_many_chunks_vs_oracle(torch, shift, slots, monkeypatch):
    """slots: QGCM_GROUP_DMA_SLOTS, staging slots in flight (3, the default; 2: every slot reused twice; 16:
    none reused); shift: the arena starts this many bytes past the pinned allocation's start (staging
    keeps host addresses mod 256).
    DMA-run path over more chunks than staging slots (slot reuse: 64-MiB chunks via
    QGCM_GROUP_DMA_CHUNK_MB), two members on device 0 with
    the batch laid out member by member: 2^19 packets, the first half of 1184..1440 B in 1472-B
    Payload.Raw slots (gaps of up to 256 B inside a run; every 1000th slot 1 KiB further on, which breaks
    the run), the second half of U{0..2000} B in 16-B packed slots; sealed against the oracle, then opened
    back and every byte of the arena checked."""
    from quantum_amd import shard

    monkeypatch.setenv("QGCM_GROUP_DMA_SLOTS", slots)
    monkeypatch.setenv("QGCM_GROUP_DMA_CHUNK_MB", "64")
    G, n = 2, 1 << 19  # ~660 MB of records: 5 chunks of 64 MiB per member, more than its 3 staging slots
    grp = shard.Group([0] * G, max_keys=64)
    try:
        rng = np.random.default_rng(0x6A05)
        keys = rng.integers(0, 256, 32 * 16, dtype=np.uint8).tobytes()
        grp.set_keys(0, keys)
        kidx = rng.integers(0, 16, n).astype(np.uint32)
        order, _ = grp.order(kidx)
        kidx = kidx[order]
        lens = rng.integers(0, 2001, n).astype(np.uint32)
        lens[: n // 2] = 1184 + lens[: n // 2] % 257  # Raw slots: 4 + L + 28 <= 1472, gaps <= 256 B
        rec = ((4 + lens.astype(np.uint64) + 28 + 15) & ~np.uint64(15))
        offs = np.zeros(n, np.uint64)
        # every 1000th slot starts 1 KiB further on: the runs break there
        offs[: n // 2] = np.arange(n // 2, dtype=np.uint64) * np.uint64(1472) + \
            np.uint64(1024) * (np.arange(n // 2, dtype=np.uint64) // np.uint64(1000))
        base = offs[n // 2 - 1] + np.uint64(1472)
        offs[n // 2:] = base + np.concatenate([[0], np.cumsum(rec[n // 2:])[:-1]]).astype(np.uint64)
        size = int(offs[-1] + rec[-1]) + 64
        whole, wptr, free = host_buffer(size + shift, True)
        arena, aptr = whole[shift:], wptr + shift
        nonces, nptr, free_n = host_buffer(12 * n, True)
        try:
            arena[:] = rng.integers(0, 256, size, dtype=np.uint8)
            idx = offs.astype(np.int64)[:, None] + np.arange(4)
            arena[idx] = np.frombuffer(AAD, np.uint8)
            nonces[:] = rng.integers(0, 256, 12 * n, dtype=np.uint8)
            plain = arena.copy()
            ref = plain.copy()
            O.aesgo_seal_descs(keys, ref, offs, lens, kidx, nonces, 4, 16)
            status = np.zeros(n, np.uint8)
            assert grp.seal_host(aptr, shard.host_descs(offs, lens, kidx), n, nptr, 4, status.ctypes.data) == 0
            assert [grp.last_path(m) for m in range(G)] == ["dma", "dma"]
            assert bool((status == 1).all()) and np.array_equal(arena, ref)
            status[:] = 0
            assert grp.open_host(aptr, shard.host_descs(offs, lens + 28, kidx), n, 4, status.ctypes.data) == 0
            assert bool((status == 1).all())
            pay = offs.astype(np.int64)
            for i in range(0, n, 997):  # sampled plaintext restored (the full arena below)
                assert np.array_equal(arena[pay[i]:pay[i] + 4 + lens[i]], plain[pay[i]:pay[i] + 4 + lens[i]])
            tail = (offs.astype(np.int64) + 4 + lens.astype(np.int64))[:, None] + np.arange(28)
            restored = arena.copy()
            restored[tail] = plain[tail]  # Open leaves tag || nonce in the slot
            assert np.array_equal(restored, plain)
        finally:
            free()
            free_n()
    finally:
        grp.close()


@pytest.mark.parametrize("G,grouped", [(1, False), (2, True), (2, False)])
def test_group_seal_with_nonces_in_the_slots(torch, G, grouped):
    """qgcm_group_seal_host with h_nonces NULL: each packet's nonce is already in its slot (the 12 bytes
    after the tag's place), as a caller that draws nonces into the slots itself lays them out.  Paths:
    one member (DMA runs), two members in qgcm_group_order's order (DMA runs) and interleaved (zero-copy);
    sealed bytes against the oracle with those nonces, then opened back."""
    from quantum_amd import shard

    grp = shard.Group([0] * G, max_keys=32)
    try:
        rng = np.random.default_rng(0x6A07 + G + 10 * grouped)
        keys = rng.integers(0, 256, 32 * 8, dtype=np.uint8).tobytes()
        grp.set_keys(0, keys)
        n = 2000
        kidx = rng.integers(0, 8, n).astype(np.uint32)
        if grouped:
            kidx = kidx[grp.order(kidx)[0]]
        lens = rng.integers(0, 3000, n).astype(np.uint32)
        rec = (4 + lens.astype(np.uint64) + 28 + 3) & ~np.uint64(3)
        offs = np.concatenate([[0], np.cumsum(rec)[:-1]]).astype(np.uint64)
        size = int(offs[-1] + rec[-1])
        arena, aptr, free = host_buffer(size, True)
        try:
            arena[:] = rng.integers(0, 256, size, dtype=np.uint8)
            idx = offs.astype(np.int64)[:, None] + np.arange(4)
            arena[idx] = np.frombuffer(AAD, np.uint8)
            nonce_at = (offs.astype(np.int64) + 4 + lens.astype(np.int64) + 16)[:, None] + np.arange(12)
            nonces = np.ascontiguousarray(arena[nonce_at].reshape(-1))
            plain = arena.copy()
            ref = plain.copy()
            O.aesgo_seal_descs(keys, ref, offs, lens, kidx, nonces, 4, 8)
            status = np.zeros(n, np.uint8)
            assert grp.seal_host(aptr, shard.host_descs(offs, lens, kidx), n, None, 4, status.ctypes.data) == 0
            want = "dma" if (G == 1 or grouped) else "zerocopy"
            assert [grp.last_path(m) for m in range(G)] == [want] * G
            assert bool((status == 1).all()) and np.array_equal(arena, ref)
            assert grp.open_host(aptr, shard.host_descs(offs, lens + 28, kidx), n, 4, status.ctypes.data) == 0
            pay = np.concatenate([np.arange(int(o), int(o) + 4 + int(L)) for o, L in zip(offs, lens)])
            assert np.array_equal(arena[pay], plain[pay])
        finally:
            free()
    finally:
        grp.close()


def test_group_unaligned_records_take_the_copy_path(torch):
    """Records packed back to back with no alignment (offsets not multiples of 4): neither DMA runs nor
    zero-copy apply (both move records dword-wise), so the member gathers them through pinned staging;
    sealed bytes against the oracle, opened back."""
    from quantum_amd import shard

    grp = shard.Group([0], max_keys=8)
    try:
        rng = np.random.default_rng(0x6A08)
        keys = rng.integers(0, 256, 32 * 4, dtype=np.uint8).tobytes()
        grp.set_keys(0, keys)
        n = 1500
        kidx = rng.integers(0, 4, n).astype(np.uint32)
        lens = rng.integers(0, 2000, n).astype(np.uint32)
        rec = 4 + lens.astype(np.uint64) + 28
        offs = np.concatenate([[0], np.cumsum(rec)[:-1]]).astype(np.uint64)
        assert bool((offs % 4 != 0).any())
        size = int(offs[-1] + rec[-1])
        arena, aptr, free = host_buffer(size, True)
        try:
            arena[:] = rng.integers(0, 256, size, dtype=np.uint8)
            arena[offs.astype(np.int64)[:, None] + np.arange(4)] = np.frombuffer(AAD, np.uint8)
            nonces, nptr, free_n = host_buffer(12 * n, True)
            nonces[:] = rng.integers(0, 256, 12 * n, dtype=np.uint8)
            plain, ref = arena.copy(), arena.copy()
            O.aesgo_seal_descs(keys, ref, offs, lens, kidx, np.ascontiguousarray(nonces), 4, 8)
            status = np.zeros(n, np.uint8)
            assert grp.seal_host(aptr, shard.host_descs(offs, lens, kidx), n, nptr, 4, status.ctypes.data) == 0
            assert grp.last_path(0) == "copy"
            assert bool((status == 1).all()) and np.array_equal(arena, ref)
            assert grp.open_host(aptr, shard.host_descs(offs, lens + 28, kidx), n, 4, status.ctypes.data) == 0
            pay = np.concatenate([np.arange(int(o), int(o) + 4 + int(L)) for o, L in zip(offs, lens)])
            assert np.array_equal(arena[pay], plain[pay])
            del nonces
            free_n()
        finally:
            free()
    finally:
        grp.close()


@pytest.mark.parametrize("n,one,align,direct", [(1, "1", 16, "1"), (64, "1", 16, "1"), (700, "1", 16, "1"),
                                                (8192, "1", 16, "0"), (8193, "1", 16, "0"), (8193, "1", 16, "1"),
                                                (65536, "1", 16, "1"), (65537, "1", 16, "1"), (700, "0", 16, "1"),
                                                (64, "1", 4, "1"), (64, "1", 16, "0"), (700, "1", 16, "0"),
                                                (700, "1", 16, "slot")])
def test_group_small_batches_one_workgroup_per_packet(torch, n, one, align, direct, monkeypatch):
    """A one-member batch of up to 8192 packets (kDescOneMax) whose records all start 16-B aligned runs one workgroup
    per packet (gcm_one_kernel reading descriptors) instead of the worklist + per-wave kernel; larger
    batches, 4-B-aligned records or QGCM_DESC_ONE=0 take the latter.  Records packed at `align` with
    random bytes in the gaps; seal against the oracle over the whole arena (gaps untouched), statuses
    start as junk, a key no member holds and opens shorter than 28 B fail with the slot untouched,
    tampered packets are zeroed.  direct: QGCM_GROUP_DIRECT -- such a batch in a pinned arena is sealed in
    place over PCIe ("1", path "direct"), or copied by DMA ("0"); "slot": direct with each nonce already in
    its slot (h_nonces NULL)."""
    from quantum_amd import shard

    monkeypatch.setenv("QGCM_DESC_ONE", one)
    monkeypatch.setenv("QGCM_GROUP_DIRECT", "0" if direct == "0" else "1")
    grp = shard.Group([0], max_keys=256)
    try:
        rng = np.random.default_rng(0x6A10 + n + align)
        nkeys = 8
        keys = rng.integers(0, 256, 32 * nkeys, dtype=np.uint8).tobytes()
        grp.set_keys(0, keys)
        kidx = rng.integers(0, nkeys, n).astype(np.uint32)
        if n > 1:
            kidx[n - max(1, n // 40):] = 200  # no member holds key 200 (at the end: the others stay one run)
        lens = rng.choice([0, 1, 15, 16, 17, 100, 1350, 1433, 4081, 9000], n).astype(np.uint32)
        mix = rng.random(n) < 0.5
        lens[mix] = rng.integers(0, 1500, int(mix.sum()))
        rec = 4 + lens.astype(np.uint64) + 28
        step = (rec + align - 1) // align * align + align * rng.integers(0, 2, n).astype(np.uint64)
        offs = np.concatenate([[0], np.cumsum(step)[:-1]]).astype(np.uint64)
        size = int(offs[-1] + step[-1])
        arena, aptr, free = host_buffer(size, True)
        ctx = grp.member(0)
        try:
            arena[:] = rng.integers(0, 256, size, dtype=np.uint8)
            arena[offs.astype(np.int64)[:, None] + np.arange(4)] = np.frombuffer(AAD, np.uint8)
            nonces, nptr, free_n = host_buffer(12 * n, True)
            nonces[:] = rng.integers(0, 256, 12 * n, dtype=np.uint8)
            if direct == "slot":  # the nonce sits after the tag's place; the call gets no nonce array
                at = (offs.astype(np.int64) + 4 + lens.astype(np.int64) + 16)[:, None] + np.arange(12)
                arena[at] = nonces.reshape(n, 12)
                nptr = None
            plain, ref = arena.copy(), arena.copy()
            ok = kidx < nkeys
            vi = np.flatnonzero(ok)
            if len(vi):
                O.aesgo_seal_descs(keys, ref, np.ascontiguousarray(offs[vi]), np.ascontiguousarray(lens[vi]),
                                   np.ascontiguousarray(kidx[vi]),
                                   np.ascontiguousarray(nonces.reshape(n, 12)[vi]).reshape(-1), 4, 8)
            c0 = ctx.launch_counts()
            status = np.full(n, 7, np.uint8)
            bad = grp.seal_host(aptr, shard.host_descs(offs, lens, kidx), n, nptr, 4, status.ctypes.data)
            c1 = ctx.launch_counts()
            path = grp.last_path(0)
            if one == "1" and align == 16 and direct != "0" and n <= DIRECT_MAX:
                assert path == "direct"
                want_one = True
            else:  # one run under kMinRun (64 KiB) goes zero-copy instead
                assert path == ("dma" if int(offs[-max(1, n // 40)]) >= 64 << 10 else "zerocopy")
                want_one = one == "1" and n <= DESC_ONE_MAX and align == 16 and path == "dma"
            assert c1["one"] - c0["one"] == (1 if want_one else 0), (c0, c1)
            assert bad == int((~ok).sum()) and np.array_equal(status, ok.astype(np.uint8))
            assert np.array_equal(arena, ref)

            tam = np.zeros(n, bool)
            tam[rng.choice(vi, size=max(1, len(vi) // 20), replace=False)] = len(vi) > 1
            for i in np.flatnonzero(tam):
                arena[int(offs[i]) + 4 + int(rng.integers(0, int(lens[i]) + 28))] ^= 0x10
            olens = lens + 28
            short = (rng.random(n) < 0.02) & ~tam
            olens[short] = rng.integers(0, 28, int(short.sum()))
            before = arena.copy()
            exp = before.copy()
            good = ok & ~short
            ost = np.zeros(n, np.uint8)
            gi = np.flatnonzero(good)
            if len(gi):
                sub = np.zeros(len(gi), np.uint8)
                O.aesgo_open_descs(keys, exp, np.ascontiguousarray(offs[gi]), np.ascontiguousarray(olens[gi]),
                                   np.ascontiguousarray(kidx[gi]), sub, 4, 8)
                ost[gi] = sub
            assert np.array_equal(ost[good], (~tam[good]).astype(np.uint8))
            status[:] = 7
            bad = grp.open_host(aptr, shard.host_descs(offs, olens, kidx), n, 4, status.ctypes.data)
            # shortened opens are rejected before the member (its batch is smaller) and can split the run
            # (gaps past kRunGap), so the open's path is its own
            m = int((olens >= 28).sum())
            if one == "1" and align == 16 and direct != "0" and m <= DIRECT_MAX:
                assert grp.last_path(0) == "direct"
                want_one = True
            else:
                want_one = one == "1" and m <= DESC_ONE_MAX and align == 16 and grp.last_path(0) == "dma"
            assert ctx.launch_counts()["one"] - c1["one"] == (1 if want_one else 0)
            assert bad == int((ost == 0).sum()) and np.array_equal(status, ost)
            assert np.array_equal(arena, exp)
            pay = [i for i in gi if not tam[i]]
            for i in pay[:: max(1, len(pay) // 200)]:
                o, L = int(offs[i]), int(lens[i])
                assert np.array_equal(arena[o:o + 4 + L], plain[o:o + 4 + L]), i
            del nonces
            free_n()
        finally:
            free()
    finally:
        grp.close()


@pytest.mark.parametrize("G,direct,pinned_nonces", [(2, "1", True), (3, "1", False), (2, "0", True)])
def test_group_interleaved_members_seal_in_place(torch, G, direct, pinned_nonces, monkeypatch):
    """Several members with their packets interleaved in one pinned arena (no DMA runs): each member's
    worker-sized share of 16-B-aligned records is sealed in place by its own GPU ("direct"), the members
    at once; QGCM_GROUP_DIRECT=0: zero-copy gather/scatter.  Against the oracle over the whole arena,
    nonces from pinned or pageable memory, then tampered packets fail and the rest open back."""
    from quantum_amd import shard

    monkeypatch.setenv("QGCM_GROUP_DIRECT", direct)
    grp = shard.Group([0] * G, max_keys=64)
    try:
        rng = np.random.default_rng(0x6A20 + G)
        nkeys = 24
        keys = rng.integers(0, 256, 32 * nkeys, dtype=np.uint8).tobytes()
        grp.set_keys(0, keys)
        n = 900
        kidx = rng.integers(0, nkeys, n).astype(np.uint32)
        assert len(set(shard.key_shard(kidx, G).tolist())) == G
        lens = rng.integers(0, 1500, n).astype(np.uint32)
        step = (4 + lens.astype(np.uint64) + 28 + 15) // 16 * 16
        offs = np.concatenate([[0], np.cumsum(step)[:-1]]).astype(np.uint64)
        size = int(offs[-1] + step[-1])
        arena, aptr, free = host_buffer(size, True)
        nonces, nptr, free_n = host_buffer(12 * n, pinned_nonces)
        try:
            arena[:] = rng.integers(0, 256, size, dtype=np.uint8)
            arena[offs.astype(np.int64)[:, None] + np.arange(4)] = np.frombuffer(AAD, np.uint8)
            nonces[:] = rng.integers(0, 256, 12 * n, dtype=np.uint8)
            plain, ref = arena.copy(), arena.copy()
            O.aesgo_seal_descs(keys, ref, offs, lens, kidx, np.ascontiguousarray(nonces), 4, 8)
            status = np.full(n, 7, np.uint8)
            assert grp.seal_host(aptr, shard.host_descs(offs, lens, kidx), n, nptr, 4, status.ctypes.data) == 0
            want = "direct" if direct == "1" else "zerocopy"
            assert [grp.last_path(m) for m in range(G)] == [want] * G
            assert bool((status == 1).all()) and np.array_equal(arena, ref)
            tam = rng.choice(n, size=30, replace=False)
            for i in tam:
                arena[int(offs[i]) + 4 + int(rng.integers(0, int(lens[i]) + 28))] ^= 0x08
            status[:] = 7
            assert grp.open_host(aptr, shard.host_descs(offs, lens + 28, kidx), n, 4, status.ctypes.data) == len(tam)
            assert [grp.last_path(m) for m in range(G)] == [want] * G
            ok = np.ones(n, bool)
            ok[tam] = False
            assert np.array_equal(status, ok.astype(np.uint8))
            for i in range(n):
                o, L = int(offs[i]), int(lens[i])
                if ok[i]:
                    assert np.array_equal(arena[o:o + 4 + L], plain[o:o + 4 + L]), i
                else:
                    assert not arena[o + 4:o + 4 + L].any(), i
        finally:
            del nonces
            free_n()
            free()
    finally:
        grp.close()


@pytest.mark.parametrize("G", [2, 3])
def test_group_mixed_alignment_members_never_overwrite(torch, G):
    """the direct (in place) path writes each record's 16-B-rounded area back, so a record
    of ANOTHER member that starts inside that rounded tail (4-B packed, right behind the record) would
    get stale bytes written over its result while both members run at once.  Records are interleaved
    over the members in one pinned arena, packed at 4-B alignment so every record starts in the
    previous one's rounded tail; a few of them 16-B aligned.  No member may go direct, and sealed and
    opened bytes must equal the oracle over the whole arena, several rounds (the race was timing-bound)."""
    from quantum_amd import shard

    grp = shard.Group([0] * G, max_keys=64)
    try:
        rng = np.random.default_rng(0x6A30 + G)
        nkeys = 24
        keys = rng.integers(0, 256, 32 * nkeys, dtype=np.uint8).tobytes()
        grp.set_keys(0, keys)
        n = 1200
        kidx = rng.integers(0, nkeys, n).astype(np.uint32)
        assert len(set(shard.key_shard(kidx, G).tolist())) == G
        lens = rng.integers(0, 1500, n).astype(np.uint32)
        step = (4 + lens.astype(np.uint64) + 28 + 3) // 4 * 4  # packed: 4-B aligned records
        step[rng.random(n) < 0.1] += 12  # some records end up 16-B aligned, most not
        offs = np.concatenate([[0], np.cumsum(step)[:-1]]).astype(np.uint64)
        assert (offs % 16 == 0).any() and (offs % 16 != 0).any()
        size = int(offs[-1] + step[-1]) + 16
        arena, aptr, free = host_buffer(size, True)
        nonces, nptr, free_n = host_buffer(12 * n, True)
        try:
            for rnd in range(4):
                arena[:] = rng.integers(0, 256, size, dtype=np.uint8)
                arena[offs.astype(np.int64)[:, None] + np.arange(4)] = np.frombuffer(AAD, np.uint8)
                nonces[:] = rng.integers(0, 256, 12 * n, dtype=np.uint8)
                plain, ref = arena.copy(), arena.copy()
                O.aesgo_seal_descs(keys, ref, offs, lens, kidx, np.ascontiguousarray(nonces), 4, 8)
                status = np.full(n, 7, np.uint8)
                assert grp.seal_host(aptr, shard.host_descs(offs, lens, kidx), n, nptr, 4, status.ctypes.data) == 0
                assert "direct" not in [grp.last_path(m) for m in range(G)]
                assert bool((status == 1).all()) and np.array_equal(arena, ref), rnd
                assert grp.open_host(aptr, shard.host_descs(offs, lens + 28, kidx), n, 4, status.ctypes.data) == 0
                assert "direct" not in [grp.last_path(m) for m in range(G)]
                # opened: the plaintext back, each slot's tag || nonce left as sealed (Open never writes them)
                want = ref.copy()
                pay = np.zeros(size, bool)
                for o, L in zip(offs.astype(np.int64), lens.astype(np.int64)):
                    pay[o + 4:o + 4 + L] = True
                want[pay] = plain[pay]
                assert bool((status == 1).all()) and np.array_equal(arena, want), rnd
        finally:
            del nonces
            free_n()
            free()
    finally:
        grp.close()


def test_group_zerocopy_records_at_the_allocation_end(torch):
    """Zero-copy path: records whose last byte is the last bytes of a one-page pinned allocation, with
    lengths that are not multiples of 4 or 16 (the gather reads whole dwords up to the next 4-B
    boundary only, the scatter writes exact bytes); sealed and opened against the oracle."""
    from quantum_amd import shard

    grp = shard.Group([0], max_keys=4)
    arena, aptr, free = host_buffer(4096, True)
    nb, nptr, free_n = host_buffer(4096, True)
    try:
        key = bytes(range(32))
        grp.set_keys(0, key)
        rng = random.Random(0x0E7)
        lens = [1, 1001, 2017]  # 4 + L + 28 = 33 / 1033 / 2049 B: the last record ends at byte 4093
        offs = [0, 40]
        offs.append(4093 - (4 + lens[2] + 28))
        assert offs[2] % 4 == 0 and offs[1] + 4 + lens[1] + 28 <= offs[2]
        arena[:] = np.frombuffer(rng.randbytes(4096), dtype=np.uint8)
        for o in offs:
            arena[o:o + 4] = np.frombuffer(AAD, dtype=np.uint8)
        nb[:36] = np.frombuffer(rng.randbytes(36), dtype=np.uint8)
        plain = arena.copy()
        ref = plain.copy()
        for i, L in enumerate(lens):
            buf = bytearray(ref[offs[i] + 4:offs[i] + 4 + L + 28].tobytes())
            O.aesgo_encrypt(key, buf, L, AAD, bytes(nb[12 * i:12 * i + 12]))
            ref[offs[i] + 4:offs[i] + 4 + L + 28] = np.frombuffer(bytes(buf), dtype=np.uint8)
        status = np.zeros(3, dtype=np.uint8)
        assert grp.seal_host(aptr, shard.host_descs(offs, lens, [0, 0, 0]), 3, nptr, 4, status.ctypes.data) == 0
        assert grp.last_zerocopy()
        assert status.tolist() == [1, 1, 1] and np.array_equal(arena, ref)
        assert grp.open_host(aptr, shard.host_descs(offs, [L + 28 for L in lens], [0, 0, 0]), 3, 4,
                             status.ctypes.data) == 0
        assert status.tolist() == [1, 1, 1]
        for i, L in enumerate(lens):
            assert np.array_equal(arena[offs[i]:offs[i] + 4 + L], plain[offs[i]:offs[i] + 4 + L])
        assert np.array_equal(arena[4093:], plain[4093:])  # nothing written past the last record
    finally:
        free()
        free_n()
        grp.close()


def test_group_members_hold_only_their_keys(torch):
    """A member's own context rejects a key another member owns (status 0, slot untouched)."""
    from quantum_amd import batch, shard

    grp = shard.Group([0, 0], max_keys=16)
    try:
        keys = [bytes([k]) * 32 for k in range(8)]
        grp.set_keys(0, b"".join(keys))
        owner = [grp.shard(k) for k in range(8)]
        for m in (0, 1):
            ctx = grp.member(m)
            arena = torch.zeros(8 * 128, dtype=torch.uint8, device="cuda")
            status = torch.full((8,), 7, dtype=torch.uint8, device="cuda")
            batch.seal_batch(ctx, arena, batch.make_descs([128 * k for k in range(8)], [64] * 8, list(range(8)), "cuda"),
                             8, None, status=status)
            assert status.cpu().tolist() == [1 if owner[k] == m else 0 for k in range(8)]
    finally:
        grp.close()


def test_group_member_threads_numa_local(torch):
    """Each member's host thread is pinned to its GPU's NUMA-local CPUs (sysfs local_cpulist of the
    PCI device, within the CPUs this process may use), SURVEY.md s8e."""
    import os

    from quantum_amd import shard

    grp = shard.Group([0, 0], max_keys=4)
    try:
        allowed = len(os.sched_getaffinity(0))
        n = [grp.member_cpus(m) for m in (0, 1)]
        assert n[0] == n[1] and 0 <= n[0] <= allowed
        if os.path.isdir("/sys/bus/pci/devices"):
            assert n[0] > 0  # the box exposes the GPU's local_cpulist
    finally:
        grp.close()


def test_config4_one_gpu_shard(torch, batch_digests):
    """8 x 2^20 packets x 1350 B on one GPU = its shard of config 4 (64 x 2^20 over 8 GPUs)."""
    from quantum_amd import batch
    from quantum_amd.crypto import Context, derive_key

    d = next(x for x in batch_digests if x["n"] == 1 << 20 and x["len"] == 1350)
    N, L, stride = 8 << 20, d["len"], d["stride"]
    ctx = Context(device=0, max_keys=4)
    ctx.set_key(0, derive_key(b"AES256Key-32Characters1234567890", bytes(range(32))))
    arena = torch.zeros(N * stride, dtype=torch.uint8, device="cuda")  # gaps zeroed, as the golden arena
    nonces = torch.empty(12 * N, dtype=torch.uint8, device="cuda")
    aad_word = int.from_bytes(AAD, "little")
    batch.fill_uniform(arena, stride, N, L, aad_word, d["seed_payload"], nonces, d["seed_nonce"])
    status = torch.zeros(N, dtype=torch.uint8, device="cuda")
    batch.seal_uniform(ctx, arena, stride, N, L, 0, nonces, status=status)
    assert int(status.sum()) == N
    h = hashlib.sha256()
    head = (1 << 20) * stride
    for i in range(0, head, 1 << 28):
        h.update(memoryview(arena[i:min(head, i + (1 << 28))].cpu().numpy()))
    assert h.hexdigest() == d["sha256_sealed"]  # the first 2^20 slots are config 2's sealed arena
    status.zero_()
    batch.open_uniform(ctx, arena, stride, N, L + 28, 0, status=status)
    assert int(status.sum()) == N
    ref = torch.empty_like(arena)
    batch.fill_uniform(ref, stride, N, L, aad_word, d["seed_payload"], None, 0)
    a2, r2 = arena.view(N, stride), ref.view(N, stride)
    assert torch.equal(a2[:, :4 + L], r2[:, :4 + L])  # every payload restored in place
    del arena, ref, a2, r2, nonces
    ctx.close()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("layout", ["ordered", "interleaved"])
def test_group_eight_members_vs_oracle(torch, layout):
    """G = 8, the node's GPU count (all members on device 0 here): a keyed batch of 40 000 packets of 96
    peers.  "ordered": laid out member by member (qgcm_group_order), so every member moves its packets
    by DMA runs; "interleaved": input order, 4-B-packed records, so members gather their shares (zero-copy
    path).  Keys installed on their owners only; sealed against the oracle over the whole arena, then
    opened back (a tampered packet per member fails with its plaintext zeroed)."""
    from quantum_amd import shard

    G, n, nkeys = 8, 40000, 96
    grp = shard.Group([0] * G, max_keys=128)
    try:
        rng = np.random.default_rng(0x6A80 + (layout == "ordered"))
        keys = rng.integers(0, 256, 32 * nkeys, dtype=np.uint8).tobytes()
        grp.set_keys(0, keys)
        kidx = rng.integers(0, nkeys, n).astype(np.uint32)
        assert len(set(shard.key_shard(kidx, G).tolist())) == G
        if layout == "ordered":
            order, counts = grp.order(kidx)
            kidx = kidx[order]
            assert int(counts.sum()) == n and (counts > 0).all()
        lens = rng.integers(0, 1500, n).astype(np.uint32)
        step = (4 + lens.astype(np.uint64) + 28 + 3) // 4 * 4
        offs = np.concatenate([[0], np.cumsum(step)[:-1]]).astype(np.uint64)
        size = int(offs[-1] + step[-1]) + 64
        arena, aptr, free = host_buffer(size, True)
        nonces, nptr, free_n = host_buffer(12 * n, True)
        try:
            arena[:] = rng.integers(0, 256, size, dtype=np.uint8)
            arena[offs.astype(np.int64)[:, None] + np.arange(4)] = np.frombuffer(AAD, np.uint8)
            nonces[:] = rng.integers(0, 256, 12 * n, dtype=np.uint8)
            plain, ref = arena.copy(), arena.copy()
            O.aesgo_seal_descs(keys, ref, offs, lens, kidx, np.ascontiguousarray(nonces), 4, 8)
            status = np.full(n, 7, np.uint8)
            assert grp.seal_host(aptr, shard.host_descs(offs, lens, kidx), n, nptr, 4, status.ctypes.data) == 0
            paths = {grp.last_path(m) for m in range(G)}
            assert paths == ({"dma"} if layout == "ordered" else {"zerocopy"}), paths
            assert bool((status == 1).all()) and np.array_equal(arena, ref)
            owner = shard.key_shard(kidx, G)
            tam = np.array([int(np.nonzero((owner == m) & (lens > 0))[0][0]) for m in range(G)])
            for i in tam:
                arena[int(offs[i]) + 4] ^= 0x10
            assert grp.open_host(aptr, shard.host_descs(offs, lens + 28, kidx), n, 4, status.ctypes.data) == G
            ok = np.ones(n, bool)
            ok[tam] = False
            assert np.array_equal(status, ok.astype(np.uint8))
            for i in range(n):
                o, L = int(offs[i]), int(lens[i])
                if ok[i]:
                    assert np.array_equal(arena[o:o + 4 + L], plain[o:o + 4 + L]), i
                else:
                    assert not arena[o + 4:o + 4 + L].any(), i
        finally:
            del nonces
            free_n()
            free()
    finally:
        grp.close()
