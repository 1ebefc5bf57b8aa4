"""The resident per-packet service (quantum_amd/csrc/resident.cpp, gcm_resident_kernel): qgcm_seal_one /
qgcm_open_one served without a launch per call, checked against the oracle (crypto/aes.go:41-62
framing) -- from many threads at once, across instance ends (idle timeout, lifetime cap, qgcm_set_keys,
qgcm_resident_stop) and next to a bulk batch on the same GPU.  The per-call tests in
tests/test_gpu_parity.py run through it too (their lengths past its 16-KiB slots take the launch path).
"""
import os
import random
import threading
import time

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

AAD = bytes([10, 99, 0, 1])


@pytest.fixture(scope="module")
def torch():
    import torch as T

    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


def make_ctx(**env):
    from quantum_amd.crypto import Context

    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return Context(device=0, max_keys=64)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def roundtrip(aes, key, L, rng, aad=AAD):
    pt = rng.randbytes(L)
    nonce = rng.randbytes(12)
    data = bytearray(pt + bytes(28))
    n, err = aes.Encrypt(data, L, aad, nonce=nonce)
    want = bytearray(pt + bytes(28))
    O.aesgo_encrypt(key, want, L, aad, nonce)
    if err is not None or n != L + 28 or bytes(data) != bytes(want):
        return f"seal L={L}"
    n, err = aes.Decrypt(data, aad)
    if err is not None or n != L or bytes(data[:L]) != pt:
        return f"open L={L}"
    return None


def test_served_by_resident_kernel(torch):
    from quantum_amd.crypto import AES

    ctx = make_ctx()
    try:
        key = bytes(range(32))
        aes = AES(key, ctx=ctx)
        rng = random.Random(1)
        before = ctx.launch_counts()
        for L in (0, 1, 15, 16, 17, 1350, 1433, 4096, 9000, 16352):  # 16352: the largest a slot holds
            assert roundtrip(aes, key, L, rng) is None, L
        after = ctx.launch_counts()
        assert after["resident"] - before["resident"] == 20 and after["one"] == before["one"]
        st = ctx.resident_stats()
        assert st["served"] >= 20 and st["launches"] >= 1 and st["slots"] == 256
        # past the slot: a gcm_one_kernel launch per call, same bytes
        assert roundtrip(aes, key, 16353, rng) is None
        assert ctx.launch_counts()["one"] == after["one"] + 2
        # tamper and short: zeroed plaintext, tag and nonce untouched; len < 28 untouched
        data = bytearray(rng.randbytes(100) + bytes(28))
        n, err = aes.Encrypt(data, 100, AAD)
        bad = bytearray(data)
        bad[5] ^= 1
        tail = bytes(bad[100:])
        _, err = aes.Decrypt(bad, AAD)
        assert err is not None and bytes(bad[:100]) == bytes(100) and bytes(bad[100:]) == tail
        short = bytearray(rng.randbytes(27))
        s0 = bytes(short)
        _, err = aes.Decrypt(short, AAD)
        assert err is not None and bytes(short) == s0
    finally:
        ctx.close()


def test_many_threads_vs_oracle(torch):
    """64 threads, each with one packet in flight, two keys, ragged lengths (some past the slot)."""
    from quantum_amd.crypto import AES

    ctx = make_ctx()
    try:
        keys = [bytes([0x41 + i]) * 32 for i in range(2)]
        aes_list = [AES(k, ctx=ctx) for k in keys]
        errors = []

        def work(t):
            rng = random.Random(0xAB00 + t)
            for _ in range(40):
                k = rng.randrange(2)
                L = rng.choice([0, 17, 64, 1350, 1433, rng.randrange(0, 9001), rng.randrange(16300, 16400)])
                e = roundtrip(aes_list[k], keys[k], L, rng, AAD if t % 3 else None)
                if e:
                    errors.append((t, e))
                    return

        ths = [threading.Thread(target=work, args=(t,)) for t in range(64)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        assert not errors, errors[:5]
        assert ctx.launch_counts()["resident"] > 0
    finally:
        ctx.close()


def test_instance_ends_and_relaunches(torch):
    """Idle timeout (1 ms), lifetime cap (3 ms) and qgcm_resident_stop end instances; requests that
    arrive at or after an end are served by the next instance, bit-exact."""
    from quantum_amd.crypto import AES

    ctx = make_ctx(QGCM_RESIDENT_IDLE_US=1000, QGCM_RESIDENT_LIFE_US=3000)
    try:
        key = os.urandom(32)
        aes = AES(key, ctx=ctx)
        rng = random.Random(2)
        assert roundtrip(aes, key, 1350, rng) is None
        time.sleep(0.05)  # past the idle timeout: the instance has left
        assert ctx.resident_stats()["running"] == 0
        l0 = ctx.resident_stats()["launches"]
        assert roundtrip(aes, key, 1350, rng) is None
        assert ctx.resident_stats()["launches"] == l0 + 1
        # back-to-back traffic from 8 threads until the 3-ms lifetime cap has ended 5 instances (~15 ms of
        # traffic; at most 2 s, so a slow box cannot turn a timing margin into a failure)
        errors = []
        done = threading.Event()

        def work(t):
            r = random.Random(100 + t)
            while not done.is_set():
                e = roundtrip(aes, key, r.randrange(0, 3000), r)
                if e:
                    errors.append(e)
                    return

        ths = [threading.Thread(target=work, args=(t,)) for t in range(8)]
        for th in ths:
            th.start()
        deadline = time.time() + 2.0
        while time.time() < deadline and ctx.resident_stats()["launches"] < l0 + 5 and not errors:
            time.sleep(0.01)
        done.set()
        for th in ths:
            th.join()
        assert not errors, errors[:3]
        assert ctx.resident_stats()["launches"] >= l0 + 5
        ctx.resident_stop()
        assert ctx.resident_stats()["running"] == 0
        assert roundtrip(aes, key, 33, rng) is None
    finally:
        ctx.close()


def test_set_keys_while_serving(torch):
    """qgcm_set_key ends the running instance (its workers cache key tables and key-valid bytes): a key
    installed while other threads are sealing is used correctly right away."""
    from quantum_amd.crypto import AES

    ctx = make_ctx()
    try:
        k0 = os.urandom(32)
        a0 = AES(k0, ctx=ctx)
        errors, stop = [], threading.Event()

        def busy():
            r = random.Random(7)
            while not stop.is_set():
                e = roundtrip(a0, k0, r.randrange(0, 2000), r)
                if e:
                    errors.append(e)
                    return

        th = threading.Thread(target=busy)
        th.start()
        rng = random.Random(3)
        for _ in range(5):
            k = os.urandom(32)
            a = AES(k, ctx=ctx)  # a new key slot, set while the instance runs
            for L in (1, 1350):
                assert roundtrip(a, k, L, rng) is None
        stop.set()
        th.join()
        assert not errors, errors[:3]
    finally:
        ctx.close()


def test_next_to_bulk_batch(torch):
    """Per-packet calls from 16 threads while a 2^19-packet uniform batch runs on the same GPU: both
    bit-exact (the bulk grid leaves the resident kernel's CUs alone)."""
    from quantum_amd import batch
    from quantum_amd.crypto import AES

    ctx = make_ctx()
    try:
        key = os.urandom(32)
        aes = AES(key, ctx=ctx)
        bkey = os.urandom(32)
        ctx.set_key(63, bkey)
        n, L = 1 << 19, 1350
        stride = batch.slot_stride(L, 64)
        arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
        nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
        status = torch.zeros(n, dtype=torch.uint8, device="cuda")
        batch.fill_uniform(arena, stride, n, L, int.from_bytes(AAD, "little"), 0x5EED0041, nonces, 0x5EED0042)
        head = arena[:4096 * stride].clone()
        errors = []
        stop = threading.Event()

        def work(t):
            r = random.Random(200 + t)
            while not stop.is_set():
                e = roundtrip(aes, key, r.randrange(0, 1500), r)
                if e:
                    errors.append(e)
                    return

        ths = [threading.Thread(target=work, args=(t,)) for t in range(16)]
        for th in ths:
            th.start()
        time.sleep(0.02)
        s = torch.cuda.Stream()
        for _ in range(3):
            batch.seal_uniform(ctx, arena, stride, n, L, 63, nonces, status=status, stream=s)
            batch.open_uniform(ctx, arena, stride, n, L + 28, 63, status=status, stream=s)
        s.synchronize()
        stop.set()
        for th in ths:
            th.join()
        assert not errors, errors[:3]
        assert int(status.sum()) == n
        ref = head.cpu().numpy()
        h = ref.copy()
        nh = nonces[:12 * 4096].cpu().numpy()  # kept alive across the call (ctypes takes a raw address)
        O.lib().oracle_seal_uniform(bkey, h.ctypes.data, stride, 4096, L, 4, nh.ctypes.data)
        batch.seal_uniform(ctx, head, stride, 4096, L, 63, nonces[:12 * 4096])
        assert np.array_equal(head.cpu().numpy(), h)
    finally:
        ctx.close()


def test_launch_path_when_disabled(torch):
    from quantum_amd.crypto import AES

    ctx = make_ctx(QGCM_RESIDENT=0)
    try:
        key = os.urandom(32)
        aes = AES(key, ctx=ctx)
        assert roundtrip(aes, key, 1350, random.Random(4)) is None
        c = ctx.launch_counts()
        assert c["resident"] == 0 and c["one"] == 2
    finally:
        ctx.close()


def test_aad_lengths_and_tamper_kinds(torch):
    """AAD of 0-4 bytes (nil additional data, as crypto_test.go:54-101 passes) and every tamper kind
    (a ciphertext byte, the last one, the tag, the nonce, the AAD), from 8 threads through the resident
    kernel: sealed bytes equal the oracle's, a tampered open fails exactly where the oracle's does,
    zeroes the plaintext and leaves tag and nonce as they were."""
    from quantum_amd.crypto import AES

    ctx = make_ctx()
    try:
        key = bytes(range(7, 39))
        aes = AES(key, ctx=ctx)
        before = ctx.launch_counts()
        errs = []

        def work(t):
            rng = random.Random(100 + t)
            for i in range(30):
                aad = [b"", b"\x0a", b"\x0a\x63", b"\x0a\x63\x00", AAD][i % 5]
                L = rng.choice([0, 5, 16, 31, 100, 1350, rng.randrange(0, 4000)])
                pt, nonce = rng.randbytes(L), rng.randbytes(12)
                data, want = bytearray(pt + bytes(28)), bytearray(pt + bytes(28))
                n, err = aes.Encrypt(data, L, aad or None, nonce=nonce)
                O.aesgo_encrypt(key, want, L, aad, nonce)
                if err is not None or n != L + 28 or data != want:
                    errs.append(f"seal t={t} L={L} aad={len(aad)}")
                    continue
                kind = i % 6
                bad, bad_aad = bytearray(data), bytearray(aad)
                if kind == 1 and L:
                    bad[rng.randrange(L)] ^= 0x80
                elif kind == 2 and L:
                    bad[L - 1] ^= 1
                elif kind == 3:
                    bad[L + rng.randrange(16)] ^= 4
                elif kind == 4:
                    bad[L + 16 + rng.randrange(12)] ^= 2
                elif kind == 5 and aad:
                    bad_aad[0] ^= 1
                ref = bytearray(bad)
                want_n = O.aesgo_decrypt(key, ref, bytes(bad_aad))
                tail = bytes(bad[L:])
                n, err = aes.Decrypt(bad, bytes(bad_aad) or None)
                if want_n < 0:
                    if err is None or bytes(bad[:L]) != bytes(L) or bytes(bad[L:]) != tail:
                        errs.append(f"tamper t={t} L={L} kind={kind}")
                elif err is not None or n != L or bytes(bad[:L]) != pt:
                    errs.append(f"open t={t} L={L} kind={kind}")

        ths = [threading.Thread(target=work, args=(t,)) for t in range(8)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        assert not errs, errs[:5]
        after = ctx.launch_counts()
        assert after["resident"] - before["resident"] == 8 * 30 * 2 and after["one"] == before["one"]
    finally:
        ctx.close()


def test_drawn_nonces_unique_and_open(torch):
    """Seals without an explicit nonce draw it from getrandom, buffered per thread (resident.cpp
    random_nonce): 8 threads x 2000 seals give 16000 distinct nonces, and every packet opens."""
    from quantum_amd.crypto import AES

    ctx = make_ctx()
    try:
        key = bytes(range(40, 72))
        aes = AES(key, ctx=ctx)
        nonces, errs = [], []
        lock = threading.Lock()

        def work(t):
            mine = []
            for i in range(2000):
                L = 64 + (i % 7)
                data = bytearray(bytes([t, i & 255]) * (L // 2) + bytes(L % 2) + bytes(28))
                n, err = aes.Encrypt(data, L, AAD)
                if err is not None or n != L + 28:
                    errs.append(f"seal t={t} i={i}")
                    continue
                mine.append(bytes(data[L + 16:L + 28]))
                if i % 50 == 0:
                    want = bytearray(data)
                    if O.aesgo_decrypt(key, want, AAD) != L:
                        errs.append(f"oracle open t={t} i={i}")
            with lock:
                nonces.extend(mine)

        ths = [threading.Thread(target=work, args=(t,)) for t in range(8)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        assert not errs, errs[:5]
        assert len(nonces) == 16000 and len(set(nonces)) == 16000
    finally:
        ctx.close()


@pytest.mark.parametrize("ahead", [1, 0])
def test_keystream_ahead_vs_oracle(torch, ahead, monkeypatch):
    """Seals without a caller's nonce announce their slot's next nonce, whose counter blocks the worker
    computes while idle (gcm_kernels.hip ks_fill); the next seal on the slot uses them.  4 threads x 400
    seals and opens: two keys, lengths across the flat-GHASH limit (up to 2016 B the keystream ahead is
    used; longer packets load comb tables over it, which must drop it) -- every sealed packet opens under
    the oracle with its drawn nonce, and with QGCM_RESIDENT_AHEAD=0 nothing is served ahead."""
    from quantum_amd.crypto import AES

    monkeypatch.setenv("QGCM_RESIDENT_AHEAD", str(ahead))  # read at qgcm_create
    ctx = make_ctx()
    try:
        keys = [bytes(range(90 + 7 * i, 122 + 7 * i)) for i in range(2)]
        aes_list = [AES(k, ctx=ctx) for k in keys]
        errs, nonces, lock = [], [], threading.Lock()

        def work(t):
            rng = random.Random(0xA11E + t)
            mine = []
            for i in range(400):
                k = 0 if i % 10 else 1
                L = rng.choice([0, 1, 17, 1350, 1350, 1433, 2000, 2016, 2017, 2032, rng.randrange(0, 2017), 3000])
                pt = rng.randbytes(L)
                data = bytearray(pt + bytes(28))
                n, err = aes_list[k].Encrypt(data, L, AAD)
                if err is not None or n != L + 28:
                    errs.append(f"seal t={t} i={i} L={L}")
                    return
                mine.append(bytes(data[L + 16:L + 28]))
                ref = bytearray(data)
                if O.aesgo_decrypt(keys[k], ref, AAD) != L or bytes(ref[:L]) != pt:
                    errs.append(f"oracle open t={t} i={i} L={L} k={k}")
                    return
                n, err = aes_list[k].Decrypt(data, AAD)
                if err is not None or n != L or bytes(data[:L]) != pt:
                    errs.append(f"open t={t} i={i} L={L}")
                    return
            with lock:
                nonces.extend(mine)

        ths = [threading.Thread(target=work, args=(t,)) for t in range(4)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        assert not errs, errs[:5]
        assert len(nonces) == 1600 and len(set(nonces)) == 1600
        hits = ctx.resident_stats()["ahead_hits"]
        if ahead:
            assert hits > 400, hits  # most seals up to 2016 B after the first on a slot
        else:
            assert hits == 0
    finally:
        ctx.close()


def test_failed_relaunch_leaves_no_waiters(torch):
    """A relaunch that fails (injected with the QGCM_RESIDENT_FAIL_AFTER test hook: every launch after the
    first fails) marks the resident path broken: the callers whose requests were posted return -1, every
    later call takes the launch path (bit-exact with the oracle), no caller stays counted asleep or
    spinning, and no further instance is launched -- the completion thread stops relaunching."""
    from quantum_amd.crypto import AES

    ctx = make_ctx(QGCM_RESIDENT_FAIL_AFTER=1, QGCM_RESIDENT_LIFE_US=300, QGCM_RESIDENT_IDLE_US=100,
                   QGCM_RESIDENT_SPIN_US=0)
    try:
        key = bytes(range(32))
        ctx.set_key(0, key)
        results, errors = [], []

        def caller(t):
            aes = AES(key, ctx=ctx)
            rng = random.Random(t)
            end = time.time() + 1.0
            while time.time() < end:
                L = rng.choice([64, 1350, 4000])
                pt = rng.randbytes(L)
                nonce = rng.randbytes(12)
                data = bytearray(pt + bytes(28))
                n, err = aes.Encrypt(data, L, AAD, nonce=nonce)
                if err is not None:
                    results.append("failed")
                    continue
                want = bytearray(pt + bytes(28))
                O.aesgo_encrypt(key, want, L, AAD, nonce)
                if n != L + 28 or bytes(data) != bytes(want):
                    errors.append(L)
                results.append("ok")

        th = [threading.Thread(target=caller, args=(t,)) for t in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors
        st = ctx.resident_stats()
        assert st["broken"] == 1 and st["launches"] == 1
        assert st["sleepers"] == 0 and st["spinners"] == 0
        assert results.count("ok") > 100  # the launch path served the calls after the failure
        time.sleep(0.05)
        st2 = ctx.resident_stats()
        assert st2["launches"] == 1 and st2["sleepers"] == 0
        before = ctx.launch_counts()["one"]
        assert roundtrip(AES(key, ctx=ctx), key, 1350, random.Random(9)) is None
        assert ctx.launch_counts()["one"] == before + 2
    finally:
        ctx.close()
