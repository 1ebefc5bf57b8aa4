"""The uniform kernel's shared tail (gcm_kernels.hip QGCM_TILE_POOL 4): a launch's first rows of tiles go
through each workgroup's LDS counter, its last rows through one global counter per launch (a ring of
zeroed counter sets in the context, one per launch in turn; a set that comes round before its last
launch has posted its generation is waited for on the new launch's stream).  Checked against the
oracle: launches with one full row, two, and several plus a ragged row (the tail starts only at two
full rows), many launches in flight on four streams at once, and a ring of two sets under six streams."""
import os
import threading

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

AAD_WORD = int.from_bytes(bytes([10, 99, 0, 1]), "little")
L = 33
STRIDE = 80  # >= 4 + L + 28, a multiple of 16


@pytest.fixture(scope="module")
def torch():
    import torch as T

    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


def _ctx(chunk=None, sets=None):
    from quantum_amd.crypto import Context

    env = {"QGCM_LAUNCH_CHUNK": chunk, "QGCM_POOL_SETS": sets}
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v is not None:
            os.environ[k] = str(v)
    try:
        return Context(device=0, max_keys=2)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _row_packets(torch) -> int:
    # one row of tiles: two 16-wave workgroups per CU, 16 packets per wave tile
    return torch.cuda.get_device_properties(0).multi_processor_count * 2 * 16 * 16


def _fill(torch, n, seed, length=L, stride=STRIDE):
    from quantum_amd import batch

    arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(arena, stride, n, length, AAD_WORD, seed, nonces, seed + 1)
    return arena, nonces


def _oracle(key, plain, n, nonces, length=L, stride=STRIDE):
    ref = plain.copy()
    O.lib().oracle_seal_uniform(key, ref.ctypes.data, stride, n, length, 4, nonces.ctypes.data)
    return ref


@pytest.mark.parametrize("rows,extra", [(1, 0), (1, 4097), (2, 0), (2, 12345), (5, -7)])
def test_shared_tail_rows_vs_oracle(torch, aesgo, rows, extra):
    from quantum_amd import batch

    key = bytes.fromhex(aesgo["key"])
    n = rows * _row_packets(torch) + extra
    c = _ctx()
    try:
        c.set_key(1, key)
        arena, nonces = _fill(torch, n, 0x7A110000 + rows)
        plain = arena.cpu().numpy()
        status = torch.zeros(n, dtype=torch.uint8, device="cuda")
        for _ in range(2):  # two launches, each with the next set of the ring
            arena.copy_(torch.from_numpy(plain).cuda())
            batch.seal_uniform(c, arena, STRIDE, n, L, 1, nonces, status=status)
            assert np.array_equal(arena.cpu().numpy(), _oracle(key, plain, n, nonces.cpu().numpy()))
            assert int(status.sum()) == n
        batch.open_uniform(c, arena, STRIDE, n, L + 28, 1, status=status)
        assert int(status.sum()) == n
        assert np.array_equal(arena.cpu().numpy().reshape(n, STRIDE)[:, :4 + L], plain.reshape(n, STRIDE)[:, :4 + L])
        assert c.launch_counts()["tail_waits"] == 0  # a 4096-set ring never comes round here
    finally:
        c.close()


def test_shared_tail_many_launches_on_four_streams(torch, aesgo):
    """Four host threads, each on its own stream, each call cut into 3 launches of 2 rows (the last
    ragged): seal, open, seal without synchronizing, 36 launches queued against a ring of 8 sets."""
    from quantum_amd import batch

    key = bytes.fromhex(aesgo["key"])
    rp = _row_packets(torch)
    n = 5 * rp + 999
    c = _ctx(chunk=2 * rp, sets=8)
    try:
        c.set_key(1, key)
        jobs = []
        for t in range(4):
            arena, nonces = _fill(torch, n, 0x51DE0000 + 16 * t)
            jobs.append((arena, nonces, torch.zeros(n, dtype=torch.uint8, device="cuda"), arena.cpu().numpy(),
                         torch.cuda.Stream()))
        torch.cuda.synchronize()
        c0 = c.launch_counts()["quad"]
        errs = []

        def work(arena, nonces, status, plain, s):
            try:
                batch.seal_uniform(c, arena, STRIDE, n, L, 1, nonces, status=None, stream=s)
                batch.open_uniform(c, arena, STRIDE, n, L + 28, 1, status=status, stream=s)
                batch.seal_uniform(c, arena, STRIDE, n, L, 1, nonces, status=None, stream=s)
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        th = [threading.Thread(target=work, args=j) for j in jobs]
        for x in th:
            x.start()
        for x in th:
            x.join()
        torch.cuda.synchronize()
        assert not errs
        assert c.launch_counts()["quad"] - c0 == 4 * 3 * 3
        for arena, nonces, status, plain, _ in jobs:
            assert int(status.sum()) == n
            assert np.array_equal(arena.cpu().numpy(), _oracle(key, plain, n, nonces.cpu().numpy()))
    finally:
        c.close()


def test_shared_tail_short_ring_waits_for_posted_generations(torch, aesgo):
    """A ring of two counter sets (QGCM_POOL_SETS=2) under six streams, two seals each without
    synchronizing: nearly every launch finds its set's previous launch (on another stream) still queued or
    running and waits, on its own stream, for the generation that launch posts.  Every stream seals its
    own copy of one arena; all must equal the oracle."""
    from quantum_amd import batch

    key = bytes.fromhex(aesgo["key"])
    n = 2 * _row_packets(torch) + 333
    ln, st = 1350, 1408  # ~0.4 ms a launch, far longer than a host call: the ring comes round on launches queued
    c = _ctx(sets=2)
    try:
        c.set_key(1, key)
        arena0, nonces = _fill(torch, n, 0x5E750000, ln, st)
        plain = arena0.cpu().numpy()
        want = _oracle(key, plain, n, nonces.cpu().numpy(), ln, st)
        streams = [torch.cuda.Stream() for _ in range(6)]
        arenas = [arena0.clone() for _ in streams]
        torch.cuda.synchronize()
        w0 = c.launch_counts()["tail_waits"]
        for rep in range(2):
            for a, s in zip(arenas, streams):
                if rep:
                    with torch.cuda.stream(s):
                        a.copy_(arena0)
                batch.seal_uniform(c, a, st, n, ln, 1, nonces, status=None, stream=s)
        torch.cuda.synchronize()
        assert c.launch_counts()["tail_waits"] > w0  # the ring came round on launches still queued
        for a in arenas:
            assert np.array_equal(a.cpu().numpy(), want)
    finally:
        c.close()
