"""Batched UDP I/O (qgcm_udp_*: socket/udp.go:35-70 with recvmmsg/sendmmsg) over
loopback on CPU, shaped like socket/socket_test.go:44-291 (UDP end to end, v4): datagrams are
Payload.Raw[:Length] slots and come back byte for byte, in order."""
import ctypes as C
import os
import random

import numpy as np
import pytest

from quantum_amd import _lib, common

STRIDE = common.MaxPacketLength


@pytest.fixture()
def pair():
    L = _lib.lib()
    a = L.qgcm_udp_socket(b"127.0.0.1", 0, 1 << 22)
    b = L.qgcm_udp_socket(b"127.0.0.1", 0, 1 << 22)
    assert a >= 0 and b >= 0
    yield L, a, b, L.qgcm_udp_port(b)
    L.qgcm_udp_close(a)
    L.qgcm_udp_close(b)


def slots(n, lens, rng):
    arena = np.zeros(n * STRIDE, np.uint8)
    for i, L in enumerate(lens):
        arena[i * STRIDE:i * STRIDE + L] = np.frombuffer(rng.randbytes(L), np.uint8)
    return arena


def test_batches_round_trip_in_order(pair):
    L, a, b, port_b = pair
    rng = random.Random(3)
    total, chunk = 3000, 32  # chunks stay inside the default socket buffer (no loss on loopback)
    lens = np.array([rng.choice([0, 4, 33, 1350 + 32, STRIDE]) if i % 9 == 0 else rng.randint(4, STRIDE)
                     for i in range(total)], np.uint32)
    src = slots(total, lens, rng)
    dst = np.zeros_like(src)
    got_lens = np.zeros(total, np.uint32)
    got = 0
    for c0 in range(0, total, chunk):
        n = min(chunk, total - c0)
        sent = L.qgcm_udp_send_slots(a, src[c0 * STRIDE:].ctypes.data, STRIDE, n, lens[c0:].ctypes.data,
                                     b"127.0.0.1", port_b)
        assert sent == n
        while got < c0 + n:
            r = L.qgcm_udp_recv_slots(b, dst[got * STRIDE:].ctypes.data, STRIDE, total - got,
                                      got_lens[got:].ctypes.data, 1000)
            assert r > 0
            got += r
    assert got == total
    assert np.array_equal(got_lens, lens)
    for i in range(total):
        s = slice(i * STRIDE, i * STRIDE + int(lens[i]))
        assert np.array_equal(dst[s], src[s]), i


def test_timeout_truncation_and_bad_args(pair):
    L, a, b, port_b = pair
    buf = np.zeros(4 * STRIDE, np.uint8)
    ln = np.zeros(4, np.uint32)
    assert L.qgcm_udp_recv_slots(b, buf.ctypes.data, STRIDE, 4, ln.ctypes.data, 10) == 0  # nothing queued
    big = np.frombuffer(os.urandom(2000), np.uint8).copy()
    one = np.array([2000], np.uint32)
    assert L.qgcm_udp_send_slots(a, big.ctypes.data, 2000, 1, one.ctypes.data, b"127.0.0.1", port_b) == 1
    # a datagram longer than the slot is cut to the slot, as recvfrom into the worker buffer cuts it
    assert L.qgcm_udp_recv_slots(b, buf.ctypes.data, STRIDE, 4, ln.ctypes.data, 1000) == 1
    assert ln[0] == STRIDE and np.array_equal(buf[:STRIDE], big[:STRIDE])
    assert L.qgcm_udp_socket(b"not-an-ip", 0, 0) == -1
    assert L.qgcm_udp_send_slots(a, buf.ctypes.data, STRIDE, 1, ln.ctypes.data, b"127.0.0.1", 70000) == -1
    assert L.qgcm_udp_recv_slots(-1, buf.ctypes.data, STRIDE, 1, ln.ctypes.data, 0) == -1


def test_multi_queue_spreads_flows():
    """socket/udp.go:55-70: NumWorkers queues on one address.  Four SO_REUSEPORT queues share a port;
    eight senders (distinct source ports = distinct flows) each send a numbered run; every datagram
    arrives exactly once, each flow on a single queue and in order, and more than one queue is used."""
    L = _lib.lib()
    q0 = L.qgcm_udp_queue(b"127.0.0.1", 0, 1 << 22)
    assert q0 >= 0
    port = L.qgcm_udp_port(q0)
    queues = [q0] + [L.qgcm_udp_queue(b"127.0.0.1", port, 1 << 22) for _ in range(3)]
    senders = [L.qgcm_udp_socket(b"127.0.0.1", 0, 1 << 22) for _ in range(8)]
    try:
        assert all(q >= 0 for q in queues) and all(s >= 0 for s in senders)
        per = 24  # per flow: stays inside the default receive buffer
        for f, s in enumerate(senders):
            buf = np.zeros(per * STRIDE, np.uint8)
            lens = np.full(per, 8, np.uint32)
            for i in range(per):
                buf[i * STRIDE:i * STRIDE + 8] = np.frombuffer(bytes([f, i]) + bytes(6), np.uint8)
            assert L.qgcm_udp_send_slots(s, buf.ctypes.data, STRIDE, per, lens.ctypes.data, b"127.0.0.1", port) == per
        seen = {}  # flow -> (queue, [seq...])
        total = 0
        for qi, q in enumerate(queues):
            dst = np.zeros(256 * STRIDE, np.uint8)
            ln = np.zeros(256, np.uint32)
            while True:
                r = L.qgcm_udp_recv_slots(q, dst.ctypes.data, STRIDE, 256, ln.ctypes.data, 200)
                if r <= 0:
                    break
                for i in range(r):
                    f, seq = int(dst[i * STRIDE]), int(dst[i * STRIDE + 1])
                    qq, seqs = seen.setdefault(f, (qi, []))
                    assert qq == qi  # a flow stays on one queue
                    seqs.append(seq)
                total += r
        assert total == 8 * per
        assert all(seqs == list(range(per)) for _, seqs in seen.values())
        assert len({q for q, _ in seen.values()}) > 1
    finally:
        for fd in queues + senders:
            L.qgcm_udp_close(fd)
