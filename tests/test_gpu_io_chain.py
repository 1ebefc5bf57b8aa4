"""The batched host I/O chain on the GPU box: the outgoing and incoming worker pipelines of one tunnel
(worker/outgoing.go:55-80, worker/incoming.go:54-79) with batched UDP (socket/udp.go:35-47) and the
device seal/open in between, over loopback:

  Payload.Raw slots -> qgcm_seal_host (pinned H2D, gfx950 seal, D2H) -> qgcm_udp_send_slots (sendmmsg)
  -> qgcm_udp_recv_slots (recvmmsg) -> qgcm_open_host -> plaintext

Every datagram on the wire is compared with the oracle's crypto/aes.go framing of the same packet
(explicit nonces), and every opened payload with what was sent; a datagram tampered in flight fails
(status 0, plaintext zeroed).  The pytest form of tools/udp_e2e.cpp.
"""
import ctypes as C
import threading
import time

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

STRIDE = 1472  # common.MaxPacketLength: one Payload.Raw per slot
AAD = bytes([10, 99, 0, 1])


@pytest.fixture(scope="module")
def torch():
    import torch as T

    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


def pinned(nbytes: int):
    from quantum_amd import _lib

    ptr = _lib.lib().qgcm_host_alloc(nbytes)
    assert ptr
    return np.frombuffer((C.c_uint8 * nbytes).from_address(ptr), dtype=np.uint8), ptr


@pytest.mark.parametrize("L", [1350, 1433, 17])
def test_udp_chain_wire_bytes_vs_oracle(torch, ctx, L):
    from quantum_amd import _lib

    lib = _lib.lib()
    rng = np.random.default_rng(0x10C + L)
    key = rng.bytes(32)
    slot = ctx.alloc_slot()
    ctx.set_key(slot, key)
    B = 4096
    tx, tx_ptr = pinned(B * STRIDE)
    rx, rx_ptr = pinned(B * STRIDE)
    non, non_ptr = pinned(12 * B)
    try:
        view = tx.reshape(B, STRIDE)
        view[:] = 0
        view[:, :4] = np.frombuffer(AAD, dtype=np.uint8)  # the sender's private IP (outgoing.go:28-35)
        view[:, 4:4 + L] = rng.integers(0, 256, (B, L), dtype=np.uint8)  # the TUN reads
        non[:] = rng.integers(0, 256, 12 * B, dtype=np.uint8)
        plain = view[:, :4 + L].copy()
        ref = tx.copy()
        O.lib().oracle_seal_uniform(key, ref.ctypes.data, STRIDE, B, L, 4, non.ctypes.data)

        st = np.zeros(B, dtype=np.uint8)
        assert lib.qgcm_seal_host(ctx.handle, tx_ptr, STRIDE, B, L, slot, non_ptr, 4, st.ctypes.data) == 0
        assert st.all()
        assert np.array_equal(tx, ref)  # sealed slots == the oracle's aes.go framing

        a = lib.qgcm_udp_socket(b"127.0.0.1", 0, 1 << 22)
        b = lib.qgcm_udp_socket(b"127.0.0.1", 0, 1 << 22)
        assert a >= 0 and b >= 0
        port = lib.qgcm_udp_port(b)
        tx_lens = np.full(B, 4 + L + 28, dtype=np.uint32)  # Payload.Length after encryption.go:36-37
        rx_lens = np.zeros(B, dtype=np.uint32)
        got = [0]
        window, per_call = 96, 32

        def receive():
            while got[0] < B:
                r = lib.qgcm_udp_recv_slots(b, rx_ptr + got[0] * STRIDE, STRIDE, min(B - got[0], per_call),
                                            rx_lens.ctypes.data + 4 * got[0], 3000)
                if r <= 0:
                    return
                got[0] += r

        th = threading.Thread(target=receive)
        th.start()
        sent = 0
        while sent < B:
            while sent - got[0] > window and th.is_alive():
                time.sleep(50e-6)  # keep the receive buffer from overflowing (a drop would be counted)
            n = min(B - sent, per_call)
            r = lib.qgcm_udp_send_slots(a, tx_ptr + sent * STRIDE, STRIDE, n, tx_lens.ctypes.data + 4 * sent,
                                        b"127.0.0.1", port)
            assert r > 0
            sent += r
        th.join(timeout=60)
        lib.qgcm_udp_close(a)
        lib.qgcm_udp_close(b)
        assert got[0] == B, f"lost {B - got[0]} datagrams"
        assert (rx_lens == 4 + L + 28).all()
        rv = rx.reshape(B, STRIDE)
        assert np.array_equal(rv[:, :4 + L + 28], ref.reshape(B, STRIDE)[:, :4 + L + 28])  # wire == oracle

        bad = {7, 1000, B - 1}
        for i in bad:  # tampered in flight
            rv[i, 4 + (i % (L + 28))] ^= 0x01
        st[:] = 7
        assert lib.qgcm_open_host(ctx.handle, rx_ptr, STRIDE, B, L + 28, slot, 4, st.ctypes.data) == len(bad)
        for i in range(B):
            if i in bad:
                assert st[i] == 0 and not rv[i, 4:4 + L].any()
            else:
                assert st[i] == 1
        good = np.array([i not in bad for i in range(B)])
        assert np.array_equal(rv[good, :4 + L], plain[good])  # incoming.go: the TUN writes
    finally:
        for p in (tx_ptr, rx_ptr, non_ptr):
            lib.qgcm_host_free(p)
