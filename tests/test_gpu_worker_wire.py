"""The unchanged callers' wire bytes against the oracle.

worker/outgoing.go:55-80 (mirror: quantum_amd.worker.Outgoing) runs the plugin chain of config 1's
harness -- plugin.Mock and plugin.Encryption (plugin/mock.go, plugin/encryption.go) -- over packets
read from a TUN stand-in, with resolve() writing the sender's private IP into Raw[0:4] as
outgoing.go:28-35 does.  Encrypt draws a fresh nonce per packet (crypto/aes.go:42-47), and the nonce
travels in the packet, so every datagram handed to the socket can be recomputed by the oracle from
(key, plaintext, AAD = Raw[0:4], that nonce): the wire must equal oracle_aesgo_encrypt's output byte
for byte.  The key is derived independently on the oracle side (OpenSSL X25519 + hashlib PBKDF2 over
the same keypairs, common/mapping.go:90-99).  Then worker/incoming.go:54-79 on the peer restores
the packets.  Each Apply is one qgcm_seal_one / qgcm_open_one call (the resident kernel), from one
worker or from four worker threads at once.
"""
import hashlib
import threading

import pytest

from oracle import oracle as O
from test_worker_host import FakeDev, FakeSock

pytestmark = pytest.mark.gpu

IP_A = bytes([10, 99, 0, 1])


@pytest.mark.parametrize("path", ["direct", "threads"])
def test_outgoing_wire_bytes_equal_oracle(ctx, path):
    import numpy as np

    from quantum_amd import common, crypto, plugin, worker

    a_pub, a_priv = crypto.GenerateECKeyPair()
    a_spub, a_spriv = crypto.GenerateECKeyPair()
    b_pub, b_priv = crypto.GenerateECKeyPair()
    b_spub, b_spriv = crypto.GenerateECKeyPair()
    aes_ab, err = crypto.MappingAES(b_pub, b_spub, a_priv, a_spriv, ctx=ctx)
    assert err is None
    aes_ba, err = crypto.MappingAES(a_pub, a_spub, b_priv, b_spriv, ctx=ctx)
    assert err is None
    # the oracle's own derivation of the A -> B key
    key = hashlib.pbkdf2_hmac("sha512", O.ossl_x25519(a_priv, b_pub), O.ossl_x25519(a_spriv, b_spub), 10000, 32)
    on = ["encryption", "mock"]
    map_a = common.Mapping(SupportedPlugins=on, AES=aes_ab)
    map_b = common.Mapping(SupportedPlugins=on, AES=aes_ba)
    rng = np.random.default_rng(0x3A1 if path == "direct" else 0x3A2)
    sizes = [0, 1, 15, 16, 17, 64, 100, 1349, 1350, 1351, common.MTU] + list(rng.integers(1, common.MTU, 40))
    pkts = [rng.bytes(int(n)) for n in sizes]
    enc, _ = plugin.New(plugin.EncryptionPlugin)
    mock, _ = plugin.New(plugin.MockPlugin)

    def resolve_out(p):
        p.Raw[0:4] = IP_A  # copy(payload.IPAddress, cfg.PrivateIP.To4())
        return p, map_a, True

    sock = FakeSock()
    dev_a = FakeDev(pkts)
    out = worker.Outgoing(dev_a, sock, resolve_out, [mock, enc])
    if path == "direct":
        buf = bytearray(common.MaxPacketLength)
        while dev_a.packets:
            assert out.pipeline(buf, 0)
    else:  # 4 worker threads, one Raw buffer each (outgoing.go:84-93), packets shared through dev_a
        lock = threading.Lock()

        class LockedDev(FakeDev):
            def Read(self, queue, buf):
                with lock:
                    return FakeDev.Read(self, queue, buf)

        dev_a.__class__ = LockedDev
        wire_lock = threading.Lock()
        orig_write = sock.Write

        def locked_write(queue, payload, mapping):
            with wire_lock:
                return orig_write(queue, payload, mapping)

        sock.Write = locked_write

        def run():
            b = bytearray(common.MaxPacketLength)
            while True:
                with lock:
                    if not dev_a.packets:
                        return
                out.pipeline(b, 0)

        ths = [threading.Thread(target=run) for _ in range(4)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=60)
    assert out.stats.Packets == len(pkts) and out.stats.Dropped == 0
    assert len(sock.wire) == len(pkts)
    by_plain = {}
    for w in sock.wire:
        assert w[:4] == IP_A and len(w) >= 4 + 28
        L = len(w) - 4 - 28
        nonce = w[-12:]
        # which plaintext: the one whose oracle seal under this wire nonce reproduces the wire
        matches = []
        for j, p in enumerate(pkts):
            if len(p) != L or j in by_plain:
                continue
            buf = bytearray(p + bytes(28))
            assert O.aesgo_encrypt(key, buf, L, IP_A, nonce) == L + 28
            if bytes(buf) == w[4:]:
                matches.append(j)
                break
        assert matches, f"wire packet of L={L} equals no oracle seal"
        by_plain[matches[0]] = w
    assert sorted(by_plain) == list(range(len(pkts)))

    # the peer's incoming pipeline restores every packet
    dev_b = FakeDev([])
    inc = worker.Incoming(dev_b, sock, lambda p: (p, map_b, True), [mock, enc])
    rbuf = bytearray(common.MaxPacketLength)
    while sock.wire:
        assert inc.pipeline(rbuf, 0)
    assert sorted(dev_b.written) == sorted(pkts)