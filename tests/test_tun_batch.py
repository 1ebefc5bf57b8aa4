"""Batched TUN I/O (qgcm_tun_*: device/tun.go:51-150 with a batch per call) on
CPU, shaped like device/device_test.go: a multi-queue TUN device is created and brought up; UDP
datagrams sent to its subnet come out of its queues as IPv4 packets in Payload.Raw[4:] slots, and
IPv4 packets written to a queue reach a local UDP socket.  Needs /dev/net/tun and CAP_NET_ADMIN
(root in this container); skipped where the kernel refuses."""
import ctypes as C
import socket
import struct

import numpy as np
import pytest

from quantum_amd import _lib, common

STRIDE = common.MaxPacketLength
HOST_IP, PEER_IP = "10.213.7.1", "10.213.7.2"


def _csum(b: bytes) -> int:
    if len(b) % 2:
        b += b"\0"
    s = sum(struct.unpack(f"!{len(b) // 2}H", b))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def _ipv4_udp(src: str, dst: str, sport: int, dport: int, payload: bytes) -> bytes:
    udp = struct.pack("!HHHH", sport, dport, 8 + len(payload), 0) + payload  # UDP checksum 0: none
    hdr = struct.pack("!BBHHHBBH4s4s", 0x45, 0, 20 + len(udp), 0x1234, 0x4000, 64, 17, 0,
                      socket.inet_aton(src), socket.inet_aton(dst))
    hdr = hdr[:10] + struct.pack("!H", _csum(hdr)) + hdr[12:]
    return hdr + udp


@pytest.fixture()
def tun():
    L = _lib.lib()
    fds = (C.c_int * 2)()
    name = C.create_string_buffer(16)
    rc = L.qgcm_tun_open(b"qgcmt%d", 2, fds, name, 16)
    if rc < 0:
        pytest.skip(f"TUN device refused (errno {-rc})")
    try:
        rc = L.qgcm_tun_up(name.value, HOST_IP.encode(), 24, 1433)  # common.MTU
        if rc < 0:
            pytest.skip(f"TUN link set-up refused (errno {-rc})")
        yield L, list(fds), name.value
    finally:
        for fd in fds:
            L.qgcm_tun_close(fd)


def test_tun_read_slots_gets_routed_datagrams(tun):
    """device/tun.go:51-57: packets the kernel routes into the device are read in batches into
    Raw[4:] slots, lens = packet length (NewTunPayload(buf, n))."""
    L, fds, _ = tun
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind((HOST_IP, 0))
    n_flows, per = 4, 16
    sent = {}
    for f in range(n_flows):
        sk = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        sk.bind((HOST_IP, 0))
        for j in range(per):
            msg = bytes([f, j]) * (50 + 7 * j)
            sk.sendto(msg, (PEER_IP, 9000 + f))
            sent[(f, j)] = msg
        sk.close()
    s.close()
    got = {}
    arena = np.zeros(256 * STRIDE, dtype=np.uint8)
    lens = np.zeros(256, dtype=np.uint32)
    for _ in range(20):
        for fd in fds:
            r = L.qgcm_tun_read_slots(fd, arena.ctypes.data, STRIDE, 256, lens.ctypes.data, 50)
            assert r >= 0
            for i in range(r):
                pkt = bytes(arena[i * STRIDE + 4:i * STRIDE + 4 + lens[i]])
                if pkt[0] >> 4 != 4 or pkt[9] != 17 or pkt[16:20] != socket.inet_aton(PEER_IP):
                    continue  # other traffic the kernel sends to the subnet (none expected)
                ihl = (pkt[0] & 15) * 4
                dport = struct.unpack("!H", pkt[ihl + 2:ihl + 4])[0]
                data = pkt[ihl + 8:]
                got[(dport - 9000, data[1])] = data
        if len(got) == len(sent):
            break
    assert got == sent


def test_tun_write_slots_reach_a_socket(tun):
    """device/tun.go:60-63: Raw[4 : 4 + lens[i]] written to a queue is delivered by the kernel."""
    L, fds, _ = tun
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.bind((HOST_IP, 0))
    rx.settimeout(2.0)
    port = rx.getsockname()[1]
    n = 24
    arena = np.zeros(n * STRIDE, dtype=np.uint8)
    lens = np.zeros(n, dtype=np.uint32)
    want = []
    for i in range(n):
        payload = bytes([i]) * (10 + 40 * i)
        pkt = _ipv4_udp(PEER_IP, HOST_IP, 7000, port, payload)
        arena[i * STRIDE + 4:i * STRIDE + 4 + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
        lens[i] = len(pkt)
        want.append(payload)
    assert L.qgcm_tun_write_slots(fds[1], arena.ctypes.data, STRIDE, n, lens.ctypes.data) == n
    got = [rx.recv(4096) for _ in range(n)]
    rx.close()
    assert got == want


def test_tun_timeout_and_bad_args(tun):
    L, fds, _ = tun
    arena = np.zeros(4 * STRIDE, dtype=np.uint8)
    lens = np.zeros(4, dtype=np.uint32)
    # the kernel may still send link-up chatter (IPv6 solicitations); once the queue stays empty
    # for a 10 ms wait the call times out with 0
    for _ in range(100):
        r = L.qgcm_tun_read_slots(fds[0], arena.ctypes.data, STRIDE, 4, lens.ctypes.data, 10)
        assert r >= 0
        if r == 0:
            break
    assert r == 0
    assert L.qgcm_tun_read_slots(-1, arena.ctypes.data, STRIDE, 4, lens.ctypes.data, 0) == -1
    assert L.qgcm_tun_read_slots(fds[0], arena.ctypes.data, 4, 4, lens.ctypes.data, 0) == -1  # no room past IP
    assert L.qgcm_tun_up(b"qgcm-nonexistent", HOST_IP.encode(), 24, 1433) < 0
    assert L.qgcm_tun_up(b"x", b"not-an-ip", 24, 1433) < 0
    assert L.qgcm_tun_open(None, 0, None, None, 0) < 0


def test_tun_multi_queue_keeps_flows_in_order(tun):
    """device/tun.go:67-93: one queue per worker.  The kernel picks a queue per flow, so each UDP
    flow's packets come out of exactly one queue, in order."""
    L, fds, _ = tun
    n_flows, per = 8, 20
    for f in range(n_flows):
        sk = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        sk.bind((HOST_IP, 0))
        for j in range(per):
            sk.sendto(bytes([f, j]) * 20, (PEER_IP, 9100))
        sk.close()
    seen = {}  # flow -> list of (queue, seq)
    arena = np.zeros(512 * STRIDE, dtype=np.uint8)
    lens = np.zeros(512, dtype=np.uint32)
    for _ in range(20):
        for q, fd in enumerate(fds):
            r = L.qgcm_tun_read_slots(fd, arena.ctypes.data, STRIDE, 512, lens.ctypes.data, 20)
            for i in range(max(r, 0)):
                pkt = bytes(arena[i * STRIDE + 4:i * STRIDE + 4 + lens[i]])
                if pkt[0] >> 4 != 4 or pkt[9] != 17 or pkt[16:20] != socket.inet_aton(PEER_IP):
                    continue
                ihl = (pkt[0] & 15) * 4
                data = pkt[ihl + 8:]
                seen.setdefault(data[0], []).append((q, data[1]))
        if sum(len(v) for v in seen.values()) == n_flows * per:
            break
    assert sorted(seen) == list(range(n_flows))
    for f, recs in seen.items():
        assert len({q for q, _ in recs}) == 1, f"flow {f} split over queues"
        assert [s for _, s in recs] == list(range(per)), f"flow {f} out of order"


@pytest.mark.parametrize("mode", ["1", "-1"])
def test_tun_read_paths(mode):
    """The other two drain forms of qgcm_tun_read_slots, each in a fresh process (the form is fixed at a
    process's first batched read): one io_uring submission of RWF_NOWAIT reads per batch
    (QGCM_TUN_URING=1) and poll + read per packet (-1); the default preadv2 form runs in this process."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, QGCM_TUN_URING=mode)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(root, "tests", "test_tun_batch.py"), "-k", "read_slots_gets_routed"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=120)
    if "1 skipped" in r.stdout:
        pytest.skip("TUN device refused in the child")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "1 passed" in r.stdout, r.stdout[-1000:]
