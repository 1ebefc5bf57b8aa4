"""Packet rate of the batched TUN calls (qgcm_tun_read_slots / qgcm_tun_write_slots, device/tun.go
:51-63 batched) through a real multi-queue TUN device on this host's kernel -- CPU only, needs
root (the GPU boxes run unprivileged, so this is measured in the build container).

  read:  sendmmsg bursts of 1350-B datagrams to the TUN subnet (qgcm_udp_send_slots), drained from
         the TUN queues by qgcm_tun_read_slots (one read() per packet, poll only before the first)
  write: 1378-B IPv4/UDP packets (1350 B payload) written by qgcm_tun_write_slots, delivered to a
         local UDP socket drained by qgcm_udp_recv_slots
Prints one JSON line per direction."""
import ctypes as C
import json
import os
import socket
import struct
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from quantum_amd import _lib, common  # noqa: E402
from tests.test_tun_batch import HOST_IP, PEER_IP, _ipv4_udp  # noqa: E402

STRIDE = common.MaxPacketLength
PAYLOAD = 1350
BATCH = 512


def main() -> None:
    total = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    L = _lib.lib()
    fds = (C.c_int * 1)()
    name = C.create_string_buffer(16)
    assert L.qgcm_tun_open(b"qgcmr%d", 1, fds, name, 16) == 0
    try:
        assert L.qgcm_tun_up(name.value, HOST_IP.encode(), 24, 1433) == 0
        fd = fds[0]
        tx = L.qgcm_udp_socket(HOST_IP.encode(), 0, 1 << 24)
        src = np.frombuffer(os.urandom(BATCH * STRIDE), dtype=np.uint8).copy()
        lens = np.full(BATCH, PAYLOAD, dtype=np.uint32)
        arena = np.zeros(BATCH * STRIDE, dtype=np.uint8)
        rl = np.zeros(BATCH, dtype=np.uint32)
        # drain link-up chatter
        while L.qgcm_tun_read_slots(fd, arena.ctypes.data, STRIDE, BATCH, rl.ctypes.data, 20) > 0:
            pass
        got, calls, t_read = 0, 0, 0.0
        t0 = time.perf_counter()
        while got < total:
            # bursts of 256: the device's transmit queue (txqueuelen) holds 500 packets
            assert L.qgcm_udp_send_slots(tx, src.ctypes.data, STRIDE, 256, lens.ctypes.data, PEER_IP.encode(), 9000) == 256
            batch_got = 0
            while batch_got < 256:
                tr = time.perf_counter()
                r = L.qgcm_tun_read_slots(fd, arena.ctypes.data, STRIDE, BATCH, rl.ctypes.data, 5)
                t_read += time.perf_counter() - tr
                if r <= 0:
                    break  # the kernel dropped the rest (queue full): count what arrived
                batch_got += r
                calls += 1
            got += batch_got
        dt = time.perf_counter() - t0
        print(json.dumps({"direction": "udp -> tun -> qgcm_tun_read_slots", "packets": got,
                          "packet_bytes": PAYLOAD + 28, "Mpps": round(got / dt / 1e6, 3),
                          "GiB_s": round(got * (PAYLOAD + 28) / dt / 2**30, 3),
                          "packets_per_call": round(got / max(calls, 1), 1),
                          "read_calls_us_per_packet": round(t_read / max(got, 1) * 1e6, 3),
                          "read_calls_Mpps": round(got / max(t_read, 1e-9) / 1e6, 2),
                          "io_uring": os.environ.get("QGCM_TUN_URING", "1") != "0"}), flush=True)
        L.qgcm_udp_close(tx)

        rx = L.qgcm_udp_socket(HOST_IP.encode(), 0, 1 << 26)
        port = L.qgcm_udp_port(rx)
        pkt = np.frombuffer(_ipv4_udp(PEER_IP, HOST_IP, 7000, port, os.urandom(PAYLOAD)), dtype=np.uint8)
        warena = np.zeros(BATCH * STRIDE, dtype=np.uint8)
        for i in range(BATCH):
            warena[i * STRIDE + 4:i * STRIDE + 4 + len(pkt)] = pkt
        wl = np.full(BATCH, len(pkt), dtype=np.uint32)
        got, sent = 0, 0
        t0 = time.perf_counter()
        while sent < total:
            w = L.qgcm_tun_write_slots(fd, warena.ctypes.data, STRIDE, BATCH, wl.ctypes.data)
            assert w == BATCH
            sent += w
            while True:
                r = L.qgcm_udp_recv_slots(rx, arena.ctypes.data, STRIDE, BATCH, rl.ctypes.data, 0)
                if r <= 0:
                    break
                got += r
        while True:
            r = L.qgcm_udp_recv_slots(rx, arena.ctypes.data, STRIDE, BATCH, rl.ctypes.data, 50)
            if r <= 0:
                break
            got += r
        dt = time.perf_counter() - t0
        print(json.dumps({"direction": "qgcm_tun_write_slots -> tun -> udp", "packets_written": sent,
                          "packets_delivered": got, "packet_bytes": int(len(pkt)),
                          "Mpps_written": round(sent / dt / 1e6, 3),
                          "GiB_s_written": round(sent * len(pkt) / dt / 2**30, 3)}), flush=True)
        L.qgcm_udp_close(rx)
    finally:
        L.qgcm_tun_close(fds[0])


if __name__ == "__main__":
    main()
