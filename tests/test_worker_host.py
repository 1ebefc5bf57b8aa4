"""Worker pipelines (worker/outgoing.go:55-80, worker/incoming.go:54-79) over the plugin mirror, on
CPU: the Mock plugin only, with in-memory TUN/UDP stand-ins (the GPU-backed chain is in
tests/test_gpu_parity.py::test_worker_pipelines_encrypt_compress)."""
import os

from quantum_amd import common, plugin, worker


class FakeDev:
    def __init__(self, packets):
        self.packets, self.written = list(packets), []

    def Read(self, queue, buf):
        if not self.packets:
            return None, False
        pkt = self.packets.pop(0)
        buf[common.PacketStart:common.PacketStart + len(pkt)] = pkt
        return common.NewTunPayload(buf, len(pkt)), True

    def Write(self, queue, payload):
        self.written.append(bytes(payload.Raw[common.PacketStart:payload.Length]))
        return True


class FakeSock:
    def __init__(self):
        self.wire = []

    def Write(self, queue, payload, mapping):
        self.wire.append(bytes(payload.Raw[:payload.Length]))
        return True

    def Read(self, queue, buf):
        if not self.wire:
            return None, False
        w = self.wire.pop(0)
        buf[:len(w)] = w
        return common.NewSockPayload(buf, len(w)), True


def test_outgoing_then_incoming_mock_chain():
    pkts = [os.urandom(n) for n in (1, 64, 1350, common.MTU)]
    mapping = common.Mapping(SupportedPlugins=[])
    resolve = lambda p: (p, mapping, True)  # noqa: E731
    dev_in, sock, dev_out = FakeDev(pkts), FakeSock(), FakeDev([])
    mock, _ = plugin.New(plugin.MockPlugin)
    out = worker.Outgoing(dev_in, sock, resolve, [mock])
    buf = bytearray(common.MaxPacketLength)
    while out.pipeline(buf, 0):
        pass
    assert out.stats.Packets == len(pkts) + 1 and out.stats.Dropped == 1  # the final empty Read
    inc = worker.Incoming(dev_out, sock, resolve, [mock])
    while inc.pipeline(buf, 0):
        pass
    assert dev_out.written == pkts
    assert inc.stats.Bytes == sum(len(p) + common.HeaderSize for p in pkts)


def test_unresolved_packets_are_dropped():
    dev, sock = FakeDev([b"x" * 10, b"y" * 20]), FakeSock()
    calls = []

    def resolve(p):
        calls.append(len(calls))
        return p, None, len(calls) % 2 == 0  # first unresolved, second routed

    out = worker.Outgoing(dev, sock, resolve, [])
    buf = bytearray(common.MaxPacketLength)
    assert out.pipeline(buf, 0) is False
    assert out.pipeline(buf, 0) is True
    assert out.stats.Dropped == 1 and len(sock.wire) == 1


def test_plugin_order_matches_main_go():
    comp, _ = plugin.New(plugin.CompressionPlugin)
    mock, _ = plugin.New(plugin.MockPlugin)
    out = worker.Outgoing(None, None, None, [mock, comp])
    inc = worker.Incoming(None, None, None, [mock, comp])
    assert [p.Name() for p in out.plugins] == ["compression", "mock"]
    assert [p.Name() for p in inc.plugins] == ["mock", "compression"]
