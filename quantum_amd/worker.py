"""Mirror of the reference's per-packet callers of the plugin chain.

worker/outgoing.go:55-80  Outgoing.pipeline: dev.Read -> resolve -> plugins[i].Apply(Outgoing) -> sock.Write
worker/incoming.go:54-79  Incoming.pipeline: sock.Read -> resolve -> plugins[i].Apply(Incoming) -> dev.Write
worker/outgoing.go:36-52  stats: one metric per packet, Dropped on any failed step, Bytes += Length

The TUN device, UDP socket and router are out of scope: they are injected as objects
with the reference's method shapes -- dev.Read(queue, buf) -> (payload, ok), sock.Write(queue,
payload, mapping) -> ok, resolve(payload) -> (payload, mapping, ok), and the mirror images -- so the
plugin chain runs exactly as the unchanged Go workers drive it.  Each worker owns one
common.MaxPacketLength buffer for its lifetime (outgoing.go:88, incoming.go:87).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field

from . import common, plugin


@dataclass
class Stats:
    """The aggregator's view of one direction (metric.Tx / metric.Rx counters)."""

    Packets: int = 0
    Dropped: int = 0
    Bytes: int = 0
    _mu: threading.Lock = field(default_factory=threading.Lock, repr=False)

    def add(self, dropped: bool, payload) -> None:
        with self._mu:
            self.Packets += 1
            self.Dropped += int(dropped)
            if payload is not None:
                self.Bytes += payload.Length


class Outgoing:
    """worker/outgoing.go: TUN -> plugins (sorted ascending, main.go:50) -> UDP."""

    def __init__(self, dev, sock, resolve, plugins: list[plugin.Plugin]):
        self.dev, self.sock, self.resolve = dev, sock, resolve
        self.plugins = plugin.Sorter(plugins)
        self.stats = Stats()
        self.stop = False

    def pipeline(self, buf: bytearray, queue: int) -> bool:
        """worker/outgoing.go:55-80."""
        payload, ok = self.dev.Read(queue, buf)
        if not ok:
            self.stats.add(True, payload)
            return False
        payload, mapping, ok = self.resolve(payload)
        if not ok:
            self.stats.add(True, payload)
            return False
        for p in self.plugins:
            payload, mapping, ok = p.Apply(plugin.Outgoing, payload, mapping)
            if not ok:
                self.stats.add(True, payload)
                return False
        if not self.sock.Write(queue, payload, mapping):
            self.stats.add(True, payload)
            return False
        self.stats.add(False, payload)
        return True

    def Start(self, queue: int) -> threading.Thread:
        """worker/outgoing.go:84-93: one thread per queue, one buffer per thread."""
        def run():
            buf = bytearray(common.MaxPacketLength)
            while not self.stop:
                self.pipeline(buf, queue)

        t = threading.Thread(target=run, daemon=True)
        t.start()
        return t

    def Stop(self) -> None:
        self.stop = True


class Incoming:
    """worker/incoming.go: UDP -> plugins (sorted descending, main.go:51) -> TUN."""

    def __init__(self, dev, sock, resolve, plugins: list[plugin.Plugin]):
        self.dev, self.sock, self.resolve = dev, sock, resolve
        self.plugins = plugin.Sorter(plugins, reverse=True)
        self.stats = Stats()
        self.stop = False

    def pipeline(self, buf: bytearray, queue: int) -> bool:
        """worker/incoming.go:54-79."""
        payload, ok = self.sock.Read(queue, buf)
        if not ok:
            self.stats.add(True, payload)
            return False
        payload, mapping, ok = self.resolve(payload)
        if not ok:
            self.stats.add(True, payload)
            return False
        for p in self.plugins:
            payload, mapping, ok = p.Apply(plugin.Incoming, payload, mapping)
            if not ok:
                self.stats.add(True, payload)
                return False
        if not self.dev.Write(queue, payload):
            self.stats.add(True, payload)
            return False
        self.stats.add(False, payload)
        return True

    def Start(self, queue: int) -> threading.Thread:
        def run():
            buf = bytearray(common.MaxPacketLength)
            while not self.stop:
                self.pipeline(buf, queue)

        t = threading.Thread(target=run, daemon=True)
        t.start()
        return t

    def Stop(self) -> None:
        self.stop = True
