"""Mirror of the reference's plugin package for the encryption path.

plugin/plugin.go:14-31   plugin names and Order constants (Compression=0 < Encryption=1 < Mock=2)
plugin/plugin.go:35-43   Direction: Incoming = 0, Outgoing = 1
plugin/plugin.go:46-58   Plugin interface: Apply, Close, Name, Order
plugin/plugin.go:60-81   Plugins / Sorter (sort by Order)
plugin/plugin.go:84-94   New(pluginType, cfg)
plugin/encryption.go     Encryption.Apply (per packet) -- here backed by the gfx950 kernels
plugin/mock.go           Mock (identity)

Apply keeps Go's contract: returns (payload, mapping, ok); ok=False means "drop the packet".
"""
from __future__ import annotations

from . import common

CompressionPlugin = "compression"
EncryptionPlugin = "encryption"
MockPlugin = "mock"

CompressionPluginOrder = 0
EncryptionPluginOrder = 1
MockPluginOrder = 2

Incoming = 0
Outgoing = 1


class Plugin:
    """plugin/plugin.go:46-58."""

    def Apply(self, direction: int, payload, mapping):  # pragma: no cover - interface
        raise NotImplementedError

    def Close(self):
        return None

    def Name(self) -> str:  # pragma: no cover - interface
        raise NotImplementedError

    def Order(self) -> int:  # pragma: no cover - interface
        raise NotImplementedError


class Encryption(Plugin):
    """plugin/encryption.go:11-59."""

    def __init__(self, cfg=None):
        self.cfg = cfg

    def Apply(self, direction: int, payload: common.Payload, mapping: common.Mapping):
        # plugin/encryption.go:17-19: peers without "encryption" pass through untouched
        if not common.StringInSlice(EncryptionPlugin, mapping.SupportedPlugins):
            return payload, mapping, True
        if direction == Incoming:
            # :22-29  Decrypt(payload.Packet, payload.IPAddress)
            length, err = mapping.AES.Decrypt(payload.Packet, payload.IPAddress)
            if err is not None:
                return payload, mapping, False
            payload.Packet = common._View(payload.Raw, common.PacketStart, common.PacketStart + length)
            payload.Length = common.HeaderSize + length
        elif direction == Outgoing:
            # :30-37  Encrypt(payload.Raw[PacketStart:], len(payload.Packet), payload.IPAddress)
            raw_tail = common._View(payload.Raw, common.PacketStart, len(payload.Raw))
            length, err = mapping.AES.Encrypt(raw_tail, len(payload.Packet), payload.IPAddress)
            if err is not None:
                return payload, mapping, False
            payload.Packet = common._View(payload.Raw, common.PacketStart, common.PacketStart + length)
            payload.Length = common.HeaderSize + length
        return payload, mapping, True

    def Close(self):
        return None

    def Name(self) -> str:
        return EncryptionPlugin

    def Order(self) -> int:
        return EncryptionPluginOrder


class Mock(Plugin):
    """plugin/mock.go:11-36."""

    def __init__(self, cfg=None):
        pass

    def Apply(self, direction, payload, mapping):
        return payload, mapping, True

    def Close(self):
        return None

    def Name(self) -> str:
        return MockPlugin

    def Order(self) -> int:
        return MockPluginOrder


def Sorter(plugins: list[Plugin], reverse: bool = False) -> list[Plugin]:
    """plugin/plugin.go:74-81 (sort.Sort(Sorter{...}) / sort.Reverse): stable sort by Order()."""
    return sorted(plugins, key=lambda p: p.Order(), reverse=reverse)


def New(pluginType: str, cfg=None):
    """plugin/plugin.go:84-94 -> (Plugin, error)."""
    if pluginType == EncryptionPlugin:
        return Encryption(cfg), None
    if pluginType == MockPlugin:
        return Mock(cfg), None
    if pluginType == CompressionPlugin:
        return None, ValueError("compression plugin is outside this build's scope (SURVEY.md s8f rank 3)")
    return None, ValueError("specified plugin is not supported")
