"""Mirror of the reference's plugin package for the encryption path.

plugin/plugin.go:14-31   plugin names and Order constants (Compression=0 < Encryption=1 < Mock=2)
plugin/plugin.go:35-43   Direction: Incoming = 0, Outgoing = 1
plugin/plugin.go:46-58   Plugin interface: Apply, Close, Name, Order
plugin/plugin.go:60-81   Plugins / Sorter (sort by Order)
plugin/plugin.go:84-94   New(pluginType, cfg)
plugin/encryption.go     Encryption.Apply (per packet) -- here backed by the gfx950 kernels
plugin/mock.go           Mock (identity)
plugin/compression.go    Compression.Apply (per packet) -- snappy block format, libqgcm host codec

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


def _snappy(fn: str, data: bytes, cap: int) -> bytes | None:
    import ctypes as C

    from . import _lib

    src = C.create_string_buffer(data, len(data)) if data else None
    dst = C.create_string_buffer(max(cap, 1))
    n = getattr(_lib.lib(), fn)(src, len(data), dst, cap)
    return None if n < 0 else dst.raw[:n]


class Compression(Plugin):
    """plugin/compression.go:11-70 (snappy Encode/Decode of Payload.Packet, copied into Raw[4:])."""

    def __init__(self, cfg=None):
        self.cfg = cfg

    def Apply(self, direction: int, payload: common.Payload, mapping: common.Mapping):
        from . import _lib

        if not common.StringInSlice(CompressionPlugin, mapping.SupportedPlugins):  # :31-33
            return payload, mapping, True
        packet = bytes(payload.Packet)
        if direction == Incoming:  # :36-43 decompress; a decode error drops the packet
            n = _lib.lib().qgcm_snappy_uncompressed_length(packet, len(packet)) if packet else -1
            # an empty result is golang/snappy's nil slice, which :37-39 treats as a failure
            out = _snappy("qgcm_snappy_uncompress", packet, n) if n > 0 else None
        elif direction == Outgoing:  # :44-51 compress
            out = _snappy("qgcm_snappy_compress", packet, _lib.lib().qgcm_snappy_max_compressed_length(len(packet)))
        else:
            return payload, mapping, True
        if out is None:
            return payload, mapping, False
        room = len(payload.Raw) - common.PacketStart
        payload.Raw[common.PacketStart:common.PacketStart + min(len(out), room)] = out[:room]  # Go copy()
        payload.Packet = common._View(payload.Raw, common.PacketStart, common.PacketStart + len(out))
        payload.Length = common.HeaderSize + len(out)
        return payload, mapping, True

    def Close(self):
        return None

    def Name(self) -> str:
        return CompressionPlugin

    def Order(self) -> int:
        return CompressionPluginOrder


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
        return Compression(cfg), None
    return None, ValueError("specified plugin is not supported")
