"""Mirror of the reference's common.Payload / constants / Mapping fields used on this path.

common/common.go:16-38   IPStart, IPEnd, IPLength, PacketStart, MaxPacketLength, HeaderSize,
                         OverflowSize, MTU
common/payload.go:7-45   Payload{Raw, Packet, IPAddress, Length}, NewTunPayload, NewSockPayload
common/mapping.go:16-55  Mapping.SupportedPlugins, Mapping.AES
common/common.go:79-86   StringInSlice
"""
from __future__ import annotations

from dataclasses import dataclass, field

IPStart = 0
IPEnd = 4
IPLength = 4
PacketStart = 4
MaxPacketLength = 1472
HeaderSize = IPLength
OverflowSize = 35
MTU = MaxPacketLength - HeaderSize - OverflowSize  # 1433


class _View:
    """A Go-slice-like window [start, stop) of a shared bytearray (no copy)."""

    __slots__ = ("buf", "start", "stop")

    def __init__(self, buf: bytearray, start: int, stop: int):
        if not (0 <= start <= stop <= len(buf)):
            raise IndexError("slice bounds out of range")
        self.buf, self.start, self.stop = buf, start, stop

    def __len__(self) -> int:
        return self.stop - self.start

    def tobytes(self) -> bytes:
        return bytes(self.buf[self.start:self.stop])

    def __bytes__(self) -> bytes:
        return self.tobytes()


@dataclass
class Payload:
    """common/payload.go:7-19."""

    Raw: bytearray
    Packet: _View
    IPAddress: _View
    Length: int


def NewTunPayload(raw: bytearray, packetLength: int) -> Payload:
    """common/payload.go:22-32: IPAddress = Raw[0:4], Packet = Raw[4:4+n], Length = 4+n."""
    return Payload(Raw=raw, IPAddress=_View(raw, IPStart, IPEnd),
                   Packet=_View(raw, PacketStart, PacketStart + packetLength),
                   Length=HeaderSize + packetLength)


def NewSockPayload(raw: bytearray, packetLength: int) -> Payload:
    """common/payload.go:35-45: IPAddress = Raw[0:4], Packet = Raw[4:n], Length = n."""
    return Payload(Raw=raw, IPAddress=_View(raw, IPStart, IPEnd),
                   Packet=_View(raw, PacketStart, packetLength), Length=packetLength)


def StringInSlice(a: str, slice_: list[str] | None) -> bool:
    """common/common.go:79-86."""
    return a in (slice_ or [])


@dataclass
class Mapping:
    """The two Mapping fields the encryption path reads (common/mapping.go:39,54)."""

    SupportedPlugins: list[str] = field(default_factory=list)
    AES: object | None = None  # quantum_amd.crypto.AES
