"""Mirror of the reference's crypto package on the encryption path, backed by libqgcm.

crypto/aes.go:15-19   SaltLength = 32, iterations = 10000
crypto/aes.go:22-26   type AES  -> AES (a key slot in a device Context)
crypto/aes.go:29-36   EncryptedSize / DecryptedSize
crypto/aes.go:41-52   Encrypt(data, length, additional) (int, error)
crypto/aes.go:57-62   Decrypt(data, additional) (int, error)
crypto/aes.go:65-83   NewAES(secret, salt) (*AES, error)
crypto/ecdh.go:13-31  GenerateECKeyPair() (pub, priv), GenerateSharedSecret(pub, priv)

Go's multiple returns become tuples: ``n, err = aes.Encrypt(...)`` with ``err`` None on success.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from . import _lib
from .common import _View

SaltLength = 32
iterations = 10000
keyLength = 32
NonceSize = 12
Overhead = 16


class ErrOpen(Exception):
    """cipher: message authentication failed (Go's errOpen)."""

    def __str__(self) -> str:  # pragma: no cover - message only
        return "cipher: message authentication failed"


class Context:
    """One device's key tables (qgcm_ctx).  Key slots are handed out by `alloc_slot`."""

    def __init__(self, device: int | None = None, max_keys: int = 4096):
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        err = C.create_string_buffer(_lib.ERRLEN)
        h = _lib.lib().qgcm_create(device, max_keys, err, _lib.ERRLEN)
        if not h:
            raise _lib.QgcmError(f"qgcm_create(device={device}): {err.value.decode()}")
        self.handle = h
        self.device = device
        self.max_keys = max_keys
        self._next = 0
        self._mu = threading.Lock()
        self._owned = True

    @classmethod
    def borrowed(cls, handle: int, device: int, max_keys: int, owner=None) -> "Context":
        """A view of a context owned elsewhere (a qgcm_group member): close() leaves it alone.  The
        view keeps `owner` alive; the owner invalidates the view (handle None) when it is closed."""
        c = cls.__new__(cls)
        c.handle, c.device, c.max_keys = handle, device, max_keys
        c._next, c._mu, c._owned, c._owner = max_keys, threading.Lock(), False, owner
        return c

    def launch_counts(self) -> dict:
        """Kernel launches that served this context's calls so far (qgcm_launch_counts)."""
        names = ("quad", "segmented", "per_wave", "one", "resident", "snappy_enc", "snappy_dec", "tail_waits")
        out = (C.c_uint64 * len(names))()
        _lib.check(_lib.lib().qgcm_launch_counts(self.handle, out, len(names)), "qgcm_launch_counts")
        return dict(zip(names, (int(x) for x in out)))

    def resident_stats(self) -> dict:
        """The resident per-packet kernel: requests served, instances launched, slots, workers running,
        seals served from a keystream computed ahead, callers asleep / spinning now, broken (1: every
        call takes the launch path)."""
        names = ("served", "launches", "slots", "running", "ahead_hits", "sleepers", "spinners", "broken")
        out = (C.c_uint64 * len(names))()
        n = _lib.check(_lib.lib().qgcm_resident_stats(self.handle, out, len(names)), "qgcm_resident_stats")
        return dict(zip(names[:n], (int(x) for x in out)))

    def resident_stop(self) -> None:
        _lib.check(_lib.lib().qgcm_resident_stop(self.handle), "qgcm_resident_stop")

    def alloc_slot(self) -> int:
        with self._mu:
            if self._next >= self.max_keys:
                raise _lib.QgcmError("out of key slots")
            k = self._next
            self._next += 1
            return k

    def _reserve(self, end: int) -> None:
        """Slots set explicitly are never handed out again by alloc_slot."""
        with self._mu:
            self._next = max(self._next, end)

    def set_key(self, slot: int, key: bytes) -> None:
        if len(key) != keyLength:
            raise ValueError("AES-256 key must be 32 bytes")
        _lib.check(_lib.lib().qgcm_set_key(self.handle, slot, key), "qgcm_set_key")
        self._reserve(slot + 1)

    def set_keys(self, first: int, keys: bytes) -> None:
        if len(keys) % keyLength:
            raise ValueError("keys must be a multiple of 32 bytes")
        _lib.check(_lib.lib().qgcm_set_keys(self.handle, first, len(keys) // keyLength, keys), "qgcm_set_keys")
        self._reserve(first + len(keys) // keyLength)

    def clear_keys(self, first: int, count: int = 1) -> None:
        """qgcm_clear_keys: slots [first, first + count) unset (their AES was released); calls naming
        them fail until a key is set there again."""
        _lib.check(_lib.lib().qgcm_clear_keys(self.handle, first, count), "qgcm_clear_keys")

    def close(self) -> None:
        if self.handle and getattr(self, "_owned", True):
            _lib.lib().qgcm_destroy(self.handle)
        self.handle = None
        self._owner = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


_default: Context | None = None
_default_mu = threading.Lock()


def default_context() -> Context:
    global _default
    with _default_mu:
        if _default is None:
            _default = Context()
        return _default


def derive_key(secret: bytes, salt: bytes) -> bytes:
    """crypto/aes.go:66: pbkdf2.Key(secret, salt, 10000, 32, sha512.New)."""
    out = C.create_string_buffer(keyLength)
    _lib.check(_lib.lib().qgcm_derive_key(secret, len(secret), salt, len(salt), out), "qgcm_derive_key")
    return out.raw


def derive_keys(secrets: bytes, salts: bytes) -> bytes:
    """Batched derive_key over count 32-byte secrets/salts (multithreaded host)."""
    n = len(secrets) // 32
    if len(secrets) != 32 * n or len(salts) != 32 * n:
        raise ValueError("secrets/salts must be count*32 bytes")
    out = C.create_string_buffer(32 * n)
    _lib.check(_lib.lib().qgcm_derive_keys(secrets, salts, n, out), "qgcm_derive_keys")
    return out.raw


def _addr(data, offset: int = 0) -> tuple[int, int, object]:
    """(address, length, keepalive) of a bytearray or _View window."""
    if isinstance(data, _View):
        buf, start, length = data.buf, data.start, len(data)
    elif isinstance(data, bytearray):
        buf, start, length = data, 0, len(data)
    else:
        raise TypeError("data must be a bytearray or a Payload slice (in-place operation)")
    if len(buf) == 0:
        return 0, 0, None
    arr = (C.c_uint8 * len(buf)).from_buffer(buf)
    return C.addressof(arr) + start + offset, length, arr


class AES:
    """crypto/aes.go:22-26 -- an AES-256-GCM AEAD bound to a device key slot."""

    def __init__(self, key: bytes, salt: bytes | None = None, ctx: Context | None = None):
        self.ctx = ctx or default_context()
        self.slot = self.ctx.alloc_slot()
        self.ctx.set_key(self.slot, key)
        self.salt = salt

    def NonceSize(self) -> int:
        return NonceSize

    def Overhead(self) -> int:
        return Overhead

    def EncryptedSize(self, data) -> int:
        """crypto/aes.go:29-31."""
        return len(data) + Overhead + NonceSize

    def DecryptedSize(self, data) -> int:
        """crypto/aes.go:34-36."""
        return len(data) - Overhead - NonceSize

    def Encrypt(self, data, length: int, additional=None, nonce: bytes | None = None):
        """crypto/aes.go:41-52.  Seals data[:length] in place; tag then nonce follow it.
        `nonce` is an injection point for parity tests (the reference always draws it)."""
        addr, cap, keep = _addr(data)
        if length < 0 or length + Overhead + NonceSize > cap:
            raise IndexError("slice bounds out of range")  # Go would panic in Seal/copy
        aad = bytes(additional) if additional is not None else b""
        n = _lib.lib().qgcm_seal_one(self.ctx.handle, self.slot, addr, length, aad or None, len(aad), nonce)
        del keep
        if n < 0:
            return -1, RuntimeError("qgcm_seal_one failed")
        return n, None

    def Decrypt(self, data, additional=None):
        """crypto/aes.go:57-62.  Opens data in place; returns (DecryptedSize(data), err)."""
        addr, length, keep = _addr(data)
        if length < NonceSize:
            raise IndexError("slice bounds out of range")  # the reference panics (negative slice)
        aad = bytes(additional) if additional is not None else b""
        n = _lib.lib().qgcm_open_one(self.ctx.handle, self.slot, addr, length, aad or None, len(aad))
        del keep
        return self.DecryptedSize(data) if n >= 0 else length - Overhead - NonceSize, (None if n >= 0 else ErrOpen())


def NewAES(secret: bytes, salt: bytes, ctx: Context | None = None):
    """crypto/aes.go:65-83 -> (*AES, error)."""
    try:
        return AES(derive_key(secret, salt), salt, ctx), None
    except Exception as e:  # pragma: no cover - mirrors Go's error return
        return None, e


def x25519_base(priv: bytes) -> bytes:
    out = C.create_string_buffer(32)
    _lib.check(_lib.lib().qgcm_x25519_base(out, priv), "qgcm_x25519_base")
    return out.raw


def x25519(priv: bytes, pub: bytes) -> bytes:
    out = C.create_string_buffer(32)
    _lib.check(_lib.lib().qgcm_x25519(out, priv, pub), "qgcm_x25519")
    return out.raw


def GenerateECKeyPair() -> tuple[bytes, bytes]:
    """crypto/ecdh.go:13-20 -> (pub, priv)."""
    priv = os.urandom(keyLength)
    return x25519_base(priv), priv


def GenerateSharedSecret(pubkey: bytes, privkey: bytes) -> bytes:
    """crypto/ecdh.go:23-31."""
    pub = (bytes(pubkey) + bytes(32))[:32]
    priv = (bytes(privkey) + bytes(32))[:32]
    return x25519(priv, pub)


def MappingAES(public_key: bytes | None, public_salt: bytes | None, private_key: bytes, private_salt: bytes,
               ctx: Context | None = None):
    """common/mapping.go:94-103 (ParseMapping): a peer's AES from its public key and salt and this
    node's private ones -> (*AES or None, error).  None when the peer published no keys (the
    reference then leaves mapping.AES nil)."""
    if public_key is None or public_salt is None:
        return None, None
    secret = GenerateSharedSecret(public_key, private_key)
    salt = GenerateSharedSecret(public_salt, private_salt)
    return NewAES(secret, salt, ctx)
