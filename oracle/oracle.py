"""ctypes view of the parity checker -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module.  The product package (quantum_amd/) never does.

* ``gcm_*`` / ``aesgo_*``: the plain-C restatement in gcm_oracle.c of crypto/aes.go:41-62
  over FIPS-197 + SP 800-38D (the Go 1.9 stdlib algorithm underneath it).
* ``ossl_*``: OpenSSL 3 libcrypto, an independent implementation used to cross-check the
  restatement, to generate golden fixtures, and as the timed CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "_build")

_u8p = C.POINTER(C.c_uint8)


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load(name: str) -> C.CDLL:
    path = os.path.join(_BUILD, name)
    if not os.path.exists(path):
        build()
    return C.CDLL(path)


_lib = None
_ossl = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        L = _load("liboracle.so")
        L.oracle_aes256_expand.argtypes = [C.c_char_p, C.c_char_p]
        L.oracle_aes256_encrypt_block.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p]
        L.oracle_gf128_mul.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p]
        L.oracle_gcm_seal.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t, C.c_char_p,
                                      C.c_size_t, C.c_char_p, C.c_char_p]
        L.oracle_gcm_open.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t, C.c_char_p,
                                      C.c_size_t, C.c_char_p, C.c_char_p]
        L.oracle_gcm_open.restype = C.c_int
        L.oracle_aesgo_encrypt.argtypes = [C.c_char_p, C.c_void_p, C.c_long, C.c_char_p, C.c_long,
                                           C.c_char_p]
        L.oracle_aesgo_encrypt.restype = C.c_long
        L.oracle_aesgo_decrypt.argtypes = [C.c_char_p, C.c_void_p, C.c_long, C.c_char_p, C.c_long]
        L.oracle_aesgo_decrypt.restype = C.c_long
        L.oracle_splitmix64_at.argtypes = [C.c_uint64, C.c_uint64]
        L.oracle_splitmix64_at.restype = C.c_uint64
        L.oracle_fill_stream.argtypes = [C.c_uint64, C.c_uint64, C.c_void_p, C.c_size_t]
        L.oracle_seal_uniform.argtypes = [C.c_char_p, C.c_void_p, C.c_size_t, C.c_long, C.c_long,
                                          C.c_long, C.c_void_p]
        L.oracle_aesgo_seal_descs.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                              C.c_void_p, C.c_long, C.c_long, C.c_long]
        L.oracle_aesgo_open_descs.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                              C.c_long, C.c_void_p, C.c_long, C.c_long]
        _lib = L
    return _lib


def ossl() -> C.CDLL:
    global _ossl
    if _ossl is None:
        L = _load("libossl_check.so")
        L.ossl_gcm_seal.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.c_char_p, C.c_int,
                                    C.c_char_p, C.c_char_p]
        L.ossl_gcm_open.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.c_char_p, C.c_int,
                                    C.c_char_p, C.c_char_p]
        L.ossl_pbkdf2_sha512.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_int, C.c_char_p,
                                         C.c_int]
        L.ossl_x25519.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p]
        L.ossl_x25519_base.argtypes = [C.c_char_p, C.c_char_p]
        L.ossl_seal_uniform.argtypes = [C.c_char_p, C.c_void_p, C.c_long, C.c_long, C.c_int, C.c_int,
                                        C.c_void_p]
        L.ossl_seal_descs.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_int, C.c_long, C.c_long]
        L.ossl_cpu_baseline.argtypes = [C.c_char_p, C.c_int, C.c_long, C.c_int]
        L.ossl_cpu_baseline.restype = C.c_double
        L.ossl_cpu_baseline_mode.argtypes = [C.c_char_p, C.c_int, C.c_long, C.c_int, C.c_int]
        L.ossl_cpu_baseline_mode.restype = C.c_double
        _ossl = L
    return _ossl


# ---------------- restatement (gcm_oracle.c) ----------------

def aes256_expand(key: bytes) -> bytes:
    rk = C.create_string_buffer(240)
    lib().oracle_aes256_expand(key, rk)
    return rk.raw


def aes256_encrypt_block(key: bytes, block: bytes) -> bytes:
    out = C.create_string_buffer(16)
    lib().oracle_aes256_encrypt_block(aes256_expand(key), block, out)
    return out.raw


def gf128_mul(x: bytes, y: bytes) -> bytes:
    out = C.create_string_buffer(16)
    lib().oracle_gf128_mul(x, y, out)
    return out.raw


def gcm_seal(key: bytes, iv: bytes, aad: bytes, pt: bytes) -> tuple[bytes, bytes]:
    ct = C.create_string_buffer(max(len(pt), 1))
    tag = C.create_string_buffer(16)
    lib().oracle_gcm_seal(key, iv, aad, len(aad), pt, len(pt), ct, tag)
    return ct.raw[: len(pt)], tag.raw


def gcm_open(key: bytes, iv: bytes, aad: bytes, ct: bytes, tag: bytes) -> bytes | None:
    pt = C.create_string_buffer(max(len(ct), 1))
    rc = lib().oracle_gcm_open(key, iv, aad, len(aad), ct, len(ct), tag, pt)
    return None if rc != 0 else pt.raw[: len(ct)]


def aesgo_encrypt(key: bytes, data: bytearray, length: int, aad: bytes | None, nonce: bytes) -> int:
    """crypto/aes.go:41-52 on a caller buffer (cap >= length+28), explicit nonce."""
    buf = (C.c_uint8 * len(data)).from_buffer(data)
    a = aad if aad else None
    return lib().oracle_aesgo_encrypt(key, C.addressof(buf), length, a, len(aad or b""), nonce)


def aesgo_decrypt(key: bytes, data: bytearray, aad: bytes | None) -> int:
    """crypto/aes.go:57-62 on the whole of `data`; returns len-28 or -1."""
    buf = (C.c_uint8 * len(data)).from_buffer(data) if len(data) else None
    addr = C.addressof(buf) if buf is not None else None
    a = aad if aad else None
    return lib().oracle_aesgo_decrypt(key, addr, len(data), a, len(aad or b""))


def splitmix64_at(seed: int, k: int) -> int:
    return lib().oracle_splitmix64_at(seed, k)


def stream_bytes(seed: int, offset: int, n: int) -> bytes:
    buf = C.create_string_buffer(max(n, 1))
    lib().oracle_fill_stream(seed, offset, buf, n)
    return buf.raw[:n]


# ---------------- OpenSSL cross-check ----------------

def ossl_gcm_seal(key: bytes, iv: bytes, aad: bytes, pt: bytes) -> tuple[bytes, bytes]:
    ct = C.create_string_buffer(len(pt) + 16)
    tag = C.create_string_buffer(16)
    if ossl().ossl_gcm_seal(key, iv, aad, len(aad), pt, len(pt), ct, tag) != 0:
        raise RuntimeError("openssl seal failed")
    return ct.raw[: len(pt)], tag.raw


def ossl_gcm_open(key: bytes, iv: bytes, aad: bytes, ct: bytes, tag: bytes) -> bytes | None:
    pt = C.create_string_buffer(len(ct) + 16)
    rc = ossl().ossl_gcm_open(key, iv, aad, len(aad), ct, len(ct), tag, pt)
    return None if rc != 0 else pt.raw[: len(ct)]


def ossl_pbkdf2_sha512(secret: bytes, salt: bytes, iters: int = 10000, n: int = 32) -> bytes:
    out = C.create_string_buffer(n)
    if ossl().ossl_pbkdf2_sha512(secret, len(secret), salt, len(salt), iters, out, n) != 0:
        raise RuntimeError("openssl pbkdf2 failed")
    return out.raw


def ossl_x25519(scalar: bytes, point: bytes) -> bytes:
    out = C.create_string_buffer(32)
    if ossl().ossl_x25519(out, scalar, point) != 0:
        raise RuntimeError("openssl x25519 failed")
    return out.raw


def ossl_x25519_base(scalar: bytes) -> bytes:
    out = C.create_string_buffer(32)
    if ossl().ossl_x25519_base(out, scalar) != 0:
        raise RuntimeError("openssl x25519 base failed")
    return out.raw


def ossl_seal_uniform(key: bytes, arena_addr: int, stride: int, n: int, L: int, aad_len: int,
                      nonces_addr: int) -> None:
    if ossl().ossl_seal_uniform(key, arena_addr, stride, n, L, aad_len, nonces_addr) != 0:
        raise RuntimeError("openssl batch seal failed")


def ossl_cpu_baseline(key: bytes, threads: int, packets_per_thread: int, L: int, mode: int = 0) -> float:
    """Wall seconds for `threads` workers each sealing + opening packets_per_thread L-byte packets.
    mode 0: a getrandom nonce per packet as crypto/aes.go:44 draws it; 1: counter nonces (no syscall)."""
    t = ossl().ossl_cpu_baseline_mode(key, threads, packets_per_thread, L, mode)
    if t < 0:
        raise RuntimeError("cpu baseline failed")
    return t


# ---------------- descriptor batches (config 3), split over host threads ----------------
# ctypes drops the GIL for the duration of each call, so chunks run on separate cores.

def _chunks(n: int, threads: int) -> list[tuple[int, int]]:
    threads = max(1, min(threads, n or 1))
    step = (n + threads - 1) // threads
    return [(lo, min(n, lo + step)) for lo in range(0, n, step)] if n else []


def _run(fn, n: int, threads: int) -> None:
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(max(1, threads)) as ex:
        list(ex.map(lambda r: fn(*r), _chunks(n, threads)))


def aesgo_seal_descs(keys: bytes, arena, offs, lens, kidx, nonces, aad_len: int = 4, threads: int = 1) -> None:
    """crypto/aes.go:41-52 on every packet of a descriptor batch, in place in `arena` (numpy uint8).
    offs uint64, lens uint32 (= L), kidx uint32, nonces uint8 (12 per packet): contiguous numpy arrays."""
    n = len(offs)
    _run(lambda lo, hi: lib().oracle_aesgo_seal_descs(keys, arena.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                                       kidx.ctypes.data, nonces.ctypes.data, aad_len, lo, hi), n,
         threads)


def aesgo_open_descs(keys: bytes, arena, offs, lens, kidx, status, aad_len: int = 4, threads: int = 1) -> None:
    """crypto/aes.go:57-62 on every packet (lens = L + 28); status[i] = 1 authentic / 0 errOpen."""
    n = len(offs)
    _run(lambda lo, hi: lib().oracle_aesgo_open_descs(keys, arena.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                                       kidx.ctypes.data, aad_len, status.ctypes.data, lo, hi), n,
         threads)


def ossl_seal_descs(keys: bytes, arena, offs, lens, kidx, nonces, aad_len: int = 4, threads: int = 1) -> None:
    """OpenSSL cross-check of aesgo_seal_descs (golden digests of full-size batches)."""
    n = len(offs)
    rcs = []

    def one(lo, hi):
        rcs.append(ossl().ossl_seal_descs(keys, arena.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                          kidx.ctypes.data, nonces.ctypes.data, aad_len, lo, hi))
    _run(one, n, threads)
    if any(rcs):
        raise RuntimeError("openssl descriptor seal failed")
