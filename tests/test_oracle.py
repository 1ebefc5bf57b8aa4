"""CPU: the parity checker itself, pinned against published vectors and OpenSSL.

The reference holds no known-answer vectors for this path (crypto/crypto_test.go:54-131 and
plugin/plugin_test.go:89-216 are round-trip/size tests with random salts), so the oracle is pinned
by the NIST GCM spec vectors and an independent implementation (OpenSSL), and by the semantics
those reference tests do pin: sizes +28/-28, nonce last, tag before it, round trip.
"""
import hashlib
import os

import pytest

from oracle import oracle as O


def test_gcm_spec_vectors(gcm_spec):
    for v in gcm_spec:
        K, IV, A, P = (bytes.fromhex(v[k]) for k in ("key", "iv", "aad", "pt"))
        ct, tag = O.gcm_seal(K, IV, A, P)
        assert ct.hex() == v["ct"] and tag.hex() == v["tag"], v["case"]
        assert O.gcm_open(K, IV, A, ct, tag) == P
        bad = bytearray(tag)
        bad[0] ^= 1
        assert O.gcm_open(K, IV, A, ct, bytes(bad)) is None


def test_aes_block_fips197_c3():
    # FIPS-197 Appendix C.3 (AES-256 example vector)
    key = bytes(range(32))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    assert O.aes256_encrypt_block(key, pt).hex() == "8ea2b7ca516745bfeafc49904b496089"


def test_gf128_identity_and_commutativity():
    one = bytes([0x80]) + bytes(15)
    x = os.urandom(16)
    y = os.urandom(16)
    assert O.gf128_mul(x, one) == x
    assert O.gf128_mul(x, y) == O.gf128_mul(y, x)


@pytest.mark.parametrize("L", [0, 1, 15, 16, 17, 100, 1350, 1433, 4096, 9000])
def test_oracle_matches_openssl_random(L):
    for _ in range(3):
        key, iv, pt = os.urandom(32), os.urandom(12), os.urandom(L)
        for aad in (b"", os.urandom(4)):
            assert O.gcm_seal(key, iv, aad, pt) == O.ossl_gcm_seal(key, iv, aad, pt)


def test_aesgo_vectors_restated(aesgo):
    """crypto/aes.go:41-52 framing: ct || tag || nonce, size L+28, in place."""
    key = bytes.fromhex(aesgo["key"])
    for v in aesgo["vectors"]:
        L, aad, nonce, pt = v["len"], bytes.fromhex(v["aad"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["pt"])
        buf = bytearray(pt + bytes(28))
        assert O.aesgo_encrypt(key, buf, L, aad, nonce) == L + 28
        assert buf.hex() == v["sealed"]
        assert O.aesgo_decrypt(key, buf, aad) == L
        assert bytes(buf[:L]) == pt


def test_aesgo_tamper_zeroes(aesgo):
    """Go 1.9 gcm Open zeroes the plaintext region on tag mismatch."""
    key = bytes.fromhex(aesgo["key"])
    for t in aesgo["tamper"]:
        buf = bytearray.fromhex(t["sealed"])
        aad = bytes.fromhex(t.get("aad", aesgo["aad"]))
        assert O.aesgo_decrypt(key, buf, aad) == -1
        assert bytes(buf[: len(buf) - 28]) == bytes(len(buf) - 28)


def test_aesgo_short_inputs():
    key = os.urandom(32)
    for n in (12, 20, 27):  # 12 <= len < 28: errOpen, untouched
        buf = bytearray(os.urandom(n))
        before = bytes(buf)
        assert O.aesgo_decrypt(key, buf, None) == -1
        assert bytes(buf) == before
    assert O.aesgo_decrypt(key, bytearray(5), None) == -1  # the reference panics here


def test_crypto_test_go_roundtrip():
    """crypto/crypto_test.go:54-101 TestAES restated: 1472 B of 0x01, nil AAD, random salt."""
    key = hashlib.pbkdf2_hmac("sha512", b"AES256Key-32Characters1234567890", os.urandom(32), 10000, 32)
    buf = bytearray(b"\x01" * 1472 + bytes(28))
    n = O.aesgo_encrypt(key, buf, 1472, None, os.urandom(12))
    assert n == 1500 and bytes(buf[:1472]) != b"\x01" * 1472
    assert O.aesgo_decrypt(key, buf, None) == 1472 and bytes(buf[:1472]) == b"\x01" * 1472


def test_kdf_vectors(kdf):
    for v in kdf["pbkdf2"]:
        out = O.ossl_pbkdf2_sha512(v["password"].encode(), v["salt"].encode(), v["iters"], v["dklen"])
        assert out.hex() == v["out"]
    p = kdf["pbkdf2_path"]
    assert hashlib.pbkdf2_hmac("sha512", p["secret"].encode(), bytes.fromhex(p["salt"]), 10000, 32).hex() == p["out"]
    for v in kdf["x25519"]:
        assert O.ossl_x25519(bytes.fromhex(v["scalar"]), bytes.fromhex(v["u"])).hex() == v["out"]
    assert O.ossl_x25519(bytes.fromhex(kdf["alice"]["priv"]), bytes.fromhex(kdf["bob"]["pub"])).hex() == kdf["shared"]


def test_splitmix_stream():
    # splitmix64 reference output for seed 0 (first value) -- Vigna's published generator
    assert O.splitmix64_at(0, 0) == 0xE220A8397B1DCDAF
    b = O.stream_bytes(0x5EED0001, 5, 11)
    full = O.stream_bytes(0x5EED0001, 0, 16)
    assert b == full[5:16]
