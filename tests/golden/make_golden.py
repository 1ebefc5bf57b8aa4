"""Generates tests/golden/*.json -- run from the repo root: python tests/golden/make_golden.py

Sources (no reference code is copied; the reference ships no known-answer vectors):
  * gcm_spec.json    NIST GCM spec AES-256 test cases 13-16 (McGrew & Viega, "The Galois/Counter
                     Mode of Operation", Appendix B), the published vectors of the algorithm the
                     reference's Go 1.9 crypto/cipher implements.  Values typed from the spec and
                     asserted against BOTH the C restatement (oracle/gcm_oracle.c) and OpenSSL.
  * aesgo.json       crypto/aes.go-framed vectors: key = NewAES("AES256Key-32Characters1234567890",
                     salt = 00..1f) (the reference tests' key, crypto/crypto_test.go:55), AAD = the
                     4-B private IP 10.99.0.1, seeded splitmix64 payloads/nonces; sealed bytes from
                     the restatement, cross-checked with OpenSSL; tamper cases.
  * kdf.json         PBKDF2-HMAC-SHA512 published vectors + the path's key; RFC 7748 X25519 vectors;
                     a 1024-peer derivation table digest (common/mapping.go:90-99).
  * batch_digest.json  SHA-256 of the sealed config-2 arena (2^20 x 1350 B) and of a smaller one.
  * config3_digest.json  BASELINE config 3 (tests/config3_workload.py): 2^20 packets of U{64..9000} B
                     under 1024 X25519+PBKDF2 peer keys; SHA-256 of the arena before sealing, sealed
                     (OpenSSL, its first 4096 packets cross-checked against the restatement) and opened.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle as O  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

TEST_SECRET = b"AES256Key-32Characters1234567890"
TEST_SALT = bytes(range(32))
AAD = bytes([10, 99, 0, 1])
SEED_PAYLOAD = 0x5EED0001
SEED_NONCE = 0x5EED0002
LENGTHS = [0, 1, 3, 4, 5, 15, 16, 17, 31, 63, 64, 65, 255, 1349, 1350, 1351, 1433, 4079, 4080, 4081, 9000]

GCM_SPEC = [
    # (case, key, iv, aad, pt, ct, tag)
    ("tc13", "00" * 32, "00" * 12, "", "", "", "530f8afbc74536b9a963b4f1c4cb738b"),
    ("tc14", "00" * 32, "00" * 12, "", "00" * 16, "cea7403d4d606b6e074ec5d3baf39d18",
     "d0d1c8a799996bf0265b98b5d48ab919"),
    ("tc15", "feffe9928665731c6d6a8f9467308308" * 2, "cafebabefacedbaddecaf888", "",
     "d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf0e2449a6b525"
     "b16aedf5aa0de657ba637b391aafd255",
     "522dc1f099567d07f47f37a32a84427d643a8cdcbfe5c0c97598a2bd2555d1aa8cb08e48590dbb3da7b08b1056828838"
     "c5f61e6393ba7a0abcc9f662898015ad", "b094dac5d93471bdec1a502270e3cc6c"),
    ("tc16", "feffe9928665731c6d6a8f9467308308" * 2, "cafebabefacedbaddecaf888",
     "feedfacedeadbeeffeedfacedeadbeefabaddad2",
     "d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf0e2449a6b525"
     "b16aedf5aa0de657ba637b39",
     "522dc1f099567d07f47f37a32a84427d643a8cdcbfe5c0c97598a2bd2555d1aa8cb08e48590dbb3da7b08b1056828838"
     "c5f61e6393ba7a0abcc9f662", "76fc6ece0f4e1768cddf8853bb2d551b"),
]

# PBKDF2-HMAC-SHA512 published vectors (password, salt, iterations, dkLen, hex)
PBKDF2 = [
    ("password", "salt", 1, 64,
     "867f70cf1ade02cff3752599a3a53dc4af34c7a669815ae5d513554e1c8cf252c02d470a285a0501bad999bfe943c08f"
     "050235d7d68b1da55e63f73b60a57fce"),
    ("password", "salt", 2, 64,
     "e1d9c16aa681708a45f5c7c4e215ceb66e011a2e9f0040713f18aefdb866d53cf76cab2868a39b9f7840edce4fef5a82"
     "be67335c77a6068e04112754f27ccf4e"),
]

# RFC 7748 s5.2 (first vector) and s6.1 (Alice/Bob)
X25519 = [
    ("a546e36bf0527c9d3b16154b82465edd62144c0ac1fc5a18506a2244ba449ac4",
     "e6db6867583030db3594c1a424b15f7c726624ec26b3353b10a903a6d0ab1c4c",
     "c3da55379de9c6908e94ea4df28d084f32eccf03491c71f754b4075577a28552"),
]
ALICE = ("77076d0a7318a57d3c16c17251b26645df4c2f87ebc0992ab177fba51db92c2a",
         "8520f0098930a754748b7ddcb43ef75a0dbf3a0d26381af4eba4a98eaa9b4e6a")
BOB = ("5dab087e624a8a4b79e17f8b83800ee66f3bb1292618b6fd1c2f8b27ff88e0eb",
       "de9edb7d7b7dc1b4d35b61c2ece435373f8343c85b78674dadfc7e146f882b4f")
SHARED = "4a5d9d5ba4ce2de1728e3bf480350f25e07e21c947d19e3376f09b3c1e161742"


def h(b: bytes) -> str:
    return b.hex()


def gcm_spec() -> list[dict]:
    out = []
    for name, k, iv, a, p, c, t in GCM_SPEC:
        K, IV, A, P = map(bytes.fromhex, (k, iv, a, p))
        ct, tag = O.gcm_seal(K, IV, A, P)
        assert (ct.hex(), tag.hex()) == (c, t), f"oracle disagrees with spec {name}"
        ct2, tag2 = O.ossl_gcm_seal(K, IV, A, P)
        assert (ct2.hex(), tag2.hex()) == (c, t), f"openssl disagrees with spec {name}"
        out.append(dict(case=name, key=k, iv=iv, aad=a, pt=p, ct=c, tag=t))
    return out


def aesgo() -> dict:
    key = O.ossl_pbkdf2_sha512(TEST_SECRET, TEST_SALT)
    vecs = []
    off = 0
    for i, L in enumerate(LENGTHS):
        for aad in (AAD, b""):
            pt = O.stream_bytes(SEED_PAYLOAD, off, L)
            nonce = O.stream_bytes(SEED_NONCE, 12 * len(vecs), 12)
            off += L
            buf = bytearray(pt + bytes(28))
            n = O.aesgo_encrypt(key, buf, L, aad, nonce)
            assert n == L + 28
            ct, tag = O.ossl_gcm_seal(key, nonce, aad, pt)
            assert bytes(buf) == ct + tag + nonce, f"openssl disagrees at L={L}"
            back = bytearray(buf)
            assert O.aesgo_decrypt(key, back, aad) == L and bytes(back[:L]) == pt
            vecs.append(dict(len=L, aad=h(aad), nonce=h(nonce), pt=h(pt), sealed=h(bytes(buf))))
    # tamper cases on the L=1350 / AAD vector: each must fail Open and zero the plaintext
    base = next(v for v in vecs if v["len"] == 1350 and v["aad"])
    sealed = bytes.fromhex(base["sealed"])
    tampers = []
    for what, idx in (("ct", 7), ("ct_last", 1349), ("tag", 1350 + 3), ("nonce", 1350 + 16 + 5)):
        t = bytearray(sealed)
        t[idx] ^= 0x01
        b = bytearray(t)
        assert O.aesgo_decrypt(key, b, AAD) == -1 and bytes(b[:1350]) == bytes(1350)
        tampers.append(dict(what=what, index=idx, sealed=h(bytes(t))))
    b = bytearray(sealed)
    assert O.aesgo_decrypt(key, b, bytes([10, 99, 0, 2])) == -1
    tampers.append(dict(what="aad", index=-1, sealed=base["sealed"], aad="0a630002"))
    return dict(secret=TEST_SECRET.decode(), salt=h(TEST_SALT), key=h(key), aad=h(AAD), seed_payload=SEED_PAYLOAD,
                seed_nonce=SEED_NONCE, vectors=vecs, tamper=tampers)


def kdf() -> dict:
    for pw, salt, it, n, want in PBKDF2:
        assert O.ossl_pbkdf2_sha512(pw.encode(), salt.encode(), it, n).hex() == want
        assert hashlib.pbkdf2_hmac("sha512", pw.encode(), salt.encode(), it, n).hex() == want
    for s, u, want in X25519:
        assert O.ossl_x25519(bytes.fromhex(s), bytes.fromhex(u)).hex() == want
    assert O.ossl_x25519_base(bytes.fromhex(ALICE[0])).hex() == ALICE[1]
    assert O.ossl_x25519_base(bytes.fromhex(BOB[0])).hex() == BOB[1]
    assert O.ossl_x25519(bytes.fromhex(ALICE[0]), bytes.fromhex(BOB[1])).hex() == SHARED
    path_key = hashlib.pbkdf2_hmac("sha512", TEST_SECRET, TEST_SALT, 10000, 32)
    # 1024-peer table (common/mapping.go:90-99): seeded private keys/salts for "me" and each peer.
    me_priv = O.stream_bytes(0x5EED0003, 0, 32)
    me_salt = O.stream_bytes(0x5EED0003, 32, 32)
    peers = []
    hsh = hashlib.sha256()
    for i in range(1024):
        p_priv = O.stream_bytes(0x5EED0004, 64 * i, 32)
        p_salt = O.stream_bytes(0x5EED0004, 64 * i + 32, 32)
        pub, pubsalt = O.ossl_x25519_base(p_priv), O.ossl_x25519_base(p_salt)
        secret = O.ossl_x25519(me_priv, pub)
        salt = O.ossl_x25519(me_salt, pubsalt)
        key = hashlib.pbkdf2_hmac("sha512", secret, salt, 10000, 32)
        hsh.update(key)
        if i < 4:
            peers.append(dict(index=i, pub=h(pub), pubsalt=h(pubsalt), secret=h(secret), salt=h(salt), key=h(key)))
    return dict(pbkdf2=[dict(password=p, salt=s, iters=i, dklen=n, out=o) for p, s, i, n, o in PBKDF2],
                pbkdf2_path=dict(secret=TEST_SECRET.decode(), salt=h(TEST_SALT), iters=10000, out=h(path_key)),
                x25519=[dict(scalar=s, u=u, out=o) for s, u, o in X25519],
                alice=dict(priv=ALICE[0], pub=ALICE[1]), bob=dict(priv=BOB[0], pub=BOB[1]), shared=SHARED,
                peers=dict(me_priv=h(me_priv), me_salt=h(me_salt), first=peers, sha256_of_1024_keys=hsh.hexdigest(),
                           seed_me=0x5EED0003, seed_peers=0x5EED0004))


def batch_arena(n: int, L: int, stride: int) -> tuple[np.ndarray, np.ndarray]:
    """Config-2 synthetic batch exactly as qgcm_fill_uniform lays it out (zeroed gaps)."""
    arena = np.zeros(n * stride, dtype=np.uint8)
    payload = np.frombuffer(O.stream_bytes(SEED_PAYLOAD, 0, n * L), dtype=np.uint8).reshape(n, L)
    view = arena.reshape(n, stride)
    view[:, :4] = np.frombuffer(AAD, dtype=np.uint8)
    view[:, 4:4 + L] = payload
    nonces = np.frombuffer(O.stream_bytes(SEED_NONCE, 0, 12 * n), dtype=np.uint8).copy()
    return arena, nonces


def batch_digest(n: int, L: int, stride: int, key: bytes, check_oracle: int) -> dict:
    arena, nonces = batch_arena(n, L, stride)
    if check_oracle:
        ref = arena[: check_oracle * stride].copy()
        O.lib().oracle_seal_uniform(key, ref.ctypes.data, stride, check_oracle, L, 4, nonces.ctypes.data)
    O.ossl_seal_uniform(key, arena.ctypes.data, stride, n, L, 4, nonces.ctypes.data)
    if check_oracle:
        assert np.array_equal(ref, arena[: check_oracle * stride]), "restatement != openssl on batch prefix"
    plain, _ = batch_arena(n, L, stride)
    return dict(n=n, len=L, stride=stride, aad=h(AAD), seed_payload=SEED_PAYLOAD, seed_nonce=SEED_NONCE,
                sha256_sealed=hashlib.sha256(arena.tobytes()).hexdigest(),
                sha256_plain=hashlib.sha256(plain.tobytes()).hexdigest(), oracle_checked_prefix=check_oracle)


def peer_keys() -> bytes:
    """The 1024 config-3 peer keys (common/mapping.go:90-99) from OpenSSL X25519 + hashlib PBKDF2."""
    import config3_workload as W

    me_priv, me_salt, privs, salts = W.peer_inputs(O)
    out = bytearray()
    for p_priv, p_salt in zip(privs, salts):
        secret = O.ossl_x25519(me_priv, O.ossl_x25519_base(p_priv))
        salt = O.ossl_x25519(me_salt, O.ossl_x25519_base(p_salt))
        out += hashlib.pbkdf2_hmac("sha512", secret, salt, 10000, 32)
    return bytes(out)


def sha_chunks(a: np.ndarray) -> str:
    hsh = hashlib.sha256()
    for i in range(0, len(a), 1 << 28):
        hsh.update(memoryview(a[i:i + (1 << 28)]))
    return hsh.hexdigest()


def config3(threads: int = 8) -> dict:
    import config3_workload as W

    keys = peer_keys()
    lens, kidx = W.lengths(), W.key_indices()
    offs, size = W.layout(lens)
    nonces = W.nonces(O)
    arena = W.host_arena(O, size, offs, kidx)
    plain_sha = sha_chunks(arena)
    check = 4096
    ref = arena.copy() if check else None
    O.ossl_seal_descs(keys, arena, offs, lens, kidx, nonces, 4, threads)
    if check:
        O.aesgo_seal_descs(keys, ref, offs[:check], lens[:check], kidx[:check], nonces, 4, threads)
        end = int(offs[check])
        assert np.array_equal(ref[:end], arena[:end]), "restatement != openssl on the config-3 prefix"
        del ref
    sealed_sha = sha_chunks(arena)
    tails = arena[W.tail_index(offs, lens)]
    opened = W.host_arena(O, size, offs, kidx)
    opened[W.tail_index(offs, lens)] = tails  # Open leaves tag || nonce in the slot
    opened_sha = sha_chunks(opened)
    return dict(n=W.N, keys=W.NKEYS, sha256_of_1024_keys=hashlib.sha256(keys).hexdigest(),
                payload_bytes=int(lens.sum()), arena_bytes=size, slot_bytes_used=int(offs[-1]) + ((4 + int(lens[-1]) + 31) & ~3),
                sha256_plain=plain_sha, sha256_sealed=sealed_sha, sha256_opened=opened_sha,
                oracle_checked_prefix=check, seeds=dict(len=W.SEED_LEN, key=W.SEED_KEY, arena=W.SEED_ARENA,
                                                        nonce=W.SEED_NONCE, me=W.SEED_ME, peers=W.SEED_PEERS))


def main() -> None:
    os.makedirs(HERE, exist_ok=True)
    json.dump(gcm_spec(), open(os.path.join(HERE, "gcm_spec.json"), "w"), indent=1)
    ag = aesgo()
    json.dump(ag, open(os.path.join(HERE, "aesgo.json"), "w"), indent=1)
    json.dump(kdf(), open(os.path.join(HERE, "kdf.json"), "w"), indent=1)
    key = bytes.fromhex(ag["key"])
    digests = [batch_digest(4096, 1350, 1392, key, 4096), batch_digest(1 << 20, 1350, 1392, key, 2048),
               batch_digest(1 << 14, 1350, 1472, key, 512)]
    json.dump(digests, open(os.path.join(HERE, "batch_digest.json"), "w"), indent=1)
    if "--no-config3" not in sys.argv:
        json.dump(config3(), open(os.path.join(HERE, "config3_digest.json"), "w"), indent=1)
    print("golden fixtures written")


if __name__ == "__main__":
    main()
