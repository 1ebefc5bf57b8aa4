"""BASELINE.json workloads, defined once for bench.py, the GPU parity tests and the golden generator.

Config 3 (the keyed, ragged workload): 2^20 packets, payload lengths ~ U{64..9000} (the first few
forced onto the counter-segment edges of the kernels: block 254/255 -> 256 is where a packet's counter
cache is re-derived, L = 4064..4097, and again at 8160..8193), 1024 per-peer keys derived as
common/mapping.go:90-99 does it (X25519 of this node's private key with the peer's public key = the
secret, the same for the salts, then crypto/aes.go:66 PBKDF2-HMAC-SHA512 x10000), key index
~ U[0, 1024), AAD = the peer's private IPv4 10.99.(k >> 8).(k & 255) in Raw[0:4]
(worker/outgoing.go:28-35 writes the sender IP there).

Slots are packed Payload.Raw records, 4-B aligned: slot i at offs[i], (4 + L + 28 + 3) & ~3 bytes.
Arena bytes before sealing: qgcm_fill_uniform over 1 MiB chunks (chunk c = [AAD_WORD][splitmix64
stream of SEED_ARENA at byte offset c * (2^20 - 4)]), then each packet's 4-B AAD.  Nonces: the
splitmix64 stream of SEED_NONCE, 12 B per packet.  Lengths and key indices: splitmix64 outputs.
tests/golden/config3_digest.json holds the SHA-256 of this arena before sealing, sealed and opened.
"""
from __future__ import annotations

import numpy as np

N = 1 << 20
NKEYS = 1024
CHUNK = 1 << 20
AAD_WORD = int.from_bytes(bytes([10, 99, 0, 1]), "little")
SEED_ME, SEED_PEERS = 0x5EED0003, 0x5EED0004  # tests/golden/kdf.json "peers"
SEED_LEN, SEED_KEY = 0x5EED0031, 0x5EED0032
SEED_ARENA, SEED_NONCE = 0x5EED0033, 0x5EED0034
FORCED = [4064, 4065, 4079, 4080, 4081, 4095, 4096, 4097, 8160, 8161, 8176, 8191, 8192, 8193, 8999, 9000,
          64, 65, 1350, 1433]


def splitmix64(seed: int, k: np.ndarray) -> np.ndarray:
    """Output k of the splitmix64 generator started at seed, vectorised (the device fill's
    splitmix_at, gcm_kernels.hip)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (k.astype(np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def stream_bytes(seed: int, offset: int, n: int) -> bytes:
    """Bytes [offset, offset + n) of the little-endian splitmix64 stream of `seed`."""
    if n <= 0:
        return b""
    k0, k1 = offset // 8, (offset + n + 7) // 8
    words = splitmix64(seed, np.arange(k0, k1, dtype=np.uint64)).astype("<u8")
    start = offset - 8 * k0
    return words.view(np.uint8)[start:start + n].tobytes()


def lengths(n: int = N) -> np.ndarray:
    i = np.arange(n, dtype=np.uint64)
    L = (np.uint64(64) + splitmix64(SEED_LEN, i) % np.uint64(8937)).astype(np.uint32)
    m = min(n, len(FORCED))
    L[:m] = FORCED[:m]
    return L


def key_indices(n: int = N) -> np.ndarray:
    return (splitmix64(SEED_KEY, np.arange(n, dtype=np.uint64)) % np.uint64(NKEYS)).astype(np.uint32)


def layout(lens: np.ndarray) -> tuple[np.ndarray, int]:
    """Packed 4-B aligned slot offsets and the arena size (whole fill chunks, >= 64 B of slack)."""
    slot = (4 + lens.astype(np.uint64) + 28 + 3) & ~np.uint64(3)
    offs = np.zeros(len(lens), dtype=np.uint64)
    offs[1:] = np.cumsum(slot)[:-1]
    used = int(offs[-1] + slot[-1]) if len(lens) else 0
    chunks = (used + 64 + CHUNK - 1) // CHUNK
    return offs, chunks * CHUNK


def aad_of_key(k: np.ndarray) -> np.ndarray:
    """(n, 4) uint8: 10.99.(k >> 8).(k & 255)."""
    a = np.empty((len(k), 4), dtype=np.uint8)
    a[:, 0], a[:, 1] = 10, 99
    a[:, 2] = (k >> 8) & 0xFF
    a[:, 3] = k & 0xFF
    return a


def peer_inputs() -> tuple[bytes, bytes, list[bytes], list[bytes]]:
    """This node's private key and salt, and each peer's private key and salt (kdf.json recipe)."""
    me_priv = stream_bytes(SEED_ME, 0, 32)
    me_salt = stream_bytes(SEED_ME, 32, 32)
    privs = [stream_bytes(SEED_PEERS, 64 * i, 32) for i in range(NKEYS)]
    salts = [stream_bytes(SEED_PEERS, 64 * i + 32, 32) for i in range(NKEYS)]
    return me_priv, me_salt, privs, salts


def peer_keys() -> bytes:
    """The 1024 peer keys through the product path (common/mapping.go:90-99): secret =
    X25519(me.priv, peer.pub), salt likewise, key = PBKDF2-HMAC-SHA512(secret, salt, 10000, 32)
    (qgcm_x25519*, qgcm_derive_keys; libqgcm keymath on the host)."""
    from .crypto import derive_keys, x25519, x25519_base

    me_priv, me_salt, privs, salts = peer_inputs()
    secrets = b"".join(x25519(me_priv, x25519_base(p)) for p in privs)
    salts_ = b"".join(x25519(me_salt, x25519_base(s)) for s in salts)
    return derive_keys(secrets, salts_)


def nonces(n: int = N) -> np.ndarray:
    return np.frombuffer(stream_bytes(SEED_NONCE, 0, 12 * n), dtype=np.uint8).copy()


def put_aads(a, offs: np.ndarray, kidx: np.ndarray) -> None:
    """Raw[0:4] of every slot = its peer's IP (numpy array, or a torch tensor on any device)."""
    idx = offs.astype(np.int64)[:, None] + np.arange(4, dtype=np.int64)
    if isinstance(a, np.ndarray):
        a[idx] = aad_of_key(kidx)
    else:
        import torch

        a[torch.from_numpy(idx).to(a.device)] = torch.from_numpy(aad_of_key(kidx)).to(a.device)


def device_arena(torch, size: int, offs: np.ndarray, kidx: np.ndarray, device="cuda"):
    """The config-3 arena built on the device (qgcm_fill_uniform over 1 MiB chunks, then the AADs)."""
    from . import batch

    arena = torch.empty(size, dtype=torch.uint8, device=device)
    batch.fill_uniform(arena, CHUNK, size // CHUNK, CHUNK - 4, AAD_WORD, SEED_ARENA, None, 0)
    put_aads(arena, offs, kidx)
    return arena


def tail_index(offs: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """(n, 28) byte indices of every slot's tag || nonce."""
    return (offs.astype(np.int64) + 4 + lens.astype(np.int64))[:, None] + np.arange(28, dtype=np.int64)


# Config 5 (compression + encryption chain, plugin/compression.go then plugin/encryption.go in the
# order main.go:50-51 sorts them): 2^20 Payload.Raw slots of common.MaxPacketLength = 1472 B, each
# [AAD 10.99.0.1][1350-B packet][zeros]; a packet's first half is seeded random bytes, its second half a
# repeated HTTP request line (compresses to ~0.64 with golang/snappy's block algorithm).  Nonces: 12 seeded
# bytes per packet.  tests/golden/config5_digest.json pins the sealed arena and lengths
# (tests/golden/make_config5_golden.py: libsnappy 1.1.8 + OpenSSL, cross-checked with the restatements).
C5_N, C5_LEN, C5_STRIDE = 1 << 20, 1350, 1472
C5_SEED_PAYLOAD, C5_SEED_NONCE = 0x5EED0005, 0x5EED0015
C5_LINE = b"GET /quantum/v1/peers HTTP/1.1\r\nHost: 10.99.0.1\r\n"


def config5_packets(n: int = C5_N, L: int = C5_LEN, stride: int = C5_STRIDE) -> np.ndarray:
    """(n, stride) uint8 host slots of config 5 (the rest of each slot zero)."""
    host = np.zeros((n, stride), np.uint8)
    rng = np.random.default_rng(C5_SEED_PAYLOAD)
    host[:, :4] = np.frombuffer(AAD_WORD.to_bytes(4, "little"), np.uint8)
    half = L // 2
    host[:, 4:4 + half] = rng.integers(0, 256, (n, half), dtype=np.uint8)
    line = np.frombuffer(C5_LINE, np.uint8)
    host[:, 4 + half:4 + L] = np.tile(line, (L - half) // len(line) + 1)[:L - half]
    return host


def config5_nonces(n: int = C5_N) -> np.ndarray:
    """n * 12 seeded nonce bytes (production seals draw them from getrandom, qgcm_random_nonces)."""
    return np.random.default_rng(C5_SEED_NONCE).integers(0, 256, 12 * n, dtype=np.uint8)
