"""CPU: the C ABI library loads, exports every symbol include/qgcm.h declares, and its host-side
key-setup math (crypto/aes.go:66 PBKDF2, crypto/ecdh.go X25519) matches the oracle.  No GPU calls."""
import ctypes as C
import hashlib
import os
import re

import pytest

from conftest import ROOT
from oracle import oracle as O

HEADER = os.path.join(ROOT, "include", "qgcm.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(qgcm_[a-z0-9_]+)\s*\(", text)))


def test_header_lists_match_binding():
    from quantum_amd import _lib

    assert declared_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_symbol():
    from quantum_amd import _lib

    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert _lib.lib().qgcm_version().decode().startswith("qgcm")


def test_nm_exports():
    import subprocess

    from quantum_amd import _lib

    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    syms = set(re.findall(r" T (qgcm_\w+)", out))
    assert set(declared_functions()) <= syms


def test_loads_after_torch_hip_runtime():
    """torch brings its own libamdhip64 (ROCm 7.0): once `import torch` has loaded it, the library binds
    to that one, so it may only need HIP symbol versions that runtime defines (hipStreamGetId, hip_7.1,
    did not load on the GPU box, profiles/r6_s24).  A fresh process: torch first, then the library."""
    import subprocess
    import sys

    from quantum_amd import _lib

    code = ("import ctypes, torch; L = ctypes.CDLL(%r); L.qgcm_version.restype = ctypes.c_char_p; "
            "print(L.qgcm_version().decode())" % _lib.LIB_PATH)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("qgcm"), r.stderr[-2000:]


def test_gfx950_code_object_present():
    from quantum_amd import _lib

    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the only offload target built


def test_derive_key_matches_pbkdf2(kdf):
    from quantum_amd import crypto

    p = kdf["pbkdf2_path"]
    assert crypto.derive_key(p["secret"].encode(), bytes.fromhex(p["salt"])).hex() == p["out"]
    for _ in range(3):
        s, salt = os.urandom(32), os.urandom(32)
        assert crypto.derive_key(s, salt) == hashlib.pbkdf2_hmac("sha512", s, salt, 10000, 32)
    # long secret (> SHA-512 block) exercises HMAC key hashing
    s = os.urandom(200)
    assert crypto.derive_key(s, b"salt") == hashlib.pbkdf2_hmac("sha512", s, b"salt", 10000, 32)


def test_derive_keys_batch():
    from quantum_amd import crypto

    secrets, salts = os.urandom(32 * 9), os.urandom(32 * 9)
    keys = crypto.derive_keys(secrets, salts)
    for i in range(9):
        want = hashlib.pbkdf2_hmac("sha512", secrets[32 * i:32 * i + 32], salts[32 * i:32 * i + 32], 10000, 32)
        assert keys[32 * i:32 * i + 32] == want


def test_x25519_rfc7748(kdf):
    from quantum_amd import crypto

    for v in kdf["x25519"]:
        assert crypto.x25519(bytes.fromhex(v["scalar"]), bytes.fromhex(v["u"])).hex() == v["out"]
    a, b = kdf["alice"], kdf["bob"]
    assert crypto.x25519_base(bytes.fromhex(a["priv"])).hex() == a["pub"]
    assert crypto.x25519_base(bytes.fromhex(b["priv"])).hex() == b["pub"]
    assert crypto.GenerateSharedSecret(bytes.fromhex(b["pub"]), bytes.fromhex(a["priv"])).hex() == kdf["shared"]


def test_x25519_random_vs_openssl():
    from quantum_amd import crypto

    for _ in range(200):
        k, u = os.urandom(32), os.urandom(32)
        assert crypto.x25519(k, u) == O.ossl_x25519(k, u)
    pub, priv = crypto.GenerateECKeyPair()
    assert pub == O.ossl_x25519_base(priv) and len(pub) == len(priv) == 32


def test_peer_table_digest(kdf):
    """common/mapping.go:90-99 for 1024 seeded peers: X25519 twice, then PBKDF2 (host, batched)."""
    from quantum_amd import crypto

    pe = kdf["peers"]
    me_priv, me_salt = bytes.fromhex(pe["me_priv"]), bytes.fromhex(pe["me_salt"])
    secrets, salts = bytearray(), bytearray()
    for i in range(1024):
        p_priv = O.stream_bytes(pe["seed_peers"], 64 * i, 32)
        p_salt = O.stream_bytes(pe["seed_peers"], 64 * i + 32, 32)
        secrets += crypto.x25519(me_priv, crypto.x25519_base(p_priv))
        salts += crypto.x25519(me_salt, crypto.x25519_base(p_salt))
    for f in pe["first"]:
        i = f["index"]
        assert secrets[32 * i:32 * i + 32].hex() == f["secret"] and salts[32 * i:32 * i + 32].hex() == f["salt"]
    keys = crypto.derive_keys(bytes(secrets), bytes(salts))
    assert hashlib.sha256(keys).hexdigest() == pe["sha256_of_1024_keys"]


def test_create_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from quantum_amd import _lib

    err = C.create_string_buffer(_lib.ERRLEN)
    assert not _lib.lib().qgcm_create(0, 16, err, _lib.ERRLEN)
    assert err.value  # an explanation, never a silent CPU fallback
    from quantum_amd.crypto import Context

    with pytest.raises(_lib.QgcmError):
        Context(device=0)


def test_null_and_bad_args_rejected():
    from quantum_amd import _lib

    L = _lib.lib()
    assert L.qgcm_derive_key(None, 1, b"x", 1, None) == _lib.QGCM_E_ARG
    assert L.qgcm_x25519(None, None, None) == _lib.QGCM_E_ARG
    assert L.qgcm_seal_uniform(None, None, 0, 0, 0, 0, None, 4, None, None) == _lib.QGCM_E_ARG
    assert L.qgcm_seal_one(None, 0, None, 0, None, 0, None) == -1
    assert L.qgcm_open_one(None, 0, None, 0, None, 0) == -1
    assert L.qgcm_strerror(_lib.QGCM_E_AUTH) == b"message authentication failed"
    err = C.create_string_buffer(_lib.ERRLEN)
    assert not L.qgcm_host_alloc(0)


def test_max_keys_bound():
    """max_keys above QGCM_MAX_KEYS (2^20 - 1) is refused before any device work: key index 2^20 - 1
    would sort onto the descriptor worklist's all-ones excluded marker (worklist.hip)."""
    from quantum_amd import _lib

    L = _lib.lib()
    for bad in (0, 1 << 20, 1 << 31):
        err = C.create_string_buffer(_lib.ERRLEN)
        assert not L.qgcm_create(0, bad, err, _lib.ERRLEN)
        assert b"max_keys" in err.value
    hdr = open(os.path.join(ROOT, "include", "qgcm.h")).read()
    assert "#define QGCM_MAX_KEYS ((1u << 20) - 1)" in hdr
