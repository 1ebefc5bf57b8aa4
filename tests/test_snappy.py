"""CPU: the snappy block codec of the compression plugin (plugin/compression.go) and the plugin
mirror.  golang/snappy (the reference's encoder) is absent; its block algorithm is Google's C++
snappy CompressFragment, and libsnappy 1.1.8 is in this image, so the encoder's exact output bytes are
pinned to libsnappy's: tests/golden/snappy.json (270 cases, tests/golden/make_snappy_golden.py) holds
them, and both libqgcm's host encoder and the pure-Python restatement oracle/snappy_oracle.py must
reproduce them.  Also: round trips, cross-decoding with libsnappy and pyarrow's snappy, malformed-input
rejection, and the reference's TestCompression shape."""
import ctypes as C
import hashlib
import json
import os
import random

import pytest

from oracle import snappy_oracle
from quantum_amd import _lib, common, plugin

import snappy_inputs as SI

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "snappy.json")


def _golden_match(case, comp: bytes) -> bool:
    if len(comp) != case["out_len"]:
        return False
    if "out_hex" in case:
        return comp.hex() == case["out_hex"]
    return hashlib.sha256(comp).hexdigest() == case["out_sha256"]


def test_host_encoder_bytes_equal_libsnappy_golden():
    with open(GOLDEN) as f:
        cases = json.load(f)["cases"]
    assert len(cases) == len(SI.cases())
    for case in cases:
        data = SI.make(case["kind"], case["n"])
        assert hashlib.sha256(data).hexdigest() == case["in_sha256"]
        comp = _compress(data)
        assert _golden_match(case, comp), (case["kind"], case["n"])
        assert _uncompress(comp, len(data)) == data


def test_oracle_restatement_equals_golden():
    with open(GOLDEN) as f:
        cases = json.load(f)["cases"]
    for case in cases:
        if case["n"] > 20000:  # pure-Python loops: the long cases are the host encoder's
            continue
        data = SI.make(case["kind"], case["n"])
        comp = snappy_oracle.encode(data)
        assert _golden_match(case, comp), (case["kind"], case["n"])
        assert snappy_oracle.decode(comp) == data


def _compress(data: bytes) -> bytes:
    L = _lib.lib()
    cap = L.qgcm_snappy_max_compressed_length(len(data))
    dst = C.create_string_buffer(cap)
    n = L.qgcm_snappy_compress(data or None, len(data), dst, cap)
    assert n > 0
    return dst.raw[:n]


def _uncompress(comp: bytes, cap: int):
    dst = C.create_string_buffer(max(cap, 1))
    n = _lib.lib().qgcm_snappy_uncompress(comp, len(comp), dst, cap)
    return None if n < 0 else dst.raw[:n]


def _corpus():
    rng = random.Random(5)
    out = [b"", b"a", b"ab", bytes(3), bytes(4), bytes(17), os.urandom(16), os.urandom(1350), os.urandom(9000),
           bytes(70000), os.urandom(70000), b"abc" * 30000]
    words = [b"GET ", b"/index.html", b" HTTP/1.1\r\n", b"Host: 10.99.0.1\r\n", b"\x00\x00", b"quantum "]
    for _ in range(40):
        n = rng.choice([5, 60, 61, 64, 65, 67, 68, 69, 128, 1350, 1433, 4096, 65536, 65537])
        s = bytearray()
        while len(s) < n:
            r = rng.random()
            if r < 0.4:
                s += rng.choice(words)
            elif r < 0.7 and s:
                a = rng.randrange(len(s))
                s += s[a:a + rng.randrange(1, 80)]
            else:
                s += bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 40)))
        out.append(bytes(s[:n]))
    return out


def test_roundtrip_and_bound():
    for data in _corpus():
        comp = _compress(data)
        assert len(comp) <= _lib.lib().qgcm_snappy_max_compressed_length(len(data))
        assert _lib.lib().qgcm_snappy_uncompressed_length(comp, len(comp)) == len(data)
        assert _uncompress(comp, len(data)) == data
    assert len(_compress(bytes(9000))) < 600  # runs compress
    assert len(_compress(b"quantum " * 200)) < 100


def _libsnappy():
    for path in ("/opt/conda/lib/libsnappy.so.1", "/opt/conda/lib/libsnappy.so"):
        if os.path.exists(path):
            lib = C.CDLL(path)
            lib.snappy_uncompress.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.POINTER(C.c_size_t)]
            lib.snappy_compress.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.POINTER(C.c_size_t)]
            lib.snappy_max_compressed_length.argtypes = [C.c_size_t]
            lib.snappy_max_compressed_length.restype = C.c_size_t
            return lib
    return None


def test_cross_decode_with_libsnappy():
    lib = _libsnappy()
    if lib is None:
        pytest.skip("libsnappy not present")
    for data in _corpus():
        comp = _compress(data)
        out = C.create_string_buffer(max(len(data), 1))
        n = C.c_size_t(len(data))
        assert lib.snappy_uncompress(comp, len(comp), out, C.byref(n)) == 0 and out.raw[:n.value] == data
        cap = lib.snappy_max_compressed_length(len(data))
        cbuf = C.create_string_buffer(cap)
        m = C.c_size_t(cap)
        assert lib.snappy_compress(data, len(data), cbuf, C.byref(m)) == 0
        assert _uncompress(cbuf.raw[:m.value], len(data)) == data  # decode-compatible with Google's encoder
        assert cbuf.raw[:m.value] == comp  # and the same bytes (the corpus here is not in the golden file)


def test_cross_decode_with_pyarrow():
    pa = pytest.importorskip("pyarrow")
    codec = pa.Codec("snappy")
    for data in _corpus():
        if not data:
            continue
        comp = _compress(data)
        assert codec.decompress(comp, decompressed_size=len(data)).to_pybytes() == data
        theirs = codec.compress(data).to_pybytes()
        assert _uncompress(theirs, len(data)) == data


def test_malformed_inputs_rejected():
    good = _compress(b"hello hello hello hello hello" * 10)
    n = len(b"hello hello hello hello hello" * 10)
    bad = [b"", b"\xff\xff\xff\xff\xff\xff", good[:-3], good[:1] + b"\x00" + good[2:], b"\x05\x02\xff",
           b"\x04\x0d\x01",  # copy with offset 1 before any output
           b"\x03\x08abc",  # literal longer than the input
           b"\x10\x0cabcd\x01\x00"]  # copy-1 with offset 0
    for b in bad:
        assert _uncompress(b, max(n, 64)) is None or len(_uncompress(b, max(n, 64))) == \
            _lib.lib().qgcm_snappy_uncompressed_length(b, len(b))
    assert _uncompress(good, n - 1) is None  # would not fit
    rng = random.Random(9)
    for _ in range(2000):  # random corruption never crashes and never overruns the output
        b = bytearray(good)
        for _ in range(rng.randrange(1, 4)):
            b[rng.randrange(len(b))] = rng.getrandbits(8)
        out = _uncompress(bytes(b), 4096)
        assert out is None or len(out) == _lib.lib().qgcm_snappy_uncompressed_length(bytes(b), len(b))


def test_slots_batch_threads():
    rng = random.Random(3)
    n, stride = 1000, 1472
    arena = bytearray(n * stride)
    lens = (C.c_uint32 * n)()
    plain = []
    for i in range(n):
        L = rng.randrange(0, 1434)
        data = (b"abcdefgh" * 200)[:L] if i % 3 else os.urandom(L)
        arena[i * stride + 4:i * stride + 4 + L] = data
        lens[i] = L
        plain.append(data)
    buf = (C.c_uint8 * len(arena)).from_buffer(arena)
    assert _lib.lib().qgcm_snappy_compress_slots(C.addressof(buf), stride, n, lens, 4) == 0
    for i in range(0, n, 97):
        comp = bytes(arena[i * stride + 4:i * stride + 4 + lens[i]])
        assert _uncompress(comp, 1433) == plain[i]
    st = (C.c_uint8 * n)()
    empty = sum(1 for p in plain if not p)  # decode to nothing: dropped (compression.go:37-39)
    assert _lib.lib().qgcm_snappy_uncompress_slots(C.addressof(buf), stride, n, lens, st, 4) == empty
    for i in range(n):
        if not plain[i]:
            assert st[i] == 0 and lens[i] == 1
            continue
        assert st[i] == 1 and lens[i] == len(plain[i])
        assert bytes(arena[i * stride + 4:i * stride + 4 + lens[i]]) == plain[i]
    del buf


def test_compression_plugin_roundtrip():
    """plugin/plugin_test.go:126-161 TestCompression."""
    comp, err = plugin.New(plugin.CompressionPlugin)
    assert err is None and comp.Name() == "compression" and comp.Order() == 0
    mapping = common.Mapping(SupportedPlugins=["compression", "encryption"], AES=None)
    buf = bytearray(os.urandom(common.MaxPacketLength))
    expected = bytes(buf)
    out = common.NewTunPayload(buf, common.MTU)
    compressed, _, ok = comp.Apply(plugin.Outgoing, out, mapping)
    assert ok
    inc = common.NewSockPayload(compressed.Raw, compressed.Length)
    _, _, ok = comp.Apply(plugin.Incoming, inc, mapping)
    assert ok and bytes(buf[:common.MTU]) == expected[:common.MTU]
    # a packet that does not decode is dropped; a peer without the plugin passes through
    bad = common.NewSockPayload(bytearray(b"\x00\x00\x00\x00\xff\xff\xff\xff\xff\xff" + bytes(20)), 30)
    _, _, ok = comp.Apply(plugin.Incoming, bad, mapping)
    assert not ok
    m2 = common.Mapping(SupportedPlugins=["encryption"], AES=None)
    p = common.NewTunPayload(bytearray(64), 40)
    assert comp.Apply(plugin.Outgoing, p, m2)[2] and p.Length == 44


def test_empty_result_is_dropped_by_the_plugin():
    """golang/snappy's Decode(nil, src) returns a nil slice when the stream decodes to 0 bytes, and
    plugin/compression.go:37-39 drops a nil packet: the empty stream b"\\x00" (what Encode gives for an
    empty packet) decodes at codec level (0 bytes) but fails at plugin level -- Apply, the slot batch
    and (GPU test) the device batch.  golang/snappy is not in the reference: parity unpinned, the
    behaviour restated from its published decode.go."""
    assert snappy_oracle.decode(b"\x00") == b""
    assert snappy_oracle.encode(b"") == b"\x00" and _compress(b"") == b"\x00"
    assert _uncompress(b"\x00", 16) == b""  # codec level: a valid, empty stream
    comp, _ = plugin.New(plugin.CompressionPlugin)
    mapping = common.Mapping(SupportedPlugins=["compression"], AES=None)
    raw = bytearray(b"\x0a\x63\x00\x01\x00" + bytes(40))
    p = common.NewSockPayload(raw, 5)
    _, _, ok = comp.Apply(plugin.Incoming, p, mapping)
    assert not ok and p.Length == 5
    stride, n = 64, 3
    arena = bytearray(stride * n)
    streams = [b"\x00", _compress(b"abc"), b"\x00"]
    lens = (C.c_uint32 * n)()
    for i, s in enumerate(streams):
        arena[i * stride + 4:i * stride + 4 + len(s)] = s
        lens[i] = len(s)
    before = bytes(arena)
    buf = (C.c_uint8 * len(arena)).from_buffer(arena)
    st = (C.c_uint8 * n)()
    assert _lib.lib().qgcm_snappy_uncompress_slots(C.addressof(buf), stride, n, lens, st, 2) == 2
    assert list(st) == [0, 1, 0] and list(lens) == [1, 3, 1]
    assert arena[:stride] == before[:stride] and arena[2 * stride:] == before[2 * stride:]
    assert bytes(arena[stride + 4:stride + 7]) == b"abc"
    del buf
