"""GPU: the device snappy codec (qgcm_snappy_compress_batch / qgcm_snappy_uncompress_batch,
snappy_kernels.hip) behind plugin/compression.go:16-51.

Bar: byte-exact.  The device encoder's output equals libsnappy 1.1.8's bytes on the golden corpus
(tests/golden/snappy.json, every case up to the device's 16 KiB limit) and the host encoder's on a
config-5-shaped batch (whole arena and lengths); the decoder restores every packet, agrees with the
host decoder on corrupted streams (which packets fail, and the bytes of those that do not), and a
failing packet's slot and length are untouched."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import snappy_inputs as SI

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "snappy.json")
DEV_MAX = 16384


@pytest.fixture(scope="module")
def torch():
    import torch as T

    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


def _lib():
    from quantum_amd import _lib as L

    return L.lib()


def _host_compress(data: bytes) -> bytes:
    L = _lib()
    cap = L.qgcm_snappy_max_compressed_length(len(data))
    dst = C.create_string_buffer(max(cap, 1))
    n = L.qgcm_snappy_compress(data or None, len(data), dst, cap)
    assert n > 0
    return dst.raw[:n]


def _host_uncompress(comp: bytes, cap: int):
    dst = C.create_string_buffer(max(cap, 1))
    n = _lib().qgcm_snappy_uncompress(comp, len(comp), dst, cap)
    return None if n < 0 else dst.raw[:n]


def _arena(torch, payloads, stride, fill=0xA5):
    n = len(payloads)
    host = np.full((n, stride), fill, dtype=np.uint8)
    for i, p in enumerate(payloads):
        host[i, 4:4 + len(p)] = np.frombuffer(p, np.uint8)
    lens = np.array([len(p) for p in payloads], dtype=np.uint32)
    return host, torch.from_numpy(host.reshape(-1).copy()).cuda(), torch.from_numpy(lens.view(np.int32).copy()).cuda()


def _run(torch, ctx, compress, arena, stride, n, lens, max_len, limit):
    from quantum_amd import batch

    status = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    fn = batch.snappy_compress if compress else batch.snappy_uncompress
    fn(ctx, arena, stride, n, lens, max_len, limit, status)
    torch.cuda.synchronize()
    return (arena.cpu().numpy().reshape(n, stride), lens.cpu().numpy().view(np.uint32).copy(),
            status.cpu().numpy())


def _match(case, comp: bytes) -> bool:
    if len(comp) != case["out_len"]:
        return False
    if "out_hex" in case:
        return comp.hex() == case["out_hex"]
    return hashlib.sha256(comp).hexdigest() == case["out_sha256"]


@pytest.fixture(scope="module")
def encoder_ctxs(torch):
    """One context per QGCM_SNAPPY_GROUP setting (read at qgcm_create)."""
    from quantum_amd.crypto import Context

    out, old = {}, os.environ.get("QGCM_SNAPPY_GROUP")
    try:
        for g in ("1", "0"):
            os.environ["QGCM_SNAPPY_GROUP"] = g
            out[g] = Context(device=0, max_keys=16)
    finally:
        if old is None:
            os.environ.pop("QGCM_SNAPPY_GROUP", None)
        else:
            os.environ["QGCM_SNAPPY_GROUP"] = old
    yield out
    for c in out.values():
        c.close()


@pytest.fixture(params=["1", "0"], ids=["group_codec", "wave_codec"])
def encoder(request, encoder_ctxs):
    """QGCM_SNAPPY_GROUP (at qgcm_create): 1 = four packets per wave for both directions (the encoder's
    pipelined miss probes and output straight into the slot, the decoder's header window and
    branch-free copies, the next packets prefetched; the default); 0 = one wave per packet.  Both must
    give the host codec's (and libsnappy's) bytes, and leave a failing packet's slot untouched.  The
    value is the context built with that setting."""
    return encoder_ctxs[request.param]


def test_device_encoder_equals_libsnappy_golden(torch, encoder):
    ctx = encoder
    with open(GOLDEN) as f:
        cases = [c for c in json.load(f)["cases"] if c["n"] <= DEV_MAX]
    datas = [SI.make(c["kind"], c["n"]) for c in cases]
    stride = (4 + max(_lib().qgcm_snappy_max_compressed_length(len(d)) for d in datas) + 3) // 4 * 4
    host, arena, lens = _arena(torch, datas, stride)
    out, ol, st = _run(torch, ctx, True, arena, stride, len(datas), lens, DEV_MAX, stride - 4)
    assert (st == 1).all()
    for i, (c, d) in enumerate(zip(cases, datas)):
        comp = out[i, 4:4 + ol[i]].tobytes()
        assert _match(c, comp), (c["kind"], c["n"])
        assert (out[i, 4 + ol[i]:] == host[i, 4 + ol[i]:]).all()  # past the output: untouched
        assert (out[i, :4] == host[i, :4]).all()
    # and back: the device decoder restores every case
    arena2 = torch.from_numpy(out.reshape(-1).copy()).cuda()
    lens2 = torch.from_numpy(ol.view(np.int32).copy()).cuda()
    in_max = _lib().qgcm_snappy_max_compressed_length(DEV_MAX)  # the decoder's input limit
    back, bl, st2 = _run(torch, ctx, False, arena2, stride, len(datas), lens2, in_max, DEV_MAX)
    for i, d in enumerate(datas):
        if not d:  # b"\x00" decodes to nothing: dropped, as compression.go:37-39 drops Go's nil slice
            assert st2[i] == 0 and bl[i] == 1 and np.array_equal(back[i], out[i])
            continue
        assert st2[i] == 1 and bl[i] == len(d) and back[i, 4:4 + len(d)].tobytes() == d


def test_device_codec_config5_batch_vs_host(torch, encoder):
    """2^14 Payload.Raw slots (stride 1472): config 5's packet shape and a mix of lengths 0..1433
    and contents; device compress == host encoder (whole arena incl. untouched bytes, lengths), then
    device uncompress restores the plaintext arena."""
    ctx = encoder
    n, stride = 1 << 14, 1472
    rng = np.random.default_rng(0x5EED0051)
    kinds = SI.KINDS
    payloads = []
    for i in range(n):
        L = 1350 if i % 2 == 0 else int(rng.integers(0, 1434))
        payloads.append(SI.make(kinds[i % len(kinds)], L, seed=i))
    host, arena, lens = _arena(torch, payloads, stride)
    limit = stride - 4 - 28  # room for the tag and nonce (run_host_chain's max_plain)
    out, ol, st = _run(torch, ctx, True, arena, stride, n, lens, stride - 4, limit)
    # host reference: compress each slot in place with the host encoder
    ref = host.copy()
    for i, p in enumerate(payloads):
        c = _host_compress(p)
        assert len(c) <= limit
        ref[i, 4:4 + len(c)] = np.frombuffer(c, np.uint8)
        assert ol[i] == len(c), i
    assert (st == 1).all()
    assert np.array_equal(out, ref)
    back, bl, st2 = _run(torch, ctx, False, torch.from_numpy(out.reshape(-1).copy()).cuda(), stride, n,
                         torch.from_numpy(ol.view(np.int32).copy()).cuda(), stride - 4, stride - 4)
    # an empty packet's stream b"\x00" decodes to nothing: dropped (compression.go:37-39), untouched
    want_st = np.array([1 if p else 0 for p in payloads], np.uint8)
    assert np.array_equal(st2, want_st)
    assert np.array_equal(bl, np.array([len(p) if p else 1 for p in payloads], np.uint32))
    plain = host.copy()
    for i, p in enumerate(payloads):  # bytes past the plaintext keep the compressed stream's bytes
        plain[i, 4 + len(p):] = out[i, 4 + len(p):]
    assert np.array_equal(back, plain)


def test_device_compress_failures_untouched(torch, encoder):
    """Longer than max_len, or compressed form over limit: status 0, slot and length untouched."""
    ctx = encoder
    stride = 2048
    payloads = [SI.make("random", 1500), SI.make("line", 1500), SI.make("random", 900), b"", SI.make("zeros", 40)]
    host, arena, lens = _arena(torch, payloads, stride)
    out, ol, st = _run(torch, ctx, True, arena, stride, len(payloads), lens, 1400, 1000)
    assert list(st) == [0, 0, 1, 1, 1]  # 1500 > max_len; ...; 900 random -> 906 <= 1000
    for i in (0, 1):
        assert np.array_equal(out[i], host[i]) and ol[i] == 1500
    for i in (2, 3, 4):
        c = _host_compress(payloads[i])
        assert ol[i] == len(c) and out[i, 4:4 + len(c)].tobytes() == c
    host, arena, lens = _arena(torch, payloads, stride)
    out, ol, st = _run(torch, ctx, True, arena, stride, len(payloads), lens, 2000, 800)
    assert list(st) == [0, 1, 0, 1, 1]  # random 1500 / 900 do not fit 800; the line does
    for i in (0, 2):  # encoded past the limit (the direct encoder wrote into the slot): restored whole
        assert np.array_equal(out[i], host[i]) and ol[i] == len(payloads[i])
    for i in (1, 3, 4):
        c = _host_compress(payloads[i])
        assert ol[i] == len(c) and out[i, 4:4 + len(c)].tobytes() == c
        assert np.array_equal(out[i, 4 + len(c):], host[i, 4 + len(c):])  # past the output: untouched


def test_device_uncompress_corrupted_streams_vs_host(torch, encoder):
    ctx = encoder
    """Random corruption of valid streams (and truncations, bad varints, offsets before the output):
    the device decoder fails exactly where the host decoder does, and otherwise writes its bytes."""
    rng = np.random.default_rng(0x5EED0052)
    goods = [_host_compress(SI.make(k, L, seed=j)) for j, (k, L) in
             enumerate([("words", 1350), ("half", 1350), ("runs", 700), ("line", 300), ("words", 4096)])]
    streams = [b"", b"\xff\xff\xff\xff\xff\xff", b"\x05\x02\xff", b"\x04\x0d\x01", b"\x03\x08abc",
               b"\x10\x0cabcd\x01\x00", b"\x80\x80\x80\x80\x10", b"\x04\xf0\xff\xff\xff\xffabcd"]
    for _ in range(3000):
        g = bytearray(goods[int(rng.integers(0, len(goods)))])
        r = rng.random()
        if r < 0.2:
            g = g[:int(rng.integers(0, len(g)))]
        else:
            for _ in range(int(rng.integers(1, 4))):
                g[int(rng.integers(0, len(g)))] = int(rng.integers(0, 256))
        streams.append(bytes(g))
    streams += goods
    cap = 4200
    stride = (4 + max(max(len(s) for s in streams), cap) + 3) // 4 * 4
    host, arena, lens = _arena(torch, streams, stride)
    out, ol, st = _run(torch, ctx, False, arena, stride, len(streams), lens, stride - 4, cap)
    for i, s in enumerate(streams):
        want = _host_uncompress(s, cap)
        if want is None or len(want) == 0:  # an empty result is Go's nil slice: dropped (compression.go:37-39)
            assert st[i] == 0 and ol[i] == len(s) and np.array_equal(out[i], host[i]), i
        else:
            assert st[i] == 1 and ol[i] == len(want) and out[i, 4:4 + len(want)].tobytes() == want, i
    assert st[-len(goods):].all()


def test_device_uncompress_empty_result_fails(torch, encoder):
    ctx = encoder
    """b"\\x00" decodes to 0 bytes: golang/snappy's Decode returns a nil slice and compression.go:37-39
    drops the packet, so the device batch fails it (slot and length untouched), as the host slots do."""
    streams = [b"\x00", _host_compress(b"abcabcabc"), b"\x00"]
    stride = 64
    host, arena, lens = _arena(torch, streams, stride)
    out, ol, st = _run(torch, ctx, False, arena, stride, len(streams), lens, stride - 4, stride - 4)
    assert list(st) == [0, 1, 0] and list(ol) == [1, 9, 1]
    assert np.array_equal(out[0], host[0]) and np.array_equal(out[2], host[2])
    assert out[1, 4:13].tobytes() == b"abcabcabc"


def test_device_codec_fuzz_vs_host(torch, encoder):
    """2^15 Payload.Raw slots of random shapes -- the corpus kinds plus two- and four-letter alphabets
    (hash collisions between consecutive probes, long back-references at short offsets) -- and lengths
    0..1433: device compress equals the host encoder (bytes, lengths, untouched tails); then a third
    of the streams get 1-3 random byte flips or a truncation, and the device decoder must agree with
    the host decoder on every stream (status, length, bytes)."""
    ctx = encoder
    n, stride = 1 << 15, 1472
    rng = np.random.default_rng(0x5EED0071)
    kinds = SI.KINDS + ["ab", "acgt"]
    payloads = []
    for i in range(n):
        k = kinds[int(rng.integers(0, len(kinds)))]
        L = int(rng.integers(0, 1434))
        if k == "ab":
            payloads.append(bytes(rng.choice(np.frombuffer(b"ab", np.uint8), L)))
        elif k == "acgt":
            payloads.append(bytes(rng.choice(np.frombuffer(b"acgt", np.uint8), L)))
        else:
            payloads.append(SI.make(k, L, seed=i))
    host, arena, lens = _arena(torch, payloads, stride)
    limit = stride - 4 - 28
    out, ol, st = _run(torch, ctx, True, arena, stride, n, lens, stride - 4, limit)
    comps = [_host_compress(p) for p in payloads]
    assert (st == 1).all()
    assert np.array_equal(ol, np.array([len(c) for c in comps], np.uint32))
    ref = host.copy()
    for i, c in enumerate(comps):
        ref[i, 4:4 + len(c)] = np.frombuffer(c, np.uint8)
    assert np.array_equal(out, ref)
    # corrupt a third of the streams in place, then decode on both sides
    streams = []
    for i, c in enumerate(comps):
        b = bytearray(c)
        if i % 3 == 0 and b:
            if rng.random() < 0.25:
                b = b[:int(rng.integers(0, len(b)))]
            else:
                for _ in range(int(rng.integers(1, 4))):
                    b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
        streams.append(bytes(b))
    host2, arena2, lens2 = _arena(torch, streams, stride)
    back, bl, st2 = _run(torch, ctx, False, arena2, stride, n, lens2, stride - 4, stride - 4)
    for i, s in enumerate(streams):
        want = _host_uncompress(s, stride - 4)
        if want is None or len(want) == 0:
            assert st2[i] == 0 and bl[i] == len(s) and np.array_equal(back[i], host2[i]), i
        else:
            assert st2[i] == 1 and bl[i] == len(want) and back[i, 4:4 + len(want)].tobytes() == want, i
