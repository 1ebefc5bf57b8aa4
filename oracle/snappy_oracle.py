"""TEST INFRASTRUCTURE ONLY (the checker, never the product path): a pure-Python restatement of the
snappy block codec that plugin/compression.go:16-27 calls (snappy.Encode(nil, raw) /
snappy.Decode(nil, raw)).

github.com/golang/snappy is not under /root/reference: quantum fetches it unpinned with `go get -u`
(Makefile:52-54), so there is no version to pin beyond "the block encoder golang/snappy has shipped
since 2016" (encode.go Encode, encode_other.go encodeBlock / emitLiteral / emitCopy; the amd64
assembly produces the same bytes).  That algorithm is also Google's C++ snappy CompressFragment, and
libsnappy 1.1.8 is in this image: tests/golden/make_snappy_golden.py records its output bytes as
fixtures, and tests/test_snappy.py checks this restatement, libqgcm's host encoder and (on the GPU)
the device encoder against them.  Pure-Python loops: small inputs only.
"""

_MUL = 0x1E35A7BD
_INPUT_MARGIN = 16 - 1                   # encode.go inputMargin
_MIN_BLOCK = 1 + 1 + _INPUT_MARGIN       # encode.go minNonLiteralBlockSize
_MAX_BLOCK = 65536                       # encode.go maxBlockSize


def _load32(b, i):
    return b[i] | b[i + 1] << 8 | b[i + 2] << 16 | b[i + 3] << 24


def _hash(u, shift):
    return ((u * _MUL) & 0xFFFFFFFF) >> shift


def _uvarint(n):
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def emit_literal(lit):
    """encode_other.go emitLiteral: tag 00, length-1 in the tag (< 60) or in 1-2 following bytes."""
    n = len(lit) - 1
    if n < 60:
        head = bytes([n << 2])
    elif n < 256:
        head = bytes([60 << 2, n])
    else:
        head = bytes([61 << 2, n & 0xFF, n >> 8])
    return head + bytes(lit)


def emit_copy(offset, length):
    """encode_other.go emitCopy: 64-byte copy-2 pieces while >= 68 remain, a 60 piece for 65-67,
    then copy-1 (len 4..11, offset < 2048) or copy-2."""
    out = bytearray()
    while length >= 68:
        out += bytes([63 << 2 | 2, offset & 0xFF, offset >> 8])
        length -= 64
    if length > 64:
        out += bytes([59 << 2 | 2, offset & 0xFF, offset >> 8])
        length -= 60
    if length >= 12 or offset >= 2048:
        out += bytes([(length - 1) << 2 | 2, offset & 0xFF, offset >> 8])
    else:
        out += bytes([(offset >> 8) << 5 | (length - 4) << 2 | 1, offset & 0xFF])
    return bytes(out)


def encode_block(src):
    """encode_other.go encodeBlock for one block of _MIN_BLOCK.._MAX_BLOCK bytes."""
    n = len(src)
    shift, ts = 24, 256
    while ts < (1 << 14) and ts < n:
        ts <<= 1
        shift -= 1
    table = [0] * (1 << 14)
    s_limit = n - _INPUT_MARGIN
    out = bytearray()
    next_emit, s = 0, 1
    next_hash = _hash(_load32(src, s), shift)
    while True:
        skip, next_s = 32, s
        while True:
            s = next_s
            step = skip >> 5
            next_s = s + step
            skip += step
            if next_s > s_limit:
                if next_emit < n:
                    out += emit_literal(src[next_emit:])
                return bytes(out)
            cand = table[next_hash]
            table[next_hash] = s
            next_hash = _hash(_load32(src, next_s), shift)
            if _load32(src, s) == _load32(src, cand):
                break
        out += emit_literal(src[next_emit:s])
        while True:
            base = s
            s += 4
            i = cand + 4
            while s < n and src[i] == src[s]:
                i += 1
                s += 1
            out += emit_copy(base - cand, s - base)
            next_emit = s
            if s >= s_limit:
                if next_emit < n:
                    out += emit_literal(src[next_emit:])
                return bytes(out)
            table[_hash(_load32(src, s - 1), shift)] = s - 1
            cur = _load32(src, s)
            h = _hash(cur, shift)
            cand = table[h]
            table[h] = s
            if cur != _load32(src, cand):
                next_hash = _hash(_load32(src, s + 1), shift)
                s += 1
                break


def encode(src):
    """encode.go Encode: uvarint length, then 64-KiB blocks (short ones as one literal)."""
    src = bytes(src)
    out = bytearray(_uvarint(len(src)))
    for base in range(0, len(src), _MAX_BLOCK):
        p = src[base:base + _MAX_BLOCK]
        out += emit_literal(p) if len(p) < _MIN_BLOCK else encode_block(p)
    return bytes(out)


def decode(src):
    """decode.go Decode: None for a malformed stream (the plugin then drops the packet,
    plugin/compression.go:22-25)."""
    src = bytes(src)
    total, shift, i = 0, 0, 0
    while True:
        if i >= len(src) or i >= 5:
            return None
        c = src[i]
        total |= (c & 0x7F) << shift
        i += 1
        if c < 0x80:
            break
        shift += 7
    if total > 0xFFFFFFFF:
        return None
    out = bytearray()
    while i < len(src):
        tag = src[i]
        i += 1
        kind = tag & 3
        if kind == 0:
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                if i + nb > len(src):
                    return None
                ln = int.from_bytes(src[i:i + nb], "little")
                i += nb
            ln += 1
            if ln > len(src) - i or len(out) + ln > total:
                return None
            out += src[i:i + ln]
            i += ln
            continue
        if kind == 1:
            if i + 1 > len(src):
                return None
            ln, off = 4 + ((tag >> 2) & 7), (tag >> 5) << 8 | src[i]
            i += 1
        elif kind == 2:
            if i + 2 > len(src):
                return None
            ln, off = 1 + (tag >> 2), src[i] | src[i + 1] << 8
            i += 2
        else:
            if i + 4 > len(src):
                return None
            ln, off = 1 + (tag >> 2), int.from_bytes(src[i:i + 4], "little")
            i += 4
        if off == 0 or off > len(out) or len(out) + ln > total:
            return None
        for _ in range(ln):
            out.append(out[-off])
    return bytes(out) if len(out) == total else None
