// snappy_codec.cpp -- the snappy block format for the compression plugin (plugin/compression.go).
//
// quantum compresses a packet with github.com/golang/snappy Encode before sealing it and
// decompresses with Decode after opening it (plugin/compression.go:16-27,35-51; chain order
// main.go:50-51).  That library is not in /root/reference (unpinned GOPATH dependency), so this is a
// from-scratch implementation of the published block format:
//
//   preamble: uncompressed length, little-endian base-128 varint
//   elements, tag byte low 2 bits:
//     00 literal   len-1 in tag bits 2..7 if < 60, else 60..63 = 1..4 following LE length bytes
//     01 copy      len 4..11 = 4 + tag bits 2..4, offset 11 bits = tag bits 5..7 : next byte
//     10 copy      len 1..64 = 1 + tag bits 2..7, offset = next 2 bytes LE
//     11 copy      len 1..64 = 1 + tag bits 2..7, offset = next 4 bytes LE
//   a copy repeats `len` bytes starting `offset` back in the output (may overlap: RLE).
//
// The encoder restates golang/snappy's block encoder (encode.go Encode + encode_other.go
// encodeBlock / emitLiteral / emitCopy, the algorithm the package has used since 2016 -- unpinned in
// the reference's GOPATH build, Makefile:52-54 -- and the one Google's C++ snappy CompressFragment
// uses): a 2^8..2^14-entry table of uint16 positions hashed by (u32 * 0x1e35a7bd) >> shift, probes
// every (skip >> 5) bytes with skip += (skip >> 5) after each miss, no probe within 15 bytes of the
// block end (inputMargin), after each copy the positions s-1 and s re-hashed and s tried at once,
// copies split into 64-byte pieces keeping >= 4 for the last, blocks of 64 KiB, inputs shorter than
// 17 bytes one literal.  Output bytes are checked equal to libsnappy 1.1.8's on a corpus
// (tests/test_snappy.py); the device encoder (snappy_kernels.hip) is checked equal to this one.  The
// decoder accepts every valid stream and rejects malformed ones without reading or writing out of
// bounds.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/qgcm.h"

namespace {

inline uint32_t load32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

inline uint32_t hash4(uint32_t v, int shift) { return (v * 0x1e35a7bdu) >> shift; }

uint8_t *emit_literal(uint8_t *op, const uint8_t *lit, size_t len) {
    const size_t n = len - 1;
    if (n < 60) {
        *op++ = (uint8_t)(n << 2);
    } else {
        int bytes = 0;
        for (size_t t = n; t; t >>= 8) ++bytes;
        *op++ = (uint8_t)((59 + bytes) << 2);
        for (int i = 0; i < bytes; ++i) *op++ = (uint8_t)(n >> (8 * i));
    }
    memcpy(op, lit, len);
    return op + len;
}

uint8_t *emit_copy_upto64(uint8_t *op, size_t offset, size_t len) {
    if (len >= 4 && len < 12 && offset < 2048) {
        *op++ = (uint8_t)(1 | ((len - 4) << 2) | ((offset >> 8) << 5));
        *op++ = (uint8_t)offset;
    } else {
        *op++ = (uint8_t)(2 | ((len - 1) << 2));
        *op++ = (uint8_t)offset;
        *op++ = (uint8_t)(offset >> 8);
    }
    return op;
}

uint8_t *emit_copy(uint8_t *op, size_t offset, size_t len) {
    while (len >= 68) {  // keep the remainder >= 4 so the 1-byte-offset form stays usable
        op = emit_copy_upto64(op, offset, 64);
        len -= 64;
    }
    if (len > 64) {
        op = emit_copy_upto64(op, offset, 60);
        len -= 60;
    }
    return emit_copy_upto64(op, offset, len);
}

constexpr size_t kInputMargin = 15;               // encode.go inputMargin (16 - 1)
constexpr size_t kMinBlock = 1 + 1 + kInputMargin;  // encode.go minNonLiteralBlockSize

// Length of the common prefix of a[0..) and b[0..), b ending at end (8 bytes at a time, the first
// differing byte from the XOR's trailing zeros; encode_other.go compares bytewise, same result).
inline size_t match_len(const uint8_t *a, const uint8_t *b, const uint8_t *end) {
    size_t m = 0;
    while (b + m + 8 <= end) {
        uint64_t x, y;
        memcpy(&x, a + m, 8);
        memcpy(&y, b + m, 8);
        if (x != y) return m + ((size_t)__builtin_ctzll(x ^ y) >> 3);
        m += 8;
    }
    while (b + m < end && a[m] == b[m]) ++m;
    return m;
}

// encode_other.go encodeBlock: one block of kMinBlock..65536 bytes.
uint8_t *encode_block(uint8_t *op, const uint8_t *src, size_t len) {
    int shift = 24;  // table of 2^8 .. 2^14 entries, the smallest >= len
    for (size_t ts = 256; ts < (1u << 14) && ts < len; ts <<= 1) --shift;
    uint16_t table[1 << 14];
    memset(table, 0, sizeof(uint16_t) << (32 - shift));
    const size_t s_limit = len - kInputMargin;
    size_t next_emit = 0, s = 1;
    uint32_t next_hash = hash4(load32(src + s), shift);
    for (;;) {
        size_t skip = 32, next_s = s, cand = 0;
        for (;;) {  // probe every (skip >> 5) bytes until a 4-byte match
            s = next_s;
            const size_t step = skip >> 5;
            next_s = s + step;
            skip += step;
            if (next_s > s_limit) goto remainder;
            cand = table[next_hash];
            table[next_hash] = (uint16_t)s;
            next_hash = hash4(load32(src + next_s), shift);
            if (load32(src + s) == load32(src + cand)) break;
        }
        op = emit_literal(op, src + next_emit, s - next_emit);
        for (;;) {  // copies back to back while the position after one starts another
            const size_t base = s;
            s += 4 + match_len(src + cand + 4, src + s + 4, src + len);
            op = emit_copy(op, base - cand, s - base);
            next_emit = s;
            if (s >= s_limit) goto remainder;
            uint64_t x;
            memcpy(&x, src + s - 1, 8);
            table[hash4((uint32_t)x, shift)] = (uint16_t)(s - 1);
            const uint32_t h = hash4((uint32_t)(x >> 8), shift);
            cand = table[h];
            table[h] = (uint16_t)s;
            if ((uint32_t)(x >> 8) != load32(src + cand)) {
                next_hash = hash4((uint32_t)(x >> 16), shift);
                ++s;
                break;
            }
        }
    }
remainder:
    if (next_emit < len) op = emit_literal(op, src + next_emit, len - next_emit);
    return op;
}

}  // namespace

extern "C" {

size_t qgcm_snappy_max_compressed_length(size_t n) { return 32 + n + n / 6; }

long qgcm_snappy_compress(const uint8_t *src, size_t n, uint8_t *dst, size_t cap) {
    if ((!src && n) || !dst || n > 0xffffffffu || cap < qgcm_snappy_max_compressed_length(n)) return -1;
    uint8_t *op = dst;
    for (size_t v = n;; v >>= 7) {  // preamble
        if (v < 0x80) {
            *op++ = (uint8_t)v;
            break;
        }
        *op++ = (uint8_t)(v | 0x80);
    }
    // blocks of at most 64 KiB, as the format's 2-byte offsets expect (encode.go Encode)
    for (size_t base = 0; base < n; base += 65536) {
        const size_t len = std::min<size_t>(65536, n - base);
        op = len < kMinBlock ? emit_literal(op, src + base, len) : encode_block(op, src + base, len);
    }
    return (long)(op - dst);
}

long qgcm_snappy_uncompressed_length(const uint8_t *src, size_t n) {
    uint64_t v = 0;
    for (size_t i = 0; i < n && i < 5; ++i) {
        v |= (uint64_t)(src[i] & 0x7f) << (7 * i);
        if (!(src[i] & 0x80)) return v > 0xffffffffu ? -1 : (long)v;
    }
    return -1;
}

long qgcm_snappy_uncompress(const uint8_t *src, size_t n, uint8_t *dst, size_t cap) {
    if (!src || (!dst && cap)) return -1;
    const long total = qgcm_snappy_uncompressed_length(src, n);
    if (total < 0 || (size_t)total > cap) return -1;
    size_t ip = 0;
    while (ip < n && (src[ip] & 0x80)) ++ip;
    ++ip;
    size_t op = 0;
    while (ip < n) {
        const uint8_t tag = src[ip++];
        size_t len, off;
        switch (tag & 3) {
            case 0: {
                len = tag >> 2;
                if (len >= 60) {
                    const size_t b = len - 59;
                    if (ip + b > n) return -1;
                    len = 0;
                    for (size_t i = 0; i < b; ++i) len |= (size_t)src[ip + i] << (8 * i);
                    ip += b;
                }
                ++len;
                if (len > n - ip || len > (size_t)total - op) return -1;
                memcpy(dst + op, src + ip, len);
                ip += len;
                op += len;
                continue;
            }
            case 1:
                if (ip + 1 > n) return -1;
                len = 4 + ((tag >> 2) & 7);
                off = ((size_t)(tag >> 5) << 8) | src[ip];
                ip += 1;
                break;
            case 2:
                if (ip + 2 > n) return -1;
                len = 1 + (tag >> 2);
                off = src[ip] | ((size_t)src[ip + 1] << 8);
                ip += 2;
                break;
            default:
                if (ip + 4 > n) return -1;
                len = 1 + (tag >> 2);
                off = load32(src + ip);
                ip += 4;
                break;
        }
        if (off == 0 || off > op || len > (size_t)total - op) return -1;
        size_t i = 0;
        if (off >= 8)  // 8 bytes at a time: a step never reads what it writes
            for (; i + 8 <= len; i += 8) memcpy(dst + op + i, dst + op + i - off, 8);
        for (; i < len; ++i) dst[op + i] = dst[op + i - off];  // overlapping copies repeat
        op += len;
    }
    return op == (size_t)total ? total : -1;
}

// Slots at i*stride in a Payload.Raw layout ([4-B IP][packet]): compresses packet i (lens[i] bytes
// at slot+4) in place, lens[i] <- compressed length (plugin/compression.go:39-47).  `threads`
// workers over the batch.  Returns the number of packets that did not fit their slot (left as is,
// lens[i] unchanged) or -1.
int qgcm_snappy_compress_slots_limit(uint8_t *arena, uint64_t stride, uint32_t n, uint32_t *lens, uint64_t limit,
                                     uint8_t *status, int threads) {
    if ((n && (!arena || !lens)) || stride < 4) return -1;
    if (limit > stride - 4) limit = stride - 4;
    std::atomic<uint32_t> next{0};
    std::atomic<int> bad{0};
    auto work = [&] {
        std::vector<uint8_t> tmp;
        for (;;) {
            const uint32_t i0 = next.fetch_add(256);
            if (i0 >= n) break;
            for (uint32_t i = i0; i < std::min(n, i0 + 256); ++i) {
                uint8_t *pkt = arena + (uint64_t)i * stride + 4;
                const size_t L = lens[i];
                if (status) status[i] = 0;
                if (L + 4 > stride) {
                    ++bad;
                    continue;
                }
                tmp.resize(qgcm_snappy_max_compressed_length(L));
                const long c = qgcm_snappy_compress(pkt, L, tmp.data(), tmp.size());
                if (c < 0 || (uint64_t)c > limit) {
                    ++bad;
                    continue;
                }
                memcpy(pkt, tmp.data(), (size_t)c);
                lens[i] = (uint32_t)c;
                if (status) status[i] = 1;
            }
        }
    };
    const int t = std::max(1, std::min(threads, 256));
    std::vector<std::thread> pool;
    for (int k = 1; k < t; ++k) pool.emplace_back(work);
    work();
    for (auto &th : pool) th.join();
    return bad.load();
}

int qgcm_snappy_compress_slots(uint8_t *arena, uint64_t stride, uint32_t n, uint32_t *lens, int threads) {
    return qgcm_snappy_compress_slots_limit(arena, stride, n, lens, stride, nullptr, threads);
}

// Inverse of qgcm_snappy_compress_slots (plugin/compression.go:35-38,41-47 Incoming): a packet that
// does not decode, would not fit its slot, or decodes to nothing (golang/snappy returns a nil slice for
// an empty result, which compression.go:37-39 treats as a failure) fails (status 0, slot untouched).
int qgcm_snappy_uncompress_slots(uint8_t *arena, uint64_t stride, uint32_t n, uint32_t *lens, uint8_t *status,
                             int threads) {
    if ((n && (!arena || !lens)) || stride < 4) return -1;
    std::atomic<uint32_t> next{0};
    std::atomic<int> bad{0};
    auto work = [&] {
        std::vector<uint8_t> tmp(stride);
        for (;;) {
            const uint32_t i0 = next.fetch_add(256);
            if (i0 >= n) break;
            for (uint32_t i = i0; i < std::min(n, i0 + 256); ++i) {
                uint8_t *pkt = arena + (uint64_t)i * stride + 4;
                const size_t L = std::min<uint64_t>(lens[i], stride - 4);
                const long u = qgcm_snappy_uncompress(pkt, L, tmp.data(), stride - 4);
                const bool ok = u > 0;  // an empty result is a nil slice in Go: compression.go:37-39 drops it
                if (ok) {
                    memcpy(pkt, tmp.data(), (size_t)u);
                    lens[i] = (uint32_t)u;
                } else {
                    ++bad;
                }
                if (status) status[i] = ok ? 1 : 0;
            }
        }
    };
    const int t = std::max(1, std::min(threads, 256));
    std::vector<std::thread> pool;
    for (int k = 1; k < t; ++k) pool.emplace_back(work);
    work();
    for (auto &th : pool) th.join();
    return bad.load();
}

}  // extern "C"
