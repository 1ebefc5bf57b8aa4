// snappy_kernels.hip -- the snappy block codec of the compression plugin on gfx950 (MI355X).
//
// Replaces, per packet, plugin/compression.go:16-27 (snappy.Encode / snappy.Decode of
// payload.Packet) and the copy back into Payload.Raw[4:] that Apply does (compression.go:39-51), for
// a batch of Payload.Raw slots at i * stride in device memory.
//
// One wave per packet.  The encoder is the block algorithm of golang/snappy's encodeBlock (restated
// in snappy_codec.cpp and oracle/snappy_oracle.py, pinned to libsnappy 1.1.8's bytes): its probe /
// insert sequence is inherently serial, so the wave runs it as one uniform control flow (every value
// that steers it is wave-uniform and kept in SGPRs) and spends its 64 lanes where the work is
// data-parallel -- staging the packet into LDS, extending a match 64 bytes per step (a ballot of
// mismatching lanes), copying literals, writing the result back with dword stores.  The packet, the
// hash table (2^8..2^14 uint16 positions) and the output are all in the wave's LDS, so the serial
// chain is LDS latency, not HBM latency, and many waves per CU overlap their chains.  The decoder
// parses tags uniformly and copies each literal / back-reference with all lanes (a copy of length
// <= 64 is one step: lane j reads out[op - off + j % off], which is already written).
//
// Byte-exact with the host encoder (tests/test_gpu_snappy.py): a packet whose output does not fit
// `limit` (compress) or `cap` (uncompress), or that does not decode, fails: status 0, slot and
// length untouched.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gcm_internal.h"

namespace qgcm {
namespace {

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
// LDS writes of this wave complete before its later LDS reads of other lanes' bytes
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ uint32_t hash4(uint32_t v, uint32_t shift) { return (v * 0x1e35a7bdu) >> shift; }

struct Wave {
    uint8_t *in;    // staged packet (+8 B of slack)
    uint8_t *out;   // output staging
    uint16_t *tab;  // encoder hash table
    uint32_t lane;

    // 4 bytes at byte offset o of the staged input (two aligned dwords, uniform result)
    __device__ __forceinline__ uint32_t load32(uint32_t o) const {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(in);
        const uint32_t lo = w[o >> 2], hi = w[(o >> 2) + 1];
        return rfl(__builtin_amdgcn_alignbyte(hi, lo, o & 3));
    }
    // the same, per lane (o differs across lanes)
    __device__ __forceinline__ uint32_t load32v(uint32_t o) const {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(in);
        return __builtin_amdgcn_alignbyte(w[(o >> 2) + 1], w[o >> 2], o & 3);
    }
    __device__ __forceinline__ void put(uint32_t o, uint32_t v) const {
        if (lane == 0) out[o] = (uint8_t)v;
    }
    __device__ __forceinline__ uint32_t tab_get(uint32_t h) const { return rfl(tab[h]); }
    __device__ __forceinline__ void tab_set(uint32_t h, uint32_t pos) const {
        if (lane == 0) tab[h] = (uint16_t)pos;
    }
    // out[op..op+len) = in[from..from+len), all lanes
    __device__ __forceinline__ void copy_in(uint32_t op, uint32_t from, uint32_t len) const {
        for (uint32_t j = lane; j < len; j += 64) out[op + j] = in[from + j];
    }
    // encode_other.go emitLiteral
    __device__ __forceinline__ uint32_t emit_literal(uint32_t op, uint32_t from, uint32_t len) const {
        const uint32_t n = len - 1;
        if (n < 60) {
            put(op, n << 2);
            op += 1;
        } else if (n < 256) {
            put(op, 60u << 2);
            put(op + 1, n);
            op += 2;
        } else {
            put(op, 61u << 2);
            put(op + 1, n & 0xff);
            put(op + 2, n >> 8);
            op += 3;
        }
        copy_in(op, from, len);
        return op + len;
    }
    __device__ __forceinline__ uint32_t copy2(uint32_t op, uint32_t off, uint32_t len) const {
        put(op, ((len - 1) << 2) | 2);
        put(op + 1, off & 0xff);
        put(op + 2, off >> 8);
        return op + 3;
    }
    // encode_other.go emitCopy
    __device__ __forceinline__ uint32_t emit_copy(uint32_t op, uint32_t off, uint32_t len) const {
        while (len >= 68) {
            op = copy2(op, off, 64);
            len -= 64;
        }
        if (len > 64) {
            op = copy2(op, off, 60);
            len -= 60;
        }
        if (len >= 12 || off >= 2048) return copy2(op, off, len);
        put(op, ((off >> 8) << 5) | ((len - 4) << 2) | 1);
        put(op + 1, off & 0xff);
        return op + 2;
    }
    // length of the common run of in[a..) and in[b..), b < n: 64 bytes per step
    __device__ __forceinline__ uint32_t match_len(uint32_t a, uint32_t b, uint32_t n) const {
        uint32_t m = 0;
        for (;;) {
            const uint32_t rem = n - (b + m);
            if (rem == 0) return m;
            const uint32_t k = rem < 64 ? rem : 64;
            const bool diff = lane < k && in[a + m + lane] != in[b + m + lane];
            const uint64_t d = ballot(diff);
            if (d) return m + (uint32_t)__builtin_ctzll(d);
            m += k;
        }
    }
};

// B probes of encodeBlock's miss loop at once, lane j = probe j, starting at position s with the
// given skip.  Each lane rebuilds what the serial loop would have done: its position (the skip
// recurrence), the table entry it would read -- the latest earlier probe of the batch with the same
// hash, else the entry from before the batch -- and its 4-byte compare; a ballot finds the first
// match, and the table receives the positions of the probes up to it (of probes sharing a hash, the
// last one).  The serial chain of two dependent LDS round trips per probe becomes a few per batch.
// Returns 0: match at s (cand set); 1: B misses (s, skip advanced); 2: the probes reached s_limit.
__device__ __forceinline__ int probe_batch(const Wave &w, uint32_t B, uint32_t &s, uint32_t &skip, uint32_t &cand,
                                           uint32_t s_limit, uint32_t shift) {
    uint32_t my_p = 0, my_next = 0xffffffffu, p = s, sk = skip, nb = 0;
    while (nb < B) {
        const uint32_t step = sk >> 5, nx = p + step;
        const bool mine = w.lane == nb;
        my_p = mine ? p : my_p;
        my_next = mine ? nx : my_next;
        ++nb;
        if (nx > s_limit) break;  // that probe is not made: the block's remainder follows
        p = nx;
        sk += step;
    }
    const bool valid = my_next <= s_limit;  // a prefix of the lanes
    const uint32_t nvalid = (uint32_t)__builtin_popcountll(ballot(valid));
    const uint32_t cur = valid ? w.load32v(my_p) : 0u;
    const uint32_t h = hash4(cur, shift);
    uint32_t c = valid ? (uint32_t)w.tab[h] : 0u;
    uint32_t nextsame = 64;  // first later probe of the batch with the same hash (64: none)
    for (uint32_t i = 0; i < nvalid; ++i) {
        const uint32_t hi = __builtin_amdgcn_readlane(h, i), pi = __builtin_amdgcn_readlane(my_p, i);
        const bool same = hi == h;
        c = same && i < w.lane ? pi : c;
        nextsame = same && i > w.lane && nextsame == 64 ? i : nextsame;
    }
    const uint64_t mm = ballot(valid && w.load32v(c) == cur);
    const uint32_t last = mm ? (uint32_t)__builtin_ctzll(mm) : 63;  // the last probe made
    if (valid && w.lane <= last && nextsame > last) w.tab[h] = (uint16_t)my_p;
    wave_lds_sync();
    if (mm) {
        s = __builtin_amdgcn_readlane(my_p, last);
        cand = __builtin_amdgcn_readlane(c, last);
        return 0;
    }
    if (nvalid < nb || nb < B) return 2;
    s = p;
    skip = sk;
    return 1;
}

// encode_other.go encodeBlock over the staged block in[0..n), kMinBlock <= n <= 65536; output
// from out[op]; returns the end of the output.  kBatch: the miss loop by probe_batch (the default),
// else probe by probe (A/B: QGCM_SNAPPY_SERIAL=1).
template <bool kBatch>
__device__ uint32_t encode_block(const Wave &w, uint32_t op, uint32_t n, uint32_t bits) {
    const uint32_t shift = 32 - bits;
    for (uint32_t j = w.lane; j < (1u << bits); j += 64) w.tab[j] = 0;
    wave_lds_sync();
    const uint32_t s_limit = n - 15;
    uint32_t next_emit = 0, s = 1;
    uint32_t next_val = kBatch ? 0u : w.load32(1);
    uint32_t next_hash = hash4(next_val, shift);
    for (;;) {
        uint32_t skip = 32, next_s = s, cand = 0;
        if constexpr (kBatch) {
            int r;
            uint32_t B = 16;  // short first batch: after a copy the next match is often near
            while ((r = probe_batch(w, B, s, skip, cand, s_limit, shift)) == 1) B = 64;
            if (r == 2) goto remainder;
        } else for (;;) {
            s = next_s;
            const uint32_t cur = next_val;  // load32(s)
            const uint32_t step = skip >> 5;
            next_s = s + step;
            skip += step;
            if (next_s > s_limit) goto remainder;
            cand = w.tab_get(next_hash);
            w.tab_set(next_hash, s);
            next_val = w.load32(next_s);
            next_hash = hash4(next_val, shift);
            if (cur == w.load32(cand)) break;
        }
        op = w.emit_literal(op, next_emit, s - next_emit);
        for (;;) {
            const uint32_t base = s;
            s += 4 + w.match_len(cand + 4, s + 4, n);
            op = w.emit_copy(op, base - cand, s - base);
            next_emit = s;
            if (s >= s_limit) goto remainder;
            w.tab_set(hash4(w.load32(s - 1), shift), s - 1);
            wave_lds_sync();
            const uint32_t cur = w.load32(s);
            const uint32_t h = hash4(cur, shift);
            cand = w.tab_get(h);
            w.tab_set(h, s);
            if (cur != w.load32(cand)) {
                if constexpr (!kBatch) {
                    next_val = w.load32(s + 1);
                    next_hash = hash4(next_val, shift);
                }
                ++s;
                break;
            }
        }
    }
remainder:
    if (next_emit < n) op = w.emit_literal(op, next_emit, n - next_emit);
    return op;
}

// slot bytes [4, 4 + len) -> LDS, whole dwords (the slot is 4-B aligned and at least 4 + len rounded
// up to 4 bytes long, since stride is a multiple of 4)
__device__ __forceinline__ void stage_in(uint8_t *dst, const uint8_t *slot, uint32_t len, uint32_t lane) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(slot + 4);
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    const uint32_t nw = (len + 3) >> 2;
    for (uint32_t j = lane; j < nw; j += 64) d[j] = src[j];
    if (lane < 2) d[nw + lane] = 0;  // slack read by load32 past the end
}

// LDS [0, len) -> slot bytes [4, 4 + len): whole dwords, the last partial dword bytewise
__device__ __forceinline__ void write_out(uint8_t *slot, const uint8_t *src, uint32_t len, uint32_t lane) {
    uint32_t *d = reinterpret_cast<uint32_t *>(slot + 4);
    const uint32_t *s = reinterpret_cast<const uint32_t *>(src);
    const uint32_t nw = len >> 2;
    for (uint32_t j = lane; j < nw; j += 64) d[j] = s[j];
    const uint32_t t = len & 3;
    if (lane < t) slot[4 + 4 * nw + lane] = src[4 * nw + lane];
}

__device__ __forceinline__ uint32_t put_varint(const Wave &w, uint32_t v) {
    uint32_t op = 0;
    while (v >= 0x80) {
        w.put(op++, (v & 0x7f) | 0x80);
        v >>= 7;
    }
    w.put(op++, v);
    return op;
}

__global__ void __launch_bounds__(256) snappy_compress_kernel(SnapArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6, waves = blockDim.x >> 6;
    uint8_t *base = smem + wv * a.wave_bytes;
    Wave w{base + a.off_in, base + a.off_out, reinterpret_cast<uint16_t *>(base), lane};
    for (uint32_t p = blockIdx.x * waves + wv; p < a.n; p += gridDim.x * waves) {
        const uint32_t len = rfl(a.lens[p]);
        uint8_t *slot = a.arena + (uint64_t)p * a.stride;
        bool ok = len <= a.max_in;
        uint32_t d = 0;
        if (ok) {
            stage_in(w.in, slot, len, lane);
            wave_lds_sync();
            uint32_t op = put_varint(w, len);
            if (len < 17) {
                if (len) op = w.emit_literal(op, 0, len);
            } else {
                uint32_t bits = 8;
                while (bits < 14 && (1u << bits) < len) ++bits;
                op = a.serial ? encode_block<false>(w, op, len, bits) : encode_block<true>(w, op, len, bits);
            }
            d = op;
            ok = d <= a.limit;
            wave_lds_sync();
            if (ok) write_out(slot, w.out, d, lane);
        }
        if (lane == 0) {
            if (ok) a.lens[p] = d;
            if (a.status) a.status[p] = ok ? 1 : 0;
            if (a.descs) a.descs[p] = qgcm_desc{(uint64_t)p * a.stride, ok ? d : QGCM_MAX_PAYLOAD, a.key_idx};
        }
        wave_lds_sync();  // the next packet's staging overwrites this one's LDS
    }
}

// decode.go Decode of in[0..n) into out (at most cap bytes); returns the length or -1
__device__ int decode(const Wave &w, uint32_t n, uint32_t cap) {
    uint32_t total = 0, ip = 0;
    for (uint32_t sh = 0;; sh += 7) {
        if (ip >= n || ip >= 5) return -1;
        const uint32_t c = rfl(w.in[ip++]);
        if (sh == 28 && (c & 0x7f) > 15) return -1;  // > 32 bits
        total |= (c & 0x7f) << sh;
        if (c < 0x80) break;
    }
    if (total > cap) return -1;
    uint32_t op = 0;
    while (ip < n) {
        const uint32_t tag = rfl(w.in[ip++]);
        uint32_t len, off;
        if ((tag & 3) == 0) {
            len = tag >> 2;
            if (len >= 60) {
                const uint32_t b = len - 59;
                if (ip + b > n) return -1;
                len = 0;
                for (uint32_t i = 0; i < b; ++i) len |= rfl(w.in[ip + i]) << (8 * i);
                ip += b;
                if (len >= 0xffffffffu) return -1;
            }
            ++len;
            if (len > n - ip || len > total - op) return -1;
            w.copy_in(op, ip, len);
            ip += len;
            op += len;
            continue;
        }
        if ((tag & 3) == 1) {
            if (ip + 1 > n) return -1;
            len = 4 + ((tag >> 2) & 7);
            off = ((tag >> 5) << 8) | rfl(w.in[ip]);
            ip += 1;
        } else if ((tag & 3) == 2) {
            if (ip + 2 > n) return -1;
            len = 1 + (tag >> 2);
            off = rfl(w.in[ip]) | (rfl(w.in[ip + 1]) << 8);
            ip += 2;
        } else {
            if (ip + 4 > n) return -1;
            len = 1 + (tag >> 2);
            off = w.load32(ip);
            ip += 4;
        }
        if (off == 0 || off > op || len > total - op) return -1;
        wave_lds_sync();  // earlier elements' bytes are in LDS before lanes read them back
        if (w.lane < len) w.out[op + w.lane] = w.out[op - off + w.lane % off];  // len <= 64
        op += len;
    }
    return op == total ? (int)total : -1;
}

__global__ void __launch_bounds__(256) snappy_uncompress_kernel(SnapArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6, waves = blockDim.x >> 6;
    uint8_t *base = smem + wv * a.wave_bytes;
    Wave w{base + a.off_in, base + a.off_out, nullptr, lane};
    for (uint32_t p = blockIdx.x * waves + wv; p < a.n; p += gridDim.x * waves) {
        if (a.status_in && rfl(a.status_in[p]) != 1) continue;  // not authentic: left to the caller
        const uint32_t stored = rfl(a.lens[p]);
        const uint32_t len = stored >= a.sub ? stored - a.sub : stored;
        uint8_t *slot = a.arena + (uint64_t)p * a.stride;
        int u = -1;
        if (stored >= a.sub && len <= a.max_in) {
            stage_in(w.in, slot, len, lane);
            wave_lds_sync();
            u = decode(w, len, a.limit);
            wave_lds_sync();
            if (u >= 0) write_out(slot, w.out, (uint32_t)u, lane);
        }
        if (lane == 0) {
            a.lens[p] = u >= 0 ? (uint32_t)u : len;  // failed: the compressed length (sub = 0: unchanged)
            if (a.status) a.status[p] = u >= 0 ? 1 : 0;
        }
        wave_lds_sync();
    }
}

}  // namespace

hipError_t launch_snappy(bool compress, const SnapArgs &a, int waves_per_wg, int grid, hipStream_t s) {
    const size_t lds = (size_t)waves_per_wg * a.wave_bytes;
    if (compress)
        hipLaunchKernelGGL(snappy_compress_kernel, dim3(grid), dim3(64 * waves_per_wg), lds, s, a);
    else
        hipLaunchKernelGGL(snappy_uncompress_kernel, dim3(grid), dim3(64 * waves_per_wg), lds, s, a);
    return hipGetLastError();
}

}  // namespace qgcm
