// snappy_kernels.hip -- the snappy block codec of the compression plugin on gfx950 (MI355X).
//
// Replaces, per packet, plugin/compression.go:16-27 (snappy.Encode / snappy.Decode of
// payload.Packet) and the copy back into Payload.Raw[4:] that Apply does (compression.go:39-51), for
// a batch of Payload.Raw slots at i * stride in device memory.
//
// The default codec (QGCM_SNAPPY_GROUP=1) codes four packets per wave, one per 16-lane group: the
// group encoder and the group decoder below.  The forms with one wave per packet come first; they
// also serve packets too long for four LDS regions per wave.
//
// One wave per packet.  The encoder is the block algorithm of golang/snappy's encodeBlock (restated
// in snappy_codec.cpp and oracle/snappy_oracle.py, pinned to libsnappy 1.1.8's bytes): its probe /
// insert sequence is inherently serial, so the wave runs it as one uniform control flow (every value
// that steers it is wave-uniform and kept in SGPRs) and spends its 64 lanes where the work is
// data-parallel -- staging the packet into LDS, extending a match 64 bytes per step (a ballot of
// mismatching lanes), copying literals, writing the result back with dword stores.  The packet, the
// hash table (2^8..2^14 uint16 positions) and the output are all in the wave's LDS, and the next
// packet is read while the current one is coded, so no HBM latency sits on the serial chain; 20
// waves per CU then share the CU's one scalar unit, which bounds the encoder (~3.7 K
// scalar instructions per 1350-B packet), so the loop is written for few scalar instructions.  The
// decoder parses tags uniformly and copies each literal / back-reference with all lanes (a copy of
// length <= 64 is one step: lane j reads out[op - off + j % off], which is already written).
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
    uint8_t *sink;  // this lane's 4 scratch bytes: lanes other than 0 store there when lane 0 stores a
                    // uniform value (one store instruction, no exec-mask branch around it)
    uint32_t lane;

    // 4 bytes at byte offset o of the staged input (two aligned dwords, uniform result)
    __device__ __forceinline__ uint32_t load32(uint32_t o) const {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(in);
        const uint32_t lo = w[o >> 2], hi = w[(o >> 2) + 1];
        return rfl(__builtin_amdgcn_alignbyte(hi, lo, o & 3));
    }
    __device__ __forceinline__ void put(uint32_t o, uint32_t v) const { *(lane ? sink : out + o) = (uint8_t)v; }
    __device__ __forceinline__ uint32_t tab_get(uint32_t h) const { return rfl(tab[h]); }
    __device__ __forceinline__ void tab_set(uint32_t h, uint32_t pos) const {
        *(lane ? reinterpret_cast<uint16_t *>(sink) : tab + h) = (uint16_t)pos;
    }
    // out[op..op+len) = in[from..from+len), all lanes
    __device__ __forceinline__ void copy_in(uint32_t op, uint32_t from, uint32_t len) const {
        for (uint32_t j = lane; j < len; j += 64) out[op + j] = in[from + j];
    }
    // the same, 256 bytes per step with every lane active: reads clamped to the last byte, writes past
    // len into the lane's sink, so no exec-mask branch per byte and one LDS round trip per 256 bytes
    __device__ __forceinline__ void copy_in4(uint32_t op, uint32_t from, uint32_t len) const {
        const uint32_t last = from + len - 1;
        for (uint32_t j = 0; j < len; j += 256) {
            uint8_t v[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) v[k] = in[min(from + j + 64 * k + lane, last)];
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const uint32_t o = j + 64 * k + lane;
                *(o < len ? out + op + o : sink) = v[k];
            }
        }
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

// encode_other.go encodeBlock over the staged block in[0..n), kMinBlock <= n <= 65536; output
// from out[op]; returns the end of the output.  One flat loop (the miss probes, and after a match the
// literal and the run of back-to-back copies) keeps the wave-uniform control flow simple for the
// compiler: every value that steers it lives in SGPRs.
__device__ uint32_t encode_block(const Wave &w, uint32_t op, uint32_t n, uint32_t bits) {
    const uint32_t shift = 32 - bits;
    for (uint32_t j = w.lane; j < (1u << bits); j += 64) w.tab[j] = 0;
    wave_lds_sync();
    const uint32_t s_limit = n - 15;
    uint32_t next_emit = 0, s = 1, skip = 32;
    uint32_t cur = w.load32(1), h = hash4(cur, shift);
    for (;;) {
        const uint32_t step = skip >> 5, next_s = s + step;
        if (next_s > s_limit) break;
        skip += step;
        uint32_t cand = w.tab_get(h);
        w.tab_set(h, s);
        const uint32_t nv = w.load32(next_s);
        if (cur != w.load32(cand)) {  // miss: probe further on
            s = next_s;
            cur = nv;
            h = hash4(nv, shift);
            continue;
        }
        op = w.emit_literal(op, next_emit, s - next_emit);
        bool more;
        do {  // copies back to back while the position after one starts another
            const uint32_t base = s;
            s += 4 + w.match_len(cand + 4, s + 4, n);
            op = w.emit_copy(op, base - cand, s - base);
            next_emit = s;
            if (s >= s_limit) break;
            w.tab_set(hash4(w.load32(s - 1), shift), s - 1);
            wave_lds_sync();
            cur = w.load32(s);
            h = hash4(cur, shift);
            cand = w.tab_get(h);
            w.tab_set(h, s);
            more = cur == w.load32(cand);
        } while (more);
        if (s >= s_limit) break;
        ++s;  // the next probe, at s + 1, starts a new miss run
        skip = 32;
        cur = w.load32(s);
        h = hash4(cur, shift);
    }
    if (next_emit < n) op = w.emit_literal(op, next_emit, n - next_emit);
    return op;
}

// The next packet of a wave is read while the wave codes the current one: its length (and input
// status) and the first `cover` bytes of its slot, two 16-B loads per lane, so a packet's HBM
// latencies overlap the previous packet's work instead of preceding its own.  The loads stay inside
// the slot whatever the packet's length: cover = min(2 KiB, stride - 4 rounded down to 16).
struct Prefetch {
    uint32_t len, st;
    uint4 r0, r1;
};
__device__ __forceinline__ uint32_t pf_cover(uint64_t stride) {
    const uint64_t whole = (stride - 4) & ~15ull;
    return whole < 2048 ? (uint32_t)whole : 2048u;
}
__device__ __forceinline__ void pf_issue(Prefetch &f, const SnapArgs &a, uint32_t q, uint32_t lane, uint32_t cover) {
    const uint8_t *src = a.arena + (uint64_t)q * a.stride + 4;
    f.len = a.lens[q];
    f.st = a.status_in ? a.status_in[q] : 1u;
    const uint32_t o0 = 16 * lane, o1 = 1024 + 16 * lane;
    f.r0 = o0 < cover ? *reinterpret_cast<const uint4 *>(src + o0) : uint4{0, 0, 0, 0};
    f.r1 = o1 < cover ? *reinterpret_cast<const uint4 *>(src + o1) : uint4{0, 0, 0, 0};
}

// slot bytes [4, 4 + len) -> LDS: the prefetched chunks, then whole dwords from cover on (the slot is
// 4-B aligned and at least 4 + len rounded up to 4 bytes long, since stride is a multiple of 4); the
// staging area holds len + 24 bytes
__device__ __forceinline__ void stage_in(uint8_t *dst, const uint8_t *slot, uint32_t len, uint32_t lane,
                                         uint32_t cover, const Prefetch &f) {
    const uint32_t o0 = 16 * lane, o1 = 1024 + 16 * lane;
    if (o0 < len && o0 < cover) *reinterpret_cast<uint4 *>(dst + o0) = f.r0;
    if (o1 < len && o1 < cover) *reinterpret_cast<uint4 *>(dst + o1) = f.r1;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(slot + 4);
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    const uint32_t nw = (len + 3) >> 2;
    for (uint32_t j = (cover >> 2) + lane; j < nw; j += 64) d[j] = src[j];
    wave_lds_sync();  // the chunks' bytes past len, then the slack zeros over them
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

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) snappy_compress_kernel(SnapArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6, waves = blockDim.x >> 6;
    uint8_t *base = smem + wv * a.wave_bytes;
    Wave w{base + a.off_in, base + a.off_out, reinterpret_cast<uint16_t *>(base), base + a.off_sink + 4 * lane, lane};
    const uint32_t cover = pf_cover(a.stride), step = gridDim.x * waves;
    uint32_t p = blockIdx.x * waves + wv;
    Prefetch f{};
    if (p < a.n) pf_issue(f, a, p, lane, cover);
    for (; p < a.n; p += step) {
        const uint32_t len = rfl(f.len);
        uint8_t *slot = a.arena + (uint64_t)p * a.stride;
        bool ok = len <= a.max_in;
        if (ok) stage_in(w.in, slot, len, lane, cover, f);
        if (p + step < a.n) pf_issue(f, a, p + step, lane, cover);  // in flight while this packet is coded
        uint32_t d = 0;
        if (ok) {
            wave_lds_sync();
            uint32_t op = put_varint(w, len);
            if (len < 17) {
                if (len) op = w.emit_literal(op, 0, len);
            } else {
                uint32_t bits = 8;
                while (bits < 14 && (1u << bits) < len) ++bits;
                op = encode_block(w, op, len, bits);
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

// ---------------------------------------------------------------------------------------------
// Group encoder: FOUR packets per wave, one per 16-lane group (QGCM_SNAPPY_GROUP, the default since
// round 4).  The one-wave-per-packet encoder above is bound by the CU's single scalar unit: every
// probe's control flow and wave-uniform values run there, ~3 K scalar instructions per 1350-B packet
// (DESIGN.md 4.6).  Here a group's state lives in VGPRs (the same value in its 16 lanes), each lane
// group runs encodeBlock on its own packet, and one instruction stream -- one set of scalar
// instructions for the loop and its exec masks -- serves four packets.  Groups in different phases
// (probing / emitting a copy run) diverge under exec masks; packets of a batch tend to move alike.
// Every group lane stores the same byte to the same address where the wave encoder let one lane
// store (no exec branch per store).  Match extension compares 4 bytes per lane (64 B per group step);
// literal copies move 4 bytes per lane.  Per packet: [hash table | staged input] in LDS (a.off_in
// within a region of a.off_sink bytes), four regions per wave; the output goes straight into the slot.
// The group decoder is at the end of the file.
constexpr uint32_t kGrp = 4, kGL = 64 / kGrp;

// Group prefetch: the next packets' first bytes -- kGPf 16-B loads per lane, 1.5 KiB per packet
// -- and lengths are loaded into registers before the current packets are coded, so a packet's HBM
// latency overlaps the previous packet's work instead of preceding its own (the wave kernels'
// Prefetch, per group).  The loads stay inside the slot: cover = min(1.5 KiB, stride - 4 rounded down
// to 16); bytes from cover on are staged with dword loads.
constexpr uint32_t kGPf = 6;
struct GPrefetch {
    uint32_t len, st;
    uint4 r[kGPf];
};
__device__ __forceinline__ uint32_t gpf_cover(uint64_t stride) {
    const uint64_t whole = (stride - 4) & ~15ull;
    return whole < 256 * kGPf ? (uint32_t)whole : 256 * kGPf;
}
__device__ __forceinline__ void gpf_issue(GPrefetch &f, const SnapArgs &a, uint32_t q, uint32_t gl, uint32_t cover) {
    if (q >= a.n) return;
    const uint8_t *src = a.arena + (uint64_t)q * a.stride + 4;
    f.len = a.lens[q];
    f.st = a.status_in ? a.status_in[q] : 1u;
#pragma unroll
    for (uint32_t k = 0; k < kGPf; ++k) {
        const uint32_t o = 16 * gl + 256 * k;
        f.r[k] = o < cover ? *reinterpret_cast<const uint4 *>(src + o) : uint4{0, 0, 0, 0};
    }
}
// slot bytes [4, 4 + sn) -> LDS (the prefetched part, then whole dwords from cover on), then 8 B of
// zero slack for load32 past the end; the staging area holds sn + 24 bytes
__device__ __forceinline__ void gstage(uint8_t *dst, const uint8_t *slot, uint32_t sn, uint32_t gl, uint32_t cover,
                                       const GPrefetch &f) {
#pragma unroll
    for (uint32_t k = 0; k < kGPf; ++k) {
        const uint32_t o = 16 * gl + 256 * k;
        if (o < sn && o < cover) *reinterpret_cast<uint4 *>(dst + o) = f.r[k];
    }
    const uint32_t *src = reinterpret_cast<const uint32_t *>(slot + 4);
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    const uint32_t nw = (sn + 3) >> 2;
    for (uint32_t j = (cover >> 2) + gl; j < nw; j += kGL) d[j] = src[j];
    if (gl < 2) d[nw + gl] = 0;  // after the 16-B stores above that may cover it (a wave's LDS ops run in order)
}

struct GWave {
    uint8_t *in, *out;  // out = the slot's packet bytes in device memory
    uint16_t *tab;
    uint32_t gl, grp;  // lane within the group, group within the wave
    uint32_t olast;    // last output index kept inside the packet's limit (writes past it land there)

    __device__ __forceinline__ uint32_t load32(uint32_t o) const {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(in);
        return __builtin_amdgcn_alignbyte(w[(o >> 2) + 1], w[o >> 2], o & 3);
    }
    __device__ __forceinline__ void put(uint32_t o, uint32_t v) const {
        out[min(o, olast)] = (uint8_t)v;
    }
    // out[op..op+len) = in[from..from+len): lane gl moves bytes 4 gl .. 4 gl + 3 of every 64
    __device__ __forceinline__ void copy_in(uint32_t op, uint32_t from, uint32_t len) const {
        for (uint32_t j = 4 * gl; j < len; j += 4 * kGL) {
            const uint32_t v = load32(from + j);
            const uint32_t k = len - j < 4 ? len - j : 4;
            put(op + j, v);
            if (k > 1) put(op + j + 1, v >> 8);
            if (k > 2) put(op + j + 2, v >> 16);
            if (k > 3) put(op + j + 3, v >> 24);
        }
    }
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
    // common run of in[a..) and in[b..), b < n: lane gl compares bytes 4 gl .. 4 gl + 3 of each 64
    __device__ __forceinline__ uint32_t match_len(uint32_t a, uint32_t b, uint32_t n) const {
        uint32_t m = 0;
        for (;;) {
            const uint32_t rem = n - (b + m);
            if (rem == 0) return m;
            const uint32_t k = rem < 4 * kGL ? rem : 4 * kGL;
            const uint32_t o = 4 * gl;
            uint32_t x = 0;
            if (o < k) {
                x = load32(a + m + o) ^ load32(b + m + o);
                const uint32_t left = k - o;
                if (left < 4) x &= 0xffffffffu >> (32 - 8 * left);
            }
            const uint64_t d = (__builtin_amdgcn_ballot_w64(x != 0) >> (kGL * grp)) & 0xffffull;
            if (d) {
                const uint32_t first = (uint32_t)__builtin_ctzll(d);  // the group's first differing dword
                const uint32_t xf = __builtin_amdgcn_ds_bpermute((int)((kGL * grp + first) << 2), (int)x);
                return m + 4 * first + ((uint32_t)__builtin_ctz(xf) >> 3);
            }
            m += k;
        }
    }
};

// encodeBlock per group.  The miss probes are software-pipelined: probe positions do not depend on
// the data (each miss moves on by skip >> 5, skip += step), so the word at the probe after next is
// loaded one probe early and the next probe's table entry is read as soon as the current entry is
// written, together with the candidate's word.  A miss then waits for one LDS round trip instead of
// two (the table entry, then the candidate's word).  The early table read is issued after the current probe's table
// write (LDS operations of a wave complete in order), so it sees that write; the bytes are those of
// encodeBlock.
__device__ uint32_t gencode_block(const GWave &w, uint32_t op, uint32_t n, uint32_t bits) {
    const uint32_t shift = 32 - bits;
    uint4 *t16 = reinterpret_cast<uint4 *>(w.tab);  // 2 << bits bytes, a multiple of 256
    for (uint32_t j = w.gl; j < (2u << bits) / 16; j += kGL) t16[j] = uint4{0, 0, 0, 0};
    wave_lds_sync();
    const uint32_t s_limit = n - 15;
    uint32_t next_emit = 0, s = 1, skip = 32;
    uint32_t cur = w.load32(1), h = hash4(cur, shift);
    uint32_t cand = w.tab[h];                       // tab[h] as of this probe
    uint32_t nv = w.load32(min(s + (skip >> 5), n));  // the word at this probe's next_s
    for (;;) {
        const uint32_t step = skip >> 5, next_s = s + step;
        if (next_s > s_limit) break;
        skip += step;
        w.tab[h] = (uint16_t)s;
        const uint32_t hn = hash4(nv, shift);
        // Every LDS read of the probe -- tab[hn] (after the write above, so as the next probe sees
        // it), the word at the probe after next (clamped) and the candidate's word -- is issued
        // before any result is used, so a probe costs one LDS round trip.  Without the fence the
        // compiler sinks the next probe's reads (used on the miss path only) below the compare, and
        // each miss waited for two: compress 4.05-4.10 -> 3.67-3.75 ms per 2^20 config-5 packets
        // (profiles/r5_s11, interleaved A/B).
        const uint32_t *iw = reinterpret_cast<const uint32_t *>(w.in);
        const uint32_t o2 = min(next_s + (skip >> 5), n);
        const uint32_t cn = w.tab[hn];
        const uint32_t a0 = iw[o2 >> 2], a1 = iw[(o2 >> 2) + 1];
        const uint32_t b0 = iw[cand >> 2], b1 = iw[(cand >> 2) + 1];
        asm volatile("" ::: "memory");
        const uint32_t nv2 = __builtin_amdgcn_alignbyte(a1, a0, o2 & 3);
        const uint32_t cw = __builtin_amdgcn_alignbyte(b1, b0, cand & 3);
        if (cur != cw) {  // miss: probe further on
            s = next_s;
            cur = nv;
            h = hn;
            cand = cn;
            nv = nv2;
            continue;
        }
        op = w.emit_literal(op, next_emit, s - next_emit);
        bool more;
        do {  // copies back to back while the position after one starts another
            const uint32_t base = s;
            s += 4 + w.match_len(cand + 4, s + 4, n);
            op = w.emit_copy(op, base - cand, s - base);
            next_emit = s;
            if (s >= s_limit) break;
            w.tab[hash4(w.load32(s - 1), shift)] = (uint16_t)(s - 1);
            wave_lds_sync();
            cur = w.load32(s);
            h = hash4(cur, shift);
            cand = w.tab[h];
            w.tab[h] = (uint16_t)s;
            more = cur == w.load32(cand);
        } while (more);
        if (s >= s_limit) break;
        ++s;
        skip = 32;
        cur = w.load32(s);
        h = hash4(cur, shift);
        wave_lds_sync();
        cand = w.tab[h];
        nv = w.load32(min(s + (skip >> 5), n));
    }
    if (next_emit < n) op = w.emit_literal(op, next_emit, n - next_emit);
    return op;
}

// The output goes straight into the slot (its input is staged in LDS, so the slot is free to
// overwrite), and a packet's LDS region holds only the hash table and the staged input: 5.5 KiB for
// a 1472-B slot, 7 waves (28 packets) per CU.  Output bytes past the packet's limit all land on its
// last kept byte; a packet whose output exceeds the limit gets its first `limit` slot bytes back from
// the staged copy (staged up to max(len, limit) bytes for that).  The next packets' first bytes are
// prefetched into registers while these are coded (GPrefetch).
__global__ void __launch_bounds__(256) snappy_compress_group_kernel(SnapArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6, waves = blockDim.x >> 6;
    const uint32_t grp = lane / kGL, gl = lane % kGL;
    uint8_t *base = smem + (wv * kGrp + grp) * a.off_sink;
    GWave w{base + a.off_in, nullptr, reinterpret_cast<uint16_t *>(base), gl, grp, a.limit - 1};
    const uint32_t step = gridDim.x * waves * kGrp, cover = gpf_cover(a.stride);
    GPrefetch f{};
    gpf_issue(f, a, (blockIdx.x * waves + wv) * kGrp + grp, gl, cover);
    for (uint32_t p0 = (blockIdx.x * waves + wv) * kGrp; p0 < a.n; p0 += step) {
        const uint32_t p = p0 + grp;
        const bool have = p < a.n;
        const uint32_t len = have ? f.len : 0u;
        uint8_t *slot = a.arena + (uint64_t)(have ? p : 0u) * a.stride;
        bool ok = have && len <= a.max_in;
        // max(len, limit) bytes staged: the restore copy of a packet whose output overflows
        if (ok) gstage(w.in, slot, max(len, a.limit), gl, cover, f);  // 4-B aligned slot, stride a multiple of 4
        gpf_issue(f, a, p + step, gl, cover);                         // in flight while these packets are coded
        w.out = slot + 4;
        wave_lds_sync();
        uint32_t d = 0;
        if (ok) {
            uint32_t op = 0, v = len;  // put_varint
            while (v >= 0x80) {
                w.put(op++, (v & 0x7f) | 0x80);
                v >>= 7;
            }
            w.put(op++, v);
            if (len < 17) {
                if (len) op = w.emit_literal(op, 0, len);
            } else {
                uint32_t bits = 8;
                while (bits < 14 && (1u << bits) < len) ++bits;
                op = gencode_block(w, op, len, bits);
            }
            d = op;
            ok = d <= a.limit;
            if (!ok) {  // overflowed: the slot's first `limit` bytes back from the staged copy
                uint32_t *dst = reinterpret_cast<uint32_t *>(slot + 4);
                const uint32_t *srcw = reinterpret_cast<const uint32_t *>(w.in);
                const uint32_t nw = a.limit >> 2;
                for (uint32_t j = gl; j < nw; j += kGL) dst[j] = srcw[j];
                const uint32_t t = a.limit & 3;
                if (gl < t) slot[4 + 4 * nw + gl] = w.in[4 * nw + gl];
            }
        }
        wave_lds_sync();
        if (have && gl == 0) {
            if (ok) a.lens[p] = d;
            if (a.status) a.status[p] = ok ? 1 : 0;
            if (a.descs) a.descs[p] = qgcm_desc{(uint64_t)p * a.stride, ok ? d : QGCM_MAX_PAYLOAD, a.key_idx};
        }
        wave_lds_sync();  // the next packets' staging overwrites these ones' LDS
    }
}

// decode.go Decode of in[0..n) into out (at most cap bytes); returns the length or -1.  Literals move
// 256 bytes per step and back-references one step of 64 lanes, every lane active (reads clamped or of
// bytes already written, writes past the element into the lane's sink): no exec-mask branch per
// element, which the CU's scalar unit -- the decoder's bound -- would otherwise issue (uncompress
// 1.56 -> 1.50 ms on config 5, 2.85 -> 2.74 on copy-heavy packets, profiles/r5_s21)
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
    const uint32_t *iw = reinterpret_cast<const uint32_t *>(w.in);
    while (ip < n) {
        // the tag and the (up to 4) bytes after it in one read of the two dwords that hold them (the
        // staging area has 8 B of slack past n), used only where the bounds checks below pass: one
        // LDS round trip per element header instead of two (uncompress 1.76-1.79 -> 1.67-1.73 ms per
        // 2^20 config-5 packets, profiles/r5_s13)
        const uint32_t q = ip >> 2;
        const uint64_t x = (((uint64_t)rfl(iw[q + 1]) << 32) | rfl(iw[q])) >> (8 * (ip & 3));
        const uint32_t tag = (uint32_t)x & 0xffu;
        ++ip;
        uint32_t len, off;
        if ((tag & 3) == 0) {
            len = tag >> 2;
            if (len >= 60) {
                const uint32_t b = len - 59;
                if (ip + b > n) return -1;
                len = (uint32_t)(x >> 8) & (0xffffffffu >> (32 - 8 * b));
                ip += b;
                if (len >= 0xffffffffu) return -1;
            }
            ++len;
            if (len > n - ip || len > total - op) return -1;
            w.copy_in4(op, ip, len);
            ip += len;
            op += len;
            continue;
        }
        if ((tag & 3) == 1) {
            if (ip + 1 > n) return -1;
            len = 4 + ((tag >> 2) & 7);
            off = ((tag >> 5) << 8) | ((uint32_t)(x >> 8) & 0xffu);
            ip += 1;
        } else if ((tag & 3) == 2) {
            if (ip + 2 > n) return -1;
            len = 1 + (tag >> 2);
            off = (uint32_t)(x >> 8) & 0xffffu;
            ip += 2;
        } else {
            if (ip + 4 > n) return -1;
            len = 1 + (tag >> 2);
            off = (uint32_t)(x >> 8);
            ip += 4;
        }
        if (off == 0 || off > op || len > total - op) return -1;
        wave_lds_sync();  // earlier elements' bytes are in LDS before lanes read them back
        {  // len <= 64; every lane reads a byte already written, lanes past len write their sink
            const uint8_t v = w.out[op - off + w.lane % off];
            *(w.lane < len ? w.out + op + w.lane : w.sink) = v;
        }
        op += len;
    }
    return op == total ? (int)total : -1;
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) snappy_uncompress_kernel(SnapArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6, waves = blockDim.x >> 6;
    uint8_t *base = smem + wv * a.wave_bytes;
    Wave w{base + a.off_in, base + a.off_out, nullptr, base + a.off_sink + 4 * lane, lane};
    const uint32_t cover = pf_cover(a.stride), step = gridDim.x * waves;
    uint32_t p = blockIdx.x * waves + wv;
    Prefetch f{};
    if (p < a.n) pf_issue(f, a, p, lane, cover);
    for (; p < a.n; p += step) {
        const bool auth = rfl(f.st) == 1;  // status_in: packets that failed to open are left to the caller
        const uint32_t stored = rfl(f.len);
        const uint32_t len = stored >= a.sub ? stored - a.sub : stored;
        uint8_t *slot = a.arena + (uint64_t)p * a.stride;
        const bool take = auth && stored >= a.sub && len <= a.max_in;
        if (take) stage_in(w.in, slot, len, lane, cover, f);
        if (p + step < a.n) pf_issue(f, a, p + step, lane, cover);  // in flight while this packet is decoded
        if (!auth) continue;
        int u = -1;
        if (take) {
            wave_lds_sync();
            u = decode(w, len, a.limit);
            // an empty result fails: golang/snappy's Decode(nil, src) returns a nil slice for it and
            // compression.go:37-39 drops a nil packet
            if (u == 0) u = -1;
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

// ---------------------------------------------------------------------------------------------
// Group decoder: four packets per wave, one per 16-lane group.  The wave decoder above runs each
// element's parse as wave-uniform scalar code for one packet, and the CU's one scalar unit is its
// bound; here each group parses its own packet in VGPRs (the same values in its 16 lanes), so one
// instruction stream serves four packets.  An element header comes from one two-dword window; a
// literal moves 4 bytes per lane per step; a back-reference (<= 64 bytes) is four reads then four
// writes per lane (i = gl, gl + 16, ...: out[op - off + i mod off], bytes earlier elements wrote), the
// lanes past the element writing into their scratch word.  Per packet: [staged input | output |
// 64 B of scratch] in LDS, wave_bytes / 4 bytes, four per wave.
struct GDec {
    uint8_t *in, *out, *sink;  // sink: this lane's scratch word
    uint32_t gl;
    __device__ __forceinline__ uint32_t load32(uint32_t o) const {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(in);
        return __builtin_amdgcn_alignbyte(w[(o >> 2) + 1], w[o >> 2], o & 3);
    }
};

// i % off for i < 64 and off >= 1 without a division: off >= 64 leaves i; below that the quotient of a
// float reciprocal with a half-step margin ((i + 0.5) / off is at least 1/128 from an integer, far more
// than the reciprocal's error; every (i, off) pair checked exhaustively), corrected once each way
__device__ __forceinline__ uint32_t mod64(uint32_t i, uint32_t off) {
    if (off >= 64) return i;
    const uint32_t q = (uint32_t)(((float)i + 0.5f) * __builtin_amdgcn_rcpf((float)off));
    int m = (int)i - (int)(q * off);
    m = m < 0 ? m + (int)off : m;
    return (uint32_t)(m >= (int)off ? m - (int)off : m);
}

// decode.go Decode of in[0..n) into out (at most cap bytes), per group; returns the length or -1
__device__ int gdecode(const GDec &w, uint32_t n, uint32_t cap) {
    const uint32_t *iw = reinterpret_cast<const uint32_t *>(w.in);
    uint32_t total = 0, ip = 0;
    {
        const uint64_t x = ((uint64_t)iw[1] << 32) | iw[0];  // the staging's 8 B of slack cover n < 8
        for (uint32_t sh = 0;; sh += 7) {
            if (ip >= n || ip >= 5) return -1;
            const uint32_t c = (uint32_t)(x >> (8 * ip)) & 0xffu;
            ++ip;
            if (sh == 28 && (c & 0x7f) > 15) return -1;  // > 32 bits
            total |= (c & 0x7f) << sh;
            if (c < 0x80) break;
        }
    }
    if (total > cap) return -1;
    uint32_t op = 0;
    while (ip < n) {
        const uint32_t q = ip >> 2;
        const uint64_t x = (((uint64_t)iw[q + 1] << 32) | iw[q]) >> (8 * (ip & 3));
        const uint32_t tag = (uint32_t)x & 0xffu;
        ++ip;
        uint32_t len, off;
        if ((tag & 3) == 0) {
            len = tag >> 2;
            if (len >= 60) {
                const uint32_t b = len - 59;  // 1..4 little-endian length bytes
                if (ip + b > n) return -1;
                len = (uint32_t)(x >> 8) & (0xffffffffu >> (32 - 8 * b));
                ip += b;
                if (len >= 0xffffffffu) return -1;
            }
            ++len;
            if (len > n - ip || len > total - op) return -1;
            for (uint32_t j = 4 * w.gl; j < len; j += 4 * kGL) {  // 4 bytes per lane, the tail to the sink
                const uint32_t v = w.load32(ip + j);
#pragma unroll
                for (uint32_t t = 0; t < 4; ++t) *(j + t < len ? w.out + op + j + t : w.sink) = (uint8_t)(v >> (8 * t));
            }
            ip += len;
            op += len;
            continue;
        }
        if ((tag & 3) == 1) {
            if (ip + 1 > n) return -1;
            len = 4 + ((tag >> 2) & 7);
            off = ((tag >> 5) << 8) | ((uint32_t)(x >> 8) & 0xffu);
            ip += 1;
        } else if ((tag & 3) == 2) {
            if (ip + 2 > n) return -1;
            len = 1 + (tag >> 2);
            off = (uint32_t)(x >> 8) & 0xffffu;
            ip += 2;
        } else {
            if (ip + 4 > n) return -1;
            len = 1 + (tag >> 2);
            off = (uint32_t)(x >> 8);
            ip += 4;
        }
        if (off == 0 || off > op || len > total - op) return -1;
        // the bytes read back were written by OTHER lanes in earlier elements: the wave's LDS ops run in
        // order, but the compiler must not move these reads above those writes (a cross-lane dependence
        // it cannot see): a compiler fence (the wave decoder's wave_lds_sync also waits; in-order LDS
        // needs only the fence)
        asm volatile("" ::: "memory");
        uint8_t v[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) v[k] = w.out[op - off + mod64(w.gl + kGL * k, off)];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t i = w.gl + kGL * k;
            *(i < len ? w.out + op + i : w.sink) = v[k];
        }
        op += len;
    }
    return op == total ? (int)total : -1;
}

__global__ void __launch_bounds__(256) snappy_uncompress_group_kernel(SnapArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6, waves = blockDim.x >> 6;
    const uint32_t grp = lane / kGL, gl = lane % kGL, region = a.wave_bytes / kGrp;
    uint8_t *base = smem + (wv * kGrp + grp) * region;
    const GDec w{base + a.off_in, base + a.off_out, base + a.off_sink + 4 * gl, gl};
    const uint32_t step = gridDim.x * waves * kGrp, cover = gpf_cover(a.stride);
    GPrefetch f{};
    gpf_issue(f, a, (blockIdx.x * waves + wv) * kGrp + grp, gl, cover);
    for (uint32_t p0 = (blockIdx.x * waves + wv) * kGrp; p0 < a.n; p0 += step) {
        const uint32_t p = p0 + grp;
        const bool have = p < a.n;
        const uint32_t stored = have ? f.len : 0u;
        const bool auth = have && f.st == 1;  // status_in: packets that failed to open are left to the caller
        const uint32_t len = stored >= a.sub ? stored - a.sub : stored;
        uint8_t *slot = a.arena + (uint64_t)(have ? p : 0u) * a.stride;
        const bool take = auth && stored >= a.sub && len <= a.max_in;
        if (take) gstage(w.in, slot, len, gl, cover, f);
        gpf_issue(f, a, p + step, gl, cover);  // in flight while these packets are decoded
        wave_lds_sync();
        int u = -1;
        if (take) {
            u = gdecode(w, len, a.limit);
            // an empty result fails: golang/snappy's Decode(nil, src) returns a nil slice for it and
            // compression.go:37-39 drops a nil packet
            if (u == 0) u = -1;
        }
        wave_lds_sync();
        if (u > 0) {  // LDS [0, u) -> slot bytes [4, 4 + u)
            uint32_t *dst = reinterpret_cast<uint32_t *>(slot + 4);
            const uint32_t *srcw = reinterpret_cast<const uint32_t *>(w.out);
            const uint32_t nw = (uint32_t)u >> 2;
            for (uint32_t j = gl; j < nw; j += kGL) dst[j] = srcw[j];
            const uint32_t t = (uint32_t)u & 3;
            if (gl < t) slot[4 + 4 * nw + gl] = w.out[4 * nw + gl];
        }
        if (auth && gl == 0) {
            a.lens[p] = u > 0 ? (uint32_t)u : len;  // failed: the compressed length (sub = 0: unchanged)
            if (a.status) a.status[p] = u > 0 ? 1 : 0;
        }
        wave_lds_sync();  // the next packets' staging overwrites these ones' LDS
    }
}

}  // namespace

hipError_t launch_snappy(bool compress, const SnapArgs &a, int waves_per_wg, int grid, hipStream_t s, int group) {
    const size_t lds = (size_t)waves_per_wg * a.wave_bytes;
    const dim3 g(grid), b(64 * waves_per_wg);
    if (compress && group)
        hipLaunchKernelGGL(snappy_compress_group_kernel, g, b, lds, s, a);
    else if (compress)
        hipLaunchKernelGGL(snappy_compress_kernel, g, b, lds, s, a);
    else if (group == 2)
        hipLaunchKernelGGL(snappy_uncompress_group_kernel, g, b, lds, s, a);
    else
        hipLaunchKernelGGL(snappy_uncompress_kernel, g, b, lds, s, a);
    return hipGetLastError();
}

}  // namespace qgcm
