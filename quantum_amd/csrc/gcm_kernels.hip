// gcm_kernels.hip -- AES-256-GCM seal/open of packet batches for gfx950 (MI355X, CDNA4).
//
// Replaces, per packet, crypto/aes.go:41-52 (Encrypt: cipher.AEAD.Seal in place, tag, nonce)
// and crypto/aes.go:57-62 (Decrypt: cipher.AEAD.Open in place), the calls that
// plugin/encryption.go:22-37 makes for every tunnelled payload.
//
// Design (DESIGN.md has the numbers):
//  * gcm_quad_kernel (the batch path): four lanes per packet (lane m owns blocks m mod 4), 16 packets
//    per wave, key-uniform wave tiles so round keys sit in SGPRs and the GHASH multiplier is uniform;
//    persistent grid of two 16-wave workgroups per CU; gcm_seg_kernel: the same engine over sorted
//    key runs (descriptor batches); gcm_one_kernel: one workgroup per packet (the per-call
//    Encrypt/Decrypt);
//  * AES-256 by T-tables in LDS: Te0/Te1 replicated 32x so a ds_read_b32 is bank-conflict free;
//    the lookup address (x<<8 | lane*4) is ONE v_perm_b32 (one all-VGPR AND-OR for byte 1 in the
//    Tab2F engine); Te2/Te3 = rot16(Te0/Te1) folded into the column XOR;
//  * CTR caching: counters of a packet differ only in the low byte for 256 consecutive blocks,
//    so rounds 1-2 collapse to 5 lookups per block (197 instead of 224 lookups per block);
//  * GHASH by comb tables of the uniform multiplier H^4 in LDS: the 5-bit comb of the default
//    single-key engine (Tab2F: 26 windows x 2 ds_read_b64, one 256-B bank row per half-table), the
//    4-bit comb elsewhere (one 256-B bank row per nibble table); each lane runs a Horner chain by H^4
//    and the four chains are recombined once per packet.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "gcm_internal.h"

namespace qgcm {

// The packet kernels use dynamic LDS only, so it starts at LDS address 0 and every table address
// below is absolute: LDS pointers are formed straight from the integer (no base add per lookup).
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u128;

struct __attribute__((aligned(4))) W4 {
    uint32_t x, y, z, w;
};

// Streamed payload block (read once per pass).  Serving the final-round S-box from L1 instead of
// LDS, with these loads non-temporal, measured 5% slower: the LDS path stays.
// QGCM_NT_DATA (side builds, A/B only): 1 = payload loads non-temporal, 2 = stores, 3 = both.
#ifndef QGCM_NT_DATA
#define QGCM_NT_DATA 0
#endif
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ W4 load_block(const W4 *p) {
    if constexpr ((QGCM_NT_DATA & 1) != 0) {
        const u32x4u v = __builtin_nontemporal_load(reinterpret_cast<const u32x4u *>(p));
        return W4{v.x, v.y, v.z, v.w};
    }
    return *p;
}
__device__ __forceinline__ void store_block(W4 *p, const W4 &v) {
    if constexpr ((QGCM_NT_DATA & 2) != 0) {
        __builtin_nontemporal_store(u32x4u{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4u *>(p));
        return;
    }
    *p = v;
}

__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
    return __builtin_amdgcn_perm(s0, s1, sel);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32, truth table of a^b^c
}
__device__ __forceinline__ uint32_t rot16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint32_t lds32(uint32_t addr) { return *(const lds_u32 *)(size_t)addr; }
__device__ __forceinline__ uint4 lds128(uint32_t addr) {
    const u32x4 v = *(const lds_u128 *)(size_t)addr;
    return uint4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ void lds_st32(uint32_t addr, uint32_t v) { *(lds_u32 *)(size_t)addr = v; }
__device__ __forceinline__ void lds_st128(uint32_t addr, uint4 v) {
    *(lds_u128 *)(size_t)addr = u32x4{v.x, v.y, v.z, v.w};
}
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x2 lds_u64;
// volatile: keeps the two halves as two ds_read_b64 (the load/store optimizer would otherwise pair
// them into ds_read2_b64, two 4 x 16-lane accesses: 8 LDS cycles instead of 2 x 2)
__device__ __forceinline__ u32x2 lds64(uint32_t addr) { return *(const volatile lds_u64 *)(size_t)addr; }

// GHASH 4-bit comb tables in LDS (descriptor per-wave kernel, latency kernel): entry e = 16 p + v
// (nibble position p, value v) is 16 B at base + 16 e, read by one ds_read_b128 (4 x 16-lane groups;
// at 12 waves/CU this measured 1.2% faster than two ds_read_b64 halves).
__device__ __forceinline__ void lds_st_comb(uint32_t base, uint32_t e, uint4 v) { lds_st128(base + e * 16u, v); }

// Te0[byte k of s] / Te1[byte k of s] from this lane's replica.
// v_perm: result byte0 = lb.byte0 (lane*4), byte1 = s.byte k, bytes 2,3 = 0.
#define TA(s, k) perm((s), lb, 0x0c0c0400u + ((k) << 8))
#define TE0(s, k) lds32(TA(s, k))
#define TE1(s, k) lds32(TA(s, k) + 128u)

// T-table addressing, parameterised for the quad kernel's engines: kB = LDS byte address of the
// tables (an immediate ds offset, so free), kAO = byte-1 lookups address by one all-VGPR AND-OR
// ((s & 0xff00) | lane base, m8 = 0xff00 held in a VGPR: ~2.7 cycles per wave64 instruction) instead
// of v_perm with an SGPR selector (~4.5 cycles; tools/microbench/valu_ops*.hip).
template <uint32_t kB, bool kAO>
struct TT {
    uint32_t lb, m8;
    __device__ __forceinline__ uint32_t a(uint32_t s, int k) const {
        if (kAO && k == 1) return __builtin_amdgcn_bitop3_b32(s, m8, lb, (0xf0 & 0xcc) | 0xaa);
        return perm(s, lb, 0x0c0c0400u + (k << 8));
    }
    __device__ __forceinline__ uint32_t t0(uint32_t s, int k) const { return lds32(a(s, k) + kB); }
    __device__ __forceinline__ uint32_t t1(uint32_t s, int k) const { return lds32(a(s, k) + kB + 128u); }
};
typedef TT<0, false> TT0;

struct Ctr {
    uint32_t K0, x3;          // round-1 column 0 without the varying term; rk0 word3 byte3
    uint32_t U0, U1, U2, U3;  // round-2 columns without the term that depends on column 0
};

// Round keys of one key slot: rk[0..59] (FIPS-197 words as LE column words) and
// rr[0..59] = rot16(rk) so that  a ^ rot16(b) ^ rk  =  a ^ rot16(b ^ rr)  costs two v_bitop3.
struct Keys {
    const uint32_t *rk;
    const uint32_t *rr;
};

// Wave priority while a round issues its 16 lookups (s_setprio n, back to 0 once they are issued):
// the instruction arbiter then favours waves about to feed the LDS over waves combining results, so
// the LDS queue runs dry less often.  Priority 1 on the full rounds: +1.9 / +3.4 / +4.6% on config 2
// in three in-process A/Bs (tools/ab_libs.py), +1.7% on config 3 (tools/ab_libs_desc.py); priority 2
// or 3, or also on the final round or the GHASH lookups, no better.  The values are
// compile-time knobs (-DQGCM_ROUND_PRIO=n etc., 0 = off) for side builds in those A/Bs.
#ifndef QGCM_ROUND_PRIO
#define QGCM_ROUND_PRIO 1
#endif
#ifndef QGCM_LAST_PRIO
#define QGCM_LAST_PRIO 0
#endif
#ifndef QGCM_GH_PRIO
#define QGCM_GH_PRIO 0
#endif

// One full AES round (SubBytes, ShiftRows, MixColumns, AddRoundKey) on LE column words:
// column c = Te0[s_c.b0] ^ Te1[s_c+1.b1] ^ rot16(Te0[s_c+2.b2] ^ Te1[s_c+3.b3]) ^ rk_c.
template <class A>
__device__ __forceinline__ void round_full(uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3, const Keys &k,
                                           int r, const A &t) {
    // All 16 lookups of the round are issued before the first combine (the asm is a scheduling
    // fence): up to 16 LDS reads in flight per wave instead of 1-2 under the 64-VGPR budget.
    // +2.9% on config 2 in an in-process A/B.
    if constexpr (QGCM_ROUND_PRIO > 0) __builtin_amdgcn_s_setprio(QGCM_ROUND_PRIO);
    const uint32_t a0 = t.t0(s2, 2), a1 = t.t1(s3, 3), a2 = t.t0(s3, 2), a3 = t.t1(s0, 3);
    const uint32_t a4 = t.t0(s0, 2), a5 = t.t1(s1, 3), a6 = t.t0(s1, 2), a7 = t.t1(s2, 3);
    const uint32_t c0 = t.t0(s0, 0), c1 = t.t1(s1, 1), c2 = t.t0(s1, 0), c3 = t.t1(s2, 1);
    const uint32_t c4 = t.t0(s2, 0), c5 = t.t1(s3, 1), c6 = t.t0(s3, 0), c7 = t.t1(s0, 1);
    asm volatile("" ::: "memory");
    if constexpr (QGCM_ROUND_PRIO > 0) __builtin_amdgcn_s_setprio(0);
    s0 = xor3(c0, c1, rot16(xor3(a0, a1, k.rr[4 * r + 0])));
    s1 = xor3(c2, c3, rot16(xor3(a2, a3, k.rr[4 * r + 1])));
    s2 = xor3(c4, c5, rot16(xor3(a4, a5, k.rr[4 * r + 2])));
    s3 = xor3(c6, c7, rot16(xor3(a6, a7, k.rr[4 * r + 3])));
}
__device__ __forceinline__ void round_full(uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3, const Keys &k,
                                           int r, uint32_t lb) {
    round_full(s0, s1, s2, s3, k, r, TT0{lb, 0});
}

// Final round (no MixColumns): S-box bytes are byte1/byte2 of Te0 and byte3 of Te1.
template <class A>
__device__ __forceinline__ void round_last(uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3, const Keys &k,
                                           const A &t) {
    const uint32_t *rk = k.rk + 56;
    // 16 lookups in flight, then combine (as round_full; +1.1% in an in-process A/B)
    if constexpr (QGCM_LAST_PRIO > 0) __builtin_amdgcn_s_setprio(QGCM_LAST_PRIO);
    const uint32_t a0 = t.t0(s1, 1), a1 = t.t0(s0, 0), a2 = t.t1(s3, 3), a3 = t.t0(s2, 2);
    const uint32_t b0 = t.t0(s2, 1), b1 = t.t0(s1, 0), b2 = t.t1(s0, 3), b3 = t.t0(s3, 2);
    const uint32_t c0 = t.t0(s3, 1), c1 = t.t0(s2, 0), c2 = t.t1(s1, 3), c3 = t.t0(s0, 2);
    const uint32_t d0 = t.t0(s0, 1), d1 = t.t0(s3, 0), d2 = t.t1(s2, 3), d3 = t.t0(s1, 2);
    asm volatile("" ::: "memory");
    if constexpr (QGCM_LAST_PRIO > 0) __builtin_amdgcn_s_setprio(0);
    s0 = xor3(perm(a0, a1, 0x0c0c0501u), perm(a2, a3, 0x07020c0cu), rk[0]);
    s1 = xor3(perm(b0, b1, 0x0c0c0501u), perm(b2, b3, 0x07020c0cu), rk[1]);
    s2 = xor3(perm(c0, c1, 0x0c0c0501u), perm(c2, c3, 0x07020c0cu), rk[2]);
    s3 = xor3(perm(d0, d1, 0x0c0c0501u), perm(d2, d3, 0x07020c0cu), rk[3]);
}
__device__ __forceinline__ void round_last(uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3, const Keys &k,
                                           uint32_t lb) {
    round_last(s0, s1, s2, s3, k, TT0{lb, 0});
}

// Precompute rounds 1-2 for counter blocks nonce || (ctr_hi << 8 | low byte).  Round 1: only
// column 0 sees the varying byte (s3.b3, via Te3); round 2: each column sees exactly one byte
// of that column 0.
// the round-key words ctr_setup reads (rk[0..4], rk[9], rk[10]; rr[5..8], rr[11]), so a caller can
// load them ahead (the latency engine does, before its staging barrier)
struct SetupKeys {
    uint32_t rk0, rk1, rk2, rk3, rk4, rr5, rr6, rr7, rr8, rk9, rk10, rr11;
};
__device__ __forceinline__ SetupKeys setup_keys(const Keys &k) {
    return SetupKeys{k.rk[0], k.rk[1], k.rk[2], k.rk[3], k.rk[4], k.rr[5],
                     k.rr[6], k.rr[7], k.rr[8], k.rk[9], k.rk[10], k.rr[11]};
}
template <class A>
__device__ __forceinline__ void ctr_setup(Ctr &c, uint32_t n0, uint32_t n1, uint32_t n2, uint32_t ctr_hi,
                                          const SetupKeys &k, const A &t) {
    const uint32_t s0 = n0 ^ k.rk0, s1 = n1 ^ k.rk1, s2 = n2 ^ k.rk2;
    const uint32_t s3 = bswap(ctr_hi << 8) ^ k.rk3;  // byte3 varies per block; unused below
    c.x3 = k.rk3 >> 24;
    c.K0 = xor3(t.t0(s0, 0), t.t1(s1, 1), rot16(t.t0(s2, 2))) ^ k.rk4;
    const uint32_t t1 = xor3(t.t0(s1, 0), t.t1(s2, 1), rot16(xor3(t.t0(s3, 2), t.t1(s0, 3), k.rr5)));
    const uint32_t t2 = xor3(t.t0(s2, 0), t.t1(s3, 1), rot16(xor3(t.t0(s0, 2), t.t1(s1, 3), k.rr6)));
    const uint32_t t3 = xor3(t.t0(s3, 0), t.t1(s0, 1), rot16(xor3(t.t0(s1, 2), t.t1(s2, 3), k.rr7)));
    c.U0 = t.t1(t1, 1) ^ rot16(xor3(t.t0(t2, 2), t.t1(t3, 3), k.rr8));
    c.U1 = xor3(t.t0(t1, 0), t.t1(t2, 1), rot16(t.t0(t3, 2))) ^ k.rk9;
    c.U2 = xor3(t.t0(t2, 0), t.t1(t3, 1), rot16(t.t1(t1, 3))) ^ k.rk10;
    c.U3 = t.t0(t3, 0) ^ rot16(xor3(t.t0(t1, 2), t.t1(t2, 3), k.rr11));
}
template <class A>
__device__ __forceinline__ void ctr_setup(Ctr &c, uint32_t n0, uint32_t n1, uint32_t n2, uint32_t ctr_hi,
                                          const Keys &k, const A &t) {
    ctr_setup(c, n0, n1, n2, ctr_hi, setup_keys(k), t);
}
__device__ __forceinline__ void ctr_setup(Ctr &c, uint32_t n0, uint32_t n1, uint32_t n2, uint32_t ctr_hi,
                                          const Keys &k, uint32_t lb) {
    ctr_setup(c, n0, n1, n2, ctr_hi, k, TT0{lb, 0});
}

// E_K(nonce || ctr) for a counter whose high 24 bits match the cache; lo = ctr & 0xff.
template <class A, uint32_t kB>
__device__ __forceinline__ void ctr_block_t(const Ctr &c, uint32_t lo, const Keys &k, const A &t, uint32_t &s0,
                                            uint32_t &s1, uint32_t &s2, uint32_t &s3) {
    const uint32_t x = lo ^ c.x3;
    const uint32_t t0 = c.K0 ^ rot16(lds32(((x << 8) | t.lb) + kB + 128u));  // Te3[x]
    s0 = c.U0 ^ t.t0(t0, 0);
    s1 = c.U1 ^ rot16(t.t1(t0, 3));  // Te3[t0.b3]
    s2 = c.U2 ^ rot16(t.t0(t0, 2));  // Te2[t0.b2]
    s3 = c.U3 ^ t.t1(t0, 1);
#pragma unroll
    for (int r = 3; r < 14; ++r) round_full(s0, s1, s2, s3, k, r, t);
    round_last(s0, s1, s2, s3, k, t);
}
__device__ __forceinline__ void ctr_block(const Ctr &c, uint32_t lo, const Keys &k, uint32_t lb, uint32_t &s0,
                                          uint32_t &s1, uint32_t &s2, uint32_t &s3) {
    ctr_block_t<TT0, 0>(c, lo, k, TT0{lb, 0}, s0, s1, s2, s3);
}

// ---------------------------------------------------------------------------------------------
// AES-256 counter-block engines for the quad kernel.  Measured on gfx950 (tools/microbench/
// valu_ops*.hip, bitop3_forms.hip): v_perm_b32, v_alignbit_b32, shifts and ANY VALU op with an SGPR
// operand issue at ~4.5 cycles per wave-instruction per SIMD; v_bitop3_b32 / v_and / v_or / v_xor with
// VGPR operands only at ~2.7.  With the T-table round at 16 lookups (32 LDS cycles per wave per CU),
// the Tab2 round's 16 v_perm + 4 v_alignbit + 4 SGPR-keyed v_bitop3 (~120 SIMD-cycles = 30 CU-cycles
// per wave-round) nearly saturate the VALU as well as the LDS.
//  Tab2: Te0/Te1 in LDS (64 KiB), Te2/Te3 = rot16 folded into the column XOR, round keys in SGPRs,
//        byte-1 lookup addresses by one all-VGPR AND-OR; GHASH by the 4-bit comb of the wave's key
//        (descriptor per-wave kernel).  Round 2 measured four T-tables in LDS (128 KiB, no rotations,
//        all-VGPR XORs) 5% slower: one 16-wave workgroup per CU instead of two.
//  Tab2F: Tab2 with the 5-bit comb GHASH (single-key batches and the segmented kernel).
template <bool kFence>
__device__ __forceinline__ void ghash_mul(uint32_t &y0, uint32_t &y1, uint32_t &y2, uint32_t &y3, uint32_t gb);

struct Tab2 {
    Keys kk;
    TT<0, true> t;
    __device__ __forceinline__ void setup(Ctr &c, uint32_t n0, uint32_t n1, uint32_t n2, uint32_t hi) const {
        ctr_setup(c, n0, n1, n2, hi, kk, t);
    }
    __device__ __forceinline__ void block(const Ctr &c, uint32_t lo, uint32_t &k0, uint32_t &k1, uint32_t &k2,
                                          uint32_t &k3) const {
        ctr_block_t<TT<0, true>, 0>(c, lo, kk, t, k0, k1, k2, k3);
    }
    __device__ __forceinline__ void ghash(uint32_t &y0, uint32_t &y1, uint32_t &y2, uint32_t &y3, uint32_t gb) const {
        ghash_mul<true>(y0, y1, y2, y3, gb);
    }
};

// GHASH multiply by the uniform H^4 through a 5-bit comb (single-key batches, engine Tab2F).  The
// 128 bits of Y (LE words y0..y3, bit t = bit t%32 of word t/32) are cut into 26 windows of 5 bits
// (the last has 3); window i's table holds, for each of its 32 values v, the product with H^4 of the
// element whose only bits are v at bits 5i..5i+4, as two 8-B halves: words 0-1 at 512 i + 8 v, words
// 2-3 at 512 i + 256 + 8 v.  A half-table is one 256-B bank row, so the 32 lanes of a ds_read_b64
// lane group read any 32 values without a conflict (64 banks for b64: MI355X_MICROARCH.md "LDS"),
// and the address of window i is ((Y >> (5i mod 32 - 3)) & 0xf8): one shift and one all-VGPR AND,
// its table offset an immediate.  26 x 2 ds_read_b64 = 52 LDS cycles per multiply against 64 for the
// 4-bit comb (2 x 32 ds_read_b64), and 25 shifts + 26 ANDs instead of 48 v_perm/shift/AND-literal ops.
constexpr uint32_t kG5Windows = 26;
constexpr uint32_t kG5Bytes = kG5Windows * 512;  // 13 KiB, at LDS address 0 (T-tables after it)

template <int kI>
__device__ __forceinline__ uint32_t g5_addr(const uint32_t (&y)[4], uint32_t mf8) {
    constexpr int p = 5 * kI, w = p >> 5, o = p & 31;
    uint32_t x;
    if constexpr (o > 27 && w < 3)
        x = __builtin_amdgcn_alignbit(y[w + 1], y[w], o - 3);  // the window crosses into the next word
    else if constexpr (o > 3)
        x = y[w] >> (o - 3);
    else if constexpr (o < 3)
        x = y[w] << (3 - o);
    else
        x = y[w];
    return x & mf8;
}

template <int kLo, int kHi>
__device__ __forceinline__ void g5_chunk(const uint32_t (&y)[4], uint32_t mf8, uint32_t &a0, uint32_t &a1,
                                         uint32_t &a2, uint32_t &a3) {
    if constexpr (kLo < kHi) {
        if constexpr (QGCM_GH_PRIO > 0) __builtin_amdgcn_s_setprio(QGCM_GH_PRIO);
        const uint32_t x = g5_addr<kLo>(y, mf8);
        const u32x2 h0 = lds64(x + kLo * 512u), h1 = lds64(x + kLo * 512u + 256u);
        if constexpr (kLo + 1 < kHi) {
            const uint32_t x2 = g5_addr<kLo + 1>(y, mf8);
            const u32x2 l0 = lds64(x2 + (kLo + 1) * 512u), l1 = lds64(x2 + (kLo + 1) * 512u + 256u);
            if constexpr (QGCM_GH_PRIO > 0) __builtin_amdgcn_s_setprio(0);
            a0 = xor3(a0, h0.x, l0.x);
            a1 = xor3(a1, h0.y, l0.y);
            a2 = xor3(a2, h1.x, l1.x);
            a3 = xor3(a3, h1.y, l1.y);
            g5_chunk<kLo + 2, kHi>(y, mf8, a0, a1, a2, a3);
        } else {
            if constexpr (QGCM_GH_PRIO > 0) __builtin_amdgcn_s_setprio(0);
            a0 ^= h0.x;
            a1 ^= h0.y;
            a2 ^= h1.x;
            a3 ^= h1.y;
        }
    }
}

__device__ __forceinline__ void ghash_mul5(uint32_t &y0, uint32_t &y1, uint32_t &y2, uint32_t &y3, uint32_t mf8) {
    const uint32_t y[4] = {y0, y1, y2, y3};
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    // four chunks (7, 6, 7, 6 windows): at most 7 x 16 B of table rows live, as the 4-bit comb's 8
    g5_chunk<0, 7>(y, mf8, a0, a1, a2, a3);
    asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)::"memory");
    g5_chunk<7, 13>(y, mf8, a0, a1, a2, a3);
    asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)::"memory");
    g5_chunk<13, 20>(y, mf8, a0, a1, a2, a3);
    asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)::"memory");
    g5_chunk<20, 26>(y, mf8, a0, a1, a2, a3);
    y0 = a0;
    y1 = a1;
    y2 = a2;
    y3 = a3;
}

// Fills the 5-bit comb of H^4 at LDS address 0 from the key's 4-bit comb of H^4 (global, entry
// 16 p + v: nibble position p = 2 * byte (high nibble) or 2 * byte + 1 (low), value v): the product
// for bit t alone is entry p = 2 (t >> 3) + (t % 8 < 4), v = 1 << (t % 4); window entries are XORs
// of those (GHASH multiplication is linear).
__device__ __forceinline__ void g5_fill(const uint4 *__restrict__ comb4, uint32_t tid, uint32_t nthreads) {
    for (uint32_t e = tid; e < kG5Windows * 32u; e += nthreads) {
        const uint32_t i = e >> 5, v = e & 31u;
        // five unconditional loads in flight (an unset bit reads the all-zero entry v = 0 of its table)
        uint4 c[5];
#pragma unroll
        for (uint32_t j = 0; j < 5; ++j) {
            const uint32_t t = 5 * i + j, tt = t < 128u ? t : 127u;
            const uint32_t vv = (((v >> j) & 1u) && t < 128u) ? (1u << (tt & 3u)) : 0u;
            c[j] = comb4[16u * (2u * (tt >> 3) + ((tt & 7u) < 4u ? 1u : 0u)) + vv];
        }
        uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
        for (uint32_t j = 0; j < 5; ++j) {
            a0 ^= c[j].x;
            a1 ^= c[j].y;
            a2 ^= c[j].z;
            a3 ^= c[j].w;
        }
        *(lds_u64 *)(size_t)(512u * i + 8u * v) = u32x2{a0, a1};
        *(lds_u64 *)(size_t)(512u * i + 256u + 8u * v) = u32x2{a2, a3};
    }
}

// Tab2F: the Tab2 round with its tables at kG5Bytes (after the 5-bit comb), byte-1 addresses by an
// all-VGPR AND-OR, and GHASH by the 5-bit comb.  LDS 77 KiB per workgroup: two 16-wave workgroups
// per CU (32 waves/CU) as Tab2.
struct Tab2F {
    Keys kk;
    TT<kG5Bytes, true> t;
    uint32_t mf8;  // 0xf8 as a VGPR
    __device__ __forceinline__ void setup(Ctr &c, uint32_t n0, uint32_t n1, uint32_t n2, uint32_t hi) const {
        ctr_setup(c, n0, n1, n2, hi, kk, t);
    }
    __device__ __forceinline__ void block(const Ctr &c, uint32_t lo, uint32_t &k0, uint32_t &k1, uint32_t &k2,
                                          uint32_t &k3) const {
        ctr_block_t<TT<kG5Bytes, true>, kG5Bytes>(c, lo, kk, t, k0, k1, k2, k3);
    }
    __device__ __forceinline__ void ghash(uint32_t &y0, uint32_t &y1, uint32_t &y2, uint32_t &y3, uint32_t) const {
        ghash_mul5(y0, y1, y2, y3, mf8);
    }
};

// a VGPR the compiler cannot fold into a constant (an SGPR or literal operand costs half rate)
__device__ __forceinline__ uint32_t vreg(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}

// Y <- Y * H in GF(2^128) via the 4-bit comb in this wave's LDS table at gb (byte1/2 of gb hold
// its base; byte0 is 0).  Entry (p, v) at gb + p*256 + v*16, p = nibble position (2*byte for the
// high nibble, 2*byte+1 for the low one), v = nibble value.
// kFence = false (latency kernel, one wave): no chunk fences, so all 32 lookups can be in flight.
template <bool kFence = true>
__device__ __forceinline__ void ghash_mul(uint32_t &y0, uint32_t &y1, uint32_t &y2, uint32_t &y3, uint32_t gb) {
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    const uint32_t yw[4] = {y0, y1, y2, y3};
    // Four chunks of 8 lookups (one input word each): at most 8 x 16 B of results live, which is all
    // the LDS queue can overlap anyway (lgkmcnt tracks 15 in flight per wave).
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t hi = yw[w] & 0xf0f0f0f0u;
        const uint32_t lo = (yw[w] << 4) & 0xf0f0f0f0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = 4 * w + k;
            const uint4 th = lds128(perm(gb, hi, 0x0c060500u | k) + (2 * j) * 256);
            const uint4 tl = lds128(perm(gb, lo, 0x0c060500u | k) + (2 * j + 1) * 256);
            a0 = xor3(a0, th.x, tl.x);
            a1 = xor3(a1, th.y, tl.y);
            a2 = xor3(a2, th.z, tl.z);
            a3 = xor3(a3, th.w, tl.w);
        }
        // chunk fence: the accumulators are consumed here and the next chunk's LDS loads cannot be
        // hoisted above it, so at most 8 x 16 B of table rows are live at once
        if constexpr (kFence) asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)::"memory");
    }
    y0 = a0;
    y1 = a1;
    y2 = a2;
    y3 = a3;
}

// Y <- Y * H with the comb table read from global memory (L2/L1-resident, wave-uniform table):
// used for the few per-packet multiplies by H in the descriptor quad kernel, whose LDS holds only
// each wave's H^4 table.
__device__ __forceinline__ void ghash_mul_global(uint32_t &y0, uint32_t &y1, uint32_t &y2, uint32_t &y3,
                                                 const uint4 *__restrict__ T) {
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    const uint32_t yw[4] = {y0, y1, y2, y3};
    const char *base = reinterpret_cast<const char *>(T);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = 4 * w + k;
            const uint32_t oh = (yw[w] >> (8 * k)) & 0xf0u;
            const uint32_t ol = ((yw[w] >> (8 * k)) & 0x0fu) << 4;
            const uint4 th = *reinterpret_cast<const uint4 *>(base + (2 * j) * 256 + oh);
            const uint4 tl = *reinterpret_cast<const uint4 *>(base + (2 * j + 1) * 256 + ol);
            a0 = xor3(a0, th.x, tl.x);
            a1 = xor3(a1, th.y, tl.y);
            a2 = xor3(a2, th.z, tl.z);
            a3 = xor3(a3, th.w, tl.w);
        }
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)::"memory");
    }
    y0 = a0;
    y1 = a1;
    y2 = a2;
    y3 = a3;
}

// [len(A)]_64 || [len(C)]_64 times H from the global comb table of H: only the table rows of the
// nonzero bytes are read (word 1 holds len(A) <= 32 bits in its top byte, word 3 holds len(C)).
__device__ __forceinline__ void ghash_lenblock_global(uint32_t aad_len, uint32_t L, const uint4 *__restrict__ T,
                                                      uint32_t &y0, uint32_t &y1, uint32_t &y2, uint32_t &y3) {
    const char *base = reinterpret_cast<const char *>(T);
    const uint32_t w1 = bswap(aad_len * 8u), w3 = bswap(L * 8u);
    const uint32_t v[5] = {w1 >> 24, w3, w3 >> 8, w3 >> 16, w3 >> 24};
    const int j[5] = {7, 12, 13, 14, 15};  // comb table pair of word w, byte k: 4 w + k
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint4 th = *reinterpret_cast<const uint4 *>(base + (2 * j[i]) * 256 + (v[i] & 0xf0u));
        const uint4 tl = *reinterpret_cast<const uint4 *>(base + (2 * j[i] + 1) * 256 + ((v[i] & 0x0fu) << 4));
        a0 = xor3(a0, th.x, tl.x);
        a1 = xor3(a1, th.y, tl.y);
        a2 = xor3(a2, th.z, tl.z);
        a3 = xor3(a3, th.w, tl.w);
    }
    y0 = a0;
    y1 = a1;
    y2 = a2;
    y3 = a3;
}

__device__ __forceinline__ uint32_t sel4(uint32_t q, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return q == 0 ? a : (q == 1 ? b : (q == 2 ? c : d));
}
__device__ __forceinline__ uint32_t lowmask(uint32_t s) { return s ? (0xffffffffu >> (32 - 8 * s)) : 0u; }
__device__ __forceinline__ void store_bytes(uint8_t *p, uint32_t v, uint32_t nbytes) {
    if (nbytes > 0) p[0] = (uint8_t)v;
    if (nbytes > 1) p[1] = (uint8_t)(v >> 8);
    if (nbytes > 2) p[2] = (uint8_t)(v >> 16);
}
__device__ __forceinline__ uint32_t load_bytes(const uint8_t *p, uint32_t nbytes) {
    uint32_t v = 0;
    if (nbytes > 0) v |= p[0];
    if (nbytes > 1) v |= (uint32_t)p[1] << 8;
    if (nbytes > 2) v |= (uint32_t)p[2] << 16;
    return v;
}

// Reads the 28-byte tag||nonce that starts at byte L of data (any alignment; data 4-aligned).
// Out: tn[0..3] = tag words, tn[4..6] = nonce words (LE), and the s = L%4 bytes before it.
// NOTE: the packet kernels address LDS absolutely from 0, so they must own NO static LDS: the
// build passes -disable-promote-alloca-to-lds, tail values are plain scalars (no private arrays
// or structs left for the compiler to spill), and init_kernels() refuses a kernel whose static
// LDS size is not 0.

// Reads the 28-byte tag||nonce that starts at byte L of data (any alignment; data 4-aligned):
// tag words g0..g3, nonce words n0..n2 (LE), and the s = L%4 payload bytes before it (prefix).
__device__ __forceinline__ void read_tail(const uint8_t *data, uint32_t L, uint32_t &g0, uint32_t &g1, uint32_t &g2,
                                          uint32_t &g3, uint32_t &n0, uint32_t &n1, uint32_t &n2) {
    const uint32_t s = L & 3u;
    const uint32_t *t = reinterpret_cast<const uint32_t *>(data + (L & ~3u));
    const uint32_t w0 = t[0], w1 = t[1], w2 = t[2], w3 = t[3], w4 = t[4], w5 = t[5], w6 = t[6];
    const uint32_t w7 = load_bytes(data + (L & ~3u) + 28, s);
    g0 = __builtin_amdgcn_alignbyte(w1, w0, s);
    g1 = __builtin_amdgcn_alignbyte(w2, w1, s);
    g2 = __builtin_amdgcn_alignbyte(w3, w2, s);
    g3 = __builtin_amdgcn_alignbyte(w4, w3, s);
    n0 = __builtin_amdgcn_alignbyte(w5, w4, s);
    n1 = __builtin_amdgcn_alignbyte(w6, w5, s);
    n2 = __builtin_amdgcn_alignbyte(w7, w6, s);
}

// The two halves of read_tail: the quad kernel reads the nonce when the packet starts and the
// received tag only when it compares it (4 fewer VGPRs live across the block loop).
__device__ __forceinline__ void read_nonce(const uint8_t *data, uint32_t L, uint32_t &n0, uint32_t &n1, uint32_t &n2) {
    const uint32_t s = L & 3u;
    const uint32_t *t = reinterpret_cast<const uint32_t *>(data + (L & ~3u));
    const uint32_t w4 = t[4], w5 = t[5], w6 = t[6];
    const uint32_t w7 = load_bytes(data + (L & ~3u) + 28, s);
    n0 = __builtin_amdgcn_alignbyte(w5, w4, s);
    n1 = __builtin_amdgcn_alignbyte(w6, w5, s);
    n2 = __builtin_amdgcn_alignbyte(w7, w6, s);
}
__device__ __forceinline__ void read_tag(const uint8_t *data, uint32_t L, uint32_t &g0, uint32_t &g1, uint32_t &g2,
                                         uint32_t &g3) {
    const uint32_t s = L & 3u;
    const uint32_t *t = reinterpret_cast<const uint32_t *>(data + (L & ~3u));
    const uint32_t w0 = t[0], w1 = t[1], w2 = t[2], w3 = t[3], w4 = t[4];
    g0 = __builtin_amdgcn_alignbyte(w1, w0, s);
    g1 = __builtin_amdgcn_alignbyte(w2, w1, s);
    g2 = __builtin_amdgcn_alignbyte(w3, w2, s);
    g3 = __builtin_amdgcn_alignbyte(w4, w3, s);
}

// Writes prefix (s = L%4 bytes, the end of the payload) followed by tag||nonce at
// data + (L & ~3): 7 dwords + s bytes, never touching bytes past L+28.
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh);  // sh in [8, 32]
}
__device__ __forceinline__ void write_tail(uint8_t *data, uint32_t L, uint32_t g0, uint32_t g1, uint32_t g2,
                                           uint32_t g3, uint32_t n0, uint32_t n1, uint32_t n2, uint32_t prefix) {
    const uint32_t s = L & 3u;
    uint32_t *t = reinterpret_cast<uint32_t *>(data + (L & ~3u));
    const uint32_t sh = 32 - 8 * s;  // 32 when s == 0
    t[0] = (uint32_t)((((uint64_t)g0 << 32) | ((uint64_t)prefix << sh)) >> sh);
    t[1] = funnel(g1, g0, sh);
    t[2] = funnel(g2, g1, sh);
    t[3] = funnel(g3, g2, sh);
    t[4] = funnel(n0, g3, sh);
    t[5] = funnel(n1, n0, sh);
    t[6] = funnel(n2, n1, sh);
    if (s) store_bytes(data + (L & ~3u) + 28, n2 >> sh, s);
}

// ---------------------------------------------------------------------------------------------
// Quad kernel (single-key batches): FOUR lanes per packet.  Lane m of a quad owns the packet's
// 16-B blocks b = m, m+4, m+8, ... so every wave instruction moves 16 contiguous 64-B granules
// (one per packet) -- full-granule HBM traffic, and only 16 packets in flight per wave, which keeps
// 16 waves per CU within the caches.  GHASH runs as four interleaved Horner chains
// Z_m <- Z_m * H^4 ^ C_b (comb table of H^4), recombined once per packet:
//   Y = sum_m Z_m * H^(e_m)  ^  [len(A)]||[len(C)] * H,   e_m = d + 1 - b_last(m) in [2, 5],
// with the additional data A folded in as block -1 of lane 3 (SP 800-38D GHASH, restated for a
// 4-way interleave; checked against the oracle in tests).  E_K(J0) is computed by lane d % 4 in the
// slot where it has no data block.
__device__ __forceinline__ uint32_t quad_xor(uint32_t v) {
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
    return v;
}

// One packet of a quad tile (4 lanes, lane m owns blocks b = m mod 4): CTR + GHASH + tag, in place.
template <bool kSeal, class Eng>
__device__ __forceinline__ void quad_packet(const Batch &b, const Eng &eng, uint32_t pkt, uint64_t off, uint32_t L,
                                            uint32_t wkey, uint32_t m, uint32_t gH4) {
    const uint4 *Hg = b.gh_table + (size_t)wkey * kGhEntries;  // comb tables of H^k (global)
    uint8_t *raw = b.arena + off;
    uint8_t *data = raw + 4;  // common.PacketStart

    uint32_t g0 = 0, g1 = 0, g2 = 0, g3 = 0, n0, n1, n2;
    if (kSeal && b.nonces) {
        const uint32_t *np = reinterpret_cast<const uint32_t *>(b.nonces + 12ull * pkt);
        n0 = np[0];
        n1 = np[1];
        n2 = np[2];
    } else {
        read_nonce(data, L, n0, n1, n2);
    }
    const uint32_t nfull = L >> 4, r = L & 15u;
    const uint32_t d = nfull + (r ? 1u : 0u);  // data blocks incl. the partial one

    // lane 3 starts its chain with the additional data block (block -1)
    uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
    if (m == 3 && b.aad_len)
        z0 = *reinterpret_cast<const uint32_t *>(raw) & (b.aad_len >= 4 ? 0xffffffffu : lowmask(b.aad_len));
    int blast = -1;

    uint32_t e0 = 0, e1 = 0, e2 = 0, e3 = 0;  // E_K(J0)
    uint32_t prefix = 0;
    {
    Ctr cc;
    uint32_t hi = 0;
    eng.setup(cc, n0, n1, n2, 0);
    for (uint32_t bi = m; bi < nfull; bi += 4) {
        const uint32_t ctr = bi + 2;  // inc32(J0) + bi
        if ((ctr >> 8) != hi) {
            hi = ctr >> 8;
            eng.setup(cc, n0, n1, n2, hi);
        }
        // the data load is issued before the AES rounds so its latency hides behind them
        W4 *p = reinterpret_cast<W4 *>(data + 16u * bi);
        const W4 in = load_block(p);
        uint32_t k0, k1, k2, k3;
        eng.block(cc, ctr & 0xffu, k0, k1, k2, k3);
        const W4 out = {in.x ^ k0, in.y ^ k1, in.z ^ k2, in.w ^ k3};
        store_block(p, out);
        const W4 &c = kSeal ? out : in;
        eng.ghash(z0, z1, z2, z3, gH4);
        z0 ^= c.x;
        z1 ^= c.y;
        z2 ^= c.z;
        z3 ^= c.w;
        blast = (int)bi;
    }
    // One more slot: the partial last block (lane nfull % 4) and E_K(J0) (lane d % 4, the lane
    // with the fewest data blocks) share one AES pass.
    const bool part = r && (nfull & 3u) == m;
    if (part || m == (d & 3u)) {
        const uint32_t ctr = part ? nfull + 2 : 1u;  // inc32(J0) + nfull, or J0
        if ((ctr >> 8) != hi) {
            hi = ctr >> 8;
            eng.setup(cc, n0, n1, n2, hi);
        }
        uint32_t k0, k1, k2, k3;
        eng.block(cc, ctr & 0xffu, k0, k1, k2, k3);
        if (part) {
            uint8_t *blk = data + 16u * nfull;
            const W4 in = *reinterpret_cast<const W4 *>(blk);  // reads into tag area: inside the slot
            const uint32_t q = r >> 2, sb = r & 3u;
            const uint32_t o0 = in.x ^ k0, o1 = in.y ^ k1, o2 = in.z ^ k2, o3 = in.w ^ k3;
            uint32_t *bw = reinterpret_cast<uint32_t *>(blk);
            if (q > 0) bw[0] = o0;
            if (q > 1) bw[1] = o1;
            if (q > 2) bw[2] = o2;
            const uint32_t oq = sel4(q, o0, o1, o2, o3) & lowmask(sb);
            W4 c = kSeal ? W4{o0, o1, o2, o3} : in;
            if (kSeal)
                prefix = oq;  // written with tag||nonce by write_tail
            else
                store_bytes(blk + 4 * q, oq, sb);
            c.x &= q > 0 ? 0xffffffffu : lowmask(sb);
            c.y &= q > 1 ? 0xffffffffu : (q == 1 ? lowmask(sb) : 0u);
            c.z &= q > 2 ? 0xffffffffu : (q == 2 ? lowmask(sb) : 0u);
            c.w &= q == 3 ? lowmask(sb) : 0u;
            eng.ghash(z0, z1, z2, z3, gH4);
            z0 ^= c.x;
            z1 ^= c.y;
            z2 ^= c.z;
            z3 ^= c.w;
            blast = (int)nfull;
        } else {
            e0 = k0;
            e1 = k1;
            e2 = k2;
            e3 = k3;
        }
    }
    }
    // Y = sum_m Z_m * H^(e_m)  ^  ([len(A)]||[len(C)]) * H,  e_m = d + 1 - b_last(m) in [2, 5]
    // (a lane without blocks has Z_m = 0 or only the AAD block, b_last = -1, d <= 3).
    {
        const uint32_t em = d + 1u - (uint32_t)blast;
        const uint32_t tsel = em == 2 ? kGhH2 : em == 3 ? kGhH3 : em == 4 ? kGhH4 : kGhH5;
        ghash_mul_global(z0, z1, z2, z3, Hg + tsel);
        uint32_t l0, l1, l2, l3;
        ghash_lenblock_global(b.aad_len, L, Hg, l0, l1, l2, l3);
        z0 = quad_xor(z0) ^ l0;
        z1 = quad_xor(z1) ^ l1;
        z2 = quad_xor(z2) ^ l2;
        z3 = quad_xor(z3) ^ l3;
    }
    e0 = quad_xor(e0);
    e1 = quad_xor(e1);
    e2 = quad_xor(e2);
    e3 = quad_xor(e3);
    const uint32_t t0 = z0 ^ e0, t1 = z1 ^ e1, t2 = z2 ^ e2, t3 = z3 ^ e3;
    // the lane owning the partial block (or lane 0) writes the tail
    const uint32_t owner = r ? (nfull & 3u) : 0u;
    if (kSeal) {
        if (m == owner) {
            write_tail(data, L, t0, t1, t2, t3, n0, n1, n2, prefix);
            if (b.status) b.status[pkt] = 1;
        }
    } else {
        read_tag(data, L, g0, g1, g2, g3);  // the tag is never written by Open
        const bool ok = ((t0 ^ g0) | (t1 ^ g1) | (t2 ^ g2) | (t3 ^ g3)) == 0;
        if (!ok) {
            // Go 1.9 crypto/cipher gcm Open: zero the would-be plaintext on tag mismatch.
            for (uint32_t bi = m; bi < nfull; bi += 4) {
                const W4 zz = {0, 0, 0, 0};
                *reinterpret_cast<W4 *>(data + 16u * bi) = zz;
            }
            if (r && m == owner) {
                uint32_t *bw = reinterpret_cast<uint32_t *>(data + 16u * nfull);
                for (uint32_t w = 0; w < (r >> 2); ++w) bw[w] = 0;
                store_bytes(data + 16u * nfull + (r & ~3u), 0, r & 3u);
            }
        }
        if (b.status && m == 0) b.status[pkt] = ok ? 1 : 0;
    }
}

// kDesc = false: single-key (uniform) batches, engine Tab2F (5-bit comb of H^4 shared by the
// workgroup), two 16-wave workgroups per CU (32 waves/CU, 64 VGPRs).  kDesc = true: the per-wave
// descriptor kernel, engine Tab2 (each wave keeps the 4-bit comb of its current key's H^4 in its own
// 8 KiB of LDS), one 12-wave workgroup per CU; it takes the tiles of the keys too short for the
// segmented kernel (and every tile when QGCM_DESC_VARIANT=13).  Both recombine the four Horner chains
// once per packet by H^2..H^5 from the global key table (L2-resident), off the LDS pipe.
// Single-key batches: where a wave's next tile comes from.  0: static, wave w of workgroup g takes tiles
// g*16 + w + k*gridDim*16 (k = 0, 1, ...).  1: the same set of tiles per workgroup, shared by its 16
// waves through an LDS counter (index i -> tile g*16 + i%16 + (i/16)*gridDim*16, i ascending), so a wave
// that runs ahead takes more of its workgroup's tiles instead of idling while slower waves finish.
// 4 (default): mode 1 over the launch's first rows of tiles, then the last QGCM_TAIL_EIGHTHS eighths of
// its rows through one global counter that every wave of the grid draws from once its workgroup's rows
// are done (b.pool; NULL: mode 1 for all tiles).  The eight XCDs run at different speeds, so with each
// workgroup's share fixed the fastest XCD's CUs idled ~4% of a launch while the slowest finished
// (tools/quad_stats.py, profiles/r6_s18); with the shared tail every XCD ends within ~2%.  Tail of 4
// eighths: +2.1% at 3.7% fewer cycles per step against mode 1 (3: +1.6%, 5 and 6: +2.0%;
// tools/ab_steady.py, profiles/r6_s20).
#ifndef QGCM_TILE_POOL
#define QGCM_TILE_POOL 4
#endif
#ifndef QGCM_TAIL_EIGHTHS
#define QGCM_TAIL_EIGHTHS 4
#endif
constexpr uint32_t kPoolCtr = kG5Bytes + kTeBytes;  // LDS word after the uniform kernel's tables

// QGCM_QUAD_STATS (side builds only, tools/quad_stats.py): per-workgroup timeline of the uniform kernel
// in a device array (100 MHz clock): [0] start after the table fill, [1] the last wave's end, [2] the
// sum of the waves' ends, [3] tiles, [4] XCC id, [5] HW_ID, [6] 2^62 - the first wave's end.
#ifdef QGCM_QUAD_STATS
__device__ unsigned long long g_quad_stats[4096 * 8];
#endif

template <bool kDesc>
constexpr int quad_waves() { return kDesc ? 12 : 16; }
template <bool kDesc>
constexpr int quad_wpe() { return kDesc ? 3 : 8; }

template <bool kSeal, bool kDesc>
__global__ void __launch_bounds__(quad_waves<kDesc>() * 64) __attribute__((amdgpu_waves_per_eu(quad_wpe<kDesc>(),
                                                                                                  quad_wpe<kDesc>())))
gcm_quad_kernel(Batch b, const uint32_t *__restrict__ rk_table) {
    constexpr uint32_t kW = quad_waves<kDesc>();
    constexpr uint32_t kT = kW * 64;
    constexpr uint32_t kTeBase = kDesc ? 0u : kG5Bytes;  // Tab2F: the 5-bit comb first, then Te
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t m = lane & 3u;          // block residue owned by this lane
    const uint32_t qd = lane >> 2;         // packet slot within the wave tile (16 per wave)
    // the short-key pass of a segmented launch with no short keys: leave before the table fill
    if (kDesc && b.tile_list && __builtin_amdgcn_readfirstlane(*b.n_list) == 0) return;

    // dword i of the 64 KiB of T-tables: row x = i/64, slot i%64 (< 32: Te0, else Te1)
    for (uint32_t i = threadIdx.x; i < kTeBytes / 4; i += kT) {
        const uint32_t x = i >> 6, slot = i & 63u;
        lds_st32(kTeBase + 4 * i, b.te[(slot >> 5) * 256u + x]);
    }
    if constexpr (!kDesc) g5_fill(b.gh_table + (size_t)b.uniform_key * kGhEntries + kGhH4, threadIdx.x, kT);
    if constexpr (!kDesc && QGCM_TILE_POOL) {
        if (threadIdx.x == 0) lds_st32(kPoolCtr, kW);  // pool indices 0..kW-1: each wave's first tile
    }
#if QGCM_TILE_POOL == 4
    if constexpr (!kDesc) {
        if (threadIdx.x == 0) lds_st32(kPoolCtr + 12, 0u);  // waves of this workgroup done
    }
#endif
    __syncthreads();

    const uint32_t lb = (lane & 31u) << 2;
    // masks as VGPRs (an SGPR or literal operand issues at half rate)
    const uint32_t m8 = vreg(0x0000ff00u), mf8 = vreg(0x000000f8u);
    // descriptors: one H^4 table per wave after the T-tables (reloaded when the wave's key changes)
    const uint32_t gH4 = kDesc ? kTeBytes + wave * kGhBytes : 0u;
    uint32_t cur_key = kDesc ? 0xffffffffu : b.uniform_key;
    const uint32_t ntiles = kDesc ? (b.tile_list ? *b.n_list : b.n_items >> 4) : ((b.n + 15) >> 4);

#ifdef QGCM_QUAD_STATS
    unsigned long long *qs = g_quad_stats + (size_t)blockIdx.x * 8u;
    uint32_t qs_tiles = 0;
    if (!kDesc && threadIdx.x == 0) {
        qs[0] = wall_clock64();
        qs[4] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        qs[5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    }
#endif
#ifdef QGCM_QUAD_STATS
#define QS_TILE() ++qs_tiles
#define QS_END()                                                  \
    do {                                                          \
        if (!kDesc && lane == 0) {                                \
            const unsigned long long t_ = wall_clock64();         \
            atomicMax(&qs[1], t_);                                \
            atomicAdd(&qs[2], t_);                                \
            atomicAdd(&qs[3], (unsigned long long)qs_tiles);      \
            atomicMax(&qs[6], (1ull << 62) - t_);                 \
        }                                                         \
    } while (0)
#else
#define QS_TILE() do { } while (0)
#define QS_END() do { } while (0)
#endif
#if QGCM_TILE_POOL == 4
    // The launch's last rows of tiles through one global counter (b.pool, a zeroed set from the context's
    // ring, one per launch):
    // each workgroup first takes its own tiles of rows [0, srow) from its LDS counter as in mode 1, then
    // every wave draws from the shared tail [srow * grid * 16, ntiles), so the XCDs, which run at
    // different speeds (tools/quad_stats.py), end together instead of idling while the slowest finishes.
    // QGCM_TAIL_EIGHTHS: eighths of the full rows left to the tail (at least one when there are two).
    uint32_t sidx = 0xffffffffu, tail0 = 0;
    if constexpr (!kDesc) {
        const uint32_t rows = ntiles / (gridDim.x * kW);
        if (b.pool && rows > 0) {  // (no full row: each wave's first tile is all there is)
            const uint32_t tail_rows = rows < 2 ? 0u : std::min(rows - 1u, std::max(1u, rows * QGCM_TAIL_EIGHTHS / 8u));
            sidx = (rows - tail_rows) * kW;
            tail0 = (rows - tail_rows) * gridDim.x * kW;
        }
    }
#endif
    uint32_t tile = blockIdx.x * kW + wave;
    if constexpr (kDesc) {  // dynamic tiles: lengths vary by 100x between tiles
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(b.tile_counter, 1u);
        tile = __builtin_amdgcn_readfirstlane(__shfl(t, 0));
    }
    for (; tile < ntiles;) {
        uint32_t pkt, L;
        bool valid;
        uint64_t off;
        uint32_t wkey = cur_key;
        if constexpr (kDesc) {
            const uint32_t wt = b.tile_list ? b.tile_list[tile] : tile;
            pkt = b.worklist[wt * 16u + qd];
            valid = pkt != 0xffffffffu;
            qgcm_desc dsc = {0, 0, 0};
            if (valid) dsc = b.descs[pkt];
            off = dsc.offset;
            L = kSeal ? dsc.len : dsc.len - QGCM_OVERHEAD;  // open descriptors with len < 28 never get here
            const uint64_t vmask = __ballot(valid);
            if (vmask != 0) {
                wkey = __builtin_amdgcn_readfirstlane(__shfl(dsc.key_idx, __ffsll((unsigned long long)vmask) - 1));
                if (wkey != cur_key) {
                    const uint4 *src = b.gh_table + (size_t)wkey * kGhEntries + kGhH4;
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        const uint32_t e = r * 64 + lane;
                        lds_st_comb(gH4, e, src[e]);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    cur_key = wkey;
                }
            }
            // next tile (wave-uniform), fetched before this one's work
            uint32_t t = 0;
            if (lane == 0) t = atomicAdd(b.tile_counter, 1u);
            const uint32_t next = __builtin_amdgcn_readfirstlane(__shfl(t, 0));
            asm volatile("" : "+v"(L));
            if (!valid) {
                tile = next;
                continue;
            }
            tile = next;
        } else {
            pkt = tile * 16u + qd;
            L = b.uniform_len;
            // Opaque per tile: stops LICM from hoisting dozens of L-derived values (masks, selectors)
            // out of the tile loop, which would hold them in registers for the whole kernel.
            asm volatile("" : "+s"(L));
            valid = pkt < b.n;
            if (!kSeal) {
                if (L < (uint32_t)QGCM_OVERHEAD) valid = false;
                L -= QGCM_OVERHEAD;
            }
            off = (uint64_t)pkt * b.stride;
            if constexpr (QGCM_TILE_POOL) {
                // the next pool index, taken now so the LDS atomic's latency hides behind this tile
                uint32_t i = 0;
                if (lane == 0) i = __atomic_fetch_add((lds_u32 *)(size_t)kPoolCtr, 1u, __ATOMIC_RELAXED);
                i = __builtin_amdgcn_readfirstlane(i);
                tile = blockIdx.x * kW + (i % kW) + (i / kW) * gridDim.x * kW;
#if QGCM_TILE_POOL == 4
                if (i >= sidx) {  // this workgroup's rows are done: the launch's tail, shared
                    uint32_t c = 0;
                    if (lane == 0) c = atomicAdd(b.pool, 1u);
                    tile = tail0 + __builtin_amdgcn_readfirstlane(c);
                }
#endif
            } else {
                tile += gridDim.x * kW;
            }
            if (!valid) {
                if (!kSeal && b.status && pkt < b.n && m == 0) b.status[pkt] = 0;
                continue;  // the whole quad leaves together
            }
        }
        const Keys kk = {rk_table + (size_t)wkey * kRkWords, rk_table + (size_t)wkey * kRkWords + 64};
        if constexpr (kDesc) {
            quad_packet<kSeal>(b, Tab2{kk, {lb, m8}}, pkt, off, L, wkey, m, gH4);
        } else {
            quad_packet<kSeal>(b, Tab2F{kk, {lb, m8}, mf8}, pkt, off, L, wkey, m, gH4);
        }
        QS_TILE();
    }
    QS_END();
#if QGCM_TILE_POOL == 4
    // the last wave of the grid zeroes the pool set for the launch that next holds it
    if constexpr (!kDesc) {
        if (b.pool) {
            uint32_t last = 0;
            if (lane == 0 && __atomic_fetch_add((lds_u32 *)(size_t)(kPoolCtr + 12), 1u, __ATOMIC_RELAXED) == kW - 1) {
                __threadfence();
                last = atomicAdd(b.pool + kPoolDoneWord, 1u) == gridDim.x - 1u ? 1u : 0u;
            }
            if (lane == 0 && last) {
                __threadfence();
                b.pool[0] = 0;
                b.pool[kPoolDoneWord] = 0;
                // the set is free for the launch that next takes it from the ring: post this launch's
                // generation to the host word (that launch waits for it if it comes round early)
                __threadfence_system();
                __hip_atomic_store(b.pool_done, b.pool_gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
#endif
}
#undef QS_TILE
#undef QS_END

#ifdef QGCM_QUAD_STATS
extern "C" int qgcm_debug_quad_stats(unsigned long long *out, int n, int reset) {
    if (n > 4096 * 8) n = 4096 * 8;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_quad_stats), (size_t)n * 8) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long zero[4096 * 8];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_quad_stats), zero, sizeof(zero)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

// ---------------------------------------------------------------------------------------------
// Descriptor batches through the Tab2F engine (BASELINE config 3: any key mix, any lengths):
// gcm_seg_kernel.  The 5-bit comb of H^4 is 13 KiB, too large for one table per wave, so the
// sixteen waves of a workgroup share ONE key's table and work on one key run of the sorted worklist
// at a time.  A run's tiles are handed out by a global counter of that run (run_next), so any number
// of workgroups can work on one run together: a single-key batch is one queue for the whole GPU,
// longest tiles first, as the per-wave kernels' global tile queue.  Runs are first dealt out one per
// workgroup from a global cursor (each run gets an owner that stays on it until it is exhausted);
// once all are owned, a workgroup whose run is done helps: from its home position (its equal share
// of the tiles) it moves forward cyclically to the next run with at least QGCM_SEG_HELP_MIN tiles
// left, and leaves when there is none.  Moving to another run is a phase change: the waves meet at a
// barrier, wave 0 finds the run, and the table is refilled when the key changes.  Runs are sorted
// longest first, so the tiles drawn last from a run are short and the barrier wait is short; the
// other workgroup of the CU keeps the LDS busy while one waits.  LDS: [0, 13K) the 5-bit comb,
// [13K, 77K) Te, then the control words: 77 KiB per workgroup, two 16-wave workgroups per CU as the
// single-key kernel.
constexpr uint32_t kSegCtl = kG5Bytes + kTeBytes;  // run, phase key (LDS words)
constexpr uint32_t kSegLds = kSegCtl + 16u;
constexpr uint32_t kSegDone = 0xffffffffu;

__device__ __forceinline__ volatile lds_u32 *seg_ctl(uint32_t i) { return (volatile lds_u32 *)(size_t)(kSegCtl + 4u * i); }

// Wave-wide search: the first t in [lo, hi] with pred(t), for a pred that is monotone and true at hi
// (63 probes per step, one load round each).
template <class P>
__device__ __forceinline__ uint32_t wave_lower_bound(uint32_t lo, uint32_t hi, uint32_t lane, P pred) {
    while (hi - lo > 63u) {
        const uint32_t step = (hi - lo + 62u) / 63u;
        const uint32_t p = min(lo + lane * step, hi);
        const uint64_t msk = __ballot(pred(p));  // lane 63 probes hi
        const uint32_t f = (uint32_t)__ffsll((unsigned long long)msk) - 1u;
        if (f == 0) return lo;
        const uint32_t nlo = lo + (f - 1u) * step + 1u, nhi = min(lo + f * step, hi);
        lo = nlo;
        hi = nhi;
    }
    const uint64_t msk = __ballot(pred(min(lo + lane, hi)));
    return lo + (uint32_t)__ffsll((unsigned long long)msk) - 1u;
}

// QGCM_SEG_STATS (side builds only, tools/seg_stats.py): per-workgroup counters of the segmented
// kernel in a device array: phases, tiles, start/end (100 MHz clock), waves' idle and busy time,
// table fills, wave 0's time finding runs; [8] XCC id, [9] HW_ID (which CU).
#ifdef QGCM_SEG_STATS
__device__ unsigned long long g_seg_stats[4096 * 16];
#define SEG_STAT_ADD(i, v) \
    do { if (lane == 0) atomicAdd(&g_seg_stats[blockIdx.x * 16u + (i)], (unsigned long long)(v)); } while (0)
#define SEG_NOW() wall_clock64()
#else
#define SEG_STAT_ADD(i, v) do { } while (0)
#define SEG_NOW() 0ull
#endif

// Wave 0: the next run to work on, published with its key (kSegDone: no tiles left anywhere).
// First the runs are dealt out one by one from a global cursor (tile_counter[0]), so each has one
// owner while unowned runs remain; after that the workgroup helps: it takes the first run at or after
// r (cyclically; r starts at the workgroup's equal share of the tiles) that has enough tiles left.  (Helping
// any in-progress run before all are owned makes workgroups pile onto the same runs and move on
// together: many short phases.)
// A helper joins only a run with at least QGCM_SEG_HELP_MIN tiles left: fewer are finished by the
// run's owner (a run's owner works on it until it is exhausted, so no tile is left behind) within
// about one tile time, and joining would cost the helper a barrier and a table refill for little work.
// QGCM_SEG_START = 1: a helper's run search starts at a pseudo-random run (hash of the workgroup and
// its last run) instead of at the run it just left, so helpers that search at the same moment do not
// move as one convoy from run to run.
#ifndef QGCM_SEG_START
#define QGCM_SEG_START 1
#endif
#ifndef QGCM_SEG_HELP_MIN
#define QGCM_SEG_HELP_MIN 16
#endif
// QGCM_SEG_LAST = n > 0: when no run has QGCM_SEG_HELP_MIN tiles left (the launch's end), a helper joins a
// run with at least n unclaimed tiles rather than leave: its CU would idle otherwise (profiles/r6_s29).
#ifndef QGCM_SEG_LAST
#define QGCM_SEG_LAST 0
#endif
__device__ __forceinline__ void seg_next_phase(const Batch &b, uint32_t &r, uint32_t nruns, bool &helping,
                                               uint32_t lane) {
    uint32_t found = kSegDone;
    if (!helping) {
        uint32_t c = 0;
        if (lane == 0) c = atomicAdd(b.tile_counter, 1u);
        c = __builtin_amdgcn_readfirstlane(__shfl(c, 0));
        if (c < nruns)
            found = c;
        else
            helping = true;
    }
    if (helping) {
        if (QGCM_SEG_START) {  // a pseudo-random start per search: helpers spread over the runs
            const uint32_t h = (blockIdx.x * 0x9E3779B1u) ^ (r * 0x85EBCA6Bu + 0x632BE5ABu);
            r = (uint32_t)(((uint64_t)(h ^ (h >> 15)) * nruns) >> 32);
        }
        // four runs per lane per step (their loads in flight together): 256 runs per step
        for (uint32_t pass = 0, need = QGCM_SEG_HELP_MIN; pass < (QGCM_SEG_LAST ? 2u : 1u) && found == kSegDone;
             ++pass, need = QGCM_SEG_LAST ? QGCM_SEG_LAST : 1u)
        for (uint32_t base = 0; base < nruns; base += 256u) {
            bool left[4];
            uint32_t idx[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t o = base + 64u * j + lane;
                uint32_t i = r + o;
                i = i >= nruns ? i - nruns : i;  // r < nruns, and only offsets o < nruns look
                idx[j] = i;
                left[j] = false;
                if (o < nruns) {
                    const uint2 run = b.runs[i];
                    left[j] = __hip_atomic_load(b.run_next + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
                                  need <= run.y - run.x;
                }
            }
#pragma unroll
            for (uint32_t j = 0; j < 4 && found == kSegDone; ++j) {
                const uint64_t msk = __ballot(left[j]);
                if (msk) found = __builtin_amdgcn_readfirstlane(__shfl(idx[j], (int)__ffsll((unsigned long long)msk) - 1));
            }
            if (found != kSegDone) break;
        }
    }
    uint32_t key = kSegDone;
    if (found != kSegDone) {
        r = found;
        key = b.tile_keys[b.runs[found].x];
    }
    if (lane == 0) {
        *seg_ctl(0) = found;
        *seg_ctl(1) = key;
    }
}

// Side-build knob for A/Bs (tools/ab_libs_desc.py): QGCM_SEG_CLAIM tiles per atomic claim.
#ifndef QGCM_SEG_CLAIM
#define QGCM_SEG_CLAIM 1
#endif

template <bool kSeal>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8)))
gcm_seg_kernel(Batch b, const uint32_t *__restrict__ rk_table) {
    constexpr uint32_t kT = 1024;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t m = lane & 3u;
    const uint32_t qd = lane >> 2;
    // no key run long enough (every tile goes to the per-wave kernel): leave before the table fill
    if (__builtin_amdgcn_readfirstlane(*b.nruns) == 0) return;
    for (uint32_t i = threadIdx.x; i < kTeBytes / 4; i += kT) {
        const uint32_t x = i >> 6, slot = i & 63u;
        lds_st32(kG5Bytes + 4 * i, b.te[(slot >> 5) * 256u + x]);
    }
    const uint32_t lb = (lane & 31u) << 2;
    const uint32_t m8 = vreg(0x0000ff00u), mf8 = vreg(0x000000f8u);
    const uint32_t ntiles = b.n_items >> 4;
    uint32_t table_key = kSegDone;
    uint32_t r = 0, nruns = 0;  // wave 0: the current run
    bool helping = false;
    if (wave == 0) {
        nruns = *b.nruns;
        // home position: the workgroup's equal share of the tiles (where its help search starts)
        const uint32_t t = (uint32_t)((uint64_t)ntiles * blockIdx.x / gridDim.x);
        // the run holding tile t: the last run that begins at or before it
        const uint32_t i = wave_lower_bound(0u, nruns, lane, [&](uint32_t j) { return j == nruns || b.runs[j].x > t; });
        r = i ? i - 1u : 0u;
        SEG_STAT_ADD(6, r);
        SEG_STAT_ADD(8, __builtin_amdgcn_s_getreg((31 << 11) | 20));  // HW_REG_XCC_ID
        SEG_STAT_ADD(9, __builtin_amdgcn_s_getreg((31 << 11) | 4));   // HW_REG_HW_ID
    }
    __syncthreads();
    [[maybe_unused]] unsigned long long t_idle = SEG_NOW();
    if (wave == 0) SEG_STAT_ADD(2, t_idle);
    [[maybe_unused]] uint32_t ntile_stat = 0;
    for (;;) {
        if (wave == 0) {
            [[maybe_unused]] const unsigned long long t0 = SEG_NOW();
            seg_next_phase(b, r, nruns, helping, lane);
            SEG_STAT_ADD(7, SEG_NOW() - t0);
        }
        __syncthreads();
        if (wave == 0) SEG_STAT_ADD(0, 1);
        const uint32_t run = __builtin_amdgcn_readfirstlane(*seg_ctl(0));
        const uint32_t key = __builtin_amdgcn_readfirstlane(*seg_ctl(1));
        if (run == kSegDone) break;
        if (key != table_key) {
            g5_fill(b.gh_table + (size_t)key * kGhEntries + kGhH4, threadIdx.x, kT);
            table_key = key;
            __syncthreads();
        }
        [[maybe_unused]] const unsigned long long t_busy = SEG_NOW();
        SEG_STAT_ADD(4, t_busy - t_idle);
        const uint2 rt = b.runs[run];
        const Tab2F e3 = {{rk_table + (size_t)key * kRkWords, rk_table + (size_t)key * kRkWords + 64}, {lb, m8}, mf8};
        // QGCM_SEG_CLAIM consecutive tiles per atomic (1 unless set in a side build)
        for (uint32_t t = 0, left = 0;; ++t, --left) {
            if (left == 0) {
                uint32_t nx = 0;
                if (lane == 0) nx = atomicAdd(b.run_next + run, (uint32_t)QGCM_SEG_CLAIM);
                t = rt.x + __builtin_amdgcn_readfirstlane(__shfl(nx, 0));
                left = QGCM_SEG_CLAIM;
            }
            if (t >= rt.y) break;
            const uint32_t pkt = b.worklist[t * 16u + qd];
            if (pkt != 0xffffffffu) {  // the padding of a key run's last tile
                const qgcm_desc dsc = b.descs[pkt];
                const uint32_t L = kSeal ? dsc.len : dsc.len - QGCM_OVERHEAD;  // open: len >= 28 here
                quad_packet<kSeal, Tab2F>(b, e3, pkt, dsc.offset, L, key, m, 0u);
            }
            ++ntile_stat;
        }
        t_idle = SEG_NOW();
        SEG_STAT_ADD(5, t_idle - t_busy);
        __syncthreads();  // the table and the control words are free again
    }
    SEG_STAT_ADD(1, ntile_stat);
    if (wave == 0) SEG_STAT_ADD(3, SEG_NOW());
}

#ifdef QGCM_SEG_STATS
extern "C" int qgcm_debug_seg_stats(unsigned long long *out, int n, int reset) {
    if (n > 4096 * 16) n = 4096 * 16;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_seg_stats), (size_t)n * 8) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long zero[4096 * 16];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_seg_stats), zero, sizeof(zero)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

// ---------------------------------------------------------------------------------------------
// Latency kernel for ONE packet (qgcm_seal_one / qgcm_open_one, the per-call form of
// crypto/aes.go:41-62 behind plugin/encryption.go:22-37).  The batch kernels give a packet 1-4
// lanes and stream it from memory block by block; for a lone packet on pinned host memory that
// means ~85 serial PCIe round trips and 22-85 serial AES+GHASH steps per MTU packet (55 us of
// kernel at 1350 B).  Here one 512-thread workgroup (8 waves, one CU)
//  1. stages the whole slot [aad|data|tag|nonce] into LDS with one pass of 16-B loads (one memory
//     round trip) while it fills the T-tables and the comb tables this packet needs;
//  2. runs the counter blocks column-sliced up to kOneSliceMax blocks (a quad per block, lane q owns
//     state column q, 4 lookups per round and lane, DPP for the other columns), one lane per block
//     beyond (block d = E_K(J0));
//  3. runs GHASH on 64 chains of 8 lanes: chain c owns the blocks whose exponent in
//     Y = sum_i B_i H^(N+1-i) is c + 2 mod 64 (the AAD block included), a Horner chain by H^64,
//     then sum_c Z_c H^c by radix-2 Estrin levels (multiply by H^(2^l), add the partner chain's
//     product), then Y = S H^2 + [len(A)]||[len(C)] H -- 1 + 6 + 1 dependent multiplies at 1350 B
//     where the quad chains took 23; each multiply is split over the chain's 8 lanes (ghash_mul8).
//     The seven comb tables (H^(2^l), l = 0..6) sit in LDS;
//  4. writes the result with 16-B stores, overlapped with GHASH: a seal stores the ciphertext rows
//     before the tag as soon as the counter blocks are done, an open stores the plaintext straight
//     from the counter lanes (the staged ciphertext stays for GHASH) and, on a tag mismatch (rare),
//     overwrites it with zeros once those stores have landed (as Go 1.9 Open: zeroed plaintext).
// DESIGN.md 4.3 has the device-side timeline of each step.
// LDS: [0, 64K) Te, [64K, 120K) comb tables of H^(2^l), [120K, 120K + kOneCap) the slot at +12
// (payload 16-B aligned), 64 B of scratch (E_K(J0), the GHASH value), 2 KiB of GHASH exchange.
constexpr uint32_t kOneThreads = 512;
constexpr uint32_t kOneTabs = 7;
constexpr uint32_t kOneBuf = kTeBytes + kOneTabs * kGhBytes;
constexpr uint32_t kOneScratch = kOneBuf + kOneCap;  // [0, 16) E_K(J0), [16, 32) the GHASH value
constexpr uint32_t kOneX = kOneScratch + 64;         // GHASH Estrin exchange: 2 x 64 chains x 16 B
constexpr uint32_t kOneLds = kOneX + 2048;
constexpr uint32_t kOneSliceMax = kOneThreads / 4;  // counter blocks (J0 included) a column-sliced pass takes
static_assert(kOneLds <= 160u * 1024u, "gfx950 LDS is 160 KiB per workgroup");
// QGCM_RES_TRACE (side builds, tools/res_trace.sh): per served request the resident kernel adds the
// device-clock intervals poll -> input staged -> result computed -> result writes acknowledged to
// g_res_trace; one_packet stamps the middle two into LDS words past the resident control block.
#ifdef QGCM_RES_TRACE
constexpr uint32_t kResTrace = ((kOneLds + 15u) & ~15u) + 16;  // inside kResCtl's 64 B: [16, 48)
__device__ __forceinline__ void res_stamp(uint32_t slot, uint32_t by = 0) {
    if (threadIdx.x == by) {
        const uint64_t t = wall_clock64();
        lds_st32(kResTrace + 8 * slot, (uint32_t)t);
        lds_st32(kResTrace + 8 * slot + 4, (uint32_t)(t >> 32));
    }
}
#endif

typedef __attribute__((address_space(3))) uint8_t lds_u8;
__device__ __forceinline__ uint32_t lds8(uint32_t addr) { return *(const lds_u8 *)(size_t)addr; }
__device__ __forceinline__ void lds_st8(uint32_t addr, uint32_t v) { *(lds_u8 *)(size_t)addr = (uint8_t)v; }
// little-endian word at any LDS byte address
__device__ __forceinline__ uint32_t lds32u(uint32_t a) {
    return lds8(a) | lds8(a + 1) << 8 | lds8(a + 2) << 16 | lds8(a + 3) << 24;
}
__device__ __forceinline__ void lds_st32u(uint32_t a, uint32_t v) {
    lds_st8(a, v);
    lds_st8(a + 1, v >> 8);
    lds_st8(a + 2, v >> 16);
    lds_st8(a + 3, v >> 24);
}
// byte mask of the first r (< 16) bytes of a block, as four LE words
__device__ __forceinline__ void block_mask(uint32_t r, uint32_t &m0, uint32_t &m1, uint32_t &m2, uint32_t &m3) {
    const uint32_t q = r >> 2, sb = r & 3u;
    m0 = q > 0 ? 0xffffffffu : lowmask(sb);
    m1 = q > 1 ? 0xffffffffu : (q == 1 ? lowmask(sb) : 0u);
    m2 = q > 2 ? 0xffffffffu : (q == 2 ? lowmask(sb) : 0u);
    m3 = q == 3 ? lowmask(sb) : 0u;
}

// 16-B accesses of pinned host memory that go around the GPU caches (buffer instructions with sc0 sc1:
// a kernel that keeps running while the host rewrites the memory must not hit stale lines, and its
// results must reach the host without an L2 write-back).  A wave's 16-B lanes leave as whole 64-B
// requests; 8-B system-scope atomics cost about a round trip each (tools/microbench/hostmem.hip: a
// 1408-B request read and written back in 5.3 us vs 31.3 us).
constexpr int kSc0Sc1 = 1 | 16;  // cache-policy bits of the buffer intrinsics on gfx950: sc0 = 1, sc1 = 16
__device__ __forceinline__ uint4 host_ld16(const void *base, uint32_t bytes, uint32_t off) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)bytes, 0x00020000);
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, kSc0Sc1);
    return uint4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ void host_st16(void *base, uint32_t bytes, uint32_t off, uint4 v) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, r, (int)off, 0, kSc0Sc1);
}

// Slot access of the latency engine.  kSys = false: plain 16-B loads and stores (the slot is device
// memory, or pinned host memory handed over at a kernel launch).  kSys = true (the resident kernel,
// whose slots in pinned host memory are rewritten by the host while the kernel runs): host_ld16 /
// host_st16 within the kResSlotBytes slot.
template <bool kSys>
__device__ __forceinline__ uint4 slot_ld16(const uint8_t *slot, uint32_t i) {
    if constexpr (kSys) return host_ld16(slot, kResSlotBytes, 16 * i);
    return reinterpret_cast<const uint4 *>(slot)[i];
}
template <bool kSys>
__device__ __forceinline__ void slot_st16(uint8_t *slot, uint32_t i, uint4 v) {
    if constexpr (kSys) {
        host_st16(slot, kResSlotBytes, 16 * i, v);
        return;
    }
    reinterpret_cast<uint4 *>(slot)[i] = v;
}
// 16 B at a 4-B aligned byte offset of the slot (an open's plaintext block j at 4 + 16 j)
template <bool kSys>
__device__ __forceinline__ void slot_st16_at(uint8_t *slot, uint32_t off, uint4 v) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(slot, 0, (int)(kSys ? kResSlotBytes : kOneCap), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, r, (int)off, 0, kSys ? kSc0Sc1 : 0);
}

// Z <- Z * T on the 8 lanes e = 0..7 of one GHASH chain (the latency engine): lane e looks up the
// four 4-bit comb windows of bytes 2e and 2e+1 of Z (entry (p, v) at gb + 256 p + 16 v, as ghash_mul),
// then the chain's 8 partial products are XOR-reduced by DPP (quad_perm within each quad, then
// row_half_mirror across the two quads of the half-row), so every lane ends with the product.
__device__ __forceinline__ void ghash_mul8(uint32_t &z0, uint32_t &z1, uint32_t &z2, uint32_t &z3, uint32_t gb,
                                           uint32_t e) {
    const uint32_t w = e >> 1, k0 = 2u * (e & 1u);
    const uint32_t y = w == 0 ? z0 : w == 1 ? z1 : w == 2 ? z2 : z3;
    const uint32_t hi = y & 0xf0f0f0f0u, lo = (y << 4) & 0xf0f0f0f0u;  // nibble values x 16
    const uint32_t r0 = gb + 1024u * e;                                // rows 4e .. 4e+3
    const uint4 t0 = lds128(r0 + ((hi >> (8 * k0)) & 0xffu));
    const uint4 t1 = lds128(r0 + 256u + ((lo >> (8 * k0)) & 0xffu));
    const uint4 t2 = lds128(r0 + 512u + ((hi >> (8 * k0 + 8)) & 0xffu));
    const uint4 t3 = lds128(r0 + 768u + ((lo >> (8 * k0 + 8)) & 0xffu));
    uint32_t a0 = xor3(t0.x, t1.x, t2.x) ^ t3.x, a1 = xor3(t0.y, t1.y, t2.y) ^ t3.y;
    uint32_t a2 = xor3(t0.z, t1.z, t2.z) ^ t3.z, a3 = xor3(t0.w, t1.w, t2.w) ^ t3.w;
    a0 = quad_xor(a0);
    a1 = quad_xor(a1);
    a2 = quad_xor(a2);
    a3 = quad_xor(a3);
    z0 = a0 ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)a0, 0x141, 0xf, 0xf, false);  // row_half_mirror
    z1 = a1 ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)a1, 0x141, 0xf, 0xf, false);
    z2 = a2 ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)a2, 0x141, 0xf, 0xf, false);
    z3 = a3 ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)a3, 0x141, 0xf, 0xf, false);
}

// Workgroup barrier for LDS data only: __syncthreads() also waits for every outstanding global
// store (its release fence is s_waitcnt vmcnt(0)), and the latency engine's result stores go to host
// memory over PCIe while it keeps computing -- waiting for their acknowledgement at each barrier cost
// ~1.5 us per packet.  Only LDS is shared through these barriers; the caller orders the stores.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Fills the replicated T-tables (64 KiB at LDS 0): loads first, stores after (one memory latency).
__device__ __forceinline__ void one_fill_te(const uint32_t *te, uint32_t tid) {
    constexpr int kTeIt = kTeBytes / 16 / kOneThreads;  // 8
    uint32_t tv[kTeIt];
#pragma unroll
    for (int k = 0; k < kTeIt; ++k) {
        const uint32_t i = tid + k * kOneThreads;
        tv[k] = te[((i >> 3) & 1u) * 256u + (i >> 4)];
    }
#pragma unroll
    for (int k = 0; k < kTeIt; ++k) {
        const uint32_t i = tid + k * kOneThreads;
        lds_st128(16 * i, uint4{tv[k], tv[k], tv[k], tv[k]});
    }
}

// Word q of the counter block E_K(nonce || ctr), ctr < 256, column-sliced: the four lanes of a quad own
// the four columns of one block's state, each looks up 4 table entries per round instead of 16 and
// takes the other columns from its quad by DPP (a lone packet is bound by the rounds' latency, which
// this cuts, not by the tables).  All four lanes of the quad call it together.
// Column q's round keys (rounds 3..13 and the last), loaded by the caller ahead of other memory reads:
// a load's wait is in issue order, so round keys issued after a packet's table reads would wait for them.
struct ColKeys {
    uint32_t rq[11], rl;
    SetupKeys sk;
};
__device__ __forceinline__ void col_keys(const Keys &kk, uint32_t q, ColKeys &ck) {
#pragma unroll
    for (int i = 0; i < 11; ++i) ck.rq[i] = kk.rr[4 * (3 + i) + q];
    ck.rl = kk.rk[56 + q];
    ck.sk = setup_keys(kk);
}
__device__ __forceinline__ uint32_t ctr_sliced_word(const Keys &kk, const ColKeys &ck, uint32_t n0, uint32_t n1,
                                                    uint32_t n2, uint32_t ctr, uint32_t q, uint32_t lb) {
    const uint32_t *rq = ck.rq, rl = ck.rl;
    Ctr cc;
    ctr_setup(cc, n0, n1, n2, 0u, ck.sk, TT0{lb, 0});  // every counter here is below 256: one segment
    const uint32_t x = (ctr & 0xffu) ^ cc.x3;
    const uint32_t tv = cc.K0 ^ rot16(lds32(((x << 8) | lb) + 128u));  // as ctr_block_t
    const uint32_t kq = (4u - q) & 3u;  // byte of tv that column q looks up: 0, 3, 2, 1
    uint32_t sv = lds32(perm(tv, lb, 0x0c0c0400u + (kq << 8)) + ((q & 1u) ? 128u : 0u));
    if (q == 1 || q == 2) sv = rot16(sv);
    sv ^= q == 0 ? cc.U0 : q == 1 ? cc.U1 : q == 2 ? cc.U2 : cc.U3;
    const TT0 t{lb, 0};
    // column q of round rr: Te0[s_q.b0] ^ Te1[s_q+1.b1] ^ rot16(Te0[s_q+2.b2] ^ Te1[s_q+3.b3] ^ rr)
#pragma unroll
    for (int i = 0; i < 11; ++i) {
        const uint32_t s1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)sv, 0x39, 0xf, 0xf, false);
        const uint32_t s2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)sv, 0x4E, 0xf, 0xf, false);
        const uint32_t s3 = (uint32_t)__builtin_amdgcn_mov_dpp((int)sv, 0x93, 0xf, 0xf, false);
        const uint32_t c0 = t.t0(sv, 0), c1 = t.t1(s1, 1), a0 = t.t0(s2, 2), a1 = t.t1(s3, 3);
        asm volatile("" ::: "memory");
        sv = xor3(c0, c1, rot16(xor3(a0, a1, rq[i])));
    }
    const uint32_t s1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)sv, 0x39, 0xf, 0xf, false);
    const uint32_t s2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)sv, 0x4E, 0xf, 0xf, false);
    const uint32_t s3 = (uint32_t)__builtin_amdgcn_mov_dpp((int)sv, 0x93, 0xf, 0xf, false);
    const uint32_t a0 = t.t0(s1, 1), a1 = t.t0(sv, 0), a2 = t.t1(s3, 3), a3 = t.t0(s2, 2);
    asm volatile("" ::: "memory");
    return xor3(perm(a0, a1, 0x0c0c0501u), perm(a2, a3, 0x07020c0cu), rl);  // as round_last
}

// Keystream ahead (the resident kernel, seals): a worker that has been told the nonce of a slot's next
// seal computes, while it has nothing else to do, that nonce's counter blocks into LDS -- kKsBlocks
// blocks of 16 B, blocks 0 .. kKsBlocks-2 = E_K(inc32(J0) + j), the last E_K(J0) -- in the comb-table
// area, which packets on the flat GHASH (every packet up to 2016 B of a key with flat tables) leave
// unused; the seal that comes with that nonce then starts its GHASH right after staging.
constexpr uint32_t kKsBlocks = kOneThreads / 4;           // one quad per block: 2032 B of payload + J0
constexpr uint32_t kKsBytes = 16 * kKsBlocks;             // 2 KiB per slot
constexpr uint32_t kKsSlots = kOneTabs * kGhBytes / kKsBytes;  // 28 slots of a worker can hold one
__device__ __forceinline__ void ks_fill(const uint32_t *__restrict__ rk_table, uint32_t key, uint32_t n0, uint32_t n1,
                                        uint32_t n2, uint32_t dst) {
    const uint32_t tid = threadIdx.x, j = tid >> 2, q = tid & 3u, lb = (tid & 31u) << 2;
    const Keys kk = {rk_table + (size_t)key * kRkWords, rk_table + (size_t)key * kRkWords + 64};
    ColKeys ck;
    col_keys(kk, q, ck);
    lds_st32(dst + 16u * j + 4u * q, ctr_sliced_word(kk, ck, n0, n1, n2, j == kKsBlocks - 1u ? 1u : j + 2u, q, lb));
}

// One packet on one kOneThreads workgroup, tables already in LDS except (fill_te) the T-tables and the
// comb tables of H^(2^l) that this packet needs beyond what `tab_key` / `tab_n` say is loaded (both
// workgroup-uniform, updated here; a caller serving several packets puts a workgroup barrier
// between two calls).  The slot (16-B aligned, (4 + Lin (+ 28 for seal) + 15) & ~15
// bytes, checked by the caller) is staged in LDS, sealed or opened there and written back whole.
// nonce: seal only, 12 B, or NULL for the nonce already in the slot.  ks_tag / ks_lds (seal, resident
// kernel): a keystream computed ahead (ks_fill), used when its tag names this key and nonce.  Returns
// the verdict (bit 0: 1 ok, 0 authentication failure; bit 1: the keystream ahead was used), the same
// on every thread.
template <bool kSeal, bool kSys>
__device__ uint32_t one_packet(const Batch &b, const uint32_t *__restrict__ rk_table, const uint8_t *in, uint8_t *out,
                               uint32_t Lin,
                               uint32_t key, uint32_t aad_len, const uint8_t *nonce, bool fill_te, uint32_t &tab_key,
                               uint32_t &tab_n, uint32_t ks_tag = 0, uint32_t ks_lds = 0) {
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t n16 = (uint32_t)((4ull + Lin + (kSeal ? QGCM_OVERHEAD : 0) + 15) >> 4);
    const uint32_t L = kSeal ? Lin : Lin - QGCM_OVERHEAD;
    const uint32_t A = kOneBuf + 12u, P = kOneBuf + 16u;  // slot base (AAD), payload base
    // 1. stage the slot: every load issued before the table fill, so the PCIe round trip overlaps it
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t i = tid + k * kOneThreads;
        if (i < n16) v[k] = slot_ld16<kSys>(in, i);
    }
    // the column-sliced counter blocks' round keys, before the table reads (see ColKeys)
    const Keys kk = {rk_table + (size_t)key * kRkWords, rk_table + (size_t)key * kRkWords + 64};
    const bool sliced = ((L + 15u) >> 4) + 1u <= kOneSliceMax;  // d + 1 blocks; workgroup-uniform
    ColKeys ck{};
    if (sliced) col_keys(kk, tid & 3u, ck);
    // The table fills load everything first and store after (one memory latency, not one per
    // iteration): Te0/Te1 words for 32 replicas per row, then the comb tables of H^(2^l) -- only the
    // ones this packet's GHASH reads (H^(2^l) for the Estrin levels up to bit-length(min(d + 2, 63)),
    // H^64 once a chain owns two exponents) and not loaded yet for this key.
    constexpr int kGhIt = kOneTabs * 512 / kOneThreads;  // 7
    const uint4 *gh = b.gh_table + (size_t)key * kGhEntries;
    const uint32_t emax = ((L + 15u) >> 4) + 2u;  // GHASH exponents 1 .. d + 2 (step 3)
    // flat GHASH (step 3) from the key's global tables of H^1 .. H^kPwPowers: no comb tables in LDS
    const bool flat = b.pw_table != nullptr && key < b.pw_keys && emax <= kPwPowers;  // workgroup-uniform
    const uint32_t ntabs = flat ? 0u : emax >= 64u ? kOneTabs : 32u - __builtin_clz(emax);
    const uint32_t t0 = key == tab_key ? tab_n : 0u;  // tables [0, t0) already hold this key's
    if (fill_te) one_fill_te(b.te, tid);
    if (ntabs > t0) {
        uint4 gv[kGhIt];
#pragma unroll
        for (int k = 0; k < kGhIt; ++k) {
            const uint32_t i = tid + k * kOneThreads, l = i >> 9;
            const uint32_t src = l == 0 ? kGhH : l == 1 ? kGhH2 : l == 2 ? kGhH4 : kGhH8 + (l - 3) * 512u;
            if (l >= t0 && l < ntabs) gv[k] = gh[src + (i & 511u)];
        }
#pragma unroll
        for (int k = 0; k < kGhIt; ++k) {
            const uint32_t i = tid + k * kOneThreads, l = i >> 9;
            if (l >= t0 && l < ntabs) lds_st_comb(kTeBytes + l * kGhBytes, i & 511u, gv[k]);
        }
        tab_key = key;
        tab_n = ntabs;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t i = tid + k * kOneThreads;
        if (i < n16) {
            const uint32_t a = A + 16 * i;
            lds_st32(a, v[k].x);
            lds_st32(a + 4, v[k].y);
            lds_st32(a + 8, v[k].z);
            lds_st32(a + 12, v[k].w);
        }
    }
    for (uint32_t i = tid + 4 * kOneThreads; i < n16; i += kOneThreads) {  // slots over 16 KiB
        const uint4 w = slot_ld16<kSys>(in, i);
        const uint32_t a = A + 16 * i;
        lds_st32(a, w.x);
        lds_st32(a + 4, w.y);
        lds_st32(a + 8, w.z);
        lds_st32(a + 12, w.w);
    }
    lds_barrier();
#ifdef QGCM_RES_TRACE
    if (kSys) res_stamp(0);
#endif

    const uint32_t lb = (lane & 31u) << 2;
    const uint32_t nfull = L >> 4, r = L & 15u;
    const uint32_t d = nfull + (r ? 1u : 0u);
    uint32_t n0, n1, n2;
    if (kSeal && nonce) {  // the nonce goes into the slot with the tag
        const uint32_t *np = reinterpret_cast<const uint32_t *>(nonce);
        n0 = np[0];
        n1 = np[1];
        n2 = np[2];
    } else {
        n0 = lds32u(P + L + 16);
        n1 = lds32u(P + L + 20);
        n2 = lds32u(P + L + 24);
    }
    uint32_t m0, m1, m2, m3;
    block_mask(r, m0, m1, m2, m3);
    // a seal whose nonce's keystream a resident worker computed ahead (ks_tag: {key + 1, nonce} in LDS,
    // ks_lds: the blocks; see ks_fill); flat packets have d + 2 <= kPwPowers, so d < kKsBlocks - 1
    const bool use_ks = kSeal && ks_tag && flat && lds32(ks_tag) == key + 1u && lds32(ks_tag + 4) == n0 &&
                        lds32(ks_tag + 8) == n1 && lds32(ks_tag + 12) == n2;  // workgroup-uniform

    // 2. Counter blocks; block d is E_K(J0) (into scratch), and emit(j, q, w) takes word q of block j's
    // keystream (masked to the payload in the partial block).  Packets of up to kOneSliceMax blocks
    // (2032 B) run column-sliced: the four lanes of a quad own the four columns of one block's state,
    // each looks up 4 table entries per round instead of 16 and takes the other columns from its quad
    // by DPP -- a lone packet is bound by the rounds' latency, which this cuts, not by the tables.
    // Longer packets: one lane per block (ctr_setup + ctr_block).
    auto ctr_run = [&](auto &&emit, auto &&emit4) {
        auto put = [&](uint32_t j, uint32_t q, uint32_t w) {
            if (j == d) {
                lds_st32(kOneScratch + 4 * q, w);
            } else {
                if (j == nfull) w &= q == 0 ? m0 : q == 1 ? m1 : q == 2 ? m2 : m3;
                emit(j, q, w);
            }
        };
        if (use_ks) {  // the keystream computed ahead for this nonce (resident kernel): LDS reads
            const uint32_t j = tid >> 2, q = tid & 3u;
            if (j <= d) put(j, q, lds32(ks_lds + 16u * (j == d ? kKsBlocks - 1u : j) + 4u * q));
        } else if (sliced) {
            const uint32_t j = tid >> 2, q = tid & 3u;
            if (j <= d) put(j, q, ctr_sliced_word(kk, ck, n0, n1, n2, j == d ? 1u : j + 2u, q, lb));  // quad-uniform
        } else {
            for (uint32_t j = tid; j <= d; j += kOneThreads) {
                const uint32_t ctr = j == d ? 1u : j + 2u;  // J0, or inc32(J0) + j
                Ctr cc;
                ctr_setup(cc, n0, n1, n2, ctr >> 8, kk, lb);
                uint32_t k0, k1, k2, k3;
                ctr_block(cc, ctr & 0xffu, kk, lb, k0, k1, k2, k3);
                if (j == d) {
                    lds_st128(kOneScratch, uint4{k0, k1, k2, k3});
                } else {
                    if (j == nfull) {
                        k0 &= m0;
                        k1 &= m1;
                        k2 &= m2;
                        k3 &= m3;
                    }
                    emit4(j, uint4{k0, k1, k2, k3});  // a whole block per lane: contiguous 16-B accesses
                }
            }
        }
    };

    // 3. GHASH over the staged ciphertext on all 512 threads, the hash into scratch + 16.  Chain c
    // (64 chains, 8 lanes each: lane e looks up the 4 comb windows of bytes 2e, 2e+1, and the chain's
    // lanes XOR their partial products by DPP, ghash_mul8) owns the blocks whose exponent in
    // Y = sum_i B_i H^(N+1-i) is c + 2 mod 64 (the AAD block included): a Horner chain by H^64, then
    // sum_c Z_c H^c by radix-2 Estrin levels (multiply by H^(2^l), add chain c + 2^l's product through
    // LDS), then Y = S H^2 + [len(A)]||[len(C)] H.  Every thread calls it (it has workgroup barriers).
    // the block of GHASH exponent ex in Y = sum_ex B_ex H^ex: the AAD block (ex = d + 2), the length
    // block (ex = 1), else ciphertext block d + 1 - ex (the partial one masked)
    auto gblock = [&](uint32_t ex) {
        if (ex == d + 2u) return uint4{aad_len ? lds32(A) & (aad_len >= 4 ? 0xffffffffu : lowmask(aad_len)) : 0u, 0u, 0u, 0u};
        if (ex == 1) return uint4{0u, bswap(aad_len * 8u), 0u, bswap(L * 8u)};
        const uint32_t bi = d + 1u - ex;
        uint4 cb = lds128(P + 16 * bi);
        if (bi == nfull) {
            cb.x &= m0;
            cb.y &= m1;
            cb.z &= m2;
            cb.w &= m3;
        }
        return cb;
    };
    // Flat GHASH for packets with d + 2 <= kPwPowers exponents: every product B_ex H^ex is independent,
    // looked up in the key's kPwBits-bit comb table of H^ex (global memory, pw_setup_kernel): chain c's
    // 8 lanes take ex = c + 1 and c + 65, lane e the windows e, e + 8, ... of the block (bits of the
    // GHASH bit stream, x^0 first).  One round of independent table reads replaces the Horner step and
    // the Estrin levels' dependent multiplies and barriers.  In three phases: flat_issue (the block reads
    // and table loads), flat_consume (their XOR; it waits for the loads, so it comes before this thread's
    // first global store -- vmcnt would wait for those too), flat_finish (the 512 partials XOR-reduced:
    // DPP within rows, readlane across them, LDS across waves).  An open issues the loads before its
    // counter blocks (the ciphertext is staged) and consumes them before its first plaintext store, so
    // the table latency hides behind the rounds.
    uint4 fr[2 * kPwLaneWins];
#pragma unroll
    for (int k = 0; k < 2 * (int)kPwLaneWins; ++k) fr[k] = uint4{0, 0, 0, 0};
    uint32_t fa0 = 0, fa1 = 0, fa2 = 0, fa3 = 0;
    bool fed = false;
    auto flat_issue = [&]() {
        const uint32_t c = tid >> 3, e = tid & 7u;
        const uint4 *pwk = b.pw_table + (size_t)key * kPwPowers * kPwEntries;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t x = c + 1u + 64u * h;
            if (x <= emax) {
                const uint4 cb = gblock(x);
                // the block as a big-endian bit stream: bit i of the stream is x^i
                const uint32_t s0 = bswap(cb.x), s1 = bswap(cb.y), s2 = bswap(cb.z), s3 = bswap(cb.w);
                const uint4 *t = pwk + (x - 1u) * kPwEntries;
#pragma unroll
                for (int k = 0; k < (int)kPwLaneWins; ++k) {
                    const uint32_t w = e + 8u * k;
                    if (w < kPwWin) {
                        const uint32_t o = w * kPwBits, jw = o >> 5;
                        const uint32_t hi = jw == 0 ? s0 : jw == 1 ? s1 : jw == 2 ? s2 : s3;
                        const uint32_t lo = jw == 0 ? s1 : jw == 1 ? s2 : jw == 2 ? s3 : 0u;
                        const uint64_t v = (uint64_t)hi << 32 | lo;
                        const uint32_t u = (uint32_t)(v >> (64u - kPwBits - (o & 31u))) & ((1u << kPwBits) - 1u);
                        fr[kPwLaneWins * h + k] = t[(w << kPwBits) + u];
                    }
                }
            }
        }
    };
    auto flat_consume = [&]() {
        uint4 a = fr[0];
#pragma unroll
        for (int k = 1; k < 2 * (int)kPwLaneWins; ++k) a = uint4{a.x ^ fr[k].x, a.y ^ fr[k].y, a.z ^ fr[k].z, a.w ^ fr[k].w};
        fa0 = a.x;
        fa1 = a.y;
        fa2 = a.z;
        fa3 = a.w;
        fed = true;
    };
    auto row_xor = [](uint32_t v) {  // XOR over the 16 lanes of each row, in every lane of it
        v = quad_xor(v);
        v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false);  // row_half_mirror
        v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xf, 0xf, false);  // row_mirror
        return __builtin_amdgcn_readlane(v, 0) ^ __builtin_amdgcn_readlane(v, 16) ^ __builtin_amdgcn_readlane(v, 32) ^
               __builtin_amdgcn_readlane(v, 48);
    };
    auto flat_finish = [&]() {
        if (!fed) flat_consume();
        const uint32_t r0 = row_xor(fa0), r1 = row_xor(fa1), r2 = row_xor(fa2), r3 = row_xor(fa3);
        if (lane == 0) lds_st128(kOneX + 16 * (tid >> 6), uint4{r0, r1, r2, r3});
        lds_barrier();
        if (tid == 0) {
            uint4 y = lds128(kOneX);
            for (uint32_t wv = 1; wv < kOneThreads / 64u; ++wv) {
                const uint4 q = lds128(kOneX + 16 * wv);
                y = uint4{y.x ^ q.x, y.y ^ q.y, y.z ^ q.z, y.w ^ q.w};
            }
            lds_st128(kOneScratch + 16, y);
        }
    };

    auto ghash = [&]() {
        if (flat) return flat_finish();
        const uint32_t c = tid >> 3, e = tid & 7u;
        uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
        // Exponents 1 (the length block) .. d + 2 (the AAD block; zero without additional data), so
        // Y = sum_c Z_c H^c with no multiply after the tree.  Chain c's exponents e = c (mod 64), highest
        // first (chain-uniform loop); chain 0's lowest is 64, hence its one more multiply by H^64.
        const uint32_t emax = d + 2u;
        const uint32_t ehi = c == 0 ? (emax & ~63u) : (c <= emax ? c + ((emax - c) & ~63u) : 0u);
        const uint32_t elo = c ? c : 64u;
        const uint32_t steps = ehi >= elo ? (ehi - elo) / 64u + 1u : 0u;  // ehi = 0: none
        for (uint32_t k = 0; k < steps; ++k) {
            const uint32_t ex = ehi - 64u * k;
            uint4 cb;
            if (ex == emax) {  // the additional data
                cb = uint4{aad_len ? lds32(A) & (aad_len >= 4 ? 0xffffffffu : lowmask(aad_len)) : 0u, 0u, 0u, 0u};
            } else if (ex == 1) {  // [len(A)]_64 || [len(C)]_64 in bits
                cb = uint4{0u, bswap(aad_len * 8u), 0u, bswap(L * 8u)};
            } else {  // ciphertext block d + 1 - ex
                const uint32_t bi = d + 1u - ex;
                cb = lds128(P + 16 * bi);
                if (bi == nfull) {
                    cb.x &= m0;
                    cb.y &= m1;
                    cb.z &= m2;
                    cb.w &= m3;
                }
            }
            if (k) ghash_mul8(z0, z1, z2, z3, kTeBytes + 6 * kGhBytes, e);  // H^64
            z0 ^= cb.x;
            z1 ^= cb.y;
            z2 ^= cb.z;
            z3 ^= cb.w;
        }
        if (c == 0 && steps) ghash_mul8(z0, z1, z2, z3, kTeBytes + 6 * kGhBytes, e);
        const uint32_t top = emax < 63u ? emax : 63u;
        const int levels = 32 - __builtin_clz(top);  // emax >= 2
        for (int l = 0; l < levels; ++l) {
            const uint32_t span = 1u << l;
            uint32_t p0 = z0, p1 = z1, p2 = z2, p3 = z3;
            if ((c & (2 * span - 1)) == span && c <= top) ghash_mul8(p0, p1, p2, p3, kTeBytes + l * kGhBytes, e);
            const bool take = (c & (2 * span - 1)) == 0;
            if (l < 3) {
                p0 = __shfl_down(p0, 8u << l, 64);
                p1 = __shfl_down(p1, 8u << l, 64);
                p2 = __shfl_down(p2, 8u << l, 64);
                p3 = __shfl_down(p3, 8u << l, 64);
            } else {
                const uint32_t xb = kOneX + 1024u * (l & 1);  // double-buffered: one barrier per level
                if (e == 0 && !take) lds_st128(xb + 16 * c, uint4{p0, p1, p2, p3});
                lds_barrier();
                if (take && c + span < 64u) {
                    const uint4 q = lds128(xb + 16 * (c + span));
                    p0 = q.x;
                    p1 = q.y;
                    p2 = q.z;
                    p3 = q.w;
                }
            }
            if (take && c + span <= top) {
                z0 ^= p0;
                z1 ^= p1;
                z2 ^= p2;
                z3 ^= p3;
            }
        }
        if (tid == 0) lds_st128(kOneScratch + 16, uint4{z0, z1, z2, z3});
    };

    auto row = [&](uint32_t i) {
        const uint32_t a = A + 16 * i;
        return uint4{lds32(a), lds32(a + 4), lds32(a + 8), lds32(a + 12)};
    };
    uint32_t ok = 1;
    if (kSeal) {
        ctr_run(
            [&](uint32_t j, uint32_t q, uint32_t w) {  // ciphertext into the staged payload
                const uint32_t a = P + 16 * j + 4 * q;
                lds_st32(a, lds32(a) ^ w);
            },
            [&](uint32_t j, uint4 k) {
                const uint4 cv = lds128(P + 16 * j);
                lds_st128(P + 16 * j, uint4{cv.x ^ k.x, cv.y ^ k.y, cv.z ^ k.z, cv.w ^ k.w});
            });
        lds_barrier();
#ifdef QGCM_RES_TRACE
        if (kSys) res_stamp(2);
#endif
        if (flat) {  // the table reads before the early stores (see flat_issue)
            flat_issue();
            flat_consume();
        }
        // the rows that end before the tag go out now; their stores complete while GHASH runs
        const uint32_t early = (4u + L) >> 4;
        for (uint32_t i = tid; i < early; i += kOneThreads) slot_st16<kSys>(out, i, row(i));
        ghash();
#ifdef QGCM_RES_TRACE
        if (kSys) res_stamp(3);
#endif
        lds_barrier();
        if (tid == 0) {
            const uint4 e = lds128(kOneScratch), y = lds128(kOneScratch + 16);
            lds_st32u(P + L, e.x ^ y.x);
            lds_st32u(P + L + 4, e.y ^ y.y);
            lds_st32u(P + L + 8, e.z ^ y.z);
            lds_st32u(P + L + 12, e.w ^ y.w);
            if (nonce) {
                lds_st32u(P + L + 16, n0);
                lds_st32u(P + L + 20, n1);
                lds_st32u(P + L + 24, n2);
            }
        }
        lds_barrier();
#ifdef QGCM_RES_TRACE
        if (kSys) res_stamp(1);
#endif
        for (uint32_t i = early + tid; i < n16; i += kOneThreads) slot_st16<kSys>(out, i, row(i));
        ok |= use_ks ? 2u : 0u;
    } else {
        // the plaintext goes straight from registers to the output (the staged ciphertext stays for
        // GHASH); on a tag mismatch it is overwritten with zeros below, once these stores have landed
        const __amdgpu_buffer_rsrc_t ro =
            __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)(kSys ? kResSlotBytes : kOneCap), 0x00020000);
        if (flat) flat_issue();  // the GHASH table reads run under the counter blocks
        ctr_run(
            [&](uint32_t j, uint32_t q, uint32_t w) {  // quads: four lanes store one block's 16 B together
                if (flat && !fed) flat_consume();
                const uint32_t off = 4 + 16 * j + 4 * q;
                __builtin_amdgcn_raw_buffer_store_b32(lds32(P + 16 * j + 4 * q) ^ w, ro, (int)off, 0,
                                                      kSys ? kSc0Sc1 : 0);
            },
            [&](uint32_t j, uint4 k) {
                const uint4 cv = lds128(P + 16 * j);
                slot_st16_at<kSys>(out, 4 + 16 * j, uint4{cv.x ^ k.x, cv.y ^ k.y, cv.z ^ k.z, cv.w ^ k.w});
            });
#ifdef QGCM_RES_TRACE
        if (kSys) res_stamp(3);
#endif
        ghash();
#ifdef QGCM_RES_TRACE
        if (kSys) res_stamp(2);
#endif
        lds_barrier();
        const uint4 e = lds128(kOneScratch), y = lds128(kOneScratch + 16);
        ok = ((e.x ^ y.x ^ lds32u(P + L)) | (e.y ^ y.y ^ lds32u(P + L + 4)) | (e.z ^ y.z ^ lds32u(P + L + 8)) |
              (e.w ^ y.w ^ lds32u(P + L + 12))) == 0;
#ifdef QGCM_RES_TRACE
        if (kSys) res_stamp(1);
#endif
        if (!ok) {  // Go 1.9 crypto/cipher gcm Open: zero the would-be plaintext on tag mismatch
            for (uint32_t jj = tid; jj < d; jj += kOneThreads) {
                const uint4 cv = lds128(P + 16 * jj);
                const uint4 z = jj == nfull ? uint4{cv.x & ~m0, cv.y & ~m1, cv.z & ~m2, cv.w & ~m3} : uint4{0, 0, 0, 0};
                lds_st128(P + 16 * jj, z);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the plaintext stores have landed
            __syncthreads();
            for (uint32_t jj = tid; jj < d; jj += kOneThreads) slot_st16_at<kSys>(out, 4 + 16 * jj, lds128(P + 16 * jj));
        }
    }
    return ok;
}

// One workgroup per packet: slot i at b.arena + i * b.stride, b.uniform_len = L (seal) or L + 28
// (open), b.uniform_key (a per-packet call is a batch of one).  Slots are 16-B aligned and
// (4 + len (+ 28 for seal) + 15) & ~15 bytes long, at most kOneCap - 16; seal nonces come from
// b.nonces (12 B per packet) when it is set, else from the slot.  b.status[packet] = verdict.
// With b.descs set (small keyed batches, run_descs_one), packet i is descs[i] instead: its record
// at a 16-B-aligned offset, no other record inside its 16-B-rounded staging area.
template <bool kSeal>
__global__ void __launch_bounds__(kOneThreads) gcm_one_kernel(Batch b, const uint32_t *__restrict__ rk_table) {
    const uint32_t tid = threadIdx.x;
    const uint32_t pkt = blockIdx.x;
    uint64_t off = (uint64_t)pkt * b.stride;
    uint32_t Lin = b.uniform_len, key = b.uniform_key;
    if (b.descs) {
        const qgcm_desc d = b.descs[pkt];
        off = d.offset;
        Lin = d.len;
        key = d.key_idx;
    }
    const uint32_t n16 = (uint32_t)((4ull + Lin + (kSeal ? QGCM_OVERHEAD : 0) + 15) >> 4);
    // as the batch kernels: a key index out of range or an open shorter than 28 B fails the packet
    // (slot untouched); so does a slot past the LDS staging area or misaligned (the host never sends one)
    if (key >= b.max_keys || !b.key_valid[key] || (!kSeal && Lin < (uint32_t)QGCM_OVERHEAD) || Lin >= kOneCap ||
        n16 * 16u > kOneCap - 16u || (off & 15u)) {
        if (tid == 0) {
            if (b.status) b.status[pkt] = 0;
            if (b.done) {  // the host waits on the flag
                __threadfence_system();
                *reinterpret_cast<volatile uint8_t *>(b.done) = 1;
            }
        }
        return;
    }
    uint32_t tab_key = 0xffffffffu, tab_n = 0;
    const uint32_t ok = one_packet<kSeal, false>(b, rk_table, b.arena + off, b.arena + off, Lin, key, b.aad_len,
                                                 kSeal && b.nonces ? b.nonces + 12ull * pkt : nullptr, true, tab_key,
                                                 tab_n);
    if (tid == 0 && b.status) b.status[pkt] = ok;
    if (b.done) {  // completion flag: every thread's stores reach the system before thread 0 sets it
        __threadfence_system();
        __syncthreads();
        if (tid == 0) {
            __threadfence_system();
            *reinterpret_cast<volatile uint8_t *>(b.done) = 1;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Resident per-packet service (resident.cpp; gcm_internal.h ResArgs has the protocol).  Each
// workgroup is a worker: it keeps gcm_one_kernel's T-tables in LDS for its whole life (and the comb
// tables of the key it served last); wave 0 polls the worker's request records, which the host writes
// into device memory over the BAR (one 16-B load per slot from the GPU's own HBM, no PCIe round trip),
// and the whole workgroup serves each new request: the input from device memory, the result into
// pinned host memory.  Measured (tools/microbench/barreq.hip, profiles/r3_s12): a 1408-B request
// served in 3.97 us per round trip from device memory against 6.22 us from pinned host memory; and
// against a build where one dispatcher wave polled for all workers and forwarded requests, direct
// polling served 414 K vs 300 K round trips/s from 16 threads (profiles/r3_s8/resident_sweep.txt).
constexpr uint32_t kResCtl = (kOneLds + 15u) & ~15u;  // LDS: [0] command, [8,16) pending mask
constexpr uint32_t kResDone = kResCtl + 64;           // the done sequence of each of the worker's slots
constexpr uint32_t kResRec = kResDone + 4 * kResMaxPerWorker;  // the request records being served
// keystream ahead (ks_fill), per slot below kKsSlots: {state, next nonce}; state 0: none, kKsPending |
// (key + 1): the nonce of the slot's next seal is known, (key + 1): its keystream is in LDS
constexpr uint32_t kResKs = kResRec + 16 * kResMaxPerWorker;
constexpr uint32_t kResLds = kResKs + 16 * kResMaxPerWorker;
constexpr uint32_t kKsPending = 0x80000000u;
static_assert(kPwPowers - 2 < kKsBlocks - 1, "a flat packet's counter blocks fit the keystream ahead");
static_assert(kResLds <= 160u * 1024u, "gfx950 LDS is 160 KiB per workgroup");
#ifdef QGCM_RES_TRACE
// per op (open 0, seal 1), sums of: poll -> staged, staged -> stamp 2, staged -> stamp 3, staged ->
// computed, computed -> acked, count, shader clocks and 100-MHz ticks poll -> acked.  Seal: stamp 2 =
// counter blocks done, 3 = GHASH done; open: 3 = counter blocks done (thread 0's), 2 = GHASH done.
__device__ unsigned long long g_res_trace[16];
#endif

__device__ __forceinline__ uint32_t ld_sys32(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <class T>
__device__ __forceinline__ T ld_agent(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_agent(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(kOneThreads) gcm_resident_kernel(Batch b, const uint32_t *__restrict__ rk_table,
                                                                   ResArgs a) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = blockIdx.x;
    const uint32_t S = a.workers * a.per_worker, P = a.per_worker, first = w * P;
    uint64_t *const ctl = reinterpret_cast<uint64_t *>(a.dev);  // [0] last activity, [1] shutdown, [2] left
    one_fill_te(b.te, tid);
    if (tid < P) lds_st32(kResDone + 4 * tid, ld_sys32(a.done + first + tid) >> 1);
    if (tid < P) lds_st32(kResKs + 16 * tid, 0u);
    uint32_t tab_key = 0xffffffffu, tab_n = 0, idle = 0;  // idle: wave 0's count of empty polls
    uint32_t hits = tid == 0 ? ld_sys32(a.hits + 16 * w) : 0u;  // seals served from a keystream ahead
    const uint32_t nks = P < kKsSlots ? P : kKsSlots;
    const uint64_t t_start = wall_clock64();
    __syncthreads();
    for (;;) {
        if (tid < 64) {  // one poll: every slot's record and the worker's stop word
            // all of a poll's loads are issued before any is used: one memory latency per poll, not
            // three or four in a row (records, stop word, shutdown word, last activity)
            uint4 m{0, 0, 0, 0};
            uint32_t stop = 0;
            uint64_t shut = 0, act = 0;
            if (lane < P) m = host_ld16(a.req, 16 * S, 16 * (first + lane));
            if (lane == 0) {
                stop = host_ld16(a.stop, 64u * a.workers, 64u * w).x;
                shut = ld_agent(ctl + 1);
                if (w == 0) act = ld_agent(ctl);  // last activity of any worker (0: none yet)
            }
            bool pend = false;
            if (lane < P) {
                pend = (m.x & 0x7fffffffu) != lds32(kResDone + 4 * lane);
                if (pend) lds_st128(kResRec + 16 * lane, m);
            }
            const uint64_t pm = __ballot(pend);
            if (lane == 0) {
                if (w == 0) {  // the instance's end: no request for idle_ticks, or life_ticks old
                    const uint64_t now = wall_clock64();
                    const int64_t q = (int64_t)(now - (act > t_start ? act : t_start));
                    if (q > (int64_t)a.idle_ticks || now - t_start > a.life_ticks) {
                        st_agent(ctl + 1, (uint64_t)1);
                        shut = 1;
                    }
                }
                stop |= shut != 0 ? 1u : 0u;
                lds_st32(kResCtl, stop ? 2u : pm ? 1u : 0u);
                lds_st32(kResCtl + 8, (uint32_t)pm);
                lds_st32(kResCtl + 12, (uint32_t)(pm >> 32));
            }
            stop = __builtin_amdgcn_readfirstlane(stop);
            if (pm) {
                idle = 0;
            } else if (!stop) {  // back off once quiet (the polls read HBM, not PCIe)
                if (++idle < 4096)
                    __builtin_amdgcn_s_sleep(1);
                else
                    __builtin_amdgcn_s_sleep(16);
            }
        }
        __syncthreads();
        const uint32_t cmd = lds32(kResCtl);  // 0: nothing to do, 1: serve, 2: serve, then leave
        uint64_t mask = lds32(kResCtl + 8) | (uint64_t)lds32(kResCtl + 12) << 32;
#ifdef QGCM_RES_TRACE
        uint64_t t_poll = wall_clock64();  // after the poll that found the requests
        uint64_t c_poll = clock64();       // shader clock, for the clock rate while serving
#endif
        if (cmd == 0) {  // idle: compute one announced nonce's keystream ahead (ks_fill)
            uint32_t jk = nks;
            for (uint32_t k = 0; k < nks; ++k)
                if (lds32(kResKs + 16 * k) & kKsPending) {
                    jk = k;
                    break;
                }
            if (jk < nks) {
                const uint4 t = lds128(kResKs + 16 * jk);
                ks_fill(rk_table, (t.x & ~kKsPending) - 1u, t.y, t.z, t.w, kTeBytes + kKsBytes * jk);
                tab_key = 0xffffffffu;  // the comb-table area now holds keystreams
                tab_n = 0;
                lds_barrier();
                if (tid == 0) lds_st32(kResKs + 16 * jk, t.x & ~kKsPending);
            }
            __syncthreads();  // every thread has read the command before wave 0 writes the next
            continue;
        }
        while (mask) {
            const uint32_t j = (uint32_t)__builtin_ctzll(mask);
            mask &= mask - 1;
            const uint32_t sl = first + j;
            const uint4 m = lds128(kResRec + 16 * j);
            const uint32_t q = m.x & 0x7fffffffu, op = m.y & 1u, aad = (m.y >> 1) & 0x7fu, Lin = m.z, key = m.w;
            const bool ahead = (m.y >> 8) & 1u;  // a seal that announces the slot's next nonce
            const uint64_t stage = (4ull + Lin + (op ? QGCM_OVERHEAD : 0) + 15) & ~15ull;
            const bool valid = aad <= 4u && key < b.max_keys && b.key_valid[key] &&
                               (op ? Lin < QGCM_MAX_PAYLOAD : Lin >= (uint32_t)QGCM_OVERHEAD) &&
                               stage <= kResSlotBytes && stage <= kOneCap - 16;
            uint32_t ok = 0;
            const uint8_t *in = a.in + (size_t)sl * kResSlotBytes;
            uint8_t *out = a.out + (size_t)sl * kResSlotBytes;
            // the announced nonce (the slot's last 16 B), read before the packet so its load overlaps it
            const bool announce = op && ahead && valid && j < nks && b.pw_table && key < b.pw_keys;
            uint4 nn{0, 0, 0, 0};
            if (announce && tid == 0) nn = host_ld16(in, kResSlotBytes, kResSlotBytes - 16);
            const uint32_t kt = op && j < nks ? kResKs + 16 * j : 0u;
            if (valid)
                ok = op ? one_packet<true, true>(b, rk_table, in, out, Lin, key, aad, nullptr, false, tab_key, tab_n, kt,
                                                 kTeBytes + kKsBytes * j)
                        : one_packet<false, true>(b, rk_table, in, out, Lin, key, aad, nullptr, false, tab_key, tab_n);
            const bool hit = (ok >> 1) & 1u;
            ok &= 1u;
            if (tab_n != 0 && tid < nks) {  // comb tables loaded over the keystreams ahead
                const uint32_t st = lds32(kResKs + 16 * tid);
                if (!(st & kKsPending)) lds_st32(kResKs + 16 * tid, 0u);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the result bytes have reached the host
            __syncthreads();
            if (tid == 0 && kt)  // this seal used (or outdated) the slot's keystream ahead; the next one's
                lds_st128(kt, announce ? uint4{kKsPending | (key + 1u), nn.x, nn.y, nn.z} : uint4{0, 0, 0, 0});
            if (tid == 0 && hit) __hip_atomic_store(a.hits + 16 * w, ++hits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#ifdef QGCM_RES_TRACE
            if (tid == 0 && valid) {
                const uint64_t t_end = wall_clock64();
                uint64_t ts[4];
                for (int k = 0; k < 4; ++k)
                    ts[k] = lds32(kResTrace + 8 * k) | (uint64_t)lds32(kResTrace + 8 * k + 4) << 32;
                unsigned long long *g = g_res_trace + 8 * op;
                atomicAdd(&g[0], (unsigned long long)(ts[0] - t_poll));
                atomicAdd(&g[1], (unsigned long long)(ts[2] - ts[0]));
                atomicAdd(&g[2], (unsigned long long)(ts[3] - ts[0]));
                atomicAdd(&g[3], (unsigned long long)(ts[1] - ts[0]));
                atomicAdd(&g[4], (unsigned long long)(t_end - ts[1]));
                atomicAdd(&g[5], 1ull);
                const uint64_t c_end = clock64();
                atomicAdd(&g[6], (unsigned long long)(c_end - c_poll));
                atomicAdd(&g[7], (unsigned long long)(t_end - t_poll));
                t_poll = t_end;  // the next pending request of this poll starts here
                c_poll = c_end;
            }
#endif
            if (tid == 0) {
                __hip_atomic_store(a.done + sl, q << 1 | ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                lds_st32(kResDone + 4 * j, q);
                __hip_atomic_fetch_max(ctl, wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        if (cmd == 2) break;
    }
    if (tid == 0) {  // the last workgroup to leave tells the host this instance is over
        const uint64_t n = __hip_atomic_fetch_add(ctl + 2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n + 1 == a.workers) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(a.over, a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

#ifdef QGCM_RES_TRACE
extern "C" int qgcm_debug_res_trace(unsigned long long out[16], int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_res_trace), 16 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_res_trace), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif

hipError_t launch_resident(const Batch &b, const ResArgs &a, hipStream_t s) {
    if (a.workers == 0 || a.per_worker == 0 || a.per_worker > kResMaxPerWorker) return hipErrorInvalidValue;
    void *args[] = {const_cast<Batch *>(&b), const_cast<uint32_t **>(&b.rk_table), const_cast<ResArgs *>(&a)};
    return hipLaunchKernel(reinterpret_cast<const void *>(&gcm_resident_kernel), dim3(a.workers),
                           dim3(kOneThreads), args, kResLds, s);
}

hipError_t launch_one(bool seal, const Batch &b, hipStream_t s) {
    if (b.n == 0 || ((uintptr_t)b.arena & 15)) return hipErrorInvalidValue;
    if (!b.descs) {  // uniform: slots that hold the 16-B-rounded staging area and fit it in LDS
        const uint64_t stage = (4ull + b.uniform_len + (seal ? QGCM_OVERHEAD : 0) + 15) & ~15ull;
        if ((b.n > 1 && (b.stride < stage || (b.stride & 15))) || stage > kOneCap - 16 ||
            (!seal && b.uniform_len < QGCM_OVERHEAD))
            return hipErrorInvalidValue;
    }
    void *args[] = {const_cast<Batch *>(&b), const_cast<uint32_t **>(&b.rk_table)};
    const void *k = seal ? reinterpret_cast<const void *>(&gcm_one_kernel<true>)
                         : reinterpret_cast<const void *>(&gcm_one_kernel<false>);
    return hipLaunchKernel(k, dim3(b.n), dim3(kOneThreads), args, kOneLds, s);
}

// Variant table: the three packet-kernel variants, named by their QGCM variant ids (qgcm_api.cpp).  The
// ids are the round-2 ones (the A/B variants measured then -- lane-per-packet, 4-bit-comb and four-table
// single-key kernels, folded J0, repeated-H recombination -- were removed in round 3; DESIGN.md keeps
// their numbers): 12 = single-key quad kernel (Tab2F), 13 = per-wave descriptor kernel (Tab2),
// 14 = segmented descriptor kernel (Tab2F) + 13 for the short keys.
struct Variant {
    const void *seal, *open;
    int waves;
    uint32_t lds;
    int wgs_per_cu;  // resident workgroups per CU the persistent grid is sized for
    bool desc;       // consumes the sorted 16-packet worklist (launch_quad_worklist)
    int complement;  // segmented: the per-wave variant that takes the short keys' tiles after it
};

// the three kernels, by slot; variant ids (12, 13, 14: the numbering of the A/B logs under profiles/ and
// of QGCM_VARIANT / QGCM_DESC_VARIANT) map onto them
static Variant g_variants[3];
static int variant_slot(int v) {
    return v == kVariantUniform ? 0 : v == kVariantDescWave ? 1 : v == kVariantDescQuad ? 2 : -1;
}

hipError_t init_kernels() {
    g_variants[0] = Variant{reinterpret_cast<const void *>(&gcm_quad_kernel<true, false>),
                                          reinterpret_cast<const void *>(&gcm_quad_kernel<false, false>),
                                          quad_waves<false>(), kG5Bytes + kTeBytes + 16u,
                                          quad_wpe<false>() * 4 / quad_waves<false>(), false, -1};
    g_variants[1] = Variant{reinterpret_cast<const void *>(&gcm_quad_kernel<true, true>),
                                           reinterpret_cast<const void *>(&gcm_quad_kernel<false, true>),
                                           quad_waves<true>(), kTeBytes + (uint32_t)quad_waves<true>() * kGhBytes,
                                           1, true, -1};
    g_variants[2] = Variant{reinterpret_cast<const void *>(&gcm_seg_kernel<true>),
                                           reinterpret_cast<const void *>(&gcm_seg_kernel<false>), 16, kSegLds, 2, true,
                                           kVariantDescWave};
    for (const Variant &v : g_variants) {
        if (!v.seal) continue;
        for (const void *k : {v.seal, v.open}) {
            hipFuncAttributes a;
            hipError_t e = hipFuncGetAttributes(&a, k);
            if (e != hipSuccess) return e;
            // absolute LDS addressing from 0 requires no static LDS in the packet kernels
            if (a.sharedSizeBytes != 0) return hipErrorInvalidKernelFile;
            e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, v.lds);
            if (e != hipSuccess) return e;
        }
    }
    for (const void *k : {reinterpret_cast<const void *>(&gcm_one_kernel<true>),
                          reinterpret_cast<const void *>(&gcm_one_kernel<false>),
                          reinterpret_cast<const void *>(&gcm_resident_kernel)}) {
        hipFuncAttributes a;
        hipError_t e = hipFuncGetAttributes(&a, k);
        if (e != hipSuccess) return e;
        if (a.sharedSizeBytes != 0) return hipErrorInvalidKernelFile;
        e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                k == reinterpret_cast<const void *>(&gcm_resident_kernel) ? kResLds : kOneLds);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

bool quad_pool_global() { return QGCM_TILE_POOL == 4; }
bool variant_valid(int v) { return variant_slot(v) >= 0 && g_variants[variant_slot(v)].seal != nullptr; }
int variant_waves(int v) { return g_variants[variant_slot(v)].waves; }
int variant_wgs_per_cu(int v) { return g_variants[variant_slot(v)].wgs_per_cu; }
bool variant_desc(int v) { return g_variants[variant_slot(v)].desc; }
int variant_complement(int v) { return g_variants[variant_slot(v)].complement; }

hipError_t launch_packets(bool seal, int variant, const Batch &b, int grid, hipStream_t s) {
    if (!variant_valid(variant)) return hipErrorInvalidValue;
    const Variant &v = g_variants[variant_slot(variant)];
    void *args[] = {const_cast<Batch *>(&b), const_cast<uint32_t **>(&b.rk_table)};
    return hipLaunchKernel(seal ? v.seal : v.open, dim3(grid), dim3(v.waves * 64), args, v.lds, s);
}

// ---------------------------------------------------------------------------------------------
// Key setup: crypto/aes.go:68-76 (aes.NewCipher + cipher.NewGCM).  One 256-thread workgroup per
// key: FIPS-197 key expansion, H = E_K(0^128), x^i * H for i < 128, then the 4-bit comb
// T_p[v] = sum over set bits of v (MSB = x^0) of x^(4p+k) * H.
__device__ __forceinline__ uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

__device__ inline void shift_x(uint8_t v[16]) {
    const int lsb = v[15] & 1;
    for (int j = 15; j > 0; --j) v[j] = (uint8_t)((v[j] >> 1) | (v[j - 1] << 7));
    v[0] >>= 1;
    if (lsb) v[0] ^= 0xe1;
}
__device__ inline uint4 pack16(const uint8_t v[16]) {
    uint4 w;
    w.x = v[0] | v[1] << 8 | v[2] << 16 | (uint32_t)v[3] << 24;
    w.y = v[4] | v[5] << 8 | v[6] << 16 | (uint32_t)v[7] << 24;
    w.z = v[8] | v[9] << 8 | v[10] << 16 | (uint32_t)v[11] << 24;
    w.w = v[12] | v[13] << 8 | v[14] << 16 | (uint32_t)v[15] << 24;
    return w;
}
// SP 800-38D Algorithm 1 on byte strings (key setup only).
__device__ inline void gf128_mul_bytes(const uint8_t X[16], const uint8_t Y[16], uint8_t Z[16]) {
    uint8_t z[16] = {0}, v[16];
    for (int i = 0; i < 16; ++i) v[i] = Y[i];
    for (int i = 0; i < 128; ++i) {
        if ((X[i >> 3] >> (7 - (i & 7))) & 1)
            for (int j = 0; j < 16; ++j) z[j] ^= v[j];
        shift_x(v);
    }
    for (int i = 0; i < 16; ++i) Z[i] = z[i];
}

__global__ void __launch_bounds__(256) key_setup_kernel(const uint8_t *keys, uint32_t first, uint32_t *rk_table,
                                                        uint4 *gh_table, const uint8_t *sbox_g) {
    __shared__ uint8_t sbox[256];
    __shared__ uint8_t rkb[240];
    constexpr int kT = kGhEntries / 512;
    __shared__ uint8_t hp[kT][16];  // H, H^4, H^2, H^3, H^5, H^8, H^16, H^32, H^64 (comb table order)
    __shared__ uint4 pw[kT][128];   // x^i * hp[t]
    const uint32_t kidx = blockIdx.x;
    const uint8_t *key = keys + 32u * kidx;
    sbox[threadIdx.x] = sbox_g[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 0; i < 32; ++i) rkb[i] = key[i];
        uint8_t rcon = 1;
        for (int i = 8; i < 60; ++i) {
            uint8_t t[4] = {rkb[4 * i - 4], rkb[4 * i - 3], rkb[4 * i - 2], rkb[4 * i - 1]};
            if (i % 8 == 0) {
                const uint8_t t0 = t[0];
                t[0] = sbox[t[1]] ^ rcon;
                t[1] = sbox[t[2]];
                t[2] = sbox[t[3]];
                t[3] = sbox[t0];
                rcon = xt(rcon);
            } else if (i % 8 == 4) {
                for (int j = 0; j < 4; ++j) t[j] = sbox[t[j]];
            }
            for (int j = 0; j < 4; ++j) rkb[4 * i + j] = rkb[4 * i - 32 + j] ^ t[j];
        }
        // H = E_K(0)
        uint8_t s[16], u[16];
        for (int i = 0; i < 16; ++i) s[i] = rkb[i];
        for (int round = 1; round <= 14; ++round) {
            for (int c = 0; c < 4; ++c)
                for (int r = 0; r < 4; ++r) u[r + 4 * c] = sbox[s[r + 4 * ((c + r) & 3)]];
            if (round != 14) {
                for (int c = 0; c < 4; ++c) {
                    const uint8_t a0 = u[4 * c], a1 = u[4 * c + 1], a2 = u[4 * c + 2], a3 = u[4 * c + 3];
                    const uint8_t all = a0 ^ a1 ^ a2 ^ a3;
                    s[4 * c + 0] = a0 ^ all ^ xt(a0 ^ a1);
                    s[4 * c + 1] = a1 ^ all ^ xt(a1 ^ a2);
                    s[4 * c + 2] = a2 ^ all ^ xt(a2 ^ a3);
                    s[4 * c + 3] = a3 ^ all ^ xt(a3 ^ a0);
                }
            } else {
                for (int i = 0; i < 16; ++i) s[i] = u[i];
            }
            for (int i = 0; i < 16; ++i) s[i] ^= rkb[16 * round + i];
        }
        // powers of H by SP 800-38D Algorithm 1 (bit-serial; setup only)
        for (int i = 0; i < 16; ++i) hp[0][i] = s[i];
        gf128_mul_bytes(s, s, hp[2]);            // H^2
        gf128_mul_bytes(hp[2], s, hp[3]);        // H^3
        gf128_mul_bytes(hp[2], hp[2], hp[1]);    // H^4
        gf128_mul_bytes(hp[1], s, hp[4]);        // H^5
        for (int t = 5; t < kT; ++t) gf128_mul_bytes(hp[t == 5 ? 1 : t - 1], hp[t == 5 ? 1 : t - 1], hp[t]);  // H^(2^(t-2))
    }
    __syncthreads();
    // x^i * H^k: multiply by x = shift toward higher bit index (right shift of the byte string),
    // reduce with R = 0xe1 || 0^120 (SP 800-38D Algorithm 1).
    if (threadIdx.x < kT) {
        uint8_t v[16];
        for (int i = 0; i < 16; ++i) v[i] = hp[threadIdx.x][i];
        for (int i = 0; i < 128; ++i) {
            pw[threadIdx.x][i] = pack16(v);
            shift_x(v);
        }
    }
    __syncthreads();
    const uint32_t slot = first + kidx;
    if (threadIdx.x < 64) {
        const int i = threadIdx.x;
        const uint32_t w = i < 60 ? (rkb[4 * i] | rkb[4 * i + 1] << 8 | rkb[4 * i + 2] << 16 |
                                     (uint32_t)rkb[4 * i + 3] << 24)
                                  : 0u;
        rk_table[(size_t)slot * kRkWords + i] = w;
        rk_table[(size_t)slot * kRkWords + 64 + i] = (w << 16) | (w >> 16);
    }
    // entries [512 t, 512 t + 512): comb table of hp[t]
    for (uint32_t e = threadIdx.x; e < kGhEntries; e += 256) {
        const uint32_t p = (e & 511u) >> 4, v = e & 15u;
        const uint4 *src = pw[e >> 9];
        uint4 acc = {0, 0, 0, 0};
        for (int k = 0; k < 4; ++k) {
            if ((v >> (3 - k)) & 1u) {
                const uint4 t = src[4 * p + k];
                acc.x ^= t.x;
                acc.y ^= t.y;
                acc.z ^= t.z;
                acc.w ^= t.w;
            }
        }
        gh_table[(size_t)slot * kGhEntries + e] = acc;
    }
}

hipError_t launch_key_setup(const uint8_t *d_keys, uint32_t first, uint32_t count, uint32_t *rk_table,
                            uint4 *gh_table, const uint8_t *d_sbox, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(key_setup_kernel, dim3(count), dim3(256), 0, s, d_keys, first, rk_table, gh_table, d_sbox);
    return hipGetLastError();
}

// The latency engine's flat GHASH tables (one_packet): the kPwBits-bit comb tables of H^1 .. H^kPwPowers
// of each key slot below pw_keys -- entry (window W, value u) = sum over the set bits k of u (MSB first)
// of x^(kPwBits W + k) * H^p, kPwEntries x 16 B per power (6 bits: 22 x 64 x 16 B = 22 KiB, 2.75 MiB
// per key, which the L2 holds; 8 bits had 64 KiB per power and 8 MiB per key).  One 256-thread
// workgroup per key, after key_setup_kernel (H is read back from the slot's 4-bit comb table of H:
// entry (p 0, v 8) = x^0 * H).  Powers by doubling levels, H^(t+1) = H^(t+1-2^l) * H^(2^l); then 16 powers
// at a time, x^i * H^k for i < 128 in LDS and the comb entries from them.
__global__ void __launch_bounds__(256) pw_setup_kernel(uint32_t first, const uint4 *gh_table, uint4 *pw,
                                                       uint32_t pw_keys) {
    __shared__ uint8_t hp[kPwPowers][16];  // H^1 .. H^128
    __shared__ uint4 xs[16][128];          // x^i * H^k for 16 powers of a batch
    const uint32_t slot = first + blockIdx.x, tid = threadIdx.x;
    if (slot >= pw_keys) return;  // workgroup-uniform
    if (tid == 0) {
        const uint4 h = gh_table[(size_t)slot * kGhEntries + kGhH + 8];
        const uint32_t w[4] = {h.x, h.y, h.z, h.w};
        for (int i = 0; i < 16; ++i) hp[0][i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
    __syncthreads();
    for (uint32_t span = 1; span < kPwPowers; span <<= 1) {
        if (tid >= span && tid < 2 * span && tid < kPwPowers) gf128_mul_bytes(hp[tid - span], hp[span - 1], hp[tid]);
        __syncthreads();
    }
    for (uint32_t b0 = 0; b0 < kPwPowers; b0 += 16) {
        {
            const uint32_t j = tid >> 4, i0 = 8 * (tid & 15u);
            uint8_t v[16];
            for (int i = 0; i < 16; ++i) v[i] = hp[b0 + j][i];
            for (uint32_t i = 0; i < i0; ++i) shift_x(v);
            for (uint32_t i = 0; i < 8; ++i) {
                xs[j][i0 + i] = pack16(v);
                shift_x(v);
            }
        }
        __syncthreads();
        for (uint32_t e = tid; e < 16u * kPwEntries; e += 256) {
            const uint32_t j = e / kPwEntries, q = e % kPwEntries, win = q >> kPwBits, u = q & ((1u << kPwBits) - 1u);
            uint4 acc = {0, 0, 0, 0};
            for (uint32_t k = 0; k < kPwBits; ++k) {
                const uint32_t i = win * kPwBits + k;  // the window's bit k (its MSB first) is x^i
                if (i < 128u && ((u >> (kPwBits - 1u - k)) & 1u)) {
                    const uint4 t = xs[j][i];
                    acc.x ^= t.x;
                    acc.y ^= t.y;
                    acc.z ^= t.z;
                    acc.w ^= t.w;
                }
            }
            pw[((size_t)slot * kPwPowers + b0 + j) * kPwEntries + q] = acc;
        }
        __syncthreads();
    }
}

hipError_t launch_pw_setup(uint32_t first, uint32_t count, const uint4 *gh_table, uint4 *pw, uint32_t pw_keys,
                           hipStream_t s) {
    if (count == 0 || !pw || first >= pw_keys) return hipSuccess;
    hipLaunchKernelGGL(pw_setup_kernel, dim3(count), dim3(256), 0, s, first, gh_table, pw, pw_keys);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Synthetic workload (BASELINE configs): splitmix64 stream bytes, random-access form.
__device__ __forceinline__ uint64_t splitmix_at(uint64_t seed, uint64_t k) {
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint8_t stream_byte(uint64_t seed, uint64_t b) {
    return (uint8_t)(splitmix_at(seed, b >> 3) >> (8 * (b & 7)));
}

__device__ __forceinline__ void fill_uniform_item(uint8_t *arena, uint64_t stride, uint32_t len, uint32_t groups,
                                                  uint32_t aad_word, uint64_t seed_payload, uint8_t *nonces,
                                                  uint64_t seed_nonce, uint64_t t) {
    const uint32_t slot = (uint32_t)(t / groups), g = (uint32_t)(t % groups);
    uint8_t *raw = arena + (uint64_t)slot * stride;
    const uint32_t dgroups = groups - 3;
    if (g < dgroups) {
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t pos = 4 * g + j;
            if (pos < 4) {
                raw[pos] = (uint8_t)(aad_word >> (8 * pos));
            } else if (pos < 4 + len) {
                raw[pos] = stream_byte(seed_payload, (uint64_t)slot * len + (pos - 4));
            }
        }
    } else if (nonces) {
        const uint32_t ng = g - dgroups;
        for (uint32_t j = 0; j < 4; ++j) {
            const uint64_t pos = 12ull * slot + 4 * ng + j;
            nonces[pos] = stream_byte(seed_nonce, pos);
        }
    }
}

// One work item per (slot, 4-byte group of the slot's first 4+L bytes), grid-stride: a dispatch's
// work-item count is a 32-bit field, and n x groups passes 2^32 at ~12.6 M slots of 1350 B (an
// unbounded grid silently filled only the first 2^32 items).
__global__ void fill_uniform_kernel(uint8_t *arena, uint64_t stride, uint32_t n, uint32_t len, uint32_t aad_word,
                                    uint64_t seed_payload, uint8_t *nonces, uint64_t seed_nonce) {
    const uint32_t groups = (4 + len + 3) / 4 + 3;  // +3 groups for the 12-byte nonce
    const uint64_t total = (uint64_t)n * groups, step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += step)
        fill_uniform_item(arena, stride, len, groups, aad_word, seed_payload, nonces, seed_nonce, t);
}

// Streaming copy: the achievable-HBM reference the roofline is also quoted against (SURVEY.md s8d
// "measure the achievable copy bandwidth with an in-repo stream kernel").  One 16-B non-temporal load and
// store per lane, one 4-KiB tile per 256-thread workgroup, a grid that covers the buffer (no loop).
// tools/microbench/copy.hip timed twelve shapes in one process on random data (profiles/r6_s2): this one
// 6.52 TB/s read + write on a 1.48-GB buffer and 6.47 on 8 GB; the round-5 form (grid-stride, each lane's
// four loads a grid apart, 8 workgroups per CU) 4.45 / 4.80, the same tile shape with cached accesses
// 5.73 / 5.61 and with four 16-B pieces per lane 5.87 / 5.75.
__global__ void __launch_bounds__(256) stream_copy_kernel(uint4 *__restrict__ dst, const uint4 *__restrict__ src,
                                                          uint64_t n16) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));  // the builtins take native vector types
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i < n16)
        __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const v4 *>(src) + i),
                                    reinterpret_cast<v4 *>(dst) + i);
}

// Record moves for the group dispatcher's zero-copy path (group.cpp): one wave per record copies
// `bytes` from src to dst (both 4-B aligned) with 16-B accesses, the rest by dwords.  Gather (pinned host -> device
// staging): the last dword may read up to 3 bytes past the record, never past a 4-B boundary, so
// never past the host allocation; the staging records are 16-B padded.  Scatter (staging -> pinned
// host): whole dwords, then the 0-3 tail bytes one by one, so nothing beyond the record is written;
// a move whose status byte is not 1 is skipped when `status` is given (a failed seal leaves the
// caller's slot untouched).
__global__ void __launch_bounds__(256) move_records_kernel(const RecMove *__restrict__ mv, uint32_t n,
                                                           const uint8_t *__restrict__ status, bool exact) {
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t r = blockIdx.x * 4u + (threadIdx.x >> 6); r < n; r += gridDim.x * 4u) {
        const RecMove m = mv[r];
        if (status && status[m.status_idx] != 1) continue;
        // 16-B accesses (4-B alignment suffices) for the whole 16-B pieces inside the record, then dwords
        const W4 *src16 = reinterpret_cast<const W4 *>(m.src);
        W4 *dst16 = reinterpret_cast<W4 *>(m.dst);
        const uint32_t n16 = m.bytes >> 4;
        for (uint32_t i = lane; i < n16; i += 64) dst16[i] = src16[i];
        const uint32_t *src = reinterpret_cast<const uint32_t *>(m.src);
        uint32_t *dst = reinterpret_cast<uint32_t *>(m.dst);
        const uint32_t nd = exact ? m.bytes >> 2 : (m.bytes + 3) >> 2;
        if (lane < nd - 4 * n16) dst[4 * n16 + lane] = src[4 * n16 + lane];
        if (exact && lane < (m.bytes & 3u)) {
            const uint32_t b = (m.bytes & ~3u) + lane;
            reinterpret_cast<uint8_t *>(m.dst)[b] = reinterpret_cast<const uint8_t *>(m.src)[b];
        }
    }
}

hipError_t launch_move_records(const RecMove *d_moves, uint32_t n, const uint8_t *d_status, bool exact, int num_cus,
                               hipStream_t s) {
    if (n == 0) return hipSuccess;
    // 8 waves per CU: PCIe-bound, and room for the other stream's kernels to run alongside
    const uint32_t blocks = (n + 3) / 4, cap = (uint32_t)num_cus * 2u;
    hipLaunchKernelGGL(move_records_kernel, dim3(blocks < cap ? blocks : cap), dim3(256), 0, s, d_moves, n, d_status,
                       exact);
    return hipGetLastError();
}

hipError_t launch_stream_copy(void *dst, const void *src, uint64_t bytes, int num_cus, hipStream_t s) {
    const uint64_t n16 = bytes / 16;
    if (n16 == 0) return hipSuccess;
    (void)num_cus;
    // a grid of one 256-lane tile per 4 KiB, launched in pieces of at most 2^30 tiles (4 TiB) each
    for (uint64_t done = 0; done < n16;) {
        const uint64_t left = n16 - done, tiles = std::min<uint64_t>((left + 255) / 256, 1ull << 30);
        const uint64_t cnt = std::min<uint64_t>(left, tiles * 256);
        hipLaunchKernelGGL(stream_copy_kernel, dim3((uint32_t)tiles), dim3(256), 0, s, static_cast<uint4 *>(dst) + done,
                           static_cast<const uint4 *>(src) + done, cnt);
        done += cnt;
    }
    return hipGetLastError();
}

hipError_t launch_fill_uniform(uint8_t *arena, uint64_t stride, uint32_t n, uint32_t len, uint32_t aad_word,
                               uint64_t seed_payload, uint8_t *nonces, uint64_t seed_nonce, hipStream_t s) {
    const uint32_t groups = (4 + len + 3) / 4 + 3;
    const uint64_t total = (uint64_t)n * groups;
    if (total == 0) return hipSuccess;
    const int bs = 256;
    const uint64_t want = (total + bs - 1) / bs, cap = 1u << 20;  // 2^28 work items per pass at most
    hipLaunchKernelGGL(fill_uniform_kernel, dim3((uint32_t)(want < cap ? want : cap)), dim3(bs), 0, s, arena, stride, n,
                       len, aad_word, seed_payload, nonces, seed_nonce);
    return hipGetLastError();
}

}  // namespace qgcm
