// keymath.cpp -- host-side key setup for the encryption path (cold path, not per packet).
//
//   crypto/aes.go:66        key = pbkdf2.Key(secret, salt, 10000, 32, sha512.New)
//   crypto/ecdh.go:13-31    curve25519.ScalarBaseMult / ScalarMult (x/crypto, RFC 7748 X25519)
//   common/mapping.go:90-99 secret = X25519(peer.PublicKey, PrivateKey),
//                           salt   = X25519(peer.PublicSalt, PrivateSalt) -> NewAES(secret, salt)
// Implemented from FIPS 180-4 (SHA-512), RFC 2104 (HMAC), RFC 8018 s5.2 (PBKDF2) and RFC 7748
// (X25519: Montgomery ladder over GF(2^255-19), radix-2^51 limbs).  No external crypto library.
#include <stdint.h>
#include <string.h>

#include <thread>
#include <vector>

#include "../../include/qgcm.h"

namespace {

// SHA-512 round constants / initial value: first 64 fractional bits of the cube / square roots
// of the first 80 / 8 primes (FIPS 180-4 s4.2.3, s5.3.5), generated from that definition.
static const uint64_t kSha512K[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL,
};
static const uint64_t kSha512H0[8] = {
    0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
    0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL,
};

inline uint64_t ror(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

struct Sha512 {
    uint64_t h[8];
    uint8_t buf[128];
    size_t fill = 0;
    uint64_t total = 0;
    Sha512() { memcpy(h, kSha512H0, sizeof h); }
    void block(const uint8_t *p) {
        uint64_t w[80];
        for (int i = 0; i < 16; ++i) {
            uint64_t v = 0;
            for (int j = 0; j < 8; ++j) v = (v << 8) | p[8 * i + j];
            w[i] = v;
        }
        for (int i = 16; i < 80; ++i) {
            const uint64_t s0 = ror(w[i - 15], 1) ^ ror(w[i - 15], 8) ^ (w[i - 15] >> 7);
            const uint64_t s1 = ror(w[i - 2], 19) ^ ror(w[i - 2], 61) ^ (w[i - 2] >> 6);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
        for (int i = 0; i < 80; ++i) {
            const uint64_t S1 = ror(e, 14) ^ ror(e, 18) ^ ror(e, 41);
            const uint64_t ch = (e & f) ^ (~e & g);
            const uint64_t t1 = k + S1 + ch + kSha512K[i] + w[i];
            const uint64_t S0 = ror(a, 28) ^ ror(a, 34) ^ ror(a, 39);
            const uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
            const uint64_t t2 = S0 + mj;
            k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
    }
    void update(const uint8_t *p, size_t n) {
        total += n;
        while (n) {
            const size_t take = (128 - fill) < n ? (128 - fill) : n;
            memcpy(buf + fill, p, take);
            fill += take; p += take; n -= take;
            if (fill == 128) { block(buf); fill = 0; }
        }
    }
    void final(uint8_t out[64]) {
        const uint64_t bits = total * 8;
        uint8_t pad = 0x80;
        update(&pad, 1);
        const uint8_t z = 0;
        while (fill != 112) update(&z, 1);
        uint8_t len[16] = {0};
        for (int j = 0; j < 8; ++j) len[15 - j] = (uint8_t)(bits >> (8 * j));
        update(len, 16);
        for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(h[i] >> (56 - 8 * j));
    }
};

// HMAC-SHA512 with precomputed inner/outer states (RFC 2104).
struct HmacSha512 {
    Sha512 inner0, outer0;
    HmacSha512(const uint8_t *key, size_t klen) {
        uint8_t k[128] = {0};
        if (klen > 128) {
            Sha512 s;
            s.update(key, klen);
            s.final(k);
        } else {
            memcpy(k, key, klen);
        }
        uint8_t ip[128], op[128];
        for (int i = 0; i < 128; ++i) { ip[i] = k[i] ^ 0x36; op[i] = k[i] ^ 0x5c; }
        inner0.update(ip, 128);
        outer0.update(op, 128);
    }
    void mac(const uint8_t *m, size_t n, uint8_t out[64]) const {
        Sha512 in = inner0, ou = outer0;
        uint8_t t[64];
        in.update(m, n);
        in.final(t);
        ou.update(t, 64);
        ou.final(out);
    }
};

// PBKDF2 (RFC 8018 s5.2) with HMAC-SHA512; dk_len <= 64 (one block) is all the path needs.
void pbkdf2_sha512(const uint8_t *pw, size_t pwlen, const uint8_t *salt, size_t slen, uint32_t iters,
                   uint8_t *out, size_t dk_len) {
    HmacSha512 prf(pw, pwlen);
    for (uint32_t blk = 1; dk_len; ++blk) {
        std::vector<uint8_t> s(slen + 4);
        memcpy(s.data(), salt, slen);
        s[slen] = (uint8_t)(blk >> 24); s[slen + 1] = (uint8_t)(blk >> 16);
        s[slen + 2] = (uint8_t)(blk >> 8); s[slen + 3] = (uint8_t)blk;
        uint8_t u[64], t[64];
        prf.mac(s.data(), s.size(), u);
        memcpy(t, u, 64);
        for (uint32_t i = 1; i < iters; ++i) {
            prf.mac(u, 64, u);
            for (int j = 0; j < 64; ++j) t[j] ^= u[j];
        }
        const size_t take = dk_len < 64 ? dk_len : 64;
        memcpy(out, t, take);
        out += take; dk_len -= take;
    }
}

// ---- X25519 over GF(2^255 - 19), five 51-bit limbs ----
typedef uint64_t fe[5];
typedef unsigned __int128 u128;
constexpr uint64_t M51 = (1ULL << 51) - 1;

inline void fe_carry(fe h) {
    uint64_t c;
    c = h[0] >> 51; h[0] &= M51; h[1] += c;
    c = h[1] >> 51; h[1] &= M51; h[2] += c;
    c = h[2] >> 51; h[2] &= M51; h[3] += c;
    c = h[3] >> 51; h[3] &= M51; h[4] += c;
    c = h[4] >> 51; h[4] &= M51; h[0] += 19 * c;
    c = h[0] >> 51; h[0] &= M51; h[1] += c;
}
inline void fe_add(fe h, const fe f, const fe g) { for (int i = 0; i < 5; ++i) h[i] = f[i] + g[i]; fe_carry(h); }
inline void fe_sub(fe h, const fe f, const fe g) {
    // f + 4p - g, limbs of f,g < 2^52
    h[0] = f[0] + 0x1FFFFFFFFFFFB4ULL - g[0];
    for (int i = 1; i < 5; ++i) h[i] = f[i] + 0x1FFFFFFFFFFFFCULL - g[i];
    fe_carry(h);
}
inline void fe_mul(fe h, const fe f, const fe g) {
    const uint64_t g1 = 19 * g[1], g2 = 19 * g[2], g3 = 19 * g[3], g4 = 19 * g[4];
    u128 r0 = (u128)f[0] * g[0] + (u128)f[1] * g4 + (u128)f[2] * g3 + (u128)f[3] * g2 + (u128)f[4] * g1;
    u128 r1 = (u128)f[0] * g[1] + (u128)f[1] * g[0] + (u128)f[2] * g4 + (u128)f[3] * g3 + (u128)f[4] * g2;
    u128 r2 = (u128)f[0] * g[2] + (u128)f[1] * g[1] + (u128)f[2] * g[0] + (u128)f[3] * g4 + (u128)f[4] * g3;
    u128 r3 = (u128)f[0] * g[3] + (u128)f[1] * g[2] + (u128)f[2] * g[1] + (u128)f[3] * g[0] + (u128)f[4] * g4;
    u128 r4 = (u128)f[0] * g[4] + (u128)f[1] * g[3] + (u128)f[2] * g[2] + (u128)f[3] * g[1] + (u128)f[4] * g[0];
    r1 += (uint64_t)(r0 >> 51); uint64_t h0 = (uint64_t)r0 & M51;
    r2 += (uint64_t)(r1 >> 51); uint64_t h1 = (uint64_t)r1 & M51;
    r3 += (uint64_t)(r2 >> 51); uint64_t h2 = (uint64_t)r2 & M51;
    r4 += (uint64_t)(r3 >> 51); uint64_t h3 = (uint64_t)r3 & M51;
    uint64_t c = (uint64_t)(r4 >> 51); uint64_t h4 = (uint64_t)r4 & M51;
    h0 += 19 * c;
    h1 += h0 >> 51; h0 &= M51;
    h[0] = h0; h[1] = h1; h[2] = h2; h[3] = h3; h[4] = h4;
}
inline void fe_mul_small(fe h, const fe f, uint64_t s) {
    u128 c = 0;
    for (int i = 0; i < 5; ++i) {
        const u128 t = (u128)f[i] * s + c;
        h[i] = (uint64_t)t & M51;
        c = t >> 51;
    }
    h[0] += 19 * (uint64_t)c;
    fe_carry(h);
}
inline void fe_cswap(fe a, fe b, uint64_t bit) {
    const uint64_t m = 0 - bit;
    for (int i = 0; i < 5; ++i) { const uint64_t t = m & (a[i] ^ b[i]); a[i] ^= t; b[i] ^= t; }
}
inline uint64_t load64(const uint8_t *p) { uint64_t v = 0; for (int i = 7; i >= 0; --i) v = (v << 8) | p[i]; return v; }
void fe_frombytes(fe h, const uint8_t s[32]) {
    h[0] = load64(s) & M51;
    h[1] = (load64(s + 6) >> 3) & M51;
    h[2] = (load64(s + 12) >> 6) & M51;
    h[3] = (load64(s + 19) >> 1) & M51;
    h[4] = (load64(s + 24) >> 12) & M51;  // drops bit 255 (RFC 7748 s5)
}
void fe_tobytes(uint8_t s[32], const fe f) {
    fe h;
    memcpy(h, f, sizeof h);
    fe_carry(h);
    fe_carry(h);
    uint64_t q = (h[0] + 19) >> 51;
    q = (h[1] + q) >> 51; q = (h[2] + q) >> 51; q = (h[3] + q) >> 51; q = (h[4] + q) >> 51;
    h[0] += 19 * q;
    h[1] += h[0] >> 51; h[0] &= M51;
    h[2] += h[1] >> 51; h[1] &= M51;
    h[3] += h[2] >> 51; h[2] &= M51;
    h[4] += h[3] >> 51; h[3] &= M51;
    h[4] &= M51;
    const uint64_t w0 = h[0] | (h[1] << 51), w1 = (h[1] >> 13) | (h[2] << 38), w2 = (h[2] >> 26) | (h[3] << 25),
                   w3 = (h[3] >> 39) | (h[4] << 12);
    const uint64_t w[4] = {w0, w1, w2, w3};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}
void fe_invert(fe out, const fe z) {
    // z^(p-2), p-2 = 2^255 - 21: square-and-multiply over the exponent bits (cold path).
    fe r = {1, 0, 0, 0, 0}, b;
    memcpy(b, z, sizeof b);
    // exponent bits, LSB first: 2^255-21 = 0x7fff...ffeb
    for (int i = 0; i < 255; ++i) {
        const int bit = (i < 8) ? ((0xebu >> i) & 1) : 1;
        if (bit) fe_mul(r, r, b);
        fe_mul(b, b, b);
    }
    memcpy(out, r, sizeof r);
}
void x25519(uint8_t out[32], const uint8_t scalar[32], const uint8_t point[32]) {
    uint8_t k[32];
    memcpy(k, scalar, 32);
    k[0] &= 248; k[31] &= 127; k[31] |= 64;
    fe x1, x2 = {1, 0, 0, 0, 0}, z2 = {0, 0, 0, 0, 0}, x3, z3 = {1, 0, 0, 0, 0};
    fe_frombytes(x1, point);
    memcpy(x3, x1, sizeof x3);
    uint64_t swap = 0;
    for (int t = 254; t >= 0; --t) {
        const uint64_t kt = (k[t >> 3] >> (t & 7)) & 1;
        swap ^= kt;
        fe_cswap(x2, x3, swap);
        fe_cswap(z2, z3, swap);
        swap = kt;
        fe A, AA, B, BB, E, Cc, D, DA, CB, t0, t1;
        fe_add(A, x2, z2); fe_mul(AA, A, A);
        fe_sub(B, x2, z2); fe_mul(BB, B, B);
        fe_sub(E, AA, BB);
        fe_add(Cc, x3, z3); fe_sub(D, x3, z3);
        fe_mul(DA, D, A); fe_mul(CB, Cc, B);
        fe_add(t0, DA, CB); fe_mul(x3, t0, t0);
        fe_sub(t1, DA, CB); fe_mul(t1, t1, t1); fe_mul(z3, x1, t1);
        fe_mul(x2, AA, BB);
        fe_mul_small(t0, E, 121665); fe_add(t0, AA, t0); fe_mul(z2, E, t0);
    }
    fe_cswap(x2, x3, swap);
    fe_cswap(z2, z3, swap);
    fe zi, r;
    fe_invert(zi, z2);
    fe_mul(r, x2, zi);
    fe_tobytes(out, r);
}

}  // namespace

extern "C" {

int qgcm_derive_key(const uint8_t *secret, size_t secret_len, const uint8_t *salt, size_t salt_len,
                    uint8_t key[QGCM_KEY_BYTES]) {
    if ((!secret && secret_len) || (!salt && salt_len) || !key) return QGCM_E_ARG;
    pbkdf2_sha512(secret, secret_len, salt, salt_len, QGCM_PBKDF2_ITERS, key, QGCM_KEY_BYTES);
    return QGCM_OK;
}

int qgcm_derive_keys(const uint8_t *secrets, const uint8_t *salts, uint32_t count, uint8_t *keys) {
    if (!count) return QGCM_OK;
    if (!secrets || !salts || !keys) return QGCM_E_ARG;
    unsigned nt = std::thread::hardware_concurrency();
    if (nt == 0) nt = 1;
    if (nt > 64) nt = 64;
    if (nt > count) nt = count;
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([=] {
            for (uint32_t i = t; i < count; i += nt)
                pbkdf2_sha512(secrets + 32ull * i, 32, salts + 32ull * i, 32, QGCM_PBKDF2_ITERS, keys + 32ull * i, 32);
        });
    for (auto &x : th) x.join();
    return QGCM_OK;
}

int qgcm_x25519_base(uint8_t pub[32], const uint8_t priv[32]) {
    if (!pub || !priv) return QGCM_E_ARG;
    uint8_t nine[32] = {9};
    x25519(pub, priv, nine);
    return QGCM_OK;
}

int qgcm_x25519(uint8_t secret[32], const uint8_t priv[32], const uint8_t peer_pub[32]) {
    if (!secret || !priv || !peer_pub) return QGCM_E_ARG;
    x25519(secret, priv, peer_pub);
    return QGCM_OK;
}

}  // extern "C"
