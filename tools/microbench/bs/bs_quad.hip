// Microbenchmark: bitsliced AES-256-CTR, one 32-block slice per lane QUAD (lane q holds state
// column q: 32 words), ShiftRows by DPP quad_perm, round-key masks from LDS.  <=128 VGPRs so four
// or more waves share a SIMD (one wave alone issues a VALU op every 4 cycles, not every 2).
// Slot k of segment s of packet P holds counter 32*s + k (slot 1 of segment 0 = J0), so the
// counter bits are fixed patterns and no input transpose is needed.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 bs_quad.hip -o bs_quad -lcrypto
#include <hip/hip_runtime.h>
#include <openssl/evp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

#include "bs_sbox.inc"

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u128;

// lane c of each quad receives the value of lane (c + R) & 3
template <int R>
__device__ __forceinline__ uint32_t qrot(uint32_t v) {
    constexpr int ctrl = ((0 + R) & 3) | (((1 + R) & 3) << 2) | (((2 + R) & 3) << 4) | (((3 + R) & 3) << 6);
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xf, 0xf, false);
}

__device__ __forceinline__ void transpose32(uint32_t *a) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t x = a[k], y = a[k + 16];
        a[k] = (x & 0x0000ffffu) | (y << 16);
        a[k + 16] = (x >> 16) | (y & 0xffff0000u);
    }
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1) {
        const uint32_t m = w == 8 ? 0x00ff00ffu : w == 4 ? 0x0f0f0f0fu : w == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
        for (int k = 0; k < 32; ++k)
            if ((k & w) == 0) {
                const uint32_t x = a[k], y = a[k + w];
                a[k] = (x & m) | ((y << w) & ~m);
                a[k + w] = ((x >> w) & m) | (y & ~m);
            }
    }
}

// One full round on this lane's column: S-box, ShiftRows (DPP), MixColumns + AddRoundKey.
// s[8r + j] = bit j of row r of this lane's column; rk = this column's 32 masks (LDS address).
__device__ __forceinline__ void quad_round(uint32_t *s, uint32_t rk_addr) {
#pragma unroll
    for (int r = 0; r < 4; ++r) bs_sbox(s + 8 * r);
    uint32_t a[4][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[0][j] = s[j];
        a[1][j] = qrot<1>(s[8 + j]);
        a[2][j] = qrot<2>(s[16 + j]);
        a[3][j] = qrot<3>(s[24 + j]);
    }
    uint32_t k[32];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const u32x4 v = *(const lds_u128 *)(size_t)(rk_addr + 16 * i);
        k[4 * i] = v.x;
        k[4 * i + 1] = v.y;
        k[4 * i + 2] = v.z;
        k[4 * i + 3] = v.w;
    }
    uint32_t u[4][8], t[8];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) u[r][j] = a[r][j] ^ a[(r + 1) & 3][j];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = u[0][j] ^ u[2][j];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        uint32_t *d = s + 8 * r;
        const uint32_t *kk = k + 8 * r;
        d[0] = x3(a[r][0], t[0], x3(u[r][7], kk[0], 0u));
        d[1] = x3(x3(a[r][1], t[1], u[r][0]), u[r][7], kk[1]);
        d[2] = x3(a[r][2], t[2], x3(u[r][1], kk[2], 0u));
        d[3] = x3(x3(a[r][3], t[3], u[r][2]), u[r][7], kk[3]);
        d[4] = x3(x3(a[r][4], t[4], u[r][3]), u[r][7], kk[4]);
        d[5] = x3(a[r][5], t[5], x3(u[r][4], kk[5], 0u));
        d[6] = x3(a[r][6], t[6], x3(u[r][5], kk[6], 0u));
        d[7] = x3(a[r][7], t[7], x3(u[r][6], kk[7], 0u));
    }
}

__device__ __forceinline__ void quad_round_last(uint32_t *s) {
#pragma unroll
    for (int r = 0; r < 4; ++r) bs_sbox(s + 8 * r);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        s[8 + j] = qrot<1>(s[8 + j]);
        s[16 + j] = qrot<2>(s[16 + j]);
        s[24 + j] = qrot<3>(s[24 + j]);
    }
}

// rkm (global): [15][128] sliced round-key masks, copied to LDS; rkw: [60] round-key words.
// Quad Q (of n_quads) -> packet P = Q / 3, segment s = Q % 3; nonce of P = {P, n1, n2}.
template <int kWpe>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kWpe, kWpe)))
bs_quad_kernel(uint32_t *__restrict__ data, uint32_t n_quads, const uint32_t *__restrict__ rkm,
               const uint32_t *__restrict__ rkw, uint32_t n1, uint32_t n2, int mode) {
    for (int i = threadIdx.x; i < 15 * 128; i += blockDim.x) *(lds_u32 *)(size_t)(4 * i) = rkm[i];
    __syncthreads();
    const uint32_t q = threadIdx.x & 3;
    const uint32_t quad0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 2;
    const uint32_t nq = (gridDim.x * blockDim.x) >> 2;
    const uint32_t rk0 = rkw[q], rk14 = rkw[56 + q];
    uint32_t acc = 0;
    for (uint32_t Q = quad0; Q < n_quads; Q += nq) {
        const uint32_t P = Q / 3, seg = Q - 3 * P;
        // this lane's column word of the counter block, before the slot pattern: nonce word q, or
        // for q = 3 the big-endian counter 32*seg (+ slot k in the low 5 bits of byte 15)
        const uint32_t w = (q == 0 ? P : q == 1 ? n1 : q == 2 ? n2 : __builtin_bswap32(32u * seg)) ^ rk0;
        uint32_t s[32];
#pragma unroll
        for (int b = 0; b < 32; ++b) s[b] = (uint32_t)(-(int32_t)((w >> b) & 1));
        if (q == 3) {
            // byte 15 = bits 24..31 of the little-endian word: its bits 0..4 are the slot index
            s[24] ^= 0xaaaaaaaau;
            s[25] ^= 0xccccccccu;
            s[26] ^= 0xf0f0f0f0u;
            s[27] ^= 0xff00ff00u;
            s[28] ^= 0xffff0000u;
        }
#pragma unroll 1
        for (int r = 1; r < 14; ++r) quad_round(s, 512 * r + 128 * q);
        quad_round_last(s);
        transpose32(s);  // s[k] = word q of keystream block (slot) k, before the last AddRoundKey
        if (mode == 0) {
#pragma unroll
            for (int k = 0; k < 32; ++k) acc ^= s[k];
        } else {
            uint32_t *p = data + (size_t)Q * 128 + q;
#pragma unroll
            for (int k = 0; k < 32; ++k) p[4 * k] ^= s[k] ^ rk14;
        }
    }
    if (mode == 0 && acc == 0x12345678u) data[0] = acc;
}

static void expand_key(const uint8_t key[32], uint32_t rkw[60]) {
    static uint8_t sbox[256];
    uint8_t p = 1, q = 1;
    do {
        p = p ^ (uint8_t)(p << 1) ^ (p & 0x80 ? 0x1b : 0);
        q ^= q << 1;
        q ^= q << 2;
        q ^= q << 4;
        if (q & 0x80) q ^= 0x09;
        const uint8_t x = q ^ (uint8_t)((q << 1) | (q >> 7)) ^ (uint8_t)((q << 2) | (q >> 6)) ^
                          (uint8_t)((q << 3) | (q >> 5)) ^ (uint8_t)((q << 4) | (q >> 4));
        sbox[p] = x ^ 0x63;
    } while (p != 1);
    sbox[0] = 0x63;
    uint8_t w[240];
    memcpy(w, key, 32);
    uint8_t rcon = 1;
    for (int i = 8; i < 60; ++i) {
        uint8_t t[4];
        memcpy(t, w + 4 * (i - 1), 4);
        if (i % 8 == 0) {
            const uint8_t t0 = t[0];
            t[0] = sbox[t[1]] ^ rcon;
            t[1] = sbox[t[2]];
            t[2] = sbox[t[3]];
            t[3] = sbox[t0];
            rcon = (uint8_t)((rcon << 1) ^ (rcon & 0x80 ? 0x1b : 0));
        } else if (i % 8 == 4) {
            for (int j = 0; j < 4; ++j) t[j] = sbox[t[j]];
        }
        for (int j = 0; j < 4; ++j) w[4 * i + j] = w[4 * (i - 8) + j] ^ t[j];
    }
    memcpy(rkw, w, 240);
}

template <int kWpe>
static void run(uint32_t *d, uint32_t n_quads, uint32_t *d_rkm, uint32_t *d_rkw, uint32_t n1, uint32_t n2,
                int grid, const uint8_t key[32], const std::vector<uint32_t> &h) {
    const size_t nwords = (size_t)n_quads * 128;
    CHECK(hipMemcpy(d, h.data(), nwords * 4, hipMemcpyHostToDevice));
    bs_quad_kernel<kWpe><<<grid, 256, 15 * 512>>>(d, n_quads, d_rkm, d_rkw, n1, n2, 1);
    CHECK(hipDeviceSynchronize());
    std::vector<uint32_t> o(nwords);
    CHECK(hipMemcpy(o.data(), d, nwords * 4, hipMemcpyDeviceToHost));
    EVP_CIPHER_CTX *ec = EVP_CIPHER_CTX_new();
    EVP_EncryptInit_ex(ec, EVP_aes_256_ecb(), NULL, key, NULL);
    EVP_CIPHER_CTX_set_padding(ec, 0);
    int bad = 0;
    for (uint32_t Q = 0; Q < n_quads; Q += (Q < 64 ? 1 : 997)) {
        const uint32_t P = Q / 3, seg = Q % 3;
        for (int k = 0; k < 32; ++k) {
            uint32_t cw[4] = {P, n1, n2, __builtin_bswap32(32u * seg + k)}, kw[4];
            uint8_t ks[16];
            int ol = 0;
            EVP_EncryptUpdate(ec, ks, &ol, (const uint8_t *)cw, 16);
            memcpy(kw, ks, 16);
            for (int c = 0; c < 4; ++c) {
                const size_t i = (size_t)Q * 128 + 4 * k + c;
                if ((o[i] ^ h[i]) != kw[c]) {
                    if (bad < 5) fprintf(stderr, "Q %u slot %d word %d: got %08x want %08x\n", Q, k, c, o[i] ^ h[i], kw[c]);
                    ++bad;
                }
            }
        }
    }
    EVP_CIPHER_CTX_free(ec);
    printf("waves/EU %d: check %s (%d bad words)\n", kWpe, bad ? "FAIL" : "ok", bad);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = 10;
    for (int mode = 0; mode < 2; ++mode) {
        bs_quad_kernel<kWpe><<<grid, 256, 15 * 512>>>(d, n_quads, d_rkm, d_rkw, n1, n2, mode);
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) bs_quad_kernel<kWpe><<<grid, 256, 15 * 512>>>(d, n_quads, d_rkm, d_rkw, n1, n2, mode);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        const double nblk = (double)n_quads * 32;
        printf("  mode %d (%s): %.3f ms, %.1f G blocks/s = %.1f GB/s keystream\n", mode,
               mode ? "xor in place" : "keystream only", ms, nblk / ms / 1e6, nblk * 16 / ms / 1e6);
    }
}

int main(int argc, char **argv) {
    const uint32_t n_quads = argc > 1 ? atoi(argv[1]) : 3u << 20;  // 2^20 packets x 3 segments
    uint8_t key[32];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 7 + 1);
    const uint32_t n1 = 0x07060504u, n2 = 0x0b0a0908u;
    uint32_t rkw[60];
    expand_key(key, rkw);
    std::vector<uint32_t> rkm(15 * 128);
    for (int r = 0; r < 15; ++r)
        for (int c = 0; c < 4; ++c)
            for (int b = 0; b < 32; ++b) rkm[128 * r + 32 * c + b] = ((rkw[4 * r + c] >> b) & 1) ? 0xffffffffu : 0u;
    const size_t nwords = (size_t)n_quads * 128;
    std::vector<uint32_t> h(nwords);
    for (size_t i = 0; i < nwords; ++i) h[i] = (uint32_t)(i * 2654435761u);
    uint32_t *d, *d_rkm, *d_rkw;
    CHECK(hipMalloc(&d, nwords * 4));
    CHECK(hipMalloc(&d_rkm, rkm.size() * 4));
    CHECK(hipMalloc(&d_rkw, 240));
    CHECK(hipMemcpy(d_rkm, rkm.data(), rkm.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_rkw, rkw, 240, hipMemcpyHostToDevice));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    run<4>(d, n_quads, d_rkm, d_rkw, n1, n2, cus * 4, key, h);
    run<5>(d, n_quads, d_rkm, d_rkw, n1, n2, cus * 5, key, h);
    run<6>(d, n_quads, d_rkm, d_rkw, n1, n2, cus * 6, key, h);
    run<8>(d, n_quads, d_rkm, d_rkw, n1, n2, cus * 8, key, h);
    return 0;
}
