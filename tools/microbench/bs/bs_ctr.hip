// Microbenchmark: bitsliced AES-256-CTR keystream on the VALU (v_bitop3 S-box), 32 blocks per lane.
// Question it answers: how fast is a VALU-bound AES on gfx950 next to the LDS-bound T-table path
// (DESIGN.md 4.1), alone and co-resident with it.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 bs_ctr.hip -o bs_ctr -lcrypto
#include <hip/hip_runtime.h>
#include <openssl/evp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

#include "bs_sbox.inc"

// 32x32 bit transpose of a[0..31] (a[k] bit b <-> a[b] bit k); an involution.
__device__ __forceinline__ void transpose32(uint32_t *a) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t x = a[k], y = a[k + 16];
        a[k] = (x & 0x0000ffffu) | (y << 16);
        a[k + 16] = (x >> 16) | (y & 0xffff0000u);
    }
#pragma unroll
    for (int k = 0; k < 32; ++k)
        if ((k & 8) == 0) {
            const uint32_t x = a[k], y = a[k + 8];
            a[k] = (x & 0x00ff00ffu) | ((y << 8) & 0xff00ff00u);
            a[k + 8] = ((x >> 8) & 0x00ff00ffu) | (y & 0xff00ff00u);
        }
#pragma unroll
    for (int k = 0; k < 32; ++k)
        if ((k & 4) == 0) {
            const uint32_t x = a[k], y = a[k + 4];
            a[k] = (x & 0x0f0f0f0fu) | ((y << 4) & 0xf0f0f0f0u);
            a[k + 4] = ((x >> 4) & 0x0f0f0f0fu) | (y & 0xf0f0f0f0u);
        }
#pragma unroll
    for (int k = 0; k < 32; ++k)
        if ((k & 2) == 0) {
            const uint32_t x = a[k], y = a[k + 2];
            a[k] = (x & 0x33333333u) | ((y << 2) & 0xccccccccu);
            a[k + 2] = ((x >> 2) & 0x33333333u) | (y & 0xccccccccu);
        }
#pragma unroll
    for (int k = 0; k < 32; ++k)
        if ((k & 1) == 0) {
            const uint32_t x = a[k], y = a[k + 1];
            a[k] = (x & 0x55555555u) | ((y << 1) & 0xaaaaaaaau);
            a[k + 1] = ((x >> 1) & 0x55555555u) | (y & 0xaaaaaaaau);
        }
}

// Sliced state s[8p + j], p = 4*col + row.  ShiftRows: s'[4c + r] = s[4((c + r) & 3) + r].
// MixColumns + AddRoundKey on the shifted state: out_i = a_i ^ t ^ xt(a_i ^ a_{i+1}) ^ rk,
// t = a0 ^ a1 ^ a2 ^ a3.
__device__ __forceinline__ void bs_round(uint32_t *s, const uint32_t *__restrict__ rk) {
#pragma unroll
    for (int p = 0; p < 16; ++p) bs_sbox(s + 8 * p);
    uint32_t o[128];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t *a[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) a[r] = s + 8 * (4 * ((c + r) & 3) + r);
        uint32_t u[4][8], t[8];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) u[r][j] = a[r][j] ^ a[(r + 1) & 3][j];
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = u[0][j] ^ u[2][j];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            uint32_t *d = o + 8 * (4 * c + r);
            const uint32_t *k = rk + 8 * (4 * c + r);
            d[0] = x3(x3(a[r][0], t[0], u[r][7]), k[0], 0u);
            d[1] = x3(x3(a[r][1], t[1], u[r][0]), u[r][7], k[1]);
            d[2] = x3(x3(a[r][2], t[2], u[r][1]), k[2], 0u);
            d[3] = x3(x3(a[r][3], t[3], u[r][2]), u[r][7], k[3]);
            d[4] = x3(x3(a[r][4], t[4], u[r][3]), u[r][7], k[4]);
            d[5] = x3(x3(a[r][5], t[5], u[r][4]), k[5], 0u);
            d[6] = x3(x3(a[r][6], t[6], u[r][5]), k[6], 0u);
            d[7] = x3(x3(a[r][7], t[7], u[r][6]), k[7], 0u);
        }
    }
#pragma unroll
    for (int w = 0; w < 128; ++w) s[w] = o[w];
}

// Final round: S-box and ShiftRows; its AddRoundKey is applied after the transpose (uniform words).
__device__ __forceinline__ void bs_round_last(uint32_t *s) {
#pragma unroll
    for (int p = 0; p < 16; ++p) bs_sbox(s + 8 * p);
    uint32_t o[128];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) o[8 * (4 * c + r) + j] = s[8 * (4 * ((c + r) & 3) + r) + j];
#pragma unroll
    for (int w = 0; w < 128; ++w) s[w] = o[w];
}

// rkm: [15][128] sliced round-key masks; rkw: [15][4] little-endian round-key words.
// Block i of the stream: counter block = n0 n1 n2 be32(i + 2) (GCM inc32 from J0 + 1).
// Lane l of group g, slot k -> block g*2048 + 64*k + l (coalesced loads).
template <int kUnroll>
__global__ void __launch_bounds__(256) bs_ctr_kernel(uint4 *__restrict__ data, uint32_t n_groups,
                                                     const uint32_t *__restrict__ rkm,
                                                     const uint32_t *__restrict__ rkw, uint32_t n0, uint32_t n1,
                                                     uint32_t n2, int mode) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    uint32_t acc = 0;
    for (uint32_t g = wave; g < n_groups; g += nwaves) {
        uint32_t s[128];
        // words 0..2: nonce ^ rk0, identical for all slots -> all-0 / all-1 words
        const uint32_t c0 = n0 ^ rkw[0], c1 = n1 ^ rkw[1], c2 = n2 ^ rkw[2];
#pragma unroll
        for (int b = 0; b < 32; ++b) {
            s[b] = (uint32_t)(-(int32_t)((c0 >> b) & 1));
            s[32 + b] = (uint32_t)(-(int32_t)((c1 >> b) & 1));
            s[64 + b] = (uint32_t)(-(int32_t)((c2 >> b) & 1));
        }
        const uint32_t base = g * 2048u + lane;
#pragma unroll
        for (int k = 0; k < 32; ++k) s[96 + k] = __builtin_bswap32(base + 64u * k + 2u) ^ rkw[3];
        transpose32(s + 96);
#pragma unroll 1
        for (int r = 1; r < 14; ++r) bs_round(s, rkm + 128 * r);
        bs_round_last(s);
#pragma unroll
        for (int c = 0; c < 4; ++c) transpose32(s + 32 * c);
        const uint32_t k0 = rkw[56], k1 = rkw[57], k2 = rkw[58], k3 = rkw[59];
        if (mode == 0) {
#pragma unroll
            for (int k = 0; k < 32; ++k) acc ^= s[k] ^ s[32 + k] ^ s[64 + k] ^ s[96 + k];
        } else {
#pragma unroll
            for (int k = 0; k < 32; ++k) {
                uint4 *p = data + (base + 64u * k);
                uint4 v = *p;
                v.x ^= s[k] ^ k0;
                v.y ^= s[32 + k] ^ k1;
                v.z ^= s[64 + k] ^ k2;
                v.w ^= s[96 + k] ^ k3;
                *p = v;
            }
        }
    }
    if (mode == 0 && acc == 0x12345678u) data[0].x = acc;
}

#ifdef BS_LIB
// co-run experiments: launch on a caller's stream (tools/microbench/bs/corun.py)
extern "C" int bs_launch(void *data, uint32_t n_groups, const uint32_t *rkm, const uint32_t *rkw, int grid,
                         int mode, void *stream) {
    bs_ctr_kernel<1><<<grid, 256, 0, (hipStream_t)stream>>>((uint4 *)data, n_groups, rkm, rkw, 0x03020100u,
                                                            0x07060504u, 0x0b0a0908u, mode);
    return (int)hipGetLastError();
}
#else
// ---- host ----
static void expand_key(const uint8_t key[32], uint32_t rkw[60]) {
    static uint8_t sbox[256];
    {
        // S-box from the inverse + affine map
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
    }
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

int main(int argc, char **argv) {
    const uint32_t n_groups = argc > 1 ? atoi(argv[1]) : 43520;  // ~2^20 x 85 blocks
    const int grid_per_cu = argc > 2 ? atoi(argv[2]) : 2;
    const int reps = 10;
    uint8_t key[32];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 7 + 1);
    const uint32_t n0 = 0x03020100u, n1 = 0x07060504u, n2 = 0x0b0a0908u;
    uint32_t rkw[60];
    expand_key(key, rkw);
    std::vector<uint32_t> rkm(15 * 128);
    for (int r = 0; r < 15; ++r)
        for (int c = 0; c < 4; ++c)
            for (int b = 0; b < 32; ++b) rkm[128 * r + 32 * c + b] = ((rkw[4 * r + c] >> b) & 1) ? 0xffffffffu : 0u;
    const size_t nblk = (size_t)n_groups * 2048;
    std::vector<uint32_t> h(nblk * 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 2654435761u);
    uint4 *d;
    uint32_t *d_rkm, *d_rkw;
    CHECK(hipMalloc(&d, nblk * 16));
    CHECK(hipMalloc(&d_rkm, rkm.size() * 4));
    CHECK(hipMalloc(&d_rkw, 60 * 4));
    CHECK(hipMemcpy(d, h.data(), nblk * 16, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_rkm, rkm.data(), rkm.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_rkw, rkw, 240, hipMemcpyHostToDevice));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int grid = prop.multiProcessorCount * grid_per_cu;
    // correctness: one pass, compare sampled blocks with OpenSSL AES-256 ECB of the counter block
    bs_ctr_kernel<1><<<grid, 256>>>(d, n_groups, d_rkm, d_rkw, n0, n1, n2, 1);
    CHECK(hipDeviceSynchronize());
    std::vector<uint32_t> o(nblk * 4);
    CHECK(hipMemcpy(o.data(), d, nblk * 16, hipMemcpyDeviceToHost));
    EVP_CIPHER_CTX *ec = EVP_CIPHER_CTX_new();
    EVP_EncryptInit_ex(ec, EVP_aes_256_ecb(), NULL, key, NULL);
    EVP_CIPHER_CTX_set_padding(ec, 0);
    int bad = 0;
    for (size_t i = 0; i < nblk; i += (i < 4096 ? 1 : 9973)) {
        uint8_t ctr[16], ks[16];
        uint32_t w[4] = {n0, n1, n2, __builtin_bswap32((uint32_t)i + 2u)};
        memcpy(ctr, w, 16);
        int ol = 0;
        EVP_EncryptUpdate(ec, ks, &ol, ctr, 16);
        uint32_t kw[4];
        memcpy(kw, ks, 16);
        for (int c = 0; c < 4; ++c)
            if ((o[4 * i + c] ^ h[4 * i + c]) != kw[c]) {
                if (bad < 5) fprintf(stderr, "block %zu word %d: got %08x want %08x\n", i, c, o[4 * i + c] ^ h[4 * i + c], kw[c]);
                ++bad;
            }
    }
    printf("check: %s (%d bad words)\n", bad ? "FAIL" : "ok", bad);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int mode = 0; mode < 2; ++mode) {
        bs_ctr_kernel<1><<<grid, 256>>>(d, n_groups, d_rkm, d_rkw, n0, n1, n2, mode);
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) bs_ctr_kernel<1><<<grid, 256>>>(d, n_groups, d_rkm, d_rkw, n0, n1, n2, mode);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("mode %d (%s): %.3f ms per %zu blocks = %.1f GB/s of keystream (%.1f G blocks/s)\n", mode,
               mode ? "xor in place" : "keystream only", ms, nblk, nblk * 16 / ms / 1e6, nblk / ms / 1e6);
    }
    return bad ? 1 : 0;
}
#endif
