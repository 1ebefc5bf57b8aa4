// Microbenchmark: does mixing GHASH comb reads (16-B rows) into the T-table AES rounds cost more
// LDS time than the sum of the parts?  Per iteration and chain: 3 T-table rounds (48 ds_read_b32,
// replicated conflict-free tables, v_perm addressing as in gcm_kernels.hip) plus the GHASH share
// of the kernel (32 comb reads per 197 lookups ~ 8 per 3 rounds) as ds_read_b128 (4 x 16-lane
// groups) or as pairs of ds_read_b64 (2 x 32-lane groups).  Registers + LDS only.
// Build: hipcc --offload-arch=gfx950 -O3 lds_mix.hip -o lds_mix
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x4 lds_u128;
typedef __attribute__((address_space(3))) u32x2 lds_u64;
__device__ __forceinline__ uint32_t lds32(uint32_t a) { return *(const lds_u32 *)(size_t)a; }
__device__ __forceinline__ u32x4 lds128(uint32_t a) { return *(const lds_u128 *)(size_t)a; }
__device__ __forceinline__ u32x2 lds64(uint32_t a) { return *(const lds_u64 *)(size_t)a; }
__device__ __forceinline__ uint32_t perm(uint32_t a, uint32_t b, uint32_t s) { return __builtin_amdgcn_perm(a, b, s); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ uint32_t rot16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
#define TA(s, k) perm((s), lb, 0x0c0c0400u + ((k) << 8))
#define TE0(s, k) lds32(TA(s, k))
#define TE1(s, k) lds32(TA(s, k) + 128u)

__device__ __forceinline__ void round_full(uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3, uint32_t rk,
                                           uint32_t lb) {
    const uint32_t a0 = TE0(s2, 2), a1 = TE1(s3, 3), a2 = TE0(s3, 2), a3 = TE1(s0, 3);
    const uint32_t a4 = TE0(s0, 2), a5 = TE1(s1, 3), a6 = TE0(s1, 2), a7 = TE1(s2, 3);
    const uint32_t c0 = TE0(s0, 0), c1 = TE1(s1, 1), c2 = TE0(s1, 0), c3 = TE1(s2, 1);
    const uint32_t c4 = TE0(s2, 0), c5 = TE1(s3, 1), c6 = TE0(s3, 0), c7 = TE1(s0, 1);
    asm volatile("" ::: "memory");
    s0 = xor3(c0, c1, rot16(xor3(a0, a1, rk)));
    s1 = xor3(c2, c3, rot16(xor3(a2, a3, rk)));
    s2 = xor3(c4, c5, rot16(xor3(a4, a5, rk)));
    s3 = xor3(c6, c7, rot16(xor3(a6, a7, rk)));
}

// MODE 0: rounds only; 1: rounds + 8 x b128 comb reads; 2: rounds + 16 x b64; 3: comb b128 only.
// Comb tables at 64 KiB: 8 tables x 16 entries x 16 B (row = 256 B), entry = nibble.
template <int MODE, int W, int WPE>
__global__ void __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
mix(uint32_t *out, int iters) {
    for (int i = threadIdx.x; i < 18432; i += W * 64) *(lds_u32 *)(size_t)(4 * i) = i * 2654435761u;
    __syncthreads();
    const uint32_t lb = (threadIdx.x & 31) << 2;
    uint32_t s0 = threadIdx.x * 977, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3;
    uint32_t z0 = s0 ^ 0x55, z1 = 0, z2 = 0, z3 = 0;
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE != 3) {
            round_full(s0, s1, s2, s3, it, lb);
            round_full(s0, s1, s2, s3, it + 1, lb);
            round_full(s0, s1, s2, s3, it + 2, lb);
        }
        if constexpr (MODE == 1 || MODE == 3) {
            const uint32_t hi = z0 & 0xf0f0f0f0u, lo = (z0 << 4) & 0xf0f0f0f0u;
            uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const u32x4 th = lds128(65536u + perm(0, hi, 0x0c0c0c00u | k) + (2 * k) * 256);
                const u32x4 tl = lds128(65536u + perm(0, lo, 0x0c0c0c00u | k) + (2 * k + 1) * 256);
                a0 = xor3(a0, th.x, tl.x);
                a1 = xor3(a1, th.y, tl.y);
                a2 = xor3(a2, th.z, tl.z);
                a3 = xor3(a3, th.w, tl.w);
            }
            z0 = a0 ^ s0;
            z1 ^= a1;
            z2 ^= a2;
            z3 ^= a3;
        }
        if constexpr (MODE == 2) {
            const uint32_t hi = z0 & 0xf0f0f0f0u, lo = (z0 << 4) & 0xf0f0f0f0u;
            uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                // the same 16-B row read as two 8-B halves (tables of 16 x 8 B = 128 B per half)
                const uint32_t ah = 65536u + (perm(0, hi, 0x0c0c0c00u | k) >> 1) + (2 * k) * 256;
                const uint32_t al = 65536u + (perm(0, lo, 0x0c0c0c00u | k) >> 1) + (2 * k + 1) * 256;
                const u32x2 th0 = lds64(ah), th1 = lds64(ah + 128), tl0 = lds64(al), tl1 = lds64(al + 128);
                a0 = xor3(a0, th0.x, tl0.x);
                a1 = xor3(a1, th0.y, tl0.y);
                a2 = xor3(a2, th1.x, tl1.x);
                a3 = xor3(a3, th1.y, tl1.y);
            }
            z0 = a0 ^ s0;
            z1 ^= a1;
            z2 ^= a2;
            z3 ^= a3;
        }
    }
    out[blockIdx.x * W * 64 + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3 ^ z0 ^ z1 ^ z2 ^ z3;
}

template <int MODE, int W, int WGS>
void run(uint32_t *d, int cus, const char *name) {
    auto k = mix<MODE, W, W * WGS / 4>;
    const int lds = 65536 + 8192;
    hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    const int iters = 2000;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(cus * WGS), dim3(W * 64), lds, 0, d, 10);
    hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(cus * WGS), dim3(W * 64), lds, 0, d, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    // modelled LDS-array cycles per iteration per wave: 48 b32 x 2, 8 b128 x 4, 16 b64 x 2
    const double cyc = (MODE == 0 ? 96 : MODE == 1 ? 128 : MODE == 2 ? 128 : 32);
    const double waves = (double)cus * WGS * W;
    const double model_ms = waves / cus * iters * cyc / 2.2e9 * 1e3;
    printf("%-22s waves/CU %2d: %.3f ms  LDS-array model at 2.2 GHz %.3f ms  (model/measured %.3f)\n", name, W * WGS,
           ms, model_ms, model_ms / ms);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *d;
    hipMalloc(&d, 256 * 1024 * 4 * 4);
    run<0, 16, 2>(d, cus, "rounds");
    run<1, 16, 2>(d, cus, "rounds+comb b128");
    run<2, 16, 2>(d, cus, "rounds+comb 2xb64");
    run<3, 16, 2>(d, cus, "comb b128 only");
    run<0, 8, 2>(d, cus, "rounds");
    run<1, 8, 2>(d, cus, "rounds+comb b128");
    run<2, 8, 2>(d, cus, "rounds+comb 2xb64");
    return 0;
}
