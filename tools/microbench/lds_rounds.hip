// Microbenchmark: achievable T-table lookup rate (ds_read_b32, replicated conflict-free tables,
// v_perm addressing) on gfx950 vs waves per CU and independent chains per lane.  No global memory
// in the timed loop.  Build: hipcc --offload-arch=gfx950 -O3 lds_rounds.hip -o lds_rounds
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t lds32(uint32_t a) { return *(const lds_u32 *)(size_t)a; }
__device__ __forceinline__ uint32_t perm(uint32_t a, uint32_t b, uint32_t s) { return __builtin_amdgcn_perm(a, b, s); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ uint32_t rot16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
#define TA(s, k) perm((s), lb, 0x0c0c0400u + ((k) << 8))
#define TE0(s, k) lds32(TA(s, k))
#define TE1(s, k) lds32(TA(s, k) + 128u)

template <int W, int N, int WPE = W / 4>
__global__ void __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
rounds(uint32_t *out, int iters, uint32_t rkseed) {
    extern __shared__ uint32_t sm[];
    for (int i = threadIdx.x; i < 16384; i += W * 64) *(lds_u32 *)(size_t)(4 * i) = i * 2654435761u;
    __syncthreads();
    const uint32_t lb = (threadIdx.x & 31) << 2;
    uint32_t s[N][4];
#pragma unroll
    for (int j = 0; j < N; ++j)
        for (int c = 0; c < 4; ++c) s[j][c] = threadIdx.x * 977 + j * 131 + c;
    for (int it = 0; it < iters; ++it) {
        const uint32_t rk = rkseed + it;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            uint32_t s0 = s[j][0], s1 = s[j][1], s2 = s[j][2], s3 = s[j][3];
            const uint32_t b0 = xor3(TE0(s2, 2), TE1(s3, 3), rk);
            const uint32_t b1 = xor3(TE0(s3, 2), TE1(s0, 3), rk);
            const uint32_t b2 = xor3(TE0(s0, 2), TE1(s1, 3), rk);
            const uint32_t b3 = xor3(TE0(s1, 2), TE1(s2, 3), rk);
            s[j][0] = xor3(TE0(s0, 0), TE1(s1, 1), rot16(b0));
            s[j][1] = xor3(TE0(s1, 0), TE1(s2, 1), rot16(b1));
            s[j][2] = xor3(TE0(s2, 0), TE1(s3, 1), rot16(b2));
            s[j][3] = xor3(TE0(s3, 0), TE1(s0, 1), rot16(b3));
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) acc ^= s[j][0] ^ s[j][1] ^ s[j][2] ^ s[j][3];
    out[blockIdx.x * W * 64 + threadIdx.x] = acc;
}

template <int W, int N, int WGS = 1>
void run(uint32_t *d, int cus) {
    auto k = rounds<W, N, W * WGS / 4>;
    hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    const int iters = 2000;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(cus * WGS), dim3(W * 64), 65536, 0, d, 10, 1u);
    hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(cus * WGS), dim3(W * 64), 65536, 0, d, iters, 1u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lookups = (double)cus * WGS * W * 64 * N * iters * 16;
    const double wave_ds = lookups / 64;           // ds_read_b32 wave-instructions
    printf("waves/CU %2d chains/lane %d: ", W * WGS, N); printf(" %.3f ms  %.1f G lookups/s  ds_b32 per CU-cycle @2.2GHz %.3f (peak 0.5)\n",
           ms, lookups / ms / 1e6, wave_ds / cus / (ms * 1e-3 * 2.2e9));
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *d;
    hipMalloc(&d, 256 * 1024 * 4 * 4);
    run<4, 1>(d, cus); run<4, 2>(d, cus); run<4, 4>(d, cus); run<4, 8>(d, cus);
    run<8, 1>(d, cus); run<8, 2>(d, cus); run<8, 4>(d, cus); run<8, 8>(d, cus);
    run<16, 1>(d, cus); run<16, 2>(d, cus); run<16, 4>(d, cus);
    run<16, 1, 2>(d, cus); run<16, 2, 2>(d, cus);
    run<12, 1, 2>(d, cus); run<8, 1, 2>(d, cus); run<8, 2, 2>(d, cus);
    return 0;
}
