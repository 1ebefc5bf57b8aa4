// Microbenchmark: LDS read throughput by access width on gfx950 (is a byte / halfword gather cheaper
// than a dword gather?).  Every lane reads its own bank replica (conflict-free), 16 independent
// reads per iteration.  "pure": one base address per iteration and rows by immediate offsets (LDS
// issue only); "lookup": a data-dependent address per read, like a table lookup.
// Build: hipcc --offload-arch=gfx950 -O3 lds_width.hip -o lds_width
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint64_t lds_u64;

template <int KIND>
__device__ __forceinline__ uint32_t rd(uint32_t a) {
    if constexpr (KIND == 0) return *(const lds_u32 *)(size_t)a;
    if constexpr (KIND == 1) return *(const lds_u8 *)(size_t)a;
    if constexpr (KIND == 2) return *(const lds_u16 *)(size_t)a;
    if constexpr (KIND == 3) {
        const uint64_t v = *(const lds_u64 *)(size_t)a;
        return (uint32_t)v ^ (uint32_t)(v >> 32);
    }
    return 0;
}

// KIND 0: b32, row x at x*256 (lane*4 within);  1: u8;  2: u16;  3: b64 (row x at x*512, lane*8).
template <int KIND, int W, int WPE, bool PURE>
__global__ void __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
k_reads(uint32_t *out, int iters) {
    for (int i = threadIdx.x; i < 16384; i += W * 64) *(lds_u32 *)(size_t)(4 * i) = i * 2654435761u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lb = KIND == 3 ? (lane & 31u) << 3 : (lane & 31u) << 2;
    uint32_t s[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) s[j] = threadIdx.x * 977u + j * 131u;
    for (int it = 0; it < iters; ++it) {
        uint32_t v[16];
        if constexpr (PURE) {
            const uint32_t base = ((s[0] & 0x3u) << (KIND == 3 ? 9 : 8)) | lb;
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = rd<KIND>(base + j * (KIND == 3 ? 2048u : 1024u));
            asm volatile("" ::: "memory");
#pragma unroll
            for (int j = 0; j < 16; j += 2) s[j] = __builtin_amdgcn_bitop3_b32(s[j], v[j], v[j + 1], 0x96);
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t x = s[j] & 0x3fu;
                v[j] = rd<KIND>(KIND == 3 ? (x << 9 | lb) : (x << 8 | lb));
            }
            asm volatile("" ::: "memory");
#pragma unroll
            for (int j = 0; j < 16; ++j) s[j] = (s[j] + v[j]) ^ (uint32_t)it;
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc ^= s[j];
    out[blockIdx.x * W * 64 + threadIdx.x] = acc;
}

template <int KIND, int W, int WGS, bool PURE = true>
void run(uint32_t *d, int cus, const char *name) {
    auto k = k_reads<KIND, W, W * WGS / 4, PURE>;
    const int lds = 65536;
    hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    const int iters = 4000;
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
    const double wave_ds = (double)cus * WGS * W * iters * 16;  // wave-instructions
    printf("%s %-4s waves/CU %2d: %.3f ms  %.1f G lane-reads/s  wave-reads per CU-cycle @2.2GHz %.3f\n",
           PURE ? "pure  " : "lookup", name, W * WGS, ms, wave_ds * 64 / ms / 1e6, wave_ds / cus / (ms * 1e-3 * 2.2e9));
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *d;
    hipMalloc(&d, 256 * 1024 * 4 * 4);
    run<0, 8, 1>(d, cus, "b32");
    run<1, 8, 1>(d, cus, "u8");
    run<2, 8, 1>(d, cus, "u16");
    run<3, 8, 1>(d, cus, "b64");
    run<0, 16, 2>(d, cus, "b32");
    run<1, 16, 2>(d, cus, "u8");
    run<2, 16, 2>(d, cus, "u16");
    run<3, 16, 2>(d, cus, "b64");
    run<0, 16, 2, false>(d, cus, "b32");
    run<1, 16, 2, false>(d, cus, "u8");
    return 0;
}
