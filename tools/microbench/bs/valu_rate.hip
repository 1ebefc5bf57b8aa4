// Microbenchmark: VALU issue rate on gfx950 for the ops of a bitsliced AES (v_bitop3_b32 with
// 3 VGPR sources, 2 VGPR + 1 SGPR, v_xor_b32, v_mov_b32_dpp) vs waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

constexpr int kRegs = 24;

template <int kOp>
__global__ void __launch_bounds__(256) valu_kernel(uint32_t *out, int iters, uint32_t sk) {
    uint32_t v[kRegs];
#pragma unroll
    for (int i = 0; i < kRegs; ++i) v[i] = threadIdx.x * (i + 1) + blockIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int rep = 0; rep < 4; ++rep)
#pragma unroll
            for (int i = 0; i < kRegs; ++i) {
                const uint32_t a = v[(i + 7) % kRegs], b = v[(i + 13) % kRegs];
                if (kOp == 0) v[i] = __builtin_amdgcn_bitop3_b32(v[i], a, b, 0x6a);
                if (kOp == 1) v[i] = __builtin_amdgcn_bitop3_b32(v[i], a, sk + rep, 0x6a);
                if (kOp == 2) v[i] = v[i] ^ a;
                if (kOp == 3) v[i] = v[i] ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)a, 0x39, 0xf, 0xf, false);
            }
        asm volatile("" ::: "memory");
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < kRegs; ++i) acc ^= v[i];
    if (acc == 0x12345u) out[0] = acc;
}

int main() {
    uint32_t *d;
    CHECK(hipMalloc(&d, 4));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char *names[4] = {"bitop3 3xVGPR", "bitop3 2xVGPR+SGPR", "v_xor_b32", "v_xor + v_mov_dpp"};
    const int iters = 4000;
    for (int op = 0; op < 4; ++op) {
        for (int wps = 1; wps <= 8; wps *= 2) {
            const int grid = cus * wps;
            auto launch = [&]() {
                if (op == 0) valu_kernel<0><<<grid, 256>>>(d, iters, 3);
                if (op == 1) valu_kernel<1><<<grid, 256>>>(d, iters, 3);
                if (op == 2) valu_kernel<2><<<grid, 256>>>(d, iters, 3);
                if (op == 3) valu_kernel<3><<<grid, 256>>>(d, iters, 3);
            };
            launch();
            CHECK(hipEventRecord(e0));
            launch();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double instrs = (double)iters * 4 * kRegs * (op == 3 ? 2 : 1);  // per wave
            const double waves_per_simd = wps;
            // cycles per instruction per SIMD at an assumed 2.4 GHz (also print instr/ns per SIMD)
            const double per_simd_instr = instrs * waves_per_simd;
            printf("%-22s waves/SIMD %d: %.3f ms, %.3f wave-instr/ns/SIMD (%.2f cyc @2.4GHz)\n", names[op], wps, ms,
                   per_simd_instr / (ms * 1e6), (ms * 1e6) * 2.4 / per_simd_instr);
        }
    }
    return 0;
}
