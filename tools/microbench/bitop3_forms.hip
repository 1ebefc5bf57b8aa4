// Microbenchmark: which v_bitop3_b32 forms issue at full rate on gfx950 (valu_ops / rot16 found XOR3 on
// three VGPRs or with an SGPR in src2 at ~2.4 cycles per wave-instruction per SIMD, AND-OR with an
// SGPR in src1 at ~4.8).  Forms: truth table {XOR3 0x96, AND-OR 0xec} x SGPR position {none, src1, src2}.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 bitop3_forms.hip -o bitop3_forms
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

#define R16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

template <int kOp>
__global__ void __launch_bounds__(1024) ops_kernel(uint32_t *out, int iters, uint32_t sk, uint64_t *clk) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t lb = (lane & 31u) << 2;
    uint32_t vm = 0xff00u ^ (lane & 0u);
    asm volatile("" : "+v"(vm));
    uint32_t msk = 0xff00u ^ (sk & 0u);
    asm volatile("" : "+s"(msk));
#define DECL(i) uint32_t x##i = (threadIdx.x * (i + 3)) * 2654435761u;
    R16(DECL)
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#define OP(i)                                                                                               \
    if constexpr (kOp == 0) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x##i) : "v"(vm), "v"(lb)); \
    if constexpr (kOp == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x##i) : "s"(msk), "v"(lb)); \
    if constexpr (kOp == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x##i) : "v"(lb), "s"(msk)); \
    if constexpr (kOp == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xec" : "+v"(x##i) : "v"(vm), "v"(lb)); \
    if constexpr (kOp == 4) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xec" : "+v"(x##i) : "s"(msk), "v"(lb)); \
    if constexpr (kOp == 5) asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xec" : "+v"(x##i) : "v"(lb), "s"(msk)); \
    if constexpr (kOp == 6) asm volatile("v_and_b32_e64 %0, %0, %1" : "+v"(x##i) : "v"(vm));                        \
    if constexpr (kOp == 7) asm volatile("v_or_b32_e64 %0, %0, %1" : "+v"(x##i) : "v"(lb));                         \
    if constexpr (kOp == 8) asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(x##i) : "v"(lb));                        \
    if constexpr (kOp == 9) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(x##i) : "v"(vm), "v"(lb));
        R16(OP)
#undef OP
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#define ACC(i) acc ^= x##i;
    R16(ACC)
    if (acc == 0x12345u) out[0] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

int main() {
    uint32_t *d;
    uint64_t *clk;
    CHECK(hipMalloc(&d, 4));
    CHECK(hipMalloc(&clk, 16));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char *names[10] = {"xor3 vvv", "xor3 vsv", "xor3 vvs", "andor vvv", "andor vsv", "andor(lb,x,s)",
                             "and_e64 vv", "or_e64 vv", "xor_e32 vv", "bfi vvv"};
    const int iters = 20000;
    for (int rep = 0; rep < 2; ++rep)
    for (int op = 0; op < 10; ++op) {
        const int wps = 8;
        const int grid = cus * wps / 4;
        auto launch = [&]() {
            switch (op) {
#define CASE(k) case k: ops_kernel<k><<<grid, 1024>>>(d, iters, 3, clk); break;
                CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9)
#undef CASE
            }
        };
        launch();
        CHECK(hipEventRecord(e0));
        launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        uint64_t c[2];
        CHECK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
        const double ghz = (double)c[0] / (double)c[1] * 0.1;
        const double ns = ms * 1e6 / ((double)iters * 16 * wps);
        printf("%-14s %.3f ms  %.3f ns/wave-instr/SIMD  clock %.2f GHz  %.2f cycles\n", names[op], ms, ns, ghz, ns * ghz);
    }
    return 0;
}
