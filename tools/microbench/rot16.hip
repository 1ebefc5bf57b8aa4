// Microbenchmark: rot16 (swap the 16-bit halves of a dword) and byte-1 address candidates on gfx950,
// 16 independent chains per wave, 8 waves per SIMD (see valu_ops.hip / valu_ops2.hip).
//   pk_add    v_pk_add_u16 d, s, 0 op_sel:[1,0] op_sel_hi:[0,1]   (halves swapped by the op_sel bits)
//   alignbyte v_alignbyte_b32 d, s, s, 2
//   alignbit  v_alignbit_b32 d, s, s, 16
//   xor_sdwa  v_xor_b32_sdwa d, a, b src1_sel:WORD_1 (the high half of b into the low half)
//   bitop3_ao v_bitop3_b32 d, s, m(SGPR), lb: (s & m) | lb -- a byte-1 LDS address in one full-rate op
//   pk_mov    v_pk_mov_b32 d[0:1], s[0:1], s[0:1] op_sel:[1,0]
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 rot16.hip -o rot16
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
    uint32_t msk = 0xff00u ^ (sk & 0u);
    asm volatile("" : "+s"(msk));
#define DECL(i) uint32_t x##i = (threadIdx.x * (i + 3)) * 2654435761u; uint64_t y##i = x##i * 0x100000001ull;
    R16(DECL)
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (kOp == 0) {
#define OP(i) asm volatile("v_pk_add_u16 %0, %0, 0 op_sel:[1,0] op_sel_hi:[0,1]" : "+v"(x##i));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 1) {
#define OP(i) asm volatile("v_alignbyte_b32 %0, %0, %0, 2" : "+v"(x##i));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 2) {
#define OP(i) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(x##i));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 3) {
#define OP(i) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(x##i) : "v"(lb));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 4) {
#define OP(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xec" : "+v"(x##i) : "s"(msk), "v"(lb));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 5) {
#define OP(i) asm volatile("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]" : "+v"(y##i));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 6) {
#define OP(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x##i) : "v"(lb));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 7) {
#define OP(i) asm volatile("v_lshlrev_b32 %0, 8, %0" : "+v"(x##i));
            R16(OP)
#undef OP
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#define ACC(i) acc ^= x##i ^ (uint32_t)y##i;
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
    const char *names[8] = {"pk_add", "alignbyte", "alignbit", "xor_sdwa", "bitop3_ao", "pk_mov", "add_u32", "lshl"};
    const int iters = 20000;
    for (int op = 0; op < 8; ++op) {
        const int wps = 8;
        const int grid = cus * wps / 4;
        auto launch = [&]() {
            switch (op) {
#define CASE(k) case k: ops_kernel<k><<<grid, 1024>>>(d, iters, 3, clk); break;
                CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7)
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
        printf("%-10s waves/SIMD %d: %.3f ms  %.3f ns/wave-instr/SIMD  clock %.2f GHz  %.2f cycles\n", names[op], wps, ms,
               ns, ghz, ns * ghz);
    }
    return 0;
}
