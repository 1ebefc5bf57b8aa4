// Microbenchmark 2: issue cost of candidate LDS-address builds for the T-table round on gfx950.
// The address of a T-table lookup is (byte k of a state word) << 8 | lane*4.  hipcc builds it with
// one v_perm_b32 (SGPR selector), which valu_ops.hip measured at ~4.2 cycles per wave-instruction per
// SIMD (v_bitop3_b32 ~2.4).  Candidates, each 16 independent chains per wave, 8 waves per SIMD:
//   sdwa_b1   v_mov_b32_sdwa a, s  dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2
//   andor     v_and_or_b32 a, s, m(SGPR), lb       (byte 1 in place)
//   bfe       v_bfe_u32 a, s, 16, 8
//   lshlor    v_lshl_or_b32 a, s, 8, lb
//   lshl_sdwa v_lshlrev_b32_sdwa a, 8, s src1_sel:BYTE_2
//   xor_e64   v_xor_b32_e64 a, a, lb
//   and       v_and_b32 a, s(SGPR), a
//   mov       v_mov_b32 a, a
// then the round mix: per lookup one address op + one ds_read_b32, plus 3 combine ops per 4 lookups
// (2 v_bitop3 + 1 v_alignbit, as round_full), for perm / sdwa / andor address builds.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 valu_ops2.hip -o valu_ops2
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
#define R4(M) M(0) M(1) M(2) M(3)

template <int kOp>
__global__ void __launch_bounds__(1024) ops_kernel(uint32_t *out, int iters, uint32_t sk, uint64_t *clk) {
    extern __shared__ uint32_t lds[];
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t i = threadIdx.x; i < 16384; i += 1024) lds[i] = (i * 2654435761u) & 0x00ff00ffu;
    __syncthreads();
    uint32_t lb = (lane & 31u) << 2;
    uint32_t sel = sk;
    uint32_t msk = 0xff00u ^ (sk & 0u);
    asm volatile("" : "+s"(msk));
#define DECL(i) uint32_t x##i = (threadIdx.x * (i + 3)) & 0x00ff00ffu; uint32_t a##i = lb;
    R16(DECL)
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (kOp == 0) {
#define OP(i) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a##i) : "v"(x##i)); \
              asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(x##i) : "v"(a##i));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 1) {
#define OP(i) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x##i) : "s"(msk), "v"(lb));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 2) {
#define OP(i) asm volatile("v_bfe_u32 %0, %0, 16, 8" : "+v"(x##i));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 3) {
#define OP(i) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(x##i) : "v"(lb));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 4) {
#define OP(i) asm volatile("v_lshlrev_b32_sdwa %0, 8, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "+v"(x##i));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 5) {
#define OP(i) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(x##i) : "v"(lb));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 6) {
#define OP(i) asm volatile("v_and_b32 %0, %1, %0" : "+v"(x##i) : "s"(msk));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 7) {
#define OP(i) asm volatile("v_mov_b32 %0, %1" : "=v"(a##i) : "v"(x##i)); asm volatile("v_mov_b32 %0, %1" : "=v"(x##i) : "v"(a##i));
            R16(OP)
#undef OP
        } else {
            // round mix: 16 x (address op + ds_read_b32), then 4 x (2 bitop3 + 1 alignbit)
#define ADDR(i)                                                                                                    \
    if constexpr (kOp == 8)                                                                                        \
        asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(a##i) : "v"(x##i), "v"(lb), "s"(sel));                   \
    else if constexpr (kOp == 9)                                                                                   \
        asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2"          \
                     : "+v"(a##i) : "v"(x##i));                                                                   \
    else                                                                                                           \
        asm volatile("v_and_or_b32 %0, %1, %2, %3" : "=v"(a##i) : "v"(x##i), "s"(msk), "v"(lb));
            R16(ADDR)
#undef ADDR
#define LD(i) asm volatile("ds_read_b32 %0, %1" : "=v"(x##i) : "v"(a##i));
            R16(LD)
#undef LD
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#define CMB(c)                                                                                                     \
    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x##c) : "v"(x##c##4), "v"(lb));               \
    asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(x##c));                                                     \
    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x##c) : "v"(x##c##8), "v"(lb));
#define x04 x4
#define x14 x5
#define x24 x6
#define x34 x7
#define x08 x8
#define x18 x9
#define x28 x10
#define x38 x11
            CMB(0) CMB(1) CMB(2) CMB(3)
#undef CMB
            // keep the chained values inside the 64 KiB table: bytes 1 and 3 of every word zero
#define MSK(i) asm volatile("v_and_b32 %0, 0xff00ff, %0" : "+v"(x##i));
            R4(MSK)
#undef MSK
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#define ACC(i) acc ^= x##i ^ a##i;
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
    const char *names[11] = {"sdwa_b1", "andor", "bfe", "lshlor", "lshl_sdwa", "xor_e64", "and", "mov",
                             "mix_perm", "mix_sdwa", "mix_andor"};
    const int per_it[11] = {32, 16, 16, 16, 16, 16, 16, 32, 48, 48, 48};  // wave-instructions per iteration
    const int iters = 20000;
    const uint32_t sel = 0x0c0c0600u;  // byte0 <- lb.byte0, byte1 <- s.byte2
    for (int op = 0; op < 11; ++op) {
        const int wps = 8;
        const int grid = cus * wps / 4;
        auto launch = [&]() {
            switch (op) {
#define CASE(k) case k: ops_kernel<k><<<grid, 1024, 65536>>>(d, iters, sel, clk); break;
                CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9) CASE(10)
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
        const double instr_per_simd = (double)iters * per_it[op] * wps;
        const double ns = ms * 1e6 / instr_per_simd;
        // the mixes: cycles per lookup per CU (16 lookups per iteration per wave, 32 waves per CU)
        const double lookups_per_cu = (double)iters * 16 * 32;
        printf("%-10s waves/SIMD %d: %.3f ms  %.3f ns/wave-instr/SIMD  clock %.2f GHz  %.2f cycles/instr/SIMD"
               "  (mix: %.2f CU-cycles per wave lookup)\n",
               names[op], wps, ms, ns, ghz, ns * ghz, ms * 1e6 * ghz / lookups_per_cu);
    }
    return 0;
}
