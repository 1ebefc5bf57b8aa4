// Microbenchmark: issue cost of the VALU forms the T-table AES round uses on gfx950, by operand kind.
//   perm_s   v_perm_b32 v, v, v, s   (address build with the selector in an SGPR -- what hipcc emits)
//   perm_v   v_perm_b32 v, v, v, v   (selector in a VGPR)
//   bitop3_v v_bitop3_b32 v, v, v, v (XOR3 on three VGPRs)
//   bitop3_s v_bitop3_b32 v, v, v, s
//   xor      v_xor_b32 v, v, v
//   align    v_alignbit_b32 v, v, v, 16 (rot16)
//   perm_s+ds  one v_perm_b32 (SGPR selector) + one conflict-free ds_read_b32 per pair, the round's mix
//   perm_v+ds  the same with the selector in a VGPR
// 16 independent chains per wave (inline asm, operands fixed), 8 waves per SIMD.  Prints ns per
// wave-instruction per SIMD and cycles at the clock read from s_memtime / s_memrealtime.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 valu_ops.hip -o valu_ops
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
    extern __shared__ uint32_t lds[];
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t i = threadIdx.x; i < 16384; i += 1024) lds[i] = i * 2654435761u;
    __syncthreads();
    uint32_t lb = (lane & 31u) << 2;
    uint32_t sel = sk;  // 0x0c0c0100-ish, opaque to the compiler
    uint32_t vsel = sk ^ threadIdx.x * 0u;
    asm volatile("" : "+v"(vsel));
#define DECL(i) uint32_t x##i = threadIdx.x * (i + 3) + 0x01000000u * i;
    R16(DECL)
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (kOp == 0) {
#define OP(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x##i) : "v"(lb), "s"(sel));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 1) {
#define OP(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x##i) : "v"(lb), "v"(vsel));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 2) {
#define OP(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x##i) : "v"(lb), "v"(vsel));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 3) {
#define OP(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x##i) : "v"(lb), "s"(sel));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 4) {
#define OP(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x##i) : "v"(lb));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 5) {
#define OP(i) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(x##i));
            R16(OP)
#undef OP
        } else if constexpr (kOp == 6 || kOp == 7) {
            // x = lds[perm(x, lb, sel)]: an address build + a lookup per chain, 16 chains in flight
#define OP(i)                                                                                  \
    if constexpr (kOp == 6)                                                                    \
        asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x##i) : "v"(lb), "s"(sel));          \
    else                                                                                       \
        asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x##i) : "v"(lb), "v"(vsel));
            R16(OP)
#undef OP
#define LD(i) asm volatile("ds_read_b32 %0, %0" : "+v"(x##i));
            R16(LD)
#undef LD
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
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
    const char *names[8] = {"perm_s", "perm_v", "bitop3_v", "bitop3_s", "xor", "align", "perm_s+ds", "perm_v+ds"};
    const int iters = 20000;
    // selector: byte1 <- s.byte1? any fixed pattern; LDS addresses stay inside 64 KiB: bytes 2,3 = 0
    const uint32_t sel = 0x0c0c0500u;
    for (int op = 0; op < 8; ++op) {
        for (int wps : {4, 8}) {
            const int grid = cus * wps / 4;  // 1024-thread workgroups: four waves per SIMD each
            auto launch = [&]() {
                switch (op) {
                    case 0: ops_kernel<0><<<grid, 1024, 65536>>>(d, iters, sel, clk); break;
                    case 1: ops_kernel<1><<<grid, 1024, 65536>>>(d, iters, sel, clk); break;
                    case 2: ops_kernel<2><<<grid, 1024, 65536>>>(d, iters, sel, clk); break;
                    case 3: ops_kernel<3><<<grid, 1024, 65536>>>(d, iters, sel, clk); break;
                    case 4: ops_kernel<4><<<grid, 1024, 65536>>>(d, iters, sel, clk); break;
                    case 5: ops_kernel<5><<<grid, 1024, 65536>>>(d, iters, sel, clk); break;
                    case 6: ops_kernel<6><<<grid, 1024, 65536>>>(d, iters, sel, clk); break;
                    case 7: ops_kernel<7><<<grid, 1024, 65536>>>(d, iters, sel, clk); break;
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
            const double ghz = (double)c[0] / (double)c[1] * 0.1;  // s_memrealtime is 100 MHz
            const int per_it = op >= 6 ? 32 : 16;                 // wave-instructions per iteration
            const double instr_per_simd = (double)iters * per_it * wps;
            const double ns = ms * 1e6 / instr_per_simd;
            printf("%-10s waves/SIMD %d: %.3f ms  %.3f ns/wave-instr/SIMD  clock %.2f GHz  %.2f cycles\n", names[op], wps,
                   ms, ns, ghz, ns * ghz);
        }
    }
    return 0;
}
