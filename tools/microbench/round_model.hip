// Microbenchmark: AES T-table round throughput on gfx950 for two LDS table designs, to decide the
// quad kernel's layout.  valu_ops*.hip / bitop3_forms.hip measured that v_perm_b32,
// v_alignbit_b32 and any VALU op with an SGPR operand issue at ~4.5 cycles per wave-instruction per
// SIMD, v_bitop3_b32 / v_and / v_xor on VGPRs only at ~2.7.
//   cur: Te0/Te1 replicated 32x (64 KiB), Te2/Te3 = rot16; per round 16 x (v_perm address (SGPR
//        selector) + ds_read_b32), per column xor3(c0, c1, rot16(xor3(a0, a1, rk_sgpr))); 2 workgroups of
//        16 waves per CU (32 waves/CU).
//   four: Te0..Te3 replicated 32x (128 KiB); per round 12 v_perm addresses + 4 byte-1 addresses as one
//        all-VGPR v_bitop3 ((s & 0xff00) | lane base), per column xor3(xor3(a, b, c), d, rk_vgpr) on VGPRs
//        only; 1 workgroup of 16 waves per CU.
//   cur1: cur with the byte-1 lookups' address as one all-VGPR AND-OR (bitop3) instead of v_perm.
//   fast: the LDS pattern of cur (64 KiB, 32 waves/CU) with the least VALU: every address one all-VGPR
//        AND-OR, columns combined as four (not AES; the ceiling of the read pattern itself).
// Each lane runs kChains independent AES-like chains (the quad kernel has 1; more = ILP experiment).
// Prints CU-cycles per round per wave (one round of one 64-lane wave = 16 lookups).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 round_model.hip -o round_model
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

__device__ __forceinline__ uint32_t lds_rd(uint32_t a) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
__device__ __forceinline__ uint32_t perm_s(uint32_t s, uint32_t lb, uint32_t sel) {
    uint32_t d;
    asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(d) : "v"(s), "v"(lb), "s"(sel));
    return d;
}
__device__ __forceinline__ uint32_t andor_v(uint32_t s, uint32_t m, uint32_t lb) {
    uint32_t d;
    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xec" : "=v"(d) : "v"(s), "v"(m), "v"(lb));
    return d;
}
__device__ __forceinline__ uint32_t xor3_vvv(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ uint32_t xor3_vvs(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "s"(c));
    return d;
}
__device__ __forceinline__ uint32_t rot16(uint32_t a) {
    uint32_t d;
    asm volatile("v_alignbit_b32 %0, %1, %1, 16" : "=v"(d) : "v"(a));
    return d;
}
__device__ __forceinline__ void wait_lds() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// selectors: byte1 <- s.byte k, byte0 <- lb.byte0 (v_perm: S0 = s bytes 4..7, S1 = lb bytes 0..3)
#define SEL(k) (0x0c0c0400u + ((k) << 8))

template <int kDesign, int kChains>
__global__ void __launch_bounds__(1024) round_kernel(uint32_t *out, int iters, const uint32_t *rk_g, uint64_t *clk) {
    extern __shared__ uint32_t lds[];
    const uint32_t tbytes = kDesign != 1 ? 65536u : 131072u;  // design 3 (fast) uses the 64 KiB layout
    for (uint32_t i = threadIdx.x; i < tbytes / 4; i += 1024) lds[i] = (i * 2654435761u) & 0xffffffffu;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t lb = (lane & 31u) << 2;
    // table offsets: cur: Te0 at +0, Te1 at +128 within 256-B rows; four: rows of 512 B? no -- four
    // tables of 64 KiB... the 4-table layout: Te0/Te1 rows as cur in [0, 64K), Te2/Te3 in [64K, 128K)
    const uint32_t lb2 = lb | 0x10000u;  // lane base of the second 64 KiB (Te2/Te3)
    uint32_t m = 0xff00u ^ (lane & 0u);
    asm volatile("" : "+v"(m));
    uint32_t rkv[4];
    for (int c = 0; c < 4; ++c) rkv[c] = rk_g[c] ^ (lane & 0u);  // per-lane copies (VGPRs)
    const uint32_t rks0 = rk_g[0], rks1 = rk_g[1], rks2 = rk_g[2], rks3 = rk_g[3];
    uint32_t s[kChains][4];
    for (int j = 0; j < kChains; ++j)
        for (int c = 0; c < 4; ++c) s[j][c] = (threadIdx.x * (4 * j + c + 1)) * 2654435761u;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        uint32_t a[kChains][16];
#pragma unroll
        for (int j = 0; j < kChains; ++j) {
            if constexpr (kDesign == 3) {  // VALU floor: every address one all-VGPR AND-OR (not AES)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    a[j][4 * c + 0] = lds_rd(andor_v(s[j][c], m, lb));
                    a[j][4 * c + 1] = lds_rd(andor_v(s[j][(c + 1) & 3], m, lb) + 128u);
                    a[j][4 * c + 2] = lds_rd(andor_v(s[j][(c + 2) & 3], m, lb));
                    a[j][4 * c + 3] = lds_rd(andor_v(s[j][(c + 3) & 3], m, lb) + 128u);
                }
            } else if constexpr (kDesign == 2) {
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    a[j][4 * c + 0] = lds_rd(perm_s(s[j][c], lb, SEL(0)));
                    a[j][4 * c + 1] = lds_rd(andor_v(s[j][(c + 1) & 3], m, lb) + 128u);
                    a[j][4 * c + 2] = lds_rd(perm_s(s[j][(c + 2) & 3], lb, SEL(2)));
                    a[j][4 * c + 3] = lds_rd(perm_s(s[j][(c + 3) & 3], lb, SEL(3)) + 128u);
                }
            } else if constexpr (kDesign == 0) {
                // column c: Te0[s_c.b0] ^ Te1[s_c+1.b1] ^ rot16(Te0[s_c+2.b2] ^ Te1[s_c+3.b3])
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    a[j][4 * c + 0] = lds_rd(perm_s(s[j][c], lb, SEL(0)));
                    a[j][4 * c + 1] = lds_rd(perm_s(s[j][(c + 1) & 3], lb, SEL(1)) + 128u);
                    a[j][4 * c + 2] = lds_rd(perm_s(s[j][(c + 2) & 3], lb, SEL(2)));
                    a[j][4 * c + 3] = lds_rd(perm_s(s[j][(c + 3) & 3], lb, SEL(3)) + 128u);
                }
            } else {
                // column c: Te0[b0] ^ Te1[b1] ^ Te2[b2] ^ Te3[b3]; byte 1 by an all-VGPR AND-OR
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    a[j][4 * c + 0] = lds_rd(perm_s(s[j][c], lb, SEL(0)));
                    a[j][4 * c + 1] = lds_rd(andor_v(s[j][(c + 1) & 3], m, lb) + 128u);
                    a[j][4 * c + 2] = lds_rd(perm_s(s[j][(c + 2) & 3], lb2, 0x0c020400u + (2 << 8)));
                    a[j][4 * c + 3] = lds_rd(perm_s(s[j][(c + 3) & 3], lb2, 0x0c020400u + (3 << 8)) + 128u);
                }
            }
        }
        wait_lds();
#pragma unroll
        for (int j = 0; j < kChains; ++j) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint32_t *x = &a[j][4 * c];
                if constexpr (kDesign != 1 && kDesign != 3) {
                    const uint32_t rk = c == 0 ? rks0 : c == 1 ? rks1 : c == 2 ? rks2 : rks3;
                    s[j][c] = xor3_vvv(x[0], x[1], rot16(xor3_vvs(x[2], x[3], rk)));
                } else {
                    s[j][c] = xor3_vvv(xor3_vvv(x[0], x[1], x[2]), x[3], rkv[c]);
                }
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    for (int j = 0; j < kChains; ++j)
        for (int c = 0; c < 4; ++c) acc ^= s[j][c];
    if (acc == 0x12345u) out[0] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

int main() {
    uint32_t *d, *rk;
    uint64_t *clk;
    CHECK(hipMalloc(&d, 4));
    CHECK(hipMalloc(&rk, 64));
    CHECK(hipMemset(rk, 0x5a, 64));
    CHECK(hipMalloc(&clk, 16));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    struct Cfg {
        const void *fn;
        int design, chains;
    };
    const Cfg cfgs[] = {{(const void *)&round_kernel<0, 1>, 0, 1}, {(const void *)&round_kernel<2, 1>, 2, 1},
                        {(const void *)&round_kernel<2, 2>, 2, 2}, {(const void *)&round_kernel<1, 1>, 1, 1},
                        {(const void *)&round_kernel<1, 2>, 1, 2}, {(const void *)&round_kernel<1, 3>, 1, 3},
                        {(const void *)&round_kernel<1, 4>, 1, 4}, {(const void *)&round_kernel<3, 1>, 3, 1},
                        {(const void *)&round_kernel<3, 2>, 3, 2}};
    const char *dn[4] = {"cur", "four", "cur1", "fast"};
    for (const Cfg &c : cfgs)
        CHECK(hipFuncSetAttribute(c.fn, hipFuncAttributeMaxDynamicSharedMemorySize, c.design == 1 ? 131072 : 65536));
    const int iters = 20000;
    for (int rep = 0; rep < 2; ++rep)
        for (const Cfg &cf : cfgs) {
            const int wgs_per_cu = cf.design == 1 ? 1 : 2;  // 16-wave workgroups: 16 / 32 waves per CU
            const int grid = cus * wgs_per_cu;
            const size_t lds = cf.design == 1 ? 131072 : 65536;
            int it_ = iters;
            void *args[] = {&d, &it_, &rk, &clk};
            CHECK(hipLaunchKernel(cf.fn, dim3(grid), dim3(1024), args, lds, nullptr));
            CHECK(hipEventRecord(e0));
            CHECK(hipLaunchKernel(cf.fn, dim3(grid), dim3(1024), args, lds, nullptr));
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            uint64_t c[2];
            CHECK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
            const double ghz = (double)c[0] / (double)c[1] * 0.1;
            const double wave_rounds_per_cu = (double)iters * cf.chains * 16 * wgs_per_cu;
            const double cyc = ms * 1e6 * ghz / wave_rounds_per_cu;
            printf("%-5s chains %d waves/CU %2d: %.3f ms  clock %.2f GHz  %.2f CU-cycles per wave-round "
                   "(LDS floor 32)  lookups/CU-cycle %.3f\n",
                   dn[cf.design], cf.chains, 16 * wgs_per_cu, ms, ghz, cyc, 16.0 / cyc);
        }
    return 0;
}
