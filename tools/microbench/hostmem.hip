// Host-memory access forms for a kernel that keeps running while the host rewrites the buffer (the
// resident per-packet kernel): per request the host writes `bytes` of fresh data and a sequence
// number; one 256-thread workgroup polls the sequence (system-scope atomic), reads the buffer with
// form F, writes it back XOR-ed with the sequence, drains, and publishes the sequence.  The host checks
// every byte (a stale read shows up as a mismatch) and times the round trip.
//   F0: 8-B relaxed system-scope atomics (global_load/store_dwordx2 sc0 sc1)
//   F1: 16-B plain loads and stores
//   F2: 16-B buffer loads/stores with sc0 sc1 (aux bits)
//   F3: 16-B buffer loads with sc1 (bypass L1), plain 16-B stores
//   F4: 16-B plain loads after a system acquire fence, plain stores + system release fence
//   F5: 16-B buffer loads sc0 sc1, 16-B buffer stores sc0 sc1 nt
//   F6: 16-B buffer loads sc0 sc1, plain 16-B stores + system release fence
//   F7: 16-B buffer loads sc0 sc1, 16-B buffer stores sc1
// Allocation: hipHostMallocCoherent (A=1) or hipHostMallocDefault (A=0).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench/hostmem.hip -o tools/bin/hostmem
// Usage: hostmem <form> <coherent> <bytes> <requests>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>

template <int F>
__device__ __forceinline__ uint4 ld16(uint8_t *buf, uint32_t i) {
    if constexpr (F == 0) {
        const uint64_t *p = reinterpret_cast<const uint64_t *>(buf) + 2 * i;
        const uint64_t a = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t c = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return uint4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)c, (uint32_t)(c >> 32)};
    } else if constexpr (F == 2 || F == 3 || F >= 5) {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 0x7fffffff, 0x00020000);
        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
        const v4 v = __builtin_amdgcn_raw_buffer_load_b128(r, 16 * i, 0, F == 3 ? 16 : 17);
        return uint4{v.x, v.y, v.z, v.w};
    } else {
        return reinterpret_cast<const uint4 *>(buf)[i];
    }
}
template <int F>
__device__ __forceinline__ void st16(uint8_t *buf, uint32_t i, uint4 v) {
    if constexpr (F == 0) {
        uint64_t *p = reinterpret_cast<uint64_t *>(buf) + 2 * i;
        __hip_atomic_store(p, (uint64_t)v.x | (uint64_t)v.y << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(p + 1, (uint64_t)v.z | (uint64_t)v.w << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if constexpr (F == 2 || F == 5 || F == 7) {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 0x7fffffff, 0x00020000);
        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(v4{v.x, v.y, v.z, v.w}, r, 16 * i, 0, F == 2 ? 17 : F == 5 ? 19 : 16);
    } else {
        reinterpret_cast<uint4 *>(buf)[i] = v;
    }
}

template <int F>
__global__ void __launch_bounds__(256) serve(uint8_t *buf, uint32_t n16, uint32_t *seq, uint32_t *done, uint32_t reqs,
                                             unsigned long long *cycles) {
    __shared__ uint32_t s_q;
    unsigned long long busy = 0;
    for (uint32_t r = 1; r <= reqs; ++r) {
        if (threadIdx.x == 0) {
            uint64_t spins = 0;
            while (__hip_atomic_load(seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != r) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins > (1ull << 28)) break;  // exit condition: the host is gone
            }
            s_q = r;
        }
        __syncthreads();
        const unsigned long long t0 = wall_clock64();
        if constexpr (F == 4) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        const uint32_t q = s_q;
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = threadIdx.x + 256 * k;
            if (i < n16) v[k] = ld16<F>(buf, i);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = threadIdx.x + 256 * k;
            if (i < n16) st16<F>(buf, i, uint4{v[k].x ^ q, v[k].y ^ q, v[k].z ^ q, v[k].w ^ q});
        }
        if constexpr (F == 4 || F == 6) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(done, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            busy += wall_clock64() - t0;
        }
    }
    if (threadIdx.x == 0) *cycles = busy;
}

int main(int argc, char **argv) {
    const int F = argc > 1 ? atoi(argv[1]) : 1;
    const bool coh = argc > 2 ? atoi(argv[2]) != 0 : true;
    const uint32_t bytes = argc > 3 ? atoi(argv[3]) : 1408;
    const uint32_t reqs = argc > 4 ? atoi(argv[4]) : 20000;
    const uint32_t n16 = (bytes + 15) / 16;
    uint8_t *buf;
    uint32_t *ctl;
    unsigned long long *d_cycles, cycles = 0;
    if (hipHostMalloc((void **)&buf, 32768, coh ? hipHostMallocCoherent : hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&ctl, 4096, hipHostMallocCoherent) != hipSuccess || hipMalloc(&d_cycles, 8) != hipSuccess)
        return 1;
    memset(ctl, 0, 4096);
    uint32_t *seq = ctl, *done = ctl + 16;
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    void (*k)(uint8_t *, uint32_t, uint32_t *, uint32_t *, uint32_t, unsigned long long *) =
        F == 0 ? serve<0> : F == 1 ? serve<1> : F == 2 ? serve<2> : F == 3 ? serve<3> : F == 4 ? serve<4>
        : F == 5 ? serve<5> : F == 6 ? serve<6> : serve<7>;
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, s, buf, n16, seq, done, reqs, d_cycles);
    // random request contents, drawn before the timed loop
    const size_t nb = 16ull * n16;
    uint8_t *pool = (uint8_t *)malloc(nb * 64 + 64);
    srand(7);
    for (size_t i = 0; i < nb * 64 + 64; ++i) pool[i] = (uint8_t)rand();
    long bad = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t r = 1; r <= reqs; ++r) {
        const uint8_t *ref = pool + (r % 64) * nb;
        memcpy(buf, ref, nb);
        __atomic_store_n(seq, r, __ATOMIC_RELEASE);
        while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != r) __builtin_ia32_pause();
        for (uint32_t i = 0; i < 16 * n16; ++i)
            if (buf[i] != (uint8_t)(ref[i] ^ (uint8_t)(r >> (8 * (i & 3))))) {
                ++bad;
                break;
            }
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    hipStreamSynchronize(s);
    hipMemcpy(&cycles, d_cycles, 8, hipMemcpyDeviceToHost);
    printf("{\"form\": %d, \"coherent\": %d, \"bytes\": %u, \"requests\": %u, \"round_trip_us\": %.2f, "
           "\"kernel_busy_us_per_req\": %.2f, \"stale_or_wrong\": %ld}\n",
           F, coh ? 1 : 0, 16 * n16, reqs, dt / reqs * 1e6, cycles / 100.0 / reqs, bad);
    return bad ? 2 : 0;
}
