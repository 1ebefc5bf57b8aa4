// Where should a resident kernel's requests live?  A kernel serves requests the host posts while it
// runs (as gcm_resident_kernel does): per request the host writes `bytes` of fresh data and a sequence
// number; one 256-thread workgroup polls the sequence, reads the data, writes it back XOR-ed with the
// sequence into pinned host memory, drains, and publishes the sequence in a host done word.  The host
// checks every byte and times the round trip.
//   mode 0: request in pinned coherent host memory (what the resident kernel does today): the GPU
//           polls over PCIe, then reads the data over PCIe (two round trips before it can work)
//   mode 1: request in fine-grained DEVICE memory that the host CPU writes through the BAR
//           (hipExtMallocWithFlags(hipDeviceMallocFinegrained), CPU access granted through HSA):
//           the host's stores are posted writes, the GPU polls and reads its own HBM
// All GPU accesses of memory the other side rewrites are 16-B buffer accesses with sc0 sc1.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench/barreq.hip -lhsa-runtime64 -o tools/bin/barreq
// Usage: barreq <mode> <bytes> <requests>
#include <emmintrin.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u ld16(const void *base, uint32_t bytes, uint32_t off) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)bytes, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 17);
}
__device__ __forceinline__ void st16(void *base, uint32_t bytes, uint32_t off, v4u v) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 17);
}

// req: [0,16) header {seq, 0, 0, 0}, [64, 64 + bytes) data.  out (host): the result.  done (host).
__global__ void __launch_bounds__(256) serve(const uint8_t *req, uint8_t *out, uint32_t n16, uint32_t *done,
                                             uint32_t reqs, unsigned long long *cycles) {
    __shared__ uint32_t s_q;
    const uint32_t span = 64 + 16 * n16;
    unsigned long long busy = 0;
    for (uint32_t r = 1; r <= reqs; ++r) {
        if (threadIdx.x == 0) {
            uint64_t spins = 0;
            uint32_t got = r;
            while (ld16(req, span, 0).x != r) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1ull << 21)) {  // exit condition: the host is gone (a few seconds)
                    got = 0;
                    break;
                }
            }
            s_q = got;
        }
        __syncthreads();
        const unsigned long long t0 = wall_clock64();
        const uint32_t q = s_q;
        if (q == 0) break;  // every thread leaves
        v4u v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = threadIdx.x + 256 * k;
            if (i < n16) v[k] = ld16(req, span, 64 + 16 * i);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = threadIdx.x + 256 * k;
            if (i < n16) st16(out, 16 * n16, 16 * i, v[k] ^ q);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_store(done, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            busy += wall_clock64() - t0;
        }
    }
    if (threadIdx.x == 0) *cycles = busy;
}

static hsa_agent_t g_cpu;
static hsa_status_t find_cpu(hsa_agent_t a, void *found) {
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
        g_cpu = a;
        *static_cast<bool *>(found) = true;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 1;
    const uint32_t bytes = argc > 2 ? atoi(argv[2]) : 1408;
    const uint32_t reqs = argc > 3 ? atoi(argv[3]) : 20000;
    const uint32_t n16 = (bytes + 15) / 16;
    if (n16 > 2048) return 1;
    uint8_t *req = nullptr, *out = nullptr;
    uint32_t *ctl = nullptr;
    unsigned long long *d_cycles = nullptr, cycles = 0;
    if (hipHostMalloc((void **)&out, 32768, hipHostMallocCoherent) != hipSuccess ||
        hipHostMalloc((void **)&ctl, 4096, hipHostMallocCoherent) != hipSuccess || hipMalloc(&d_cycles, 8) != hipSuccess)
        return 1;
    memset(ctl, 0, 4096);
    if (mode == 0) {
        if (hipHostMalloc((void **)&req, 65536, hipHostMallocCoherent) != hipSuccess) return 1;
    } else {
        if (hipExtMallocWithFlags((void **)&req, 65536, hipDeviceMallocFinegrained) != hipSuccess) {
            fprintf(stderr, "fine-grained device allocation failed\n");
            return 3;
        }
        bool found = false;
        hsa_iterate_agents(find_cpu, &found);
        const hsa_status_t st = found ? hsa_amd_agents_allow_access(1, &g_cpu, nullptr, req) : HSA_STATUS_ERROR;
        hipPointerAttribute_t at;
        const bool attr = hipPointerGetAttributes(&at, req) == hipSuccess;
        fprintf(stderr, "allow_access(cpu) = %d, hostPointer = %p, devicePointer = %p\n", (int)st,
                attr ? at.hostPointer : nullptr, attr ? at.devicePointer : nullptr);
        if (st != HSA_STATUS_SUCCESS) return 4;
    }
    memset(req, 0, 64 + 16 * n16);  // the first host write into the region (faults here if it is not mapped)
    _mm_sfence();
    uint32_t *done = ctl;
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipLaunchKernelGGL(serve, dim3(1), dim3(256), 0, s, req, out, n16, done, reqs, d_cycles);
    const size_t nb = 16ull * n16;
    uint8_t *pool = (uint8_t *)malloc(nb * 64 + 64);
    srand(7);
    for (size_t i = 0; i < nb * 64 + 64; ++i) pool[i] = (uint8_t)rand();
    long bad = 0;
    double post_ns = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t r = 1; r <= reqs; ++r) {
        const uint8_t *ref = pool + (r % 64) * nb;
        const auto p0 = std::chrono::steady_clock::now();
        for (size_t o = 0; o < nb; o += 16)
            _mm_storeu_si128(reinterpret_cast<__m128i *>(req + 64 + o), _mm_loadu_si128(reinterpret_cast<const __m128i *>(ref + o)));
        _mm_sfence();  // the data is visible before the sequence (write-combined BAR mapping in mode 1)
        _mm_store_si128(reinterpret_cast<__m128i *>(req), _mm_set_epi32(0, 0, 0, (int)r));
        _mm_sfence();
        post_ns += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - p0).count();
        const auto w0 = std::chrono::steady_clock::now();
        bool lost = false;
        while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != r) {
            __builtin_ia32_pause();
            if (std::chrono::steady_clock::now() - w0 > std::chrono::seconds(2)) {
                lost = true;  // the kernel never saw the request: stop (it leaves after its spin bound, a few seconds)
                break;
            }
        }
        if (lost) {
            fprintf(stderr, "request %u not served\n", r);
            bad = -1;
            break;
        }
        for (uint32_t i = 0; i < nb; ++i)
            if (out[i] != (uint8_t)(ref[i] ^ (uint8_t)(r >> (8 * (i & 3))))) {
                ++bad;
                break;
            }
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (bad >= 0) {
        (void)hipStreamSynchronize(s);
        (void)hipMemcpy(&cycles, d_cycles, 8, hipMemcpyDeviceToHost);
    }
    printf("{\"mode\": %d, \"request_in\": \"%s\", \"bytes\": %u, \"requests\": %u, \"round_trip_us\": %.2f, "
           "\"host_post_us\": %.2f, \"kernel_busy_us_per_req\": %.2f, \"stale_or_wrong\": %ld}\n",
           mode, mode ? "device fine-grained (host writes over the BAR)" : "pinned host", (unsigned)nb, reqs, dt / reqs * 1e6,
           post_ns / reqs / 1000.0, cycles / 100.0 / reqs, bad);
    return bad ? 2 : 0;  // a lost request: the kernel exits after its own spin bound
}
