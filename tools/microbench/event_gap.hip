// Microbenchmark: what an event record and a stream wait between back-to-back launches on one stream
// cost on gfx950 (the uniform path's pool-set ring records an event after each launch and waits on the
// event of the set's previous launch).  A ~100-us kernel (every wave sleeps until a deadline) launched
// 500 times per mode; the time per launch above mode 0 is the gap the packets add.
//   0 plain launches
//   1 hipEventRecord(ring[i % 16]) after each launch
//   2 hipStreamWaitEvent(ring[i % 16]) (recorded 16 launches earlier, same stream) before, record after
//   3 hipStreamWaitEvent only (events recorded once, long complete)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 event_gap.hip -o event_gap
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

__global__ void spin_kernel(uint64_t ticks, uint32_t *out) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0 && blockIdx.x == 0xffffffffu) out[0] = 1;
}

int main() {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *d;
    CHECK(hipMalloc(&d, 4));
    hipEvent_t ring[16], t0, t1;
    for (auto &e : ring) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CHECK(hipEventCreate(&t0));
    CHECK(hipEventCreate(&t1));
    for (auto &e : ring) CHECK(hipEventRecord(e, s));
    const int n = 500;
    const uint64_t ticks = 10000;  // 100 us at the 100-MHz wall clock
    const char *names[4] = {"plain", "record", "wait+record", "wait"};
    double base = 0;
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 0; mode < 4; ++mode) {
            for (int i = 0; i < 20; ++i) spin_kernel<<<512, 64, 0, s>>>(ticks, d);
            CHECK(hipEventRecord(t0, s));
            for (int i = 0; i < n; ++i) {
                if (mode >= 2) CHECK(hipStreamWaitEvent(s, ring[i % 16], 0));
                spin_kernel<<<512, 64, 0, s>>>(ticks, d);
                if (mode == 1 || mode == 2) CHECK(hipEventRecord(ring[i % 16], s));
            }
            CHECK(hipEventRecord(t1, s));
            CHECK(hipEventSynchronize(t1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, t0, t1));
            const double us = ms * 1e3 / n;
            if (mode == 0) base = us;
            printf("{\"rep\": %d, \"mode\": \"%s\", \"us_per_launch\": %.3f, \"over_plain_us\": %.3f}\n", rep,
                   names[mode], us, us - base);
        }
    }
    return 0;
}
