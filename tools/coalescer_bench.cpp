// Throughput of the per-packet Encrypt/Decrypt contract from many threads:
// T threads, each a stand-in for one of quantum's worker goroutines, seal then open P-byte packets
// in a loop through (a) qgcm_coalescer_seal/open and (b) qgcm_seal_one/open_one, for S seconds each.
// Build: g++ -O2 -std=c++17 -Iinclude tools/coalescer_bench.cpp -Lquantum_amd -lqgcm -lpthread
//        -Wl,-rpath,$PWD/quantum_amd -o gpurun_out/coalescer_bench
// Usage: coalescer_bench [threads=64] [payload=1350] [seconds=3] [max_batch=8192] [max_wait_us=200]
#include <qgcm.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

using Clock = std::chrono::steady_clock;

struct Result {
    double pkts_per_s, gib_per_s, fail;
};

template <typename Seal, typename Open>
Result run(int threads, int payload, double seconds, Seal seal, Open open) {
    std::atomic<bool> go{false}, stop{false};
    std::atomic<long> done{0}, failed{0};
    std::vector<std::thread> ths;
    for (int t = 0; t < threads; ++t) {
        ths.emplace_back([&, t] {
            std::vector<uint8_t> buf(payload + QGCM_OVERHEAD), ref(payload);
            const uint8_t aad[4] = {10, 99, 0, (uint8_t)t};
            for (int i = 0; i < payload; ++i) ref[i] = (uint8_t)(i * 31 + t);
            while (!go.load()) std::this_thread::yield();
            long n = 0, bad = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                memcpy(buf.data(), ref.data(), payload);
                if (seal(buf.data(), payload, aad) != payload + QGCM_OVERHEAD) ++bad;
                if (open(buf.data(), payload + QGCM_OVERHEAD, aad) != payload ||
                    memcmp(buf.data(), ref.data(), payload) != 0)
                    ++bad;
                ++n;
            }
            done += n;
            failed += bad;
        });
    }
    const auto t0 = Clock::now();
    go = true;
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    stop = true;
    for (auto &th : ths) th.join();
    const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
    const double pk = done.load() / dt;  // packets sealed AND opened per second
    return Result{pk, 2.0 * pk * payload / (1 << 30), (double)failed.load()};
}

int main(int argc, char **argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 64;
    const int payload = argc > 2 ? atoi(argv[2]) : 1350;
    const double seconds = argc > 3 ? atof(argv[3]) : 3.0;
    const uint32_t max_batch = argc > 4 ? atoi(argv[4]) : 8192;
    const uint32_t max_wait = argc > 5 ? atoi(argv[5]) : 200;
    char err[QGCM_ERRLEN];
    qgcm_ctx *ctx = qgcm_create(0, 4, err, sizeof err);
    if (!ctx) {
        fprintf(stderr, "qgcm_create: %s\n", err);
        return 1;
    }
    uint8_t key[32];
    const char *secret = "AES256Key-32Characters1234567890";
    uint8_t salt[32];
    for (int i = 0; i < 32; ++i) salt[i] = (uint8_t)i;
    if (qgcm_derive_key((const uint8_t *)secret, 32, salt, 32, key) != QGCM_OK || qgcm_set_key(ctx, 0, key) != QGCM_OK)
        return 1;
    qgcm_coalescer *co = qgcm_coalescer_create(ctx, max_batch, max_wait, 1472, 4, err, sizeof err);
    if (!co) {
        fprintf(stderr, "qgcm_coalescer_create: %s\n", err);
        return 1;
    }
    const Result rc = run(
        threads, payload, seconds,
        [&](uint8_t *d, long n, const uint8_t *a) { return qgcm_coalescer_seal(co, 0, d, n, a, 4); },
        [&](uint8_t *d, long n, const uint8_t *a) { return qgcm_coalescer_open(co, 0, d, n, a, 4); });
    const Result r1 = run(
        threads, payload, seconds / 3,
        [&](uint8_t *d, long n, const uint8_t *a) { return qgcm_seal_one(ctx, 0, d, n, a, 4, nullptr); },
        [&](uint8_t *d, long n, const uint8_t *a) { return qgcm_open_one(ctx, 0, d, n, a, 4); });
    printf("{\"bench\": \"coalescer\", \"threads\": %d, \"payload\": %d, \"max_batch\": %u, \"max_wait_us\": %u, "
           "\"coalesced\": {\"pkts_per_s\": %.0f, \"GiB_s\": %.3f, \"failures\": %.0f}, "
           "\"per_packet_calls\": {\"pkts_per_s\": %.0f, \"GiB_s\": %.3f, \"failures\": %.0f}}\n",
           threads, payload, max_batch, max_wait, rc.pkts_per_s, rc.gib_per_s, rc.fail, r1.pkts_per_s, r1.gib_per_s,
           r1.fail);
    qgcm_coalescer_destroy(co);
    qgcm_destroy(ctx);
    return rc.fail == 0 && r1.fail == 0 ? 0 : 2;
}
