// Per-packet Encrypt/Decrypt calls (crypto/aes.go:41-62 from quantum's worker goroutines,
// worker/outgoing.go:83-93) from T threads, each with one packet in flight: seal then open of a
// P-byte packet in a loop for S seconds, checked against the original bytes.  Two contexts in one
// process on the same GPU: the resident kernel (default) and QGCM_RESIDENT=0 (a gcm_one_kernel launch
// per call).  With "bulk", a host thread runs qgcm_seal_host / qgcm_open_host over 2^18 x 1350 B on
// its own context meanwhile (the per-packet rate next to bulk traffic), and reports its rate too.
// Build: g++ -O2 -std=c++17 -Iinclude tools/per_packet_bench.cpp -Lquantum_amd -lqgcm -lpthread
//        -Wl,-rpath,$PWD/quantum_amd -o gpurun_out/per_packet_bench
// Usage: per_packet_bench [threads=64] [payload=1350] [seconds=2] [bulk=0] [mode=both|resident|launch]
#include <dlfcn.h>
#include <qgcm.h>
#include <sys/resource.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

using Clock = std::chrono::steady_clock;

static qgcm_ctx *make_ctx(bool resident) {
    setenv("QGCM_RESIDENT", resident ? "1" : "0", 1);
    char err[QGCM_ERRLEN];
    qgcm_ctx *ctx = qgcm_create(0, 4, err, sizeof err);
    if (!ctx) {
        fprintf(stderr, "qgcm_create: %s\n", err);
        exit(1);
    }
    uint8_t key[32], salt[32];
    for (int i = 0; i < 32; ++i) salt[i] = (uint8_t)i;
    const char *secret = "AES256Key-32Characters1234567890";
    if (qgcm_derive_key((const uint8_t *)secret, 32, salt, 32, key) != QGCM_OK || qgcm_set_key(ctx, 0, key) != QGCM_OK)
        exit(1);
    return ctx;
}

// cgroup-v2 CPU throttling of this job (a CPU quota throttles the whole process once the period's
// budget is spent; spinning callers spend it) and the process's CPU time
struct CpuStat {
    unsigned long long nr_throttled = 0, throttled_usec = 0;
    double cpu_s = 0;
};
static CpuStat cpu_stat() {
    CpuStat c;
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.stat", "r")) {
        char k[64];
        unsigned long long v;
        while (fscanf(f, "%63s %llu", k, &v) == 2) {
            if (!strcmp(k, "nr_throttled")) c.nr_throttled = v;
            if (!strcmp(k, "throttled_usec")) c.throttled_usec = v;
        }
        fclose(f);
    }
    struct rusage ru;
    if (getrusage(RUSAGE_SELF, &ru) == 0)
        c.cpu_s = ru.ru_utime.tv_sec + ru.ru_stime.tv_sec + 1e-6 * (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec);
    return c;
}

struct Result {
    double rt_per_s, fail, p50_us, p99_us;
};

static Result run(qgcm_ctx *ctx, int threads, int payload, double seconds) {
    std::atomic<bool> go{false}, stop{false};
    std::atomic<long> done{0}, failed{0};
    std::vector<std::vector<float>> lat(threads);
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
                const auto a = Clock::now();
                if (qgcm_seal_one(ctx, 0, buf.data(), payload, aad, 4, nullptr) != payload + QGCM_OVERHEAD) ++bad;
                if (qgcm_open_one(ctx, 0, buf.data(), payload + QGCM_OVERHEAD, aad, 4) != payload ||
                    memcmp(buf.data(), ref.data(), payload) != 0)
                    ++bad;
                if ((n & 7) == 0) lat[t].push_back(std::chrono::duration<float, std::micro>(Clock::now() - a).count());
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
    std::vector<float> all;
    for (auto &v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    auto pct = [&](double p) { return all.empty() ? 0.0 : (double)all[(size_t)(p * (all.size() - 1))]; };
    return Result{done.load() / dt, (double)failed.load(), pct(0.5), pct(0.99)};
}

int main(int argc, char **argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 64;
    const int payload = argc > 2 ? atoi(argv[2]) : 1350;
    const double seconds = argc > 3 ? atof(argv[3]) : 2.0;
    const bool bulk = argc > 4 && atoi(argv[4]) != 0;
    const std::string mode = argc > 5 ? argv[5] : "both";
    // the bulk load: its own context (launch path), pinned host arena, seal/open in a loop
    std::atomic<bool> bulk_stop{false};
    std::atomic<long> bulk_calls{0};
    std::thread bulk_th;
    const uint32_t bn = 1u << 18, bl = 1350;
    const uint64_t bstride = 1408;
    if (bulk) {
        qgcm_ctx *bctx = make_ctx(false);
        uint8_t *arena = (uint8_t *)qgcm_host_alloc(bn * bstride);
        uint8_t *non = (uint8_t *)qgcm_host_alloc(12ull * bn);
        memset(arena, 0x5a, bn * bstride);
        memset(non, 0x33, 12ull * bn);
        bulk_th = std::thread([=, &bulk_stop, &bulk_calls] {
            while (!bulk_stop.load()) {
                qgcm_seal_host(bctx, arena, bstride, bn, bl, 0, non, 4, nullptr);
                qgcm_open_host(bctx, arena, bstride, bn, bl + QGCM_OVERHEAD, 0, 4, nullptr);
                bulk_calls += 2;
            }
            qgcm_host_free(arena);
            qgcm_host_free(non);
            qgcm_destroy(bctx);
        });
        std::this_thread::sleep_for(std::chrono::milliseconds(200));
    }
    int rc = 0;
    for (const bool resident : {true, false}) {
        if ((resident && mode == "launch") || (!resident && mode == "resident")) continue;
        qgcm_ctx *ctx = make_ctx(resident);
        run(ctx, threads, payload, 0.2);  // warm up (first launch, staging slots)
        const long b0 = bulk_calls.load();
        const auto tb = Clock::now();
        // a QGCM_RES_TRACE side build of the library exports the resident kernel's device-side intervals
        using TraceFn = int (*)(unsigned long long *, int);
        const TraceFn trace = (TraceFn)dlsym(RTLD_DEFAULT, "qgcm_debug_res_trace");
        unsigned long long tr[16] = {};
        if (trace) trace(tr, 1);
        const CpuStat c0 = cpu_stat();
        const Result r = run(ctx, threads, payload, seconds);
        const CpuStat c1 = cpu_stat();
        const double wall = std::chrono::duration<double>(Clock::now() - tb).count();
        const double bulk_gibs = (bulk_calls.load() - b0) / 2.0 * 2.0 * bn * bl /
                                 std::chrono::duration<double>(Clock::now() - tb).count() / (1 << 30);
        uint64_t st[5] = {0, 0, 0, 0, 0}, lc[QGCM_KERNEL_COUNTERS] = {};
        qgcm_resident_stats(ctx, st, 5);
        qgcm_launch_counts(ctx, lc, QGCM_KERNEL_COUNTERS);
        printf("{\"bench\": \"per_packet\", \"path\": \"%s\", \"threads\": %d, \"payload\": %d, \"bulk_alongside\": %s, "
               "\"round_trips_per_s\": %.0f, \"GiB_s\": %.3f, \"call_pair_p50_us\": %.1f, \"call_pair_p99_us\": %.1f, "
               "\"failures\": %.0f, \"resident_served\": %llu, \"resident_launches\": %llu, \"one_kernel_launches\": %llu, "
               "\"ahead_hits\": %llu",
               resident ? "resident" : "launch", threads, payload, bulk ? "true" : "false", r.rt_per_s,
               2.0 * r.rt_per_s * payload / (1 << 30), r.p50_us, r.p99_us, r.fail, (unsigned long long)st[0],
               (unsigned long long)st[1], (unsigned long long)lc[QGCM_KERNEL_ONE], (unsigned long long)st[4]);
        if (bulk) printf(", \"bulk_GiB_s\": %.2f", bulk_gibs);
        if (trace && resident && trace(tr, 0) == 0) {
            for (int op = 1; op >= 0; --op) {
                const unsigned long long *g = tr + 8 * op, n = g[5];
                if (!n) continue;
                printf(", \"device_us_%s\": {\"poll_to_staged\": %.2f, \"%s\": %.2f, \"%s\": %.2f, \"staged_to_computed\": %.2f, "
                       "\"computed_to_acked\": %.2f, \"requests\": %llu, \"shader_MHz\": %.0f}",
                       op ? "seal" : "open", g[0] / 100.0 / n, op ? "staged_to_ctr_done" : "staged_to_ghash_done",
                       g[1] / 100.0 / n, op ? "staged_to_ghash_done" : "staged_to_ctr_done", g[2] / 100.0 / n,
                       g[3] / 100.0 / n, g[4] / 100.0 / n, n, g[7] ? g[6] * 100.0 / g[7] : 0.0);
            }
        }
        // host CPU time per seal+open pair (the process's CPU seconds over the timed run / pairs served):
        // what the per-call drop-in costs quantum's host next to the CPU plugin chain's figure
        const double busy = (c1.cpu_s - c0.cpu_s) / wall;
        const char *sp = getenv("QGCM_RESIDENT_SPINNERS");
        printf(", \"cpus_busy\": %.2f, \"cpu_us_per_pair\": %.2f, \"spinners_env\": \"%s\", \"cgroup_throttled\": %llu, "
               "\"cgroup_throttled_ms\": %.1f",
               busy, r.rt_per_s > 0 ? busy / r.rt_per_s * 1e6 : 0.0, sp ? sp : "default", c1.nr_throttled - c0.nr_throttled,
               (c1.throttled_usec - c0.throttled_usec) / 1000.0);
        printf("}\n");
        fflush(stdout);
        if (r.fail) rc = 2;
        qgcm_destroy(ctx);
    }
    if (bulk) {
        bulk_stop = true;
        bulk_th.join();
    }
    return rc;
}
