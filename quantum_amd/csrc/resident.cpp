// resident.cpp -- the per-packet Encrypt/Decrypt contract (crypto/aes.go:41-62, one packet per
// plugin/encryption.go Apply from each of quantum's 2 x NumWorkers goroutines, worker/outgoing.go:83-93,
// worker/incoming.go:82-92) without a kernel launch per call.
//
// A resident kernel (gcm_kernels.hip gcm_resident_kernel) keeps `workers` workgroups on the GPU; each
// owns `per_worker` request slots.  A call takes a free slot of the least-loaded worker, writes its
// packet and then the slot's request record into DEVICE memory through the BAR (fine-grained VRAM the
// CPU may write: posted, write-combined stores, ordered by sfence), and waits on the slot's done word
// in pinned host memory (spinning, then asleep on a futex that a completion thread wakes); the worker,
// polling its records in its own HBM, seals or opens the packet and writes the result and the verdict
// into host memory.  No hipLaunch, no stream and no hardware queue per call, and no PCIe read on the
// request path.
//
// Lifetime: an instance ends by itself when it has seen no request for QGCM_RESIDENT_IDLE_US or is
// QGCM_RESIDENT_LIFE_US old (so work queued behind it on a shared hardware queue, or a
// device-wide synchronize, waits a bounded time), and on qgcm_resident_stop / qgcm_set_keys (the
// workers cache key tables) / qgcm_destroy.  Before leaving, every worker serves what is pending; a
// request posted after that is seen by its caller (the instance's `over` word names its generation)
// and the caller launches the next instance, which serves it.  At most one instance runs at a time.
#include <emmintrin.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <linux/futex.h>
#include <sched.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <pthread.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <thread>

#include "gcm_internal.h"

namespace qgcm {

struct Resident {
    int device = 0;
    Batch base{};
    uint32_t W = 16, P = 16, S = 256;
    uint64_t idle_ticks = 200000, life_ticks = 800000;  // 100 MHz: 2 ms, 8 ms
    uint8_t *host = nullptr;  // pinned coherent region: done words, over, the result slots
    uint8_t *devm = nullptr;  // fine-grained device region the CPU writes: records, stop words, request slots
    uint32_t *done = nullptr, *over = nullptr, *stop = nullptr, *hits = nullptr;
    uint4 *req = nullptr;
    uint8_t *in = nullptr, *out = nullptr;
    uint8_t *d_ctl = nullptr;  // device control words (kResDevBytes)
    hipStream_t stream = nullptr;
    std::unique_ptr<uint32_t[]> seqh;                  // last sequence per slot (owned by the slot holder)
    // keystream ahead (QGCM_RESIDENT_AHEAD, default on): each seal announces the nonce of its slot's
    // next seal, whose counter blocks the worker then computes while idle (gcm_kernels.hip ks_fill).
    // Per slot, owned by the slot holder: that nonce, and the fork generation + 1 it was drawn in (0:
    // none) -- a forked child must not use its parent's announced nonce.
    bool ahead = true;
    std::unique_ptr<uint8_t[]> next_nonce;
    std::unique_ptr<uint32_t[]> next_gen;
    std::unique_ptr<std::atomic<uint32_t>[]> busy;     // slot taken
    // per worker, each on its own cache line (every call updates them): requests served, callers
    // spinning now.  A caller's home worker is fixed per thread (quantum's workers are long-lived
    // locked OS threads), so concurrent callers touch different lines.
    struct alignas(64) WorkerCounts {
        std::atomic<uint64_t> served{0};
        std::atomic<int32_t> spinners{0};
    };
    std::unique_ptr<WorkerCounts[]> wc;
    std::mutex launch_mu;  // held across a launch, and by resident_pause until resident_resume
    std::atomic<uint32_t> gen{0};  // generation of the current (or last) instance; 0 = never launched
    std::atomic<bool> broken{false};
    std::atomic<uint64_t> launches{0};
    uint64_t fail_after = ~0ull;  // QGCM_RESIDENT_FAIL_AFTER: test hook, launches after which relaunch fails
    // callers that stop spinning sleep on a futex; one completion thread watches their done words
    uint64_t spin_ns = 20000;                           // QGCM_RESIDENT_SPIN_US
    int32_t max_spinners = 8;  // QGCM_RESIDENT_SPINNERS (default: half the CPU share), spread over workers
    int32_t max_spin_w = 1;    // spinners per worker: ceil(max_spinners / W)
    std::unique_ptr<std::atomic<uint32_t>[]> want;      // per slot: the sequence a sleeping caller waits for
    std::unique_ptr<std::atomic<uint32_t>[]> wake;      // per slot futex word
    std::atomic<uint32_t> sleepers{0};                  // futex word of the completion thread
    std::atomic<bool> quit{false};
    std::thread waker;
    std::mutex waker_mu;
};

namespace {

long futex(std::atomic<uint32_t> *w, int op, uint32_t val, const struct timespec *ts) {
    return syscall(SYS_futex, reinterpret_cast<uint32_t *>(w), op, val, ts, nullptr, 0);
}

uint64_t env_u64(const char *name, uint64_t dflt) {
    const char *v = getenv(name);
    return v && *v ? strtoull(v, nullptr, 10) : dflt;
}

// CPUs this process may use: the affinity mask, capped by a cgroup-v2 CPU quota (the GPU boxes give
// a job 16 CPUs of a 256-CPU host by quota, with all 256 in the mask).
int cpu_share() {
    cpu_set_t set;
    int n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 1;
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        unsigned long period = 0;
        if (fscanf(f, "%31s %lu", q, &period) == 2 && strcmp(q, "max") != 0 && period) {
            const unsigned long quota = strtoul(q, nullptr, 10);
            const int c = (int)((quota + period - 1) / period);
            if (c >= 1 && c < n) n = c;
        }
        fclose(f);
    }
    return n < 1 ? 1 : n;
}

// Launches instance g + 1 if instance g (0: none yet) has ended and nobody has launched since.
int relaunch(Resident *r, uint32_t g) {
    std::lock_guard<std::mutex> lk(r->launch_mu);
    if (r->broken.load(std::memory_order_acquire)) return QGCM_E_HIP;  // callers take the launch path now
    if (r->gen.load(std::memory_order_acquire) != g) return QGCM_OK;  // another caller did it
    if (r->launches.load(std::memory_order_relaxed) >= r->fail_after) {  // the test hook's injected failure
        r->broken = true;
        return QGCM_E_HIP;
    }
    if (hipSetDevice(r->device) != hipSuccess) return QGCM_E_HIP;
    // instance g has written `over` (its last worker is leaving): wait for the launch to retire
    if (g != 0 && hipStreamSynchronize(r->stream) != hipSuccess) {
        r->broken = true;
        return QGCM_E_HIP;
    }
    ResArgs a{};
    a.req = r->req;
    a.stop = r->stop;
    a.in = r->in;
    a.out = r->out;
    a.done = r->done;
    a.over = r->over;
    a.hits = r->hits;
    a.dev = r->d_ctl;
    a.workers = r->W;
    a.per_worker = r->P;
    a.gen = g + 1;
    a.idle_ticks = r->idle_ticks;
    a.life_ticks = r->life_ticks;
    if (hipMemsetAsync(r->d_ctl, 0, kResDevBytes, r->stream) != hipSuccess ||
        launch_resident(r->base, a, r->stream) != hipSuccess) {
        r->broken = true;
        return QGCM_E_HIP;
    }
    r->launches.fetch_add(1, std::memory_order_relaxed);
    r->gen.store(g + 1, std::memory_order_release);
    return QGCM_OK;
}

bool instance_over(const Resident *r, uint32_t g) {
    return g == 0 || __atomic_load_n(r->over, __ATOMIC_ACQUIRE) == g;
}

// The completion thread: while callers sleep, it watches their slots' done words and wakes each caller
// whose verdict has arrived (and launches the next instance when one ends with callers waiting).
void waker_loop(Resident *r) {
    while (!r->quit.load(std::memory_order_acquire)) {
        if (r->sleepers.load(std::memory_order_acquire) == 0) {
            const struct timespec ts = {0, 10 * 1000 * 1000};
            futex(&r->sleepers, FUTEX_WAIT_PRIVATE, 0, &ts);
            continue;
        }
        for (uint32_t s = 0; s < r->S; ++s) {
            const uint32_t w = r->want[s].load(std::memory_order_acquire);
            if (w && (__atomic_load_n(&r->done[s], __ATOMIC_ACQUIRE) >> 1) == w && r->wake[s].exchange(1) == 0)
                futex(&r->wake[s], FUTEX_WAKE_PRIVATE, 1, nullptr);
        }
        const uint32_t g = r->gen.load(std::memory_order_acquire);
        if (!r->broken.load(std::memory_order_acquire) && instance_over(r, g)) relaunch(r, g);
        sched_yield();  // hand the CPU to a runnable caller when the job's CPUs are all busy
    }
}

// The device region: fine-grained VRAM (the GPU reads it around its caches) that the host CPU is
// allowed to write (HSA access for the CPU agent: a BAR mapping at the same address).
hsa_status_t find_cpu_agent(hsa_agent_t a, void *out) {
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
        *static_cast<hsa_agent_t *>(out) = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

bool device_region(Resident *r, size_t bytes) {
    if (hipExtMallocWithFlags(reinterpret_cast<void **>(&r->devm), bytes, hipDeviceMallocFinegrained) != hipSuccess) {
        r->devm = nullptr;
        return false;
    }
    static const bool hsa_up = hsa_init() == HSA_STATUS_SUCCESS;  // the runtime HIP runs on (a reference)
    hsa_agent_t cpu{0};
    return hsa_up && hsa_iterate_agents(find_cpu_agent, &cpu) == HSA_STATUS_INFO_BREAK && cpu.handle &&
           hsa_amd_agents_allow_access(1, &cpu, nullptr, r->devm) == HSA_STATUS_SUCCESS;
}

}  // namespace

// 12 bytes from getrandom (crypto/rand in crypto/aes.go:44), drawn 4 KiB at a time per thread: one
// syscall per 341 nonces instead of one per packet.  A forked child must never reuse its parent's
// unread bytes (a repeated GCM nonce under one key is fatal), so the buffer is dropped when the
// process's fork generation (bumped in the child by a pthread_atfork handler) has changed.
namespace {
std::atomic<uint32_t> g_fork_gen{0};
void on_fork_child() { g_fork_gen.fetch_add(1, std::memory_order_relaxed); }
}  // namespace
bool random_nonce(uint8_t out[12]) {
    static std::once_flag once;
    std::call_once(once, [] { pthread_atfork(nullptr, nullptr, on_fork_child); });
    struct Buf {
        uint8_t b[4092];  // a multiple of 12
        uint32_t pos = sizeof(b);
        uint32_t gen = 0;
    };
    thread_local Buf t;
    const uint32_t gen = g_fork_gen.load(std::memory_order_relaxed);
    if (t.pos + 12 > sizeof(t.b) || t.gen != gen) {
        size_t got = 0;
        while (got < sizeof(t.b)) {
            const ssize_t n = getrandom(t.b + got, sizeof(t.b) - got, 0);
            if (n < 0) {
                if (errno == EINTR) continue;
                return false;
            }
            got += (size_t)n;
        }
        t.pos = 0;
        t.gen = gen;
    }
    memcpy(out, t.b + t.pos, 12);
    memset(t.b + t.pos, 0, 12);  // consumed bytes do not linger
    t.pos += 12;
    return true;
}

ResidentConfig resident_config_from_env() {
    ResidentConfig c;
    c.workers = env_u64("QGCM_RESIDENT_WORKERS", 16);
    c.slots = env_u64("QGCM_RESIDENT_SLOTS", 16);
    c.spin_us = env_u64("QGCM_RESIDENT_SPIN_US", 20);
    // callers beyond this many sleep at once instead of spinning: with many more callers than CPUs,
    // spinning ones take the CPUs that posting callers, the completion thread and other host work need
    c.spinners = env_u64("QGCM_RESIDENT_SPINNERS", (uint64_t)std::max(1, cpu_share() / 2));
    c.idle_us = env_u64("QGCM_RESIDENT_IDLE_US", 2000);
    c.life_us = env_u64("QGCM_RESIDENT_LIFE_US", 8000);
    c.fail_after = env_u64("QGCM_RESIDENT_FAIL_AFTER", ~0ull);  // test hook
    c.ahead = env_u64("QGCM_RESIDENT_AHEAD", 1) != 0;
    return c;
}

Resident *resident_create(int device, const Batch &base, int num_cus, const ResidentConfig &cfg) {
    auto r = std::make_unique<Resident>();
    r->device = device;
    r->base = base;
    r->W = (uint32_t)cfg.workers;
    r->P = (uint32_t)cfg.slots;
    if (r->W < 1 || (int)r->W > num_cus / 2 || r->P < 1 || r->P > kResMaxPerWorker) return nullptr;
    r->S = r->W * r->P;
    r->spin_ns = cfg.spin_us * 1000;
    r->max_spinners = (int32_t)cfg.spinners;
    r->idle_ticks = cfg.idle_us * 100;  // s_memrealtime: 100 MHz
    r->life_ticks = cfg.life_us * 100;
    r->fail_after = cfg.fail_after;
    // host region: done, over, then the result slots; device region: the stop words (a 64-B line per
    // worker), the request records, then the request slots
    const size_t o_over = (4ull * r->S + 63) & ~63ull, o_hits = o_over + 64;
    const size_t o_out = (o_hits + 64ull * r->W + 4095) & ~4095ull;
    const size_t host_bytes = o_out + (size_t)kResSlotBytes * r->S;
    const size_t o_req = 64ull * r->W, o_in = (o_req + 16ull * r->S + 4095) & ~4095ull;
    const size_t dev_bytes = o_in + (size_t)kResSlotBytes * r->S;
    if (hipSetDevice(device) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&r->host), host_bytes, hipHostMallocCoherent) != hipSuccess)
        return nullptr;
    memset(r->host, 0, o_out);
    if (!device_region(r.get(), dev_bytes)) {
        resident_destroy(r.release());
        return nullptr;
    }
    r->done = reinterpret_cast<uint32_t *>(r->host);
    r->over = reinterpret_cast<uint32_t *>(r->host + o_over);
    r->hits = reinterpret_cast<uint32_t *>(r->host + o_hits);
    r->out = r->host + o_out;
    r->stop = reinterpret_cast<uint32_t *>(r->devm);
    r->req = reinterpret_cast<uint4 *>(r->devm + o_req);
    r->in = r->devm + o_in;
    memset(r->devm, 0, o_in);  // stop words and records, through the BAR
    _mm_sfence();
    r->seqh.reset(new uint32_t[r->S]());
    r->ahead = cfg.ahead;
    r->next_nonce.reset(new uint8_t[12ull * r->S]());
    r->next_gen.reset(new uint32_t[r->S]());
    r->busy.reset(new std::atomic<uint32_t>[r->S]);
    for (uint32_t i = 0; i < r->S; ++i) r->busy[i] = 0;
    r->wc.reset(new Resident::WorkerCounts[r->W]);
    r->max_spin_w = std::max<int32_t>(1, (r->max_spinners + (int32_t)r->W - 1) / (int32_t)r->W);
    r->want.reset(new std::atomic<uint32_t>[r->S]);
    r->wake.reset(new std::atomic<uint32_t>[r->S]);
    for (uint32_t i = 0; i < r->S; ++i) r->want[i] = r->wake[i] = 0;
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
    if (hipMalloc(reinterpret_cast<void **>(&r->d_ctl), kResDevBytes) != hipSuccess ||
        hipStreamCreateWithPriority(&r->stream, hipStreamNonBlocking, hi) != hipSuccess) {
        resident_destroy(r.release());
        return nullptr;
    }
    return r.release();
}

// Ends the running instance (if any) after it has served what is pending (launch_mu held); the next call
// relaunches.
static int quiesce_locked(Resident *r) {
    const uint32_t g = r->gen.load(std::memory_order_acquire);
    if (g == 0) return QGCM_OK;
    for (uint32_t w = 0; w < r->W; ++w) __atomic_store_n(&r->stop[16 * w], 1u, __ATOMIC_RELEASE);
    _mm_sfence();
    const hipError_t e = hipSetDevice(r->device) == hipSuccess ? hipStreamSynchronize(r->stream) : hipErrorUnknown;
    for (uint32_t w = 0; w < r->W; ++w) __atomic_store_n(&r->stop[16 * w], 0u, __ATOMIC_RELEASE);
    _mm_sfence();
    if (e != hipSuccess) {
        r->broken = true;
        return QGCM_E_HIP;
    }
    return QGCM_OK;
}

int resident_quiesce(Resident *r) {
    if (!r) return QGCM_OK;
    std::lock_guard<std::mutex> lk(r->launch_mu);
    return quiesce_locked(r);
}

// qgcm_set_keys: ends the running instance and keeps the next one from starting until resident_resume, so
// no request is served from key tables (or keystreams computed ahead) cached across the key change.
int resident_pause(Resident *r) {
    if (!r) return QGCM_OK;
    r->launch_mu.lock();
    return quiesce_locked(r);
}

void resident_resume(Resident *r) {
    if (r) r->launch_mu.unlock();
}

void resident_destroy(Resident *r) {
    if (!r) return;
    r->quit = true;
    futex(&r->sleepers, FUTEX_WAKE_PRIVATE, 1, nullptr);
    if (r->waker.joinable()) r->waker.join();
    resident_quiesce(r);
    hipSetDevice(r->device);
    if (r->stream) hipStreamDestroy(r->stream);
    if (r->d_ctl) hipFree(r->d_ctl);
    if (r->host) hipHostFree(r->host);
    if (r->devm) hipFree(r->devm);
    delete r;
}

int resident_workers_running(const Resident *r) {
    if (!r) return 0;
    const uint32_t g = r->gen.load(std::memory_order_acquire);
    return instance_over(r, g) ? 0 : (int)r->W;
}

void resident_stats(const Resident *r, uint64_t out[kResStats]) {
    uint64_t served = 0, hits = 0;
    for (uint32_t w = 0; r && w < r->W; ++w) {
        served += r->wc[w].served.load(std::memory_order_relaxed);
        hits += __atomic_load_n(&r->hits[16 * w], __ATOMIC_RELAXED);
    }
    out[0] = served;
    out[1] = r ? r->launches.load() : 0;
    out[2] = r ? r->W * (uint64_t)r->P : 0;
    out[3] = (uint64_t)resident_workers_running(r);
    out[4] = hits;
    int64_t spinning = 0;
    for (uint32_t w = 0; r && w < r->W; ++w) spinning += r->wc[w].spinners.load(std::memory_order_relaxed);
    out[5] = r ? r->sleepers.load(std::memory_order_relaxed) : 0;
    out[6] = (uint64_t)std::max<int64_t>(0, spinning);
    out[7] = r && r->broken.load() ? 1 : 0;
}

namespace {
// A caller's waiting state: spinning (counted per worker) or asleep (want[s] set, counted in sleepers).
// finish() undoes both; the destructor calls it on every early return (timeout, failed relaunch), so the
// completion thread does not keep watching for a caller that has left.
struct WaitState {
    Resident *r;
    uint32_t s, w;
    bool spinning = false, asleep = false;
    void finish() {
        if (asleep) {
            r->want[s].store(0, std::memory_order_relaxed);
            r->sleepers.fetch_sub(1);
            asleep = false;
        }
        if (spinning) {
            r->wc[w].spinners.fetch_sub(1, std::memory_order_relaxed);
            spinning = false;
        }
    }
    ~WaitState() { finish(); }
};
}  // namespace

long resident_call(Resident *r, bool seal, uint32_t key, uint8_t *data, long len, const uint8_t *aad,
                   uint32_t aad_len, const uint8_t *nonce) {
    const uint64_t stage = (4ull + (uint64_t)len + (seal ? QGCM_OVERHEAD : 0) + 15) & ~15ull;
    if (!r || r->broken || stage > kResSlotBytes || stage > kOneCap - 16) return kResNotServed;
    // a free slot of this thread's home worker, else of the next workers in turn
    static std::atomic<uint32_t> next_thread{0};
    thread_local const uint32_t t_index = next_thread.fetch_add(1, std::memory_order_relaxed);
    const uint32_t home = t_index % r->W;
    uint32_t s = 0, w = home;
    for (uint32_t tries = 0;; ++tries) {
        bool got = false;
        for (uint32_t k = 0; k < r->W && !got; ++k) {
            const uint32_t ww = (home + k) % r->W;
            for (uint32_t i = 0; i < r->P; ++i) {
                const uint32_t c = ww * r->P + (i + tries) % r->P;
                uint32_t z = 0;
                if (r->busy[c].load(std::memory_order_relaxed) == 0 &&
                    r->busy[c].compare_exchange_strong(z, 1, std::memory_order_acquire)) {
                    s = c;
                    w = ww;
                    got = true;
                    break;
                }
            }
        }
        if (got) break;
        sched_yield();  // every slot in flight
    }
    // the nonce: the caller's, else the one this slot's previous seal announced, else a fresh one
    // (crypto/aes.go:44 rand.Read(nonce)); a seal without a caller's nonce announces the next one
    uint8_t nb[12];
    bool announce = false;
    if (seal && nonce) {
        memcpy(nb, nonce, 12);
    } else if (seal) {
        const uint32_t fg = g_fork_gen.load(std::memory_order_relaxed) + 1;
        uint8_t *nx = &r->next_nonce[12ull * s];
        const bool have = r->ahead && r->next_gen[s] == fg;
        if (have)
            memcpy(nb, nx, 12);
        r->next_gen[s] = 0;  // used (or stale) either way
        if (!have && !random_nonce(nb)) {
            r->busy[s].store(0, std::memory_order_release);
            return -1;
        }
        if (r->ahead && stage + 16 <= kResSlotBytes && random_nonce(nx)) {
            r->next_gen[s] = fg;
            announce = true;
        }
    }
    // the request into device memory (write-combined stores through the BAR) with its record's fields
    // under the old sequence (which the worker has served, so it ignores the record), then the new
    // sequence; sfence orders the first stores before it and pushes it out
    uint8_t *slot = r->in + (size_t)s * kResSlotBytes;
    uint32_t hdr = 0;
    if (aad_len) memcpy(&hdr, aad, aad_len);
    memcpy(slot, &hdr, 4);
    memcpy(slot + 4, data, (size_t)len);
    if (seal) memcpy(slot + 4 + len + 16, nb, 12);
    if (announce) memcpy(slot + kResSlotBytes - 16, &r->next_nonce[12ull * s], 12);
    const uint32_t q0 = r->seqh[s];
    uint32_t q = (q0 + 1) & 0x7fffffffu;
    if (q == 0) q = 1;
    r->seqh[s] = q;
    _mm_store_si128(reinterpret_cast<__m128i *>(&r->req[s]),
                    _mm_set_epi32((int)key, (int)len, (int)((seal ? 1u : 0u) | aad_len << 1 | (announce ? 1u : 0u) << 8),
                                  (int)q0));
    _mm_sfence();  // the slot bytes and the record's fields before the sequence
    __atomic_store_n(reinterpret_cast<uint32_t *>(&r->req[s]), q, __ATOMIC_RELAXED);
    _mm_sfence();
    long rc = 0;
    uint32_t g = r->gen.load(std::memory_order_acquire);
    if (instance_over(r, g) && relaunch(r, g) != QGCM_OK) return -1;  // broken: the slot stays taken
    uint32_t v = 0;
    const auto t0 = std::chrono::steady_clock::now();
    WaitState ws{r, s, w};
    ws.spinning = r->wc[w].spinners.fetch_add(1, std::memory_order_relaxed) < r->max_spin_w;
    if (!ws.spinning) r->wc[w].spinners.fetch_sub(1, std::memory_order_relaxed);
    const uint64_t spin_ns = ws.spinning ? r->spin_ns : 0;
    for (uint32_t spins = 0;; ++spins) {
        v = __atomic_load_n(&r->done[s], __ATOMIC_ACQUIRE);
        if ((v >> 1) == q) break;
        if ((spins & 63) == 63 || ws.asleep || spin_ns == 0) {
            g = r->gen.load(std::memory_order_acquire);
            // the instance ended with this request still pending: launch the next one
            if (instance_over(r, g) && relaunch(r, g) != QGCM_OK) return -1;  // broken: the slot stays taken
            const auto waited = std::chrono::steady_clock::now() - t0;
            if (waited > std::chrono::seconds(5)) {
                r->broken = true;  // never observed; the slot stays taken (the device may still serve it)
                return -1;
            }
            // past the spin budget: sleep until the completion thread sees the verdict (with many more
            // callers than CPUs, spinning ones would take the CPUs the posting ones need)
            if (!ws.asleep && (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(waited).count() >= spin_ns) {
                if (ws.spinning) {
                    r->wc[w].spinners.fetch_sub(1, std::memory_order_relaxed);
                    ws.spinning = false;
                }
                if (!r->waker.joinable()) {
                    std::lock_guard<std::mutex> lk(r->waker_mu);
                    if (!r->waker.joinable()) r->waker = std::thread(waker_loop, r);
                }
                r->wake[s].store(0, std::memory_order_relaxed);
                r->want[s].store(q, std::memory_order_release);
                if (r->sleepers.fetch_add(1) == 0) futex(&r->sleepers, FUTEX_WAKE_PRIVATE, 1, nullptr);
                ws.asleep = true;
                continue;  // re-check done before the first wait
            }
        }
        if (ws.asleep) {
            const struct timespec ts = {0, 200 * 1000};
            futex(&r->wake[s], FUTEX_WAIT_PRIVATE, 0, &ts);
        } else {
            __builtin_ia32_pause();
        }
    }
    ws.finish();  // before the slot is released: its next holder may set want[s]
    r->wc[w].served.fetch_add(1, std::memory_order_relaxed);
    const uint8_t *res = r->out + (size_t)s * kResSlotBytes;
    if (seal) {
        rc = -1;
        if (v & 1) {  // a rejected seal leaves the caller's buffer untouched
            memcpy(data, res + 4, (size_t)len + QGCM_OVERHEAD);
            rc = len + QGCM_OVERHEAD;
        }
    } else {
        memcpy(data, res + 4, (size_t)len - QGCM_OVERHEAD);  // plaintext, or zeros on auth failure
        rc = (v & 1) ? len - QGCM_OVERHEAD : -1;
    }
    r->busy[s].store(0, std::memory_order_release);
    return rc;
}

}  // namespace qgcm
