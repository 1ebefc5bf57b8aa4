// coalescer.cpp -- many threads' per-packet Encrypt/Decrypt calls gathered into device batches.
//
// quantum calls plugin.Apply once per packet from 2 x NumWorkers goroutines, each locked to an OS
// thread (main.go:41-48,72-75; worker/outgoing.go:55-93, worker/incoming.go:54-92).  A GPU batch
// only pays off at thousands of packets, so qgcm_coalescer_seal/open keep the exact per-packet
// contract of crypto/aes.go:41-62 (blocking; L+28 / len-28 or -1; plaintext zeroed on auth failure)
// while the packets of concurrent callers ride the same batch:
//
//   caller: reserve a slot in the FILLING batch (mutex) -> copy AAD||data into the pinned slot (no
//           lock) -> wait for the batch -> copy the result back (no lock) -> release the slot.
//   flusher (one thread per direction): flushes when the batch holds max_batch packets, runs out of
//           arena bytes, its first packet has waited max_wait_us, or no packet arrived for
//           max_wait_us / 8 (min 5 us); waits for in-flight copies,
//           draws the batch's nonces with ONE getrandom (crypto/aes.go:44 draws per packet), then
//           H2D -> qgcm_{seal,open}_batch -> D2H on its own stream.
//
// kDepth batches per direction rotate FREE -> FILLING -> FLUSHING -> DONE -> FREE, so the next batch
// fills while one is on the device and callers of the previous one copy out.
//
// Completion is published without the lane mutex: the flusher bumps the batch's 32-bit `done`
// sequence and wakes its waiters with one futex call; callers check it, spin briefly, then sleep on
// the futex, and hand the batch back with an atomic reader count (the last reader recycles it under
// the mutex).  With a condition variable every notify_all made all of a batch's callers re-acquire
// the lane mutex one after another before they could copy out.
#include <hip/hip_runtime.h>
#include <linux/futex.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>

#include "gcm_internal.h"

using Clock = std::chrono::steady_clock;

namespace {

constexpr int kDepth = 3;
enum class St { Free, Filling, Flushing, Done };

struct CBatch {
    uint8_t *h_arena = nullptr, *d_arena = nullptr;
    qgcm_desc *h_descs = nullptr, *d_descs = nullptr;
    uint8_t *h_nonces = nullptr, *d_nonces = nullptr;
    uint8_t *h_status = nullptr, *d_status = nullptr;
    uint32_t n = 0;         // reserved slots
    uint64_t used = 0;      // reserved arena bytes
    uint32_t writers = 0;   // callers still copying in
    std::atomic<uint32_t> readers{0};  // callers still to copy out
    std::atomic<uint32_t> done{0};     // completion sequence: bumped once per flush (futex word)
    int rc = QGCM_OK;       // batch-level result (written before `done` is bumped)
    St st = St::Free;
    Clock::time_point first, last;  // first and latest reservation
};

long futex(std::atomic<uint32_t> *w, int op, uint32_t v) {
    return syscall(SYS_futex, reinterpret_cast<uint32_t *>(w), op, v, nullptr, nullptr, 0);
}

// Wait until *w != seen: a short spin (a batch on the latency kernel lands in tens of us), then sleep
// on the futex.
void wait_change(std::atomic<uint32_t> *w, uint32_t seen) {
    for (int i = 0; i < 64; ++i) {
        if (w->load(std::memory_order_acquire) != seen) return;
        __builtin_ia32_pause();
    }
    while (w->load(std::memory_order_acquire) == seen) futex(w, FUTEX_WAIT_PRIVATE, seen);
}

struct Lane {
    bool seal = true;
    std::mutex mu;
    std::condition_variable cv_caller;  // space in the filling batch, or a batch finished
    std::condition_variable cv_flush;   // flusher: batch full / writers done / deadline / stop
    CBatch b[kDepth];
    int fill = 0;  // index of the batch callers reserve in
    hipStream_t stream = nullptr;
    uint8_t *done = nullptr;  // pinned, one byte per packet: set by its workgroup (latency-kernel flushes)
    std::thread thr;
};

}  // namespace

struct qgcm_coalescer {
    qgcm_ctx *ctx = nullptr;
    int device = 0;
    uint32_t max_batch = 0, max_packet = 0, aad_len = 4;
    bool one_kernel = false;  // small batches through the latency kernel (slots fit its LDS staging)
    std::chrono::microseconds max_wait{0}, quiet{0};
    uint64_t cap_bytes = 0;
    bool stop = false;
    Lane lanes[2];  // 0 = seal, 1 = open
};

namespace {

uint64_t slot_bytes(bool seal, uint32_t len) {
    return (4ull + len + (seal ? QGCM_OVERHEAD : 0) + 15) & ~15ull;  // AAD word + packet (+ tag||nonce)
}

// Flusher thread of one direction.
void flusher(qgcm_coalescer *c, Lane *ln) {
    hipSetDevice(c->device);
    std::unique_lock<std::mutex> lk(ln->mu);
    for (;;) {
        CBatch &B = ln->b[ln->fill];
        const bool full = B.st == St::Filling && (B.n == c->max_batch || B.used + slot_bytes(ln->seal, c->max_packet) >
                                                                               c->cap_bytes);
        // due: the oldest packet has waited max_wait, or arrivals paused for quiet_us (closed-loop
        // callers -- one packet in flight per worker -- have all submitted: waiting longer only
        // adds latency)
        const auto now = Clock::now();
        const bool due = B.st == St::Filling && B.n > 0 &&
                         (now >= B.first + c->max_wait || now >= B.last + c->quiet);
        if (!(full || due)) {
            if (c->stop && (B.st != St::Filling || B.n == 0)) break;
            if (B.st == St::Filling && B.n > 0)
                ln->cv_flush.wait_until(lk, std::min(B.first + c->max_wait, B.last + c->quiet));
            else
                ln->cv_flush.wait(lk);
            continue;
        }
        // close this batch; callers move on to the next one as soon as it is free
        B.st = St::Flushing;
        const int idx = ln->fill;
        ln->fill = (ln->fill + 1) % kDepth;
        if (ln->b[ln->fill].st == St::Free) ln->b[ln->fill].st = St::Filling;
        ln->cv_caller.notify_all();
        ln->cv_flush.wait(lk, [&] { return ln->b[idx].writers == 0; });
        const uint32_t n = B.n;
        const uint64_t used = B.used;
        lk.unlock();

        int rc = QGCM_OK;
        hipStream_t s = ln->stream;
        // one draw for the batch (qgcm_random_nonces: getrandom, resumed after partial reads and EINTR)
        if (ln->seal && qgcm_random_nonces(B.h_nonces, n) != QGCM_OK) rc = QGCM_E_ARG;
        const bool one = c->one_kernel && n <= qgcm::kOneBatchMax;
        if (rc == QGCM_OK && one) {
            // small batch: one latency-kernel workgroup per packet, zero-copy on the pinned batch
            // (one launch instead of H2D copies + worklist build + batch kernel + D2H copies)
            memset(ln->done, 0, n);
            rc = qgcm::run_one_descs(c->ctx, ln->seal, B.h_arena, B.h_descs, n, ln->seal ? B.h_nonces : nullptr,
                                     c->aad_len, B.h_status, s, ln->done);
            // completion by the workgroups' flags (each set after a system-scope fence behind its slot
            // and status), not by a stream synchronization; the stream is the fallback after 1 s (it
            // also reports faults)
            const auto t0 = Clock::now();
            for (uint32_t i = 0, spins = 0; rc == QGCM_OK && i < n; ++spins) {
                if (__atomic_load_n(ln->done + i, __ATOMIC_ACQUIRE)) {
                    ++i;
                    continue;
                }
                __builtin_ia32_pause();
                if ((spins & 1023) == 1023 && Clock::now() - t0 > std::chrono::seconds(1)) break;
            }
        } else if (rc == QGCM_OK) {
            if (hipMemcpyAsync(B.d_arena, B.h_arena, used, hipMemcpyHostToDevice, s) != hipSuccess ||
                hipMemcpyAsync(B.d_descs, B.h_descs, sizeof(qgcm_desc) * n, hipMemcpyHostToDevice, s) != hipSuccess ||
                (ln->seal && hipMemcpyAsync(B.d_nonces, B.h_nonces, 12ull * n, hipMemcpyHostToDevice, s) != hipSuccess))
                rc = QGCM_E_HIP;
            if (rc == QGCM_OK)
                rc = ln->seal ? qgcm_seal_batch(c->ctx, B.d_arena, B.d_descs, n, B.d_nonces, c->aad_len, B.d_status, s)
                              : qgcm_open_batch(c->ctx, B.d_arena, B.d_descs, n, c->aad_len, B.d_status, s);
            if (rc == QGCM_OK &&
                (hipMemcpyAsync(B.h_arena, B.d_arena, used, hipMemcpyDeviceToHost, s) != hipSuccess ||
                 hipMemcpyAsync(B.h_status, B.d_status, n, hipMemcpyDeviceToHost, s) != hipSuccess))
                rc = QGCM_E_HIP;
        }
        bool landed = one && rc == QGCM_OK;
        for (uint32_t i = 0; landed && i < n; ++i) landed = __atomic_load_n(ln->done + i, __ATOMIC_ACQUIRE) != 0;
        if (!landed && hipStreamSynchronize(s) != hipSuccess) rc = QGCM_E_HIP;

        lk.lock();
        B.rc = rc;
        B.readers.store(n, std::memory_order_relaxed);
        B.st = St::Done;
        B.done.fetch_add(1, std::memory_order_release);  // publishes rc, status and the slots
        futex(&B.done, FUTEX_WAKE_PRIVATE, INT32_MAX);
    }
}

// One packet through a lane: the Encrypt/Decrypt contract.  Returns the result length or -1.
long submit(qgcm_coalescer *c, Lane *ln, uint32_t key_idx, uint8_t *data, uint32_t len, const uint8_t *aad) {
    const uint64_t sb = slot_bytes(ln->seal, len);
    std::unique_lock<std::mutex> lk(ln->mu);
    int idx;
    uint32_t i;
    uint64_t off;
    for (;;) {
        if (c->stop) return -1;
        CBatch &B = ln->b[ln->fill];
        if (B.st == St::Filling && B.n < c->max_batch && B.used + sb <= c->cap_bytes) {
            idx = ln->fill;
            i = B.n++;
            off = B.used;
            B.used += sb;
            B.writers++;
            B.last = Clock::now();
            if (i == 0) {
                B.first = B.last;
                ln->cv_flush.notify_one();  // arms the latency deadline
            }
            if (B.n == c->max_batch) ln->cv_flush.notify_one();
            break;
        }
        if (B.st == St::Filling) ln->cv_flush.notify_one();  // no room: flush it
        ln->cv_caller.wait(lk);
    }
    CBatch &B = ln->b[idx];
    // the flush of this batch bumps `done` past this value (it cannot have happened yet: this caller
    // is still a writer)
    const uint32_t seen = B.done.load(std::memory_order_relaxed);
    lk.unlock();

    uint8_t *slot = B.h_arena + off;
    if (c->aad_len) memcpy(slot, aad, c->aad_len);
    memcpy(slot + 4, data, len);
    B.h_descs[i] = qgcm_desc{off, len, key_idx};

    lk.lock();
    if (--B.writers == 0) ln->cv_flush.notify_one();
    lk.unlock();
    wait_change(&B.done, seen);
    const int rc = B.rc;

    long out = -1;
    if (rc == QGCM_OK) {
        const bool ok = B.h_status[i] == 1;
        if (ln->seal) {
            if (ok) {
                memcpy(data, slot + 4, (size_t)len + QGCM_OVERHEAD);
                out = (long)len + QGCM_OVERHEAD;
            }
        } else {
            memcpy(data, slot + 4, (size_t)len - QGCM_OVERHEAD);  // plaintext, or zeros on auth failure
            out = ok ? (long)len - QGCM_OVERHEAD : -1;
        }
    }

    if (B.readers.fetch_sub(1, std::memory_order_acq_rel) == 1) {  // the last reader recycles the batch
        lk.lock();
        B.n = 0;
        B.used = 0;
        B.st = (&B == &ln->b[ln->fill]) ? St::Filling : St::Free;
        ln->cv_caller.notify_all();
        ln->cv_flush.notify_one();
    }
    return out;
}

void free_lane(Lane &ln) {
    for (CBatch &B : ln.b) {
        if (B.h_arena) hipHostFree(B.h_arena);
        if (B.h_descs) hipHostFree(B.h_descs);
        if (B.h_nonces) hipHostFree(B.h_nonces);
        if (B.h_status) hipHostFree(B.h_status);
        hipFree(B.d_arena);
        hipFree(B.d_descs);
        hipFree(B.d_nonces);
        hipFree(B.d_status);
    }
    if (ln.stream) hipStreamDestroy(ln.stream);
    if (ln.done) hipHostFree(ln.done);
}

void set_err(char *err, size_t errlen, const char *msg) {
    if (err && errlen) {
        strncpy(err, msg, errlen - 1);
        err[errlen - 1] = 0;
    }
}

}  // namespace

extern "C" {

qgcm_coalescer *qgcm_coalescer_create(qgcm_ctx *ctx, uint32_t max_batch, uint32_t max_wait_us, uint32_t max_packet,
                                      uint32_t aad_len, char *err, size_t errlen) {
    if (!ctx || max_batch == 0 || max_batch > (1u << 22) || max_packet >= QGCM_MAX_PAYLOAD || aad_len > 4) {
        set_err(err, errlen, "qgcm_coalescer_create: bad argument");
        return nullptr;
    }
    auto *c = new qgcm_coalescer;
    c->ctx = ctx;
    c->device = qgcm::ctx_device(ctx);
    c->max_batch = max_batch;
    c->max_packet = max_packet;
    c->aad_len = aad_len;
    c->max_wait = std::chrono::microseconds(max_wait_us);
    c->quiet = std::chrono::microseconds(max_wait_us / 8 > 5 ? max_wait_us / 8 : 5);
    c->cap_bytes = (uint64_t)max_batch * slot_bytes(true, max_packet);
    c->one_kernel = qgcm::ctx_one_kernel(ctx) && slot_bytes(true, max_packet) <= qgcm::kOneCap - 16;
    bool ok = hipSetDevice(c->device) == hipSuccess;
    for (int d = 0; d < 2 && ok; ++d) {
        Lane &ln = c->lanes[d];
        ln.seal = d == 0;
        ok = hipStreamCreateWithFlags(&ln.stream, hipStreamNonBlocking) == hipSuccess &&
             hipHostMalloc(reinterpret_cast<void **>(&ln.done), qgcm::kOneBatchMax, hipHostMallocDefault) == hipSuccess;
        for (CBatch &B : ln.b) {
            ok = ok && hipHostMalloc(&B.h_arena, c->cap_bytes, hipHostMallocDefault) == hipSuccess &&
                 hipHostMalloc(&B.h_descs, sizeof(qgcm_desc) * max_batch, hipHostMallocDefault) == hipSuccess &&
                 hipHostMalloc(&B.h_nonces, 12ull * max_batch, hipHostMallocDefault) == hipSuccess &&
                 hipHostMalloc(&B.h_status, max_batch, hipHostMallocDefault) == hipSuccess &&
                 hipMalloc(&B.d_arena, c->cap_bytes) == hipSuccess &&
                 hipMalloc(&B.d_descs, sizeof(qgcm_desc) * max_batch) == hipSuccess &&
                 hipMalloc(&B.d_nonces, 12ull * max_batch) == hipSuccess &&
                 hipMalloc(&B.d_status, max_batch) == hipSuccess;
        }
        ln.b[0].st = St::Filling;
    }
    if (!ok) {
        for (Lane &ln : c->lanes) free_lane(ln);
        delete c;
        set_err(err, errlen, "qgcm_coalescer_create: allocation failed");
        return nullptr;
    }
    for (Lane &ln : c->lanes) ln.thr = std::thread(flusher, c, &ln);
    return c;
}

void qgcm_coalescer_destroy(qgcm_coalescer *c) {
    if (!c) return;
    for (Lane &ln : c->lanes) {
        std::lock_guard<std::mutex> g(ln.mu);
        c->stop = true;
        ln.cv_flush.notify_all();
        ln.cv_caller.notify_all();
    }
    for (Lane &ln : c->lanes)
        if (ln.thr.joinable()) ln.thr.join();
    for (Lane &ln : c->lanes) free_lane(ln);
    delete c;
}

long qgcm_coalescer_seal(qgcm_coalescer *c, uint32_t key_idx, uint8_t *data, long length, const uint8_t *aad,
                         uint32_t aad_len) {
    if (!c || !data || length < 0 || length > (long)c->max_packet || (aad_len && !aad)) return -1;
    if (aad_len != c->aad_len) return qgcm_seal_one(c->ctx, key_idx, data, length, aad, aad_len, nullptr);
    if (!qgcm::ctx_key_ready(c->ctx, key_idx)) return -1;
    return submit(c, &c->lanes[0], key_idx, data, (uint32_t)length, aad);
}

long qgcm_coalescer_open(qgcm_coalescer *c, uint32_t key_idx, uint8_t *data, long len, const uint8_t *aad,
                         uint32_t aad_len) {
    if (!c || (!data && len) || len < 0 || (aad_len && !aad)) return -1;
    if (len < QGCM_OVERHEAD) return -1;  // crypto/aes.go:58-60 (the reference panics below 12)
    if (len - QGCM_OVERHEAD > (long)c->max_packet) return -1;
    if (aad_len != c->aad_len) return qgcm_open_one(c->ctx, key_idx, data, len, aad, aad_len);
    if (!qgcm::ctx_key_ready(c->ctx, key_idx)) return -1;
    return submit(c, &c->lanes[1], key_idx, data, (uint32_t)len, aad);
}

}  // extern "C"
