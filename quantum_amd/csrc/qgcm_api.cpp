// qgcm_api.cpp -- the C ABI of include/qgcm.h over the gfx950 kernels in gcm_kernels.hip.
//
// Host responsibilities only: argument checks (the Go methods' error contract), device key
// tables, stream plumbing and pinned staging.  All cryptographic work on packets runs on the
// GPU; there is no CPU fallback -- without a usable HIP device qgcm_create returns NULL.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <future>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/qgcm.h"
#include "chain_claim.h"
#include "gcm_internal.h"

using namespace qgcm;

constexpr int kPipeStreams = 3;         // copy-in / kernel / copy-out stages
constexpr uint64_t kPipeChunk = 32ull << 20;  // bytes of slots per pipeline chunk (chained path)
constexpr uint64_t kHostChunk = 64ull << 20;  // run_host: bytes of slots per chunk
constexpr uint64_t kHostRing = 4ull << 30;    // run_host: device staging budget (HBM is 288 GB)

struct qgcm_ctx {
    int device = 0;
    int num_cus = 0;
    uint32_t max_keys = 0;
    int uniform_variant = kVariantUniform;  // kernel variant for single-key batches (QGCM_VARIANT)
    int desc_variant = kVariantDescQuad;    // kernel variant for descriptor batches (QGCM_DESC_VARIANT)
    int wgs_per_cu_override = 0;            // persistent-grid workgroups per CU (QGCM_WGS_PER_CU, tuning)
    bool one_kernel = true;                 // seal_one/open_one use the latency kernel (QGCM_ONE_KERNEL)
    bool variant_forced = false;            // QGCM_VARIANT given: uniform batches always run that variant
    uint32_t desc_one_max = kDescOneMax;        // small keyed batches (run_descs_one), QGCM_DESC_ONE_MAX
    uint32_t direct_max = kDirectMax;           // ... sealed in place in pinned host memory, QGCM_DIRECT_MAX
    uint32_t one_uniform_max = kOneUniformMax;  // uniform batches up to this many packets take the
                                                // latency kernel (QGCM_ONE_UNIFORM_MAX, tuning)
    uint32_t launch_chunk = kLaunchChunk;       // uniform batches launch at most this many packets per
                                                // kernel (QGCM_LAUNCH_CHUNK, tuning; 0 = one launch)
    uint32_t desc_chunk = kDescChunk;           // descriptor batches: packets per sorted chunk
                                                // (QGCM_DESC_CHUNK, tuning; 0 = one launch)
    // A/B switches, read once at qgcm_create like every other knob (a getenv per call would race a
    // setenv from another thread): QGCM_DESC_ONE=0 sends small keyed batches to the worklist path,
    // QGCM_HOST_DIRECT=0 stops qgcm_seal_host sealing worker-sized pinned arenas in place,
    // QGCM_SMALL_WORKLIST=0 builds small batches' worklists by the multi-launch path
    bool desc_one_on = true, host_direct = true, small_wl = true;
    // the snappy + GCM chain's A/B knobs, read at qgcm_create too: QGCM_CHAIN_CHUNK_MB (bytes of slots
    // per chunk), QGCM_CHAIN_SLOTS (chunks in flight), QGCM_CHAIN_DEV_AHEAD / QGCM_CHAIN_DEV_BACKLOG
    // (the host/device codec split; backlog -1 = two chunks' items), QGCM_SNAPPY_GROUP (the device
    // encoder: four packets per wave, or one wave per packet)
    uint64_t chain_chunk = kPipeChunk;
    int chain_slots = kPipeStreams, chain_dev_ahead = 2, chain_dev_backlog = -1;
    bool snappy_group = true;
    int snappy_per_cu = 0;  // QGCM_SNAPPY_PER_CU: cap on resident codec waves per CU (0 = as the LDS allows; A/B knob)
    // the chain's host codec workers run one per physical core, the GPU's NUMA-local cores and the least
    // busy first (cpu_topo.cpp; QGCM_CHAIN_PIN=0 at qgcm_create: left to the scheduler).  The core list
    // comes from a 30-ms sample of the host's load, taken per device in the background from the first
    // qgcm_create on and again once it is older than kCodecCpusMaxAge (codec_cpu_list); a chained call
    // pins only when the list has a core for every worker, so no two workers share one CPU.
    bool chain_pin = true;
    std::mutex codec_cpus_mu;
    std::vector<int> codec_cpus;
    uint32_t *d_rk = nullptr;
    uint4 *d_gh = nullptr;
    uint4 *d_pw = nullptr;   // per-packet flat GHASH: comb tables of H^1..H^kPwPowers, key slots < pw_keys
    uint32_t pw_keys = 0;    // (2.75 MiB per key; QGCM_FLAT_GHASH_KEYS, default min(max_keys, 256), 0 = off)
    uint32_t *d_te = nullptr;
    uint8_t *d_sbox = nullptr;
    uint8_t *d_key_valid = nullptr;  // device view of key_set (descriptor batches check it per packet)
    std::vector<uint8_t> key_set;  // host view of which slots are populated
    std::mutex key_mu;

    // descriptor-batch workspace (worklist), guarded by ws_mu for the whole enqueue
    std::mutex ws_mu;
    void *d_qws = nullptr;  // sorted quad worklist workspace
    size_t qws_cap = 0;

    // per-packet and host-batch staging, guarded by io_mu
    std::mutex io_mu;
    // per-packet calls (qgcm_seal_one / qgcm_open_one): a pool of pinned staging slots, each with
    // its own stream and lock, so concurrent callers (quantum's worker goroutines) run their
    // one-workgroup kernels side by side instead of queueing on one slot
    struct OneSlot {
        std::mutex mu;
        hipStream_t stream = nullptr;
        uint8_t *h = nullptr;
        size_t cap = 0;
    };
    static constexpr int kOneSlots = 8;
    // pool slots stay small (the latency kernel's LDS staging limit): payloads up to ~32 KiB, which
    // covers every packet quantum sends (MTU 1433, jumbo 9000); larger calls share one big slot
    static constexpr size_t kOneSlotCap = kOneCap + 4096;
    OneSlot one[kOneSlots];
    OneSlot big;  // calls whose staging exceeds kOneSlotCap (released after the call past 64 MiB)
    std::atomic<uint32_t> one_rr{0};

    // host-batch pipeline (qgcm_seal_host / qgcm_open_host), guarded by io_mu
    hipStream_t pipe[kPipeStreams] = {};
    std::vector<hipEvent_t> ev_in, ev_kern, ev_out;  // run_host: per device chunk slot
    uint64_t host_chunk = kHostChunk, host_ring = kHostRing;  // QGCM_PIPE_CHUNK_MB / QGCM_PIPE_RING_MB
    uint8_t *d_ring = nullptr;  // chunk slots (run_host: up to host_ring bytes; chained path: one per stream)
    size_t ring_cap = 0;
    uint8_t *h_stat = nullptr;  // pinned status bytes of the whole host batch
    size_t hstat_cap = 0;
    uint8_t *d_side = nullptr;  // run_host: nonces (12 n) and status (n) of the whole batch
    size_t side_cap = 0;
    qgcm_desc *h_desc = nullptr;  // pinned descriptor staging of the chained (snappy + GCM) path
    uint32_t *h_lens = nullptr;   // pinned length staging of its device-codec chunks (hdesc_cap entries)
    std::vector<hipStream_t> chain_extra;  // chained path: streams past pipe[] (QGCM_CHAIN_SLOTS > 3)
    size_t hdesc_cap = 0;

    // orders reuse of the descriptor workspace across streams (guarded by ws_mu)
    hipEvent_t ws_done = nullptr;
    bool ws_pending = false;

    // the uniform kernel's shared tail (gcm_kernels.hip QGCM_TILE_POOL): a ring of kPoolSets zeroed
    // counter sets in device memory, one per launch in turn, whatever its stream, with nothing queued
    // between launches (an event record there costs ~3 us, profiles/r6_s23).  The grid's last wave
    // zeroes its set and posts the launch's generation to h_pool_done[k] (pinned); a set comes round
    // again kPoolSets launches later, and if its last launch has not posted yet the new launch first waits
    // for it on its own stream (hipStreamWaitValue32).  Guarded by pool_mu.
    uint32_t *d_pool = nullptr;
    uint32_t *h_pool_done = nullptr;
    uint32_t pool_gen[kPoolSets] = {};  // generation of each set's last launch (0: none yet)
    uint32_t pool_launches = 0;
    uint32_t pool_sets = kPoolSets;  // sets in use (QGCM_POOL_SETS: a short ring, so tests reach the wait)
    std::mutex pool_mu;

    std::atomic<uint64_t> launches[QGCM_KERNEL_COUNTERS] = {};  // qgcm_launch_counts
    void count(int k, uint64_t v = 1) { launches[k].fetch_add(v, std::memory_order_relaxed); }

    // where the chained snappy + GCM calls run the codec: 0 host, 1 host/device split, 2 device
    // (QGCM_CHAIN_DEVICE, qgcm_chain_codec)
    std::atomic<int> chain_codec{1};

    // resident per-packet service (resident.cpp), created on the first per-packet call
    bool res_on = true;  // QGCM_RESIDENT=0: every per-packet call launches gcm_one_kernel
    qgcm::ResidentConfig res_cfg{};  // QGCM_RESIDENT_*, read at qgcm_create
    std::atomic<qgcm::Resident *> res{nullptr};
    std::atomic<bool> res_failed{false};
    std::mutex res_mu;
};

namespace {

thread_local bool tl_dummy;

int env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}

uint8_t gf8_mul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) p ^= a;
        const uint8_t hi = a & 0x80;
        a <<= 1;
        if (hi) a ^= 0x1b;
        b >>= 1;
    }
    return p;
}

// FIPS-197 S-box from its definition; Te0[x] = (2S, S, S, 3S) as a little-endian word,
// Te1 = rotl8(Te0).
void build_tables(uint8_t sbox[256], uint32_t te[512]) {
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x) {
            uint8_t r = 1, b = (uint8_t)x;
            for (int e = 254; e; e >>= 1) {
                if (e & 1) r = gf8_mul(r, b);
                b = gf8_mul(b, b);
            }
            inv = r;
        }
        auto rl = [](uint8_t v, int s) { return (uint8_t)((v << s) | (v >> (8 - s))); };
        sbox[x] = inv ^ rl(inv, 1) ^ rl(inv, 2) ^ rl(inv, 3) ^ rl(inv, 4) ^ 0x63;
    }
    for (int x = 0; x < 256; ++x) {
        const uint32_t s = sbox[x], s2 = gf8_mul((uint8_t)s, 2), s3 = s2 ^ s;
        const uint32_t t0 = s2 | (s << 8) | (s << 16) | (s3 << 24);
        te[x] = t0;
        te[256 + x] = (t0 << 8) | (t0 >> 24);
    }
}

void set_err(char *err, int errlen, const char *msg) {
    if (err && errlen > 0) snprintf(err, (size_t)errlen, "%s", msg);
}

int hip_fail(hipError_t e) { return e == hipSuccess ? QGCM_OK : QGCM_E_HIP; }

int grid_for(const qgcm_ctx *ctx, uint32_t n_items, int variant) {
    // CUs held by a running resident per-packet kernel (one workgroup each) are left to it
    const int cus = std::max(1, ctx->num_cus - resident_workers_running(ctx->res.load(std::memory_order_acquire)));
    const uint32_t waves = (uint32_t)variant_waves(variant);
    const uint32_t tiles = (n_items + 15) / 16;  // 16-packet wave tiles
    const uint32_t wgs = (tiles + waves - 1) / waves;
    // persistent grid: the resident workgroups (each fills its own LDS tables once)
    const uint32_t per_cu = ctx->wgs_per_cu_override > 0 ? (uint32_t)ctx->wgs_per_cu_override
                                                         : (uint32_t)variant_wgs_per_cu(variant);
    const uint32_t cap = (uint32_t)cus * per_cu;
    return (int)(wgs < cap ? (wgs ? wgs : 1) : cap);
}

Batch base_batch(const qgcm_ctx *ctx) {
    Batch b{};
    b.rk_table = ctx->d_rk;
    b.gh_table = ctx->d_gh;
    b.pw_table = ctx->d_pw;
    b.pw_keys = ctx->pw_keys;
    b.te = ctx->d_te;
    b.key_valid = ctx->d_key_valid;
    b.max_keys = ctx->max_keys;
    return b;
}

int run_uniform(qgcm_ctx *ctx, bool seal, uint8_t *arena, uint64_t stride, uint32_t n, uint32_t len,
                uint32_t key_idx, const uint8_t *nonces, uint32_t aad_len, uint8_t *status, hipStream_t s);

// seal_one / open_one: the latency kernel when the slot fits its LDS staging area, else the batch
// kernel on a batch of one (QGCM_ONE_KERNEL=0 forces the latter, for A/B runs).
// With the latency kernel the call completes on its flag (status[1], written last by the kernel,
// after a system-scope fence) instead of hipStreamSynchronize: the host spins on pinned memory for
// up to 1 s, then falls back to the stream (which also reports a failed launch or a fault).
int run_one(qgcm_ctx *ctx, bool seal, uint8_t *slot, uint64_t stride, uint32_t len, uint32_t key_idx,
            uint32_t aad_len, uint8_t *status, hipStream_t s) {
    if (ctx->one_kernel && stride <= kOneCap - 16 && !(stride & 15) && !((uintptr_t)slot & 15)) {
        volatile uint8_t *done = status + 1;
        *done = 0;
        Batch b = base_batch(ctx);
        b.done = status + 1;
        b.arena = slot;
        b.status = status;
        b.stride = stride;
        b.uniform_len = len;
        b.uniform_key = key_idx;
        b.n = 1;
        b.n_items = 64;
        b.aad_len = aad_len;
        if (launch_one(seal, b, s) != hipSuccess) return QGCM_E_HIP;
        ctx->count(QGCM_KERNEL_ONE);
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spins = 0; *done == 0; ++spins) {
            __builtin_ia32_pause();
            if ((spins & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) break;
        }
        if (*done == 0) return hip_fail(hipStreamSynchronize(s));
        std::atomic_thread_fence(std::memory_order_acquire);
        return QGCM_OK;
    }
    const int rc = run_uniform(ctx, seal, slot, stride, 1, len, key_idx, nullptr, aad_len, status, s);
    return rc == QGCM_OK ? hip_fail(hipStreamSynchronize(s)) : rc;
}

// The context's resident per-packet service, created on first use (nullptr: off or unavailable).
Resident *get_resident(qgcm_ctx *ctx) {
    Resident *r = ctx->res.load(std::memory_order_acquire);
    if (r || !ctx->res_on || ctx->res_failed.load(std::memory_order_relaxed)) return r;
    std::lock_guard<std::mutex> g(ctx->res_mu);
    r = ctx->res.load(std::memory_order_acquire);
    if (!r) {
        r = resident_create(ctx->device, base_batch(ctx), ctx->num_cus, ctx->res_cfg);
        if (!r) ctx->res_failed = true;
        ctx->res.store(r, std::memory_order_release);
    }
    return r;
}

// Lock-free: every per-packet call asks, from all worker threads at once (key_set is sized once at
// qgcm_create and its bytes are written under key_mu, set after the device tables are ready).
bool key_ok(qgcm_ctx *ctx, uint32_t k) {
    if (k >= ctx->max_keys) return false;
    return __atomic_load_n(&ctx->key_set[k], __ATOMIC_ACQUIRE) != 0;
}

}  // namespace

bool qgcm::ctx_one_kernel(const qgcm_ctx *ctx) { return ctx->one_kernel; }
hipStream_t qgcm::ctx_pipe(qgcm_ctx *ctx, int k) { return ctx->pipe[k]; }
std::mutex &qgcm::ctx_io_mu(qgcm_ctx *ctx) { return ctx->io_mu; }

uint32_t qgcm::descs_one_max(const qgcm_ctx *ctx) {
    return ctx->one_kernel && !ctx->variant_forced && ctx->desc_one_on ? ctx->desc_one_max : 0u;
}

// Device-accessible address of pinned host memory [p, p + bytes) inside one allocation, or 0.
uint64_t qgcm::pinned_view(const void *p, uint64_t bytes) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeHost || !a.devicePointer) {
        (void)hipGetLastError();  // pageable memory reports an error: clear it
        return 0;
    }
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, a.devicePointer) != hipSuccess || !base) {
        (void)hipGetLastError();
        return 0;
    }
    const uint64_t dv = reinterpret_cast<uint64_t>(a.devicePointer), b = reinterpret_cast<uint64_t>(base);
    return dv >= b && dv + bytes <= b + size ? dv : 0;
}

uint32_t qgcm::direct_max(const qgcm_ctx *ctx) { return descs_one_max(ctx) ? ctx->direct_max : 0u; }

int qgcm::run_descs_one(qgcm_ctx *ctx, bool seal, uint8_t *d_arena, const qgcm_desc *d_descs, uint32_t n,
                        const uint8_t *d_nonces, uint32_t aad_len, uint8_t *d_status, hipStream_t s) {
    if (!ctx || !n || !d_arena || !d_descs || aad_len > 4 || n > QGCM_MAX_BATCH || !descs_one_max(ctx) ||
        ((uintptr_t)d_arena & 15))
        return QGCM_E_ARG;
    if (hipSetDevice(ctx->device) != hipSuccess) return QGCM_E_HIP;
    Batch b = base_batch(ctx);
    b.arena = d_arena;
    b.descs = d_descs;
    b.nonces = seal ? d_nonces : nullptr;
    b.status = d_status;
    b.n = n;
    b.n_items = (n + 63) & ~63u;
    b.aad_len = aad_len;
    if (launch_one(seal, b, s) != hipSuccess) return QGCM_E_HIP;
    ctx->count(QGCM_KERNEL_ONE);
    return QGCM_OK;
}

namespace {

int run_uniform(qgcm_ctx *ctx, bool seal, uint8_t *arena, uint64_t stride, uint32_t n, uint32_t len,
                uint32_t key_idx, const uint8_t *nonces, uint32_t aad_len, uint8_t *status, hipStream_t s) {
    if (!ctx || (!arena && n) || aad_len > 4 || n > QGCM_MAX_BATCH) return QGCM_E_ARG;
    if (((uintptr_t)arena & 3) || (stride & 3) || (nonces && ((uintptr_t)nonces & 3))) return QGCM_E_ARG;
    if (n && stride < (uint64_t)len + 4 + (seal ? QGCM_OVERHEAD : 0)) return QGCM_E_ARG;
    if ((seal || len >= QGCM_OVERHEAD) && len - (seal ? 0u : (uint32_t)QGCM_OVERHEAD) >= QGCM_MAX_PAYLOAD)
        return QGCM_E_ARG;
    if (!key_ok(ctx, key_idx)) return QGCM_E_KEY;
    if (n == 0) return QGCM_OK;
    if (hipSetDevice(ctx->device) != hipSuccess) return QGCM_E_HIP;
    Batch b = base_batch(ctx);
    b.arena = arena;
    b.nonces = seal ? nonces : nullptr;
    b.status = status;
    b.stride = stride;
    b.uniform_len = len;
    b.uniform_key = key_idx;
    b.n = n;
    b.n_items = (uint32_t)(((uint64_t)n + 63) & ~63ull);
    b.aad_len = aad_len;
    // Small batches (one workgroup wave: n <= kOneUniformMax) take the latency kernel, one
    // workgroup per packet, when the slots allow it and no kernel variant is forced (QGCM_VARIANT).
    const uint64_t stage = (4ull + len + (seal ? QGCM_OVERHEAD : 0) + 15) & ~15ull;
    if (ctx->one_kernel && !ctx->variant_forced && n <= ctx->one_uniform_max && !(stride & 15) &&
        !((uintptr_t)arena & 15) && stage <= stride && stage <= kOneCap - 16) {
        if (launch_one(seal, b, s) != hipSuccess) return QGCM_E_HIP;
        ctx->count(QGCM_KERNEL_ONE);
        return QGCM_OK;
    }
    const int v = ctx->uniform_variant;
    // Large batches go out as back-to-back launches of launch_chunk packets on the same stream: one
    // 2^23-packet launch ran at 768 GiB/s, the same batch as 2^19-packet launches at 827, at 2^20 packets
    // either form 826-829 (tools/exp_chunked.py).
    const uint32_t chunk = ctx->launch_chunk ? ctx->launch_chunk : n;
    for (uint32_t p = 0; p < n; p += chunk) {
        const uint32_t m = std::min(chunk, n - p);
        Batch c = b;
        c.arena = arena + (uint64_t)p * stride;
        c.nonces = b.nonces ? b.nonces + 12ull * p : nullptr;
        c.status = status ? status + p : nullptr;
        c.n = m;
        c.n_items = (uint32_t)(((uint64_t)m + 63) & ~63ull);
        const int grid = grid_for(ctx, c.n_items, v);
        // the shared tail needs two full rows of tiles (gcm_kernels.hip); smaller launches go without it
        const uint64_t rows = ((uint64_t)c.n_items / 16) / ((uint64_t)grid * (uint64_t)variant_waves(v));
        if (ctx->d_pool && rows >= 2) {
            std::lock_guard<std::mutex> g(ctx->pool_mu);
            const uint32_t k = ctx->pool_launches % ctx->pool_sets;
            if (ctx->pool_gen[k] && __atomic_load_n(ctx->h_pool_done + k, __ATOMIC_ACQUIRE) != ctx->pool_gen[k]) {
                if (hipStreamWaitValue32(s, ctx->h_pool_done + k, ctx->pool_gen[k], hipStreamWaitValueEq, 0xffffffffu) !=
                    hipSuccess)
                    return QGCM_E_HIP;
                ctx->count(QGCM_KERNEL_TAIL_WAITS);
            }
            if (++ctx->pool_launches == 0) ctx->pool_launches = 1;
            c.pool = ctx->d_pool + (size_t)k * kPoolSetWords;
            c.pool_done = ctx->h_pool_done + k;
            c.pool_gen = ctx->pool_launches;  // unique among the sets' outstanding generations
            if (launch_packets(seal, v, c, grid, s) != hipSuccess) return QGCM_E_HIP;
            ctx->pool_gen[k] = c.pool_gen;  // (a launch that never started posts nothing to wait for)
        } else if (launch_packets(seal, v, c, grid, s) != hipSuccess) {
            return QGCM_E_HIP;
        }
        ctx->count(QGCM_KERNEL_QUAD);
    }
    return QGCM_OK;
}

int run_descs_locked(qgcm_ctx *ctx, bool seal, const qgcm_desc *descs, uint32_t n, hipStream_t s, Batch b,
                     uint8_t *arena, const uint8_t *nonces, uint32_t aad_len, uint8_t *status);

int run_descs(qgcm_ctx *ctx, bool seal, uint8_t *arena, const qgcm_desc *descs, uint32_t n, const uint8_t *nonces,
              uint32_t aad_len, uint8_t *status, hipStream_t s) {
    if (!ctx || (n && (!arena || !descs)) || aad_len > 4 || n > QGCM_MAX_BATCH) return QGCM_E_ARG;
    if (((uintptr_t)arena & 3) || (nonces && ((uintptr_t)nonces & 3))) return QGCM_E_ARG;
    if (n == 0) return QGCM_OK;
    if (hipSetDevice(ctx->device) != hipSuccess) return QGCM_E_HIP;
    // statuses start at 0 (packets left out of the worklist keep it); small batches' worklist kernel
    // zeroes them itself
    if (status && !small_worklist(n, ctx->small_wl) && hipMemsetAsync(status, 0, n, s) != hipSuccess) return QGCM_E_HIP;
    // The workspace is reused by the next call on any stream: serialize descriptor batches per ctx.
    std::lock_guard<std::mutex> g(ctx->ws_mu);
    // ...and on the device: this batch's worklist build must not start before the previous batch's
    // kernel (possibly on another stream) has finished reading the workspace.
    if (ctx->ws_pending && hipStreamWaitEvent(s, ctx->ws_done, 0) != hipSuccess) return QGCM_E_HIP;
    const int rc = run_descs_locked(ctx, seal, descs, n, s, base_batch(ctx), arena, nonces, aad_len, status);
    if (rc == QGCM_OK) {
        if (hipEventRecord(ctx->ws_done, s) != hipSuccess) return QGCM_E_HIP;
        ctx->ws_pending = true;
    }
    return rc;
}

int run_descs_locked(qgcm_ctx *ctx, bool seal, const qgcm_desc *descs, uint32_t n, hipStream_t s, Batch b,
                     uint8_t *arena, const uint8_t *nonces, uint32_t aad_len, uint8_t *status) {
    b.arena = arena;
    b.descs = descs;
    b.nonces = seal ? nonces : nullptr;
    b.status = status;
    b.n = n;
    b.aad_len = aad_len;
    const int v = ctx->desc_variant;
    if (ctx->desc_chunk && n > ctx->desc_chunk) {
        // back-to-back chunks on this stream, each with its own sorted worklist (the workspace is
        // reused in stream order); descriptors, nonces and status are chunk-relative, offsets absolute
        for (uint32_t p = 0; p < n; p += ctx->desc_chunk) {
            const uint32_t m = std::min(ctx->desc_chunk, n - p);
            const int rc = run_descs_locked(ctx, seal, descs + p, m, s, b, arena, nonces ? nonces + 12ull * p : nullptr,
                                            aad_len, status ? status + p : nullptr);
            if (rc != QGCM_OK) return rc;
        }
        return QGCM_OK;
    }
    {
        uint32_t items = 0;
        const size_t need = quad_worklist_bytes(n, ctx->max_keys, &items);
        if (need > ctx->qws_cap) {
            if (ctx->d_qws) hipFree(ctx->d_qws);
            ctx->d_qws = nullptr;
            ctx->qws_cap = 0;
            if (hipMalloc(&ctx->d_qws, need) != hipSuccess) return QGCM_E_NOMEM;
            ctx->qws_cap = need;
        }
        QuadWorklist q{};
        if (launch_quad_worklist(descs, n, ctx->max_keys, ctx->d_key_valid, seal, ctx->d_qws, ctx->qws_cap, &q, s,
                                 status, small_worklist(n, ctx->small_wl)) != hipSuccess)
            return QGCM_E_HIP;
        b.worklist = q.worklist;
        b.tile_keys = q.tile_keys;
        b.runs = q.runs;
        b.run_next = q.run_next;
        b.nruns = q.nruns;
        b.tile_counter = q.tile_counter;
        b.n_items = q.n_items;
        // a key is a run once it has kSegMinTiles tiles, i.e. (kSegMinTiles - 1) * 16 + 1 packets (the
        // worklist's ceil(count / 16)); a smaller batch cannot give any key a run, so only the segmented
        // kernel's complement (the per-wave kernel) is launched
        const int vc = variant_complement(v);
        if (vc < 0 || n > (kSegMinTiles - 1) * 16u) {
            if (launch_packets(seal, v, b, grid_for(ctx, b.n_items, v), s) != hipSuccess) return QGCM_E_HIP;
            ctx->count(v == kVariantDescQuad ? QGCM_KERNEL_SEGMENTED : QGCM_KERNEL_PER_WAVE);
        }
        if (vc < 0) return QGCM_OK;
        // the short keys' tiles (fewer than kSegMinTiles per key) through the per-wave kernel; its
        // dynamic tile counter is the next word of the zeroed counter block
        b.tile_list = q.short_tiles;
        b.n_list = q.nshort;
        b.tile_counter = q.tile_counter + 3;
        if (launch_packets(seal, vc, b, grid_for(ctx, b.n_items, vc), s) != hipSuccess) return QGCM_E_HIP;
        ctx->count(QGCM_KERNEL_PER_WAVE);
        return QGCM_OK;
    }
}

// Per-packet streams are created at the highest priority the device offers, so a per-packet call
// does not queue behind a long batch kernel on the (few, GPU_MAX_HW_QUEUES) hardware queues.
hipError_t create_one_stream(hipStream_t *s) {
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi);
}

// Takes a free per-packet staging slot (the first one whose lock is free, starting round-robin; all
// busy: waits on one) and makes its pinned buffer hold `bytes` (the kernel works on it in place,
// zero-copy).  Pool slots are capped at kOneSlotCap bytes, so they never grow on the hot path past
// the first call; larger payloads go through the one big slot.  Returns nullptr on allocation failure.
qgcm_ctx::OneSlot *acquire_one(qgcm_ctx *ctx, size_t bytes, std::unique_lock<std::mutex> &lk) {
    const uint32_t start = ctx->one_rr.fetch_add(1, std::memory_order_relaxed);
    qgcm_ctx::OneSlot *sl = nullptr;
    if (bytes > qgcm_ctx::kOneSlotCap) {
        sl = &ctx->big;
        lk = std::unique_lock<std::mutex>(sl->mu);
    }
    for (int i = 0; i < qgcm_ctx::kOneSlots && !sl; ++i) {
        qgcm_ctx::OneSlot &c = ctx->one[(start + i) % qgcm_ctx::kOneSlots];
        std::unique_lock<std::mutex> l(c.mu, std::try_to_lock);
        if (l.owns_lock()) {
            lk = std::move(l);
            sl = &c;
        }
    }
    if (!sl) {
        sl = &ctx->one[start % qgcm_ctx::kOneSlots];
        lk = std::unique_lock<std::mutex>(sl->mu);
    }
    if (!sl->stream && create_one_stream(&sl->stream) != hipSuccess) {
        sl->stream = nullptr;
        return nullptr;
    }
    if (bytes > sl->cap) {
        size_t want = sl == &ctx->big ? bytes : qgcm_ctx::kOneSlotCap;
        if (sl != &ctx->big)
            while (want < bytes) want <<= 1;
        if (sl->h) hipHostFree(sl->h);
        sl->h = nullptr;
        sl->cap = 0;
        if (hipHostMalloc(&sl->h, want, hipHostMallocDefault) != hipSuccess) return nullptr;
        sl->cap = want;
    }
    return sl;
}

// The big slot keeps up to 64 MiB pinned between calls; beyond that it is released after the call
// (on every return path: the guard runs while the slot's lock is still held).
struct BigRelease {
    qgcm_ctx *ctx;
    qgcm_ctx::OneSlot *sl;
    ~BigRelease() {
        if (!sl || sl != &ctx->big || sl->cap <= (64u << 20)) return;
        hipHostFree(sl->h);
        sl->h = nullptr;
        sl->cap = 0;
    }
};

}  // namespace

// The chain's codec core list for a device (qgcm_ctx::chain_pin), off the caller's path: the first
// context of a device starts the 30-ms load sample, later ones share it, and a list older than
// kCodecCpusMaxAge starts a new sample (a long-running process must not pin by stale load figures).
// Returns the newest finished list, or the first sample still running.
static constexpr auto kCodecCpusMaxAge = std::chrono::seconds(60);
static std::shared_future<std::vector<int>> codec_cpu_list(int device) {
    struct Lists {
        std::shared_future<std::vector<int>> ready, next;
        std::chrono::steady_clock::time_point at;
    };
    static std::mutex mu;
    static std::map<int, Lists> lists;
    auto sample = [device] {
        return std::async(std::launch::async, [device] {
                   cpu_set_t local;
                   const bool have = qgcm::gpu_local_cpus(device, &local) > 0;
                   return qgcm::spread_cpus(have ? &local : nullptr, 30);
               }).share();
    };
    const auto now = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> g(mu);
    auto it = lists.find(device);
    if (it == lists.end()) {
        Lists l;
        l.next = sample();
        l.at = now;
        lists.emplace(device, l);
        return l.next;
    }
    Lists &l = it->second;
    if (l.next.valid() && l.next.wait_for(std::chrono::seconds(0)) == std::future_status::ready) {
        l.ready = l.next;
        l.next = {};
    }
    if (!l.next.valid() && now - l.at > kCodecCpusMaxAge) {
        l.next = sample();
        l.at = now;
    }
    return l.ready.valid() ? l.ready : l.next;
}

extern "C" {

const char *qgcm_version(void) { return "qgcm 0.1.0 (gfx950)"; }

int qgcm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

const char *qgcm_strerror(int code) {
    switch (code) {
        case QGCM_OK: return "ok";
        case QGCM_E_ARG: return "invalid argument";
        case QGCM_E_HIP: return "HIP runtime error";
        case QGCM_E_KEY: return "key index not set or out of range";
        case QGCM_E_AUTH: return "message authentication failed";
        case QGCM_E_NOMEM: return "out of device or pinned memory";
        default: return "unknown error";
    }
}

qgcm_ctx *qgcm_create(int device, uint32_t max_keys, char *err, int errlen) {
    (void)tl_dummy;
    if (max_keys == 0 || max_keys > QGCM_MAX_KEYS) {
        set_err(err, errlen, "max_keys must be in [1, 2^20 - 1]");
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        set_err(err, errlen, "no such HIP device");
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        set_err(err, errlen, "hipSetDevice failed");
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        set_err(err, errlen, "hipGetDeviceProperties failed");
        return nullptr;
    }
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        char m[QGCM_ERRLEN];
        snprintf(m, sizeof m, "device %d is %s; libqgcm is built for gfx950 only", device, prop.gcnArchName);
        set_err(err, errlen, m);
        return nullptr;
    }
    {
        // the kernel variant table (and each kernel's LDS limit) before the variant overrides below
        // consult it; serialized for contexts created from several threads
        static std::mutex init_mu;
        std::lock_guard<std::mutex> g(init_mu);
        if (init_kernels() != hipSuccess) {
            set_err(err, errlen, "kernel setup failed");
            return nullptr;
        }
    }
    auto *ctx = new qgcm_ctx();
    ctx->device = device;
    ctx->num_cus = prop.multiProcessorCount;
    ctx->max_keys = max_keys;
    ctx->key_set.assign(max_keys, 0);
    if (const char *v = getenv("QGCM_VARIANT")) {  // kernel variant overrides (tuning and tests)
        const int iv = atoi(v);
        if (variant_valid(iv) && !variant_desc(iv)) {
            ctx->uniform_variant = iv;
            ctx->variant_forced = true;
        }
    }
    if (const char *v = getenv("QGCM_WGS_PER_CU")) ctx->wgs_per_cu_override = atoi(v);
    if (const char *v = getenv("QGCM_ONE_KERNEL")) ctx->one_kernel = atoi(v) != 0;
    if (const char *v = getenv("QGCM_CHAIN_DEVICE")) ctx->chain_codec = std::max(0, std::min(2, atoi(v)));
    if (const char *v = getenv("QGCM_RESIDENT")) ctx->res_on = atoi(v) != 0;
    ctx->res_cfg = qgcm::resident_config_from_env();
    if (const char *v = getenv("QGCM_ONE_UNIFORM_MAX")) ctx->one_uniform_max = (uint32_t)std::max(0, atoi(v));
    if (const char *v = getenv("QGCM_DESC_ONE_MAX")) ctx->desc_one_max = (uint32_t)std::max(0, atoi(v));
    if (const char *v = getenv("QGCM_DIRECT_MAX")) ctx->direct_max = (uint32_t)std::max(0, atoi(v));
    if (const char *v = getenv("QGCM_LAUNCH_CHUNK"))  // rounded down to whole 64-packet tiles
        ctx->launch_chunk = (uint32_t)std::max(0, atoi(v)) & ~63u;
    if (const char *v = getenv("QGCM_DESC_CHUNK")) ctx->desc_chunk = (uint32_t)std::max(0, atoi(v));
    if (const char *v = getenv("QGCM_PIPE_CHUNK_MB")) ctx->host_chunk = (uint64_t)std::max(1, atoi(v)) << 20;
    if (const char *v = getenv("QGCM_PIPE_RING_MB")) ctx->host_ring = (uint64_t)std::max(1, atoi(v)) << 20;
    if (const char *v = getenv("QGCM_DESC_VARIANT")) {
        const int iv = atoi(v);
        if (variant_valid(iv) && variant_desc(iv)) ctx->desc_variant = iv;
    }
    auto off = [](const char *name) {
        const char *v = getenv(name);
        return v && !strcmp(v, "0");
    };
    ctx->chain_chunk = (uint64_t)std::max(1, env_int("QGCM_CHAIN_CHUNK_MB", (int)(kPipeChunk >> 20))) << 20;
    ctx->chain_slots = std::max(1, std::min(16, env_int("QGCM_CHAIN_SLOTS", kPipeStreams)));
    ctx->chain_dev_ahead = std::max(1, env_int("QGCM_CHAIN_DEV_AHEAD", 2));
    ctx->chain_dev_backlog = env_int("QGCM_CHAIN_DEV_BACKLOG", -1);
    ctx->snappy_group = env_int("QGCM_SNAPPY_GROUP", 1) != 0;
    ctx->snappy_per_cu = std::max(0, env_int("QGCM_SNAPPY_PER_CU", 0));
    ctx->chain_pin = env_int("QGCM_CHAIN_PIN", 1) != 0;
    ctx->desc_one_on = !off("QGCM_DESC_ONE");
    ctx->host_direct = !off("QGCM_HOST_DIRECT");
    ctx->small_wl = !off("QGCM_SMALL_WORKLIST");
    uint8_t sbox[256];
    uint32_t te[512];
    build_tables(sbox, te);
    bool ok = hipMalloc(&ctx->d_rk, (size_t)max_keys * kRkWords * 4) == hipSuccess &&
              hipMalloc(&ctx->d_gh, (size_t)max_keys * kGhEntries * 16) == hipSuccess &&
              hipMalloc(&ctx->d_key_valid, max_keys) == hipSuccess &&
              // unset slots hold zeros, never stale memory, and are marked invalid
              hipMemset(ctx->d_rk, 0, (size_t)max_keys * kRkWords * 4) == hipSuccess &&
              hipMemset(ctx->d_gh, 0, (size_t)max_keys * kGhEntries * 16) == hipSuccess &&
              hipMemset(ctx->d_key_valid, 0, max_keys) == hipSuccess &&
              hipMalloc(&ctx->d_te, sizeof te) == hipSuccess && hipMalloc(&ctx->d_sbox, sizeof sbox) == hipSuccess &&
              hipMemcpy(ctx->d_te, te, sizeof te, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(ctx->d_sbox, sbox, sizeof sbox, hipMemcpyHostToDevice) == hipSuccess &&
              hipEventCreateWithFlags(&ctx->ws_done, hipEventDisableTiming) == hipSuccess;
    ctx->pw_keys = (uint32_t)std::min<int64_t>(max_keys, std::max(0, env_int("QGCM_FLAT_GHASH_KEYS", 256)));
    if (ok && ctx->pw_keys &&
        (hipMalloc(&ctx->d_pw, (size_t)ctx->pw_keys * kPwPowers * kPwEntries * 16) != hipSuccess ||
         hipMemset(ctx->d_pw, 0, (size_t)ctx->pw_keys * kPwPowers * kPwEntries * 16) != hipSuccess)) {
        hipFree(ctx->d_pw);  // no room: the per-packet path keeps the Horner + Estrin GHASH
        ctx->d_pw = nullptr;
        ctx->pw_keys = 0;
    }
    for (int k = 0; ok && k < kPipeStreams; ++k)
        ok = hipStreamCreateWithFlags(&ctx->pipe[k], hipStreamNonBlocking) == hipSuccess;
    ctx->pool_sets = (uint32_t)std::max(1, std::min((int)kPoolSets, env_int("QGCM_POOL_SETS", (int)kPoolSets)));
    if (ok && quad_pool_global()) {
        const size_t bytes = (size_t)kPoolSets * kPoolSetWords * 4;
        ok = hipMalloc(&ctx->d_pool, bytes) == hipSuccess && hipMemset(ctx->d_pool, 0, bytes) == hipSuccess &&
             hipHostMalloc(&ctx->h_pool_done, kPoolSets * 4, hipHostMallocCoherent | hipHostMallocMapped) ==
                 hipSuccess;
        if (ok) memset(ctx->h_pool_done, 0, kPoolSets * 4);
    }
    if (!ok) {
        set_err(err, errlen, "device allocation / kernel setup failed");
        qgcm_destroy(ctx);
        return nullptr;
    }
    if (ctx->chain_pin) (void)codec_cpu_list(ctx->device);  // starts the first load sample
    return ctx;
}

void qgcm_destroy(qgcm_ctx *ctx) {
    if (!ctx) return;
    resident_destroy(ctx->res.exchange(nullptr));  // before the device-wide synchronize below
    hipSetDevice(ctx->device);
    hipDeviceSynchronize();
    hipFree(ctx->d_rk);
    hipFree(ctx->d_gh);
    hipFree(ctx->d_pw);
    hipFree(ctx->d_te);
    hipFree(ctx->d_sbox);
    hipFree(ctx->d_key_valid);
    hipFree(ctx->d_qws);
    auto free_slot = [](qgcm_ctx::OneSlot &sl) {
        if (sl.h) hipHostFree(sl.h);
        if (sl.stream) hipStreamDestroy(sl.stream);
    };
    for (auto &sl : ctx->one) free_slot(sl);
    free_slot(ctx->big);
    hipFree(ctx->d_ring);
    hipFree(ctx->d_side);
    if (ctx->h_stat) hipHostFree(ctx->h_stat);
    if (ctx->h_desc) hipHostFree(ctx->h_desc);
    if (ctx->h_lens) hipHostFree(ctx->h_lens);
    for (hipStream_t x : ctx->chain_extra) hipStreamDestroy(x);
    for (hipStream_t p : ctx->pipe)
        if (p) hipStreamDestroy(p);
    if (ctx->ws_done) hipEventDestroy(ctx->ws_done);
    hipFree(ctx->d_pool);
    if (ctx->h_pool_done) hipHostFree(ctx->h_pool_done);
    for (auto *v : {&ctx->ev_in, &ctx->ev_kern, &ctx->ev_out})
        for (hipEvent_t e : *v) hipEventDestroy(e);
    delete ctx;
}

int qgcm_set_keys(qgcm_ctx *ctx, uint32_t first_idx, uint32_t count, const uint8_t *keys) {
    if (!ctx || (count && !keys)) return QGCM_E_ARG;
    if ((uint64_t)first_idx + count > ctx->max_keys) return QGCM_E_KEY;
    if (count == 0) return QGCM_OK;
    if (hipSetDevice(ctx->device) != hipSuccess) return QGCM_E_HIP;
    uint8_t *d_keys = nullptr;
    if (hipMalloc(&d_keys, (size_t)count * 32) != hipSuccess) return QGCM_E_NOMEM;
    // The key setup runs on the context's kernel stream (no stream created per call: every stream a
    // process creates moves HIP's stream -> hardware-queue assignment on, and two pipeline stages that
    // end up on one hardware queue serialize their copies).
    std::lock_guard<std::mutex> io(ctx->io_mu);
    hipStream_t s = ctx->pipe[1];
    // a running resident instance holds key tables (and keystreams computed ahead, key-valid bytes) in
    // its caches: end it BEFORE the tables change and start no new one until the new keys are published.
    // res_mu is held for the whole update, so a per-packet call that finds no service cannot create one
    // meanwhile (get_resident takes res_mu to create; an instance created mid-update would cache the
    // tables being rewritten, and nothing would end it)
    std::lock_guard<std::mutex> res_lk(ctx->res_mu);
    Resident *res = ctx->res.load(std::memory_order_acquire);
    (void)resident_pause(res);  // a failure marks the resident path broken: calls take the launch path
    int rc = QGCM_OK;
    if (hipMemcpyAsync(d_keys, keys, (size_t)count * 32, hipMemcpyHostToDevice, s) != hipSuccess ||
        launch_key_setup(d_keys, first_idx, count, ctx->d_rk, ctx->d_gh, ctx->d_sbox, s) != hipSuccess ||
        launch_pw_setup(first_idx, count, ctx->d_gh, ctx->d_pw, ctx->pw_keys, s) != hipSuccess ||
        hipMemsetAsync(ctx->d_key_valid + first_idx, 1, count, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        rc = QGCM_E_HIP;
    hipFree(d_keys);
    if (rc == QGCM_OK) {
        std::lock_guard<std::mutex> g(ctx->key_mu);
        for (uint32_t i = 0; i < count; ++i) __atomic_store_n(&ctx->key_set[first_idx + i], (uint8_t)1, __ATOMIC_RELEASE);
    }
    resident_resume(res);  // the next per-packet call starts a fresh instance
    return rc;
}

int qgcm_set_key(qgcm_ctx *ctx, uint32_t key_idx, const uint8_t key[QGCM_KEY_BYTES]) {
    return qgcm_set_keys(ctx, key_idx, 1, key);
}

int qgcm_clear_keys(qgcm_ctx *ctx, uint32_t first_idx, uint32_t count) {
    if (!ctx) return QGCM_E_ARG;
    if ((uint64_t)first_idx + count > ctx->max_keys) return QGCM_E_KEY;
    if (count == 0) return QGCM_OK;
    if (hipSetDevice(ctx->device) != hipSuccess) return QGCM_E_HIP;
    std::lock_guard<std::mutex> io(ctx->io_mu);
    hipStream_t s = ctx->pipe[1];
    // the host map first (new per-packet calls and uniform batches fail from here on), then the device
    // map the descriptor batches check; the resident instance caches key-valid bytes, so it ends first
    std::lock_guard<std::mutex> res_lk(ctx->res_mu);
    Resident *res = ctx->res.load(std::memory_order_acquire);
    (void)resident_pause(res);
    {
        std::lock_guard<std::mutex> g(ctx->key_mu);
        for (uint32_t i = 0; i < count; ++i) __atomic_store_n(&ctx->key_set[first_idx + i], (uint8_t)0, __ATOMIC_RELEASE);
    }
    int rc = QGCM_OK;
    if (hipMemsetAsync(ctx->d_key_valid + first_idx, 0, count, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        rc = QGCM_E_HIP;
    resident_resume(res);
    return rc;
}

int qgcm_seal_batch(qgcm_ctx *ctx, uint8_t *d_arena, const qgcm_desc *d_descs, uint32_t n, const uint8_t *d_nonces,
                    uint32_t aad_len, uint8_t *d_status, void *stream) {
    return run_descs(ctx, true, d_arena, d_descs, n, d_nonces, aad_len, d_status, (hipStream_t)stream);
}

int qgcm_open_batch(qgcm_ctx *ctx, uint8_t *d_arena, const qgcm_desc *d_descs, uint32_t n, uint32_t aad_len,
                    uint8_t *d_status, void *stream) {
    return run_descs(ctx, false, d_arena, d_descs, n, nullptr, aad_len, d_status, (hipStream_t)stream);
}

int qgcm_seal_uniform(qgcm_ctx *ctx, uint8_t *d_arena, uint64_t stride, uint32_t n, uint32_t len, uint32_t key_idx,
                      const uint8_t *d_nonces, uint32_t aad_len, uint8_t *d_status, void *stream) {
    return run_uniform(ctx, true, d_arena, stride, n, len, key_idx, d_nonces, aad_len, d_status, (hipStream_t)stream);
}

int qgcm_open_uniform(qgcm_ctx *ctx, uint8_t *d_arena, uint64_t stride, uint32_t n, uint32_t len, uint32_t key_idx,
                      uint32_t aad_len, uint8_t *d_status, void *stream) {
    if (n > QGCM_MAX_BATCH) return QGCM_E_ARG;
    if (len < QGCM_OVERHEAD && n) {
        // every packet fails Open; the slots stay untouched (ciphertext shorter than the tag)
        if (!ctx) return QGCM_E_ARG;
        if (d_status) {
            if (hipSetDevice(ctx->device) != hipSuccess) return QGCM_E_HIP;
            return hip_fail(hipMemsetAsync(d_status, 0, n, (hipStream_t)stream));
        }
        return QGCM_OK;
    }
    return run_uniform(ctx, false, d_arena, stride, n, len, key_idx, nullptr, aad_len, d_status, (hipStream_t)stream);
}

long qgcm_seal_one(qgcm_ctx *ctx, uint32_t key_idx, uint8_t *data, long length, const uint8_t *aad, uint32_t aad_len,
                   const uint8_t *nonce) {
    if (!ctx || !data || length < 0 || length >= (long)QGCM_MAX_PAYLOAD || aad_len > 4 || (aad_len && !aad)) return -1;
    if (!key_ok(ctx, key_idx)) return -1;
    if (Resident *r = get_resident(ctx)) {  // no launch per call (and no HIP call); draws the nonce if NULL
        const long rc = resident_call(r, true, key_idx, data, length, aad, aad_len, nonce);
        if (rc != kResNotServed) {
            ctx->count(QGCM_KERNEL_RESIDENT);
            return rc;
        }
    }
    uint8_t nb[12];
    if (nonce) {
        memcpy(nb, nonce, 12);
    } else if (!random_nonce(nb)) {  // crypto/aes.go:44 rand.Read(nonce)
        return -1;
    }
    if (hipSetDevice(ctx->device) != hipSuccess) return -1;
    const uint64_t stride = ((uint64_t)length + 4 + QGCM_OVERHEAD + 15) & ~15ull;
    std::unique_lock<std::mutex> lk;
    qgcm_ctx::OneSlot *sl = acquire_one(ctx, stride + 16, lk);
    if (!sl) return -1;
    const BigRelease rel{ctx, sl};
    uint8_t *h = sl->h;
    memset(h, 0, stride);
    if (aad_len) memcpy(h, aad, aad_len);
    memcpy(h + 4, data, (size_t)length);
    memcpy(h + 4 + length + 16, nb, 12);
    // Zero-copy: the kernel seals the pinned staging slot in place over PCIe (one packet: no DMA
    // setups; the copy-in / copy-out form took ~3x longer per call)
    hipStream_t s = sl->stream;
    h[stride] = 0;
    if (run_one(ctx, true, h, stride, (uint32_t)length, key_idx, aad_len, h + stride, s) != QGCM_OK) return -1;
    if (h[stride] != 1) return -1;
    memcpy(data, h + 4, (size_t)length + QGCM_OVERHEAD);
    return length + QGCM_OVERHEAD;
}

long qgcm_open_one(qgcm_ctx *ctx, uint32_t key_idx, uint8_t *data, long len, const uint8_t *aad, uint32_t aad_len) {
    if (!ctx || (!data && len) || len < 0 || len - QGCM_OVERHEAD >= (long)QGCM_MAX_PAYLOAD || aad_len > 4 || (aad_len && !aad)) return -1;
    if (len < QGCM_OVERHEAD) return -1;  // crypto/aes.go:58-60: errOpen (the reference panics below 12)
    if (!key_ok(ctx, key_idx)) return -1;
    if (Resident *r = get_resident(ctx)) {  // no launch per call (and no HIP call)
        const long rc = resident_call(r, false, key_idx, data, len, aad, aad_len, nullptr);
        if (rc != kResNotServed) {
            ctx->count(QGCM_KERNEL_RESIDENT);
            return rc;
        }
    }
    if (hipSetDevice(ctx->device) != hipSuccess) return -1;
    const uint64_t stride = ((uint64_t)len + 4 + 15) & ~15ull;
    std::unique_lock<std::mutex> lk;
    qgcm_ctx::OneSlot *sl = acquire_one(ctx, stride + 16, lk);
    if (!sl) return -1;
    const BigRelease rel{ctx, sl};
    uint8_t *h = sl->h;
    memset(h, 0, stride);
    if (aad_len) memcpy(h, aad, aad_len);
    memcpy(h + 4, data, (size_t)len);
    hipStream_t s = sl->stream;  // zero-copy on the pinned staging slot, as qgcm_seal_one
    h[stride] = 0;
    if (run_one(ctx, false, h, stride, (uint32_t)len, key_idx, aad_len, h + stride, s) != QGCM_OK) return -1;
    memcpy(data, h + 4, (size_t)len - QGCM_OVERHEAD);  // plaintext, or zeros on auth failure
    return h[stride] == 1 ? len - QGCM_OVERHEAD : -1;
}

// Host batches, pipelined: the batch is cut into ~64 MiB chunks, each with its own device slot while
// the batch fits the staging budget (4 GiB of the 288 GB HBM; larger batches rotate through the
// slots).  One stream per stage -- copy-in, kernel, copy-out -- ordered by per-slot events: chunk c's
// kernel waits for its copy-in, its copy-out for its kernel, and (only when slots rotate) the copy-in
// of chunk c + nslots for chunk c's copy-out.  Each PCIe direction thus sees an uninterrupted queue
// of copies (a stream per chunk doing H2D -> kernel -> D2H in order made the next copy-in of that
// stream wait behind its copy-out: 30.5 GiB/s; per-stage streams with 4 rotating 32 MiB slots: 35.6).
// Pinned caller memory (qgcm_host_alloc, hipHostMalloc/Register) is DMA'd in place; pageable memory
// still works but HIP stages it, which serializes the copies.
static int run_host(qgcm_ctx *ctx, bool seal, uint8_t *h_arena, uint64_t stride, uint32_t n, uint32_t len,
                    uint32_t key_idx, const uint8_t *h_nonces, uint32_t aad_len, uint8_t *h_status) {
    if (!ctx || (n && !h_arena) || aad_len > 4 || (stride & 3)) return QGCM_E_ARG;
    if (n && stride < (uint64_t)len + 4 + (seal ? QGCM_OVERHEAD : 0)) return QGCM_E_ARG;
    if ((seal || len >= QGCM_OVERHEAD) && len - (seal ? 0u : (uint32_t)QGCM_OVERHEAD) >= QGCM_MAX_PAYLOAD)
        return QGCM_E_ARG;
    if (!key_ok(ctx, key_idx)) return QGCM_E_KEY;
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(ctx->io_mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return QGCM_E_HIP;
    if (n > ctx->hstat_cap) {
        if (ctx->h_stat) hipHostFree(ctx->h_stat);
        ctx->h_stat = nullptr;
        ctx->hstat_cap = 0;
        if (hipHostMalloc(&ctx->h_stat, n, hipHostMallocDefault) != hipSuccess) return QGCM_E_NOMEM;
        ctx->hstat_cap = n;
    }
    {
        // Direct: a worker-sized batch in a pinned arena with 16-B-aligned slots that hold the rounded
        // staging area is sealed in place over PCIe, one workgroup per packet (gcm_one_kernel on the
        // arena's device view), nonces and statuses in pinned memory too: one launch, no copies
        // (QGCM_HOST_DIRECT=0 at qgcm_create: off)
        const uint64_t area = (4ull + len + (seal ? QGCM_OVERHEAD : 0) + 15) & ~15ull;
        uint64_t va = 0, vn = 0, vst = 0;
        if (ctx->host_direct && n <= direct_max(ctx) && (uint64_t)n * stride <= kDirectMaxBytes &&
            !ctx->variant_forced && !(stride & 15) &&
            area <= stride && area <= kOneCap - 16 && (seal || len >= QGCM_OVERHEAD) &&
            (va = pinned_view(h_arena, (uint64_t)n * stride)) && !(va & 15) &&
            (!(seal && h_nonces) || (vn = pinned_view(h_nonces, 12ull * n))) && !(vn & 3) &&
            (vst = pinned_view(ctx->h_stat, n))) {
            Batch b = base_batch(ctx);
            b.arena = reinterpret_cast<uint8_t *>(va);
            b.nonces = reinterpret_cast<const uint8_t *>(vn);
            b.status = reinterpret_cast<uint8_t *>(vst);
            b.stride = stride;
            b.uniform_len = len;
            b.uniform_key = key_idx;
            b.n = n;
            b.n_items = (uint32_t)(((uint64_t)n + 63) & ~63ull);
            b.aad_len = aad_len;
            hipStream_t s = ctx->pipe[0];
            if (launch_one(seal, b, s) != hipSuccess) return QGCM_E_HIP;
            ctx->count(QGCM_KERNEL_ONE);
            if (hipStreamSynchronize(s) != hipSuccess) return QGCM_E_HIP;
            int bad = 0;
            for (uint32_t i = 0; i < n; ++i) bad += ctx->h_stat[i] != 1;
            if (h_status) memcpy(h_status, ctx->h_stat, n);
            return bad;
        }
    }
    uint64_t cpk = (ctx->host_chunk / stride) & ~63ull;  // packets per chunk, whole 64-packet tiles
    if (cpk < 64) cpk = 64;
    if (cpk > n) cpk = n;
    const uint64_t nchunks = (n + cpk - 1) / cpk;
    const bool non = seal && h_nonces;
    const uint64_t slot = (cpk * stride + 255) & ~255ull;
    const uint64_t fit = std::max<uint64_t>(2, ctx->host_ring / slot);
    const int nslots = (int)std::min<uint64_t>(nchunks, fit);
    while (ctx->ev_in.size() < (size_t)nslots) {
        hipEvent_t e[3] = {};
        for (hipEvent_t &x : e)
            if (hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess) {
                for (hipEvent_t y : e)
                    if (y) hipEventDestroy(y);
                return QGCM_E_HIP;
            }
        ctx->ev_in.push_back(e[0]);
        ctx->ev_kern.push_back(e[1]);
        ctx->ev_out.push_back(e[2]);
    }
    if (slot * nslots > ctx->ring_cap) {
        if (ctx->d_ring) hipFree(ctx->d_ring);
        ctx->d_ring = nullptr;
        ctx->ring_cap = 0;
        if (hipMalloc(&ctx->d_ring, slot * nslots) != hipSuccess) return QGCM_E_NOMEM;
        ctx->ring_cap = slot * nslots;
    }
    // nonces and status of the whole batch travel in one copy each (per-chunk side copies cost a
    // DMA setup each: 2 per chunk)
    const uint64_t non_bytes = non ? (12ull * n + 255) & ~255ull : 0;  // nonces first: 4-B aligned words
    const uint64_t side = non_bytes + n;
    if (side > ctx->side_cap) {
        if (ctx->d_side) hipFree(ctx->d_side);
        ctx->d_side = nullptr;
        ctx->side_cap = 0;
        if (hipMalloc(&ctx->d_side, side) != hipSuccess) return QGCM_E_NOMEM;
        ctx->side_cap = side;
    }
    uint8_t *d_non_all = ctx->d_side, *d_stat_all = ctx->d_side + non_bytes;
    // one copy-in stream: alternating two (two SDMA queues) measured 27.3 vs 38.0 GiB/s.  A batch of one
    // chunk (a worker's recvmmsg batch) has nothing to overlap: copy-in, kernel and copy-out go on one
    // stream, with no cross-stream events and one synchronize
    const bool one = nchunks == 1;
    hipStream_t s_in = ctx->pipe[0], s_k = one ? s_in : ctx->pipe[1], s_out = one ? s_in : ctx->pipe[2];
    auto link = [&](hipEvent_t e, hipStream_t from, hipStream_t to) {  // `to` waits for `from`'s work so far
        return from == to || (hipEventRecord(e, from) == hipSuccess && hipStreamWaitEvent(to, e, 0) == hipSuccess);
    };
    int rc = QGCM_OK;
    if (non && hipMemcpyAsync(d_non_all, h_nonces, 12ull * n, hipMemcpyHostToDevice, s_in) != hipSuccess)
        rc = QGCM_E_HIP;
    for (uint64_t c = 0; c < nchunks && rc == QGCM_OK; ++c) {
        const int k = (int)(c % nslots);
        uint8_t *d = ctx->d_ring + k * slot;
        const uint64_t c0 = c * cpk, cn = (n - c0) < cpk ? (n - c0) : cpk;
        uint8_t *h = h_arena + c0 * stride;
        // slot k is free once the copy-out of chunk c - nslots has landed
        if ((c >= (uint64_t)nslots && hipStreamWaitEvent(s_in, ctx->ev_out[k], 0) != hipSuccess) ||
            hipMemcpyAsync(d, h, cn * stride, hipMemcpyHostToDevice, s_in) != hipSuccess ||
            !link(ctx->ev_in[k], s_in, s_k)) {
            rc = QGCM_E_HIP;
            break;
        }
        if (!seal && len < QGCM_OVERHEAD)
            rc = hip_fail(hipMemsetAsync(d_stat_all + c0, 0, cn, s_k));
        else
            rc = run_uniform(ctx, seal, d, stride, (uint32_t)cn, len, key_idx, non ? d_non_all + 12 * c0 : nullptr,
                             aad_len, d_stat_all + c0, s_k);
        if (rc == QGCM_OK &&
            (!link(ctx->ev_kern[k], s_k, s_out) ||
             hipMemcpyAsync(h, d, cn * stride, hipMemcpyDeviceToHost, s_out) != hipSuccess ||
             (!one && hipEventRecord(ctx->ev_out[k], s_out) != hipSuccess)))
            rc = QGCM_E_HIP;
    }
    if (rc == QGCM_OK && ((!one && hipStreamWaitEvent(s_out, ctx->ev_kern[(nchunks - 1) % nslots], 0) != hipSuccess) ||
                          hipMemcpyAsync(ctx->h_stat, d_stat_all, n, hipMemcpyDeviceToHost, s_out) != hipSuccess))
        rc = QGCM_E_HIP;
    for (hipStream_t p : {s_in, s_k, s_out}) {
        if (one && p != s_in) continue;
        if (hipStreamSynchronize(p) != hipSuccess) rc = QGCM_E_HIP;
    }
    if (rc != QGCM_OK) return rc;
    int bad = 0;
    for (uint32_t i = 0; i < n; ++i) bad += ctx->h_stat[i] != 1;
    if (h_status) memcpy(h_status, ctx->h_stat, n);
    return bad;
}

// Device snappy batch (snappy_kernels.hip), defined below.
static int run_snappy(qgcm_ctx *ctx, bool compress, uint8_t *d_arena, uint64_t stride, uint32_t n, uint32_t *d_lens,
                      uint32_t max_in, uint32_t limit, uint8_t *d_status, const uint8_t *d_status_in,
                      qgcm_desc *d_descs, uint32_t key_idx, uint32_t sub, hipStream_t s);

// Compression + Encryption chain over host batches (BASELINE config 5; plugin order main.go:50-51:
// outgoing compression.go then encryption.go, incoming the reverse).  Chunks of ~32 MiB of slots go
// through three streams (a stream per chunk: H2D, kernels, D2H in order, three rotating slots).
// Each chunk's codec runs either on the host -- a pool of `threads` workers for the whole call,
// 256-packet items -- or on the device (snappy_kernels.hip, the same bytes):
//  * seal: host workers compress items ahead from the front of the batch; when a stream slot frees
//    up and fewer than QGCM_CHAIN_DEV_AHEAD (2) compressed host chunks are waiting, the device takes
//    the LAST untouched chunk (whole chunks from the back, claimed against the workers' front by one
//    atomic word), ships it uncompressed and compresses it in place before the seal.  The host codec
//    and PCIe thus set the split themselves: the device takes what the host cores cannot keep up with.
//  * open: chunk by chunk in order; a chunk is decoded on the device when the host workers' backlog
//    (released, not yet decoded items) exceeds QGCM_CHAIN_DEV_BACKLOG items (default two chunks),
//    else after its D2H on the host.
// A device chunk crosses PCIe at full width on the uncompressed side (the host cannot size the rows
// before the kernel ran); a host chunk's rows are as wide as its longest record.  QGCM_CHAIN_DEVICE:
// 0 = host codec only, 1 = the split above (default), 2 = device codec only (A/B knobs).
namespace {

struct CodecPool {
    static constexpr uint32_t kItem = 256;  // packets per work item
    ChunkClaims claim;                      // seal: host items from the front, device chunks from the back
    std::atomic<uint64_t> next{0};          // open: next item to claim
    std::atomic<uint64_t> limit{0};         // open: items released to the workers
    std::atomic<bool> stop{false};
    std::unique_ptr<std::atomic<uint32_t>[]> done;  // finished items per chunk
    std::unique_ptr<std::atomic<uint8_t>[]> on_dev;  // open: chunk decoded on the device (items skipped)
    std::vector<std::thread> workers;

    void wait_chunk(uint64_t c, uint32_t items) const {
        while (done[c].load(std::memory_order_acquire) < items) std::this_thread::yield();
    }
    void join() {
        stop = true;
        for (auto &t : workers) t.join();
        workers.clear();
    }
    ~CodecPool() {
        if (!workers.empty()) join();
    }
};

}  // namespace

static int run_host_chain(qgcm_ctx *ctx, bool seal, uint8_t *h_arena, uint64_t stride, uint32_t n, uint32_t *lens,
                          uint32_t key_idx, const uint8_t *h_nonces, uint32_t aad_len, int threads,
                          uint8_t *h_status) {
    if (!ctx || (n && (!h_arena || !lens)) || aad_len > 4 || (stride & 3) || stride < 4 + QGCM_OVERHEAD)
        return QGCM_E_ARG;
    if (!key_ok(ctx, key_idx)) return QGCM_E_KEY;
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(ctx->io_mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return QGCM_E_HIP;
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    const uint64_t chunk_bytes = ctx->chain_chunk;  // QGCM_CHAIN_CHUNK_MB at qgcm_create
    const int dev_mode = ctx->chain_codec.load();
    uint64_t cpk = (chunk_bytes / stride) & ~255ull;  // whole codec items per chunk
    if (cpk < 256) cpk = 256;
    if (cpk > n) cpk = n;
    const uint64_t nchunks = (n + cpk - 1) / cpk;
    const bool non = seal && h_nonces;
    const uint64_t off_non = al(cpk * stride), off_st = off_non + (non ? al(12 * cpk) : 0);
    const uint64_t off_desc = off_st + al(cpk), off_lens = off_desc + al(16 * cpk), slot = off_lens + al(4 * cpk);
    // chunks in flight, one stream and staging slot each (QGCM_CHAIN_SLOTS at qgcm_create; default 3)
    const int want_slots = ctx->chain_slots;
    const int nslots = nchunks < (uint64_t)want_slots ? (int)nchunks : want_slots;
    while ((int)ctx->chain_extra.size() + kPipeStreams < nslots) {
        hipStream_t x = nullptr;
        if (hipStreamCreateWithFlags(&x, hipStreamNonBlocking) != hipSuccess) return QGCM_E_HIP;
        ctx->chain_extra.push_back(x);
    }
    auto stream_of = [&](int k) { return k < kPipeStreams ? ctx->pipe[k] : ctx->chain_extra[k - kPipeStreams]; };
    // every packet a slot can hold fits the device codec, so a chunk's result does not depend on where
    // its codec ran
    const bool dev_ok = dev_mode > 0 && stride - 4 <= kSnapDevMax;
    if (slot * nslots > ctx->ring_cap) {
        if (ctx->d_ring) hipFree(ctx->d_ring);
        ctx->d_ring = nullptr;
        ctx->ring_cap = 0;
        if (hipMalloc(&ctx->d_ring, slot * nslots) != hipSuccess) return QGCM_E_NOMEM;
        ctx->ring_cap = slot * nslots;
    }
    if (n > ctx->hstat_cap) {
        if (ctx->h_stat) hipHostFree(ctx->h_stat);
        ctx->h_stat = nullptr;
        ctx->hstat_cap = 0;
        if (hipHostMalloc(&ctx->h_stat, n, hipHostMallocDefault) != hipSuccess) return QGCM_E_NOMEM;
        ctx->hstat_cap = n;
    }
    if (cpk * nslots > ctx->hdesc_cap) {
        for (void *p : {(void *)ctx->h_desc, (void *)ctx->h_lens})
            if (p) hipHostFree(p);
        ctx->h_desc = nullptr;
        ctx->h_lens = nullptr;
        ctx->hdesc_cap = 0;
        if (hipHostMalloc(reinterpret_cast<void **>(&ctx->h_desc), cpk * nslots * sizeof(qgcm_desc),
                          hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void **>(&ctx->h_lens), cpk * nslots * sizeof(uint32_t),
                          hipHostMallocDefault) != hipSuccess)
            return QGCM_E_NOMEM;
        ctx->hdesc_cap = cpk * nslots;
    }
    std::vector<uint8_t> codec(n, 1);  // host codec status per packet (device status: ctx->h_stat)
    const uint32_t max_plain = (uint32_t)(stride - 4 - QGCM_OVERHEAD);
    const uint32_t per_chunk = (uint32_t)((cpk + CodecPool::kItem - 1) / CodecPool::kItem);
    const uint64_t total_items = (n + CodecPool::kItem - 1) / CodecPool::kItem;
    auto items_in = [&](uint64_t c) {
        const uint64_t c0 = c * cpk, cn = (n - c0) < cpk ? (n - c0) : cpk;
        return (uint32_t)((cn + CodecPool::kItem - 1) / CodecPool::kItem);
    };
    CodecPool pool;
    pool.done.reset(new std::atomic<uint32_t>[nchunks]);
    pool.on_dev.reset(new std::atomic<uint8_t>[nchunks]);
    for (uint64_t c = 0; c < nchunks; ++c) {
        pool.done[c] = 0;
        pool.on_dev[c] = 0;
    }
    pool.claim.reset(nchunks, total_items, per_chunk);
    auto process = [&](uint64_t it, std::vector<uint8_t> &tmp) {
        const uint64_t i0 = it * CodecPool::kItem, i1 = std::min<uint64_t>(n, i0 + CodecPool::kItem);
        for (uint64_t i = i0; i < i1; ++i) {
            uint8_t *pkt = h_arena + i * stride + 4;
            if (seal) {
                // compression.go:44-51; a packet whose compressed form leaves no room for the
                // tag and nonce fails, untouched
                const long c = lens[i] <= max_plain ? qgcm_snappy_compress(pkt, lens[i], tmp.data(), tmp.size()) : -1;
                if (c < 0 || (uint64_t)c > max_plain) {
                    codec[i] = 0;
                } else {
                    memcpy(pkt, tmp.data(), (size_t)c);
                    lens[i] = (uint32_t)c;
                }
            } else if (ctx->h_stat[i] == 1) {  // compression.go:35-43, on authentic packets only
                const uint32_t sl = lens[i] - QGCM_OVERHEAD;
                const long u = qgcm_snappy_uncompress(pkt, sl, tmp.data(), stride - 4);
                if (u <= 0) {  // an empty result is Go's nil slice: compression.go:37-39 drops it
                    codec[i] = 0;
                    lens[i] = sl;
                } else {
                    memcpy(pkt, tmp.data(), (size_t)u);
                    lens[i] = (uint32_t)u;
                }
            }
        }
    };
    auto work = [&] {
        std::vector<uint8_t> tmp(std::max<uint64_t>(stride, qgcm_snappy_max_compressed_length(stride)));
        for (;;) {
            uint64_t it;
            if (seal) {  // claim the front item unless the device owns its chunk
                const int64_t c = pool.stop ? -1 : pool.claim.claim_item();
                if (c < 0) return;
                it = (uint64_t)c;
            } else {
                it = pool.next.load();
                for (;;) {
                    if (it >= total_items || pool.stop) return;
                    if (it < pool.limit.load(std::memory_order_acquire)) {
                        if (pool.next.compare_exchange_weak(it, it + 1)) break;
                    } else {
                        std::this_thread::yield();
                        it = pool.next.load();
                    }
                }
            }
            if (seal || !pool.on_dev[it / per_chunk].load(std::memory_order_acquire)) process(it, tmp);
            pool.done[it / per_chunk].fetch_add(1, std::memory_order_release);
        }
    };
    const int nt = (seal && dev_ok && dev_mode == 2) ? 0 : std::max(1, std::min(threads, 256));
    std::vector<int> cores;  // one CPU per worker, or empty: left to the scheduler
    if (ctx->chain_pin && nt > 0) {
        std::lock_guard<std::mutex> g(ctx->codec_cpus_mu);
        const auto f = codec_cpu_list(ctx->device);
        if (f.valid() && (ctx->codec_cpus.empty() || f.wait_for(std::chrono::seconds(0)) == std::future_status::ready))
            ctx->codec_cpus = f.get();
        if ((size_t)nt <= ctx->codec_cpus.size()) cores = ctx->codec_cpus;
    }
    for (int t = 0; t < nt; ++t)
        pool.workers.emplace_back([&work, cpu = cores.empty() ? -1 : cores[(size_t)t]] {
            if (cpu >= 0) qgcm::pin_to_cpu(cpu);
            work();
        });
    // seal: the device takes a chunk when fewer than ahead_min compressed host chunks are waiting as a
    // stream slot frees up (the host codec is about to stall the pipeline); open: when more than
    // backlog_max released items wait for the host decoder
    const uint64_t ahead_min = (uint64_t)ctx->chain_dev_ahead;
    const uint64_t backlog_max = ctx->chain_dev_backlog >= 0 ? (uint64_t)ctx->chain_dev_backlog : 2ull * per_chunk;
    std::vector<int64_t> slot_chunk(nslots, -1);
    // a slot's previous chunk has landed: device chunks' lengths back to the caller; open: release
    // its items to the host workers (device chunks' items are skipped)
    auto finalize = [&](int k) {
        const int64_t c = slot_chunk[k];
        if (c < 0) return;
        const uint64_t c0 = c * cpk, cn = (n - c0) < cpk ? (n - c0) : cpk;
        if (pool.on_dev[c]) memcpy(lens + c0, ctx->h_lens + (uint64_t)k * cpk, 4 * cn);
        slot_chunk[k] = -1;
    };
    int rc = QGCM_OK;
    uint64_t host_next = 0, released = 0;
    for (uint64_t e = 0; rc == QGCM_OK; ++e) {
        const int k = (int)(e % nslots);
        hipStream_t s = stream_of(k);
        if (slot_chunk[k] >= 0) {
            if (hipStreamSynchronize(s) != hipSuccess) {
                rc = QGCM_E_HIP;
                break;
            }
            const int64_t prev = slot_chunk[k];
            finalize(k);
            if (!seal) {  // chunks are enqueued in order on open: release up to the one that landed
                released = std::max<uint64_t>(released, (uint64_t)(prev + 1) * per_chunk);
                pool.limit.store(std::min<uint64_t>(released, total_items), std::memory_order_release);
            }
        }
        int64_t c = -1;
        bool dev = false;
        if (seal) {
            for (;;) {
                const uint64_t dlo = pool.claim.device_from();
                if (host_next >= dlo) break;
                uint64_t ready = 0;  // compressed host chunks waiting, up to ahead_min
                while (ready < ahead_min && host_next + ready < dlo &&
                       pool.done[host_next + ready].load(std::memory_order_acquire) == items_in(host_next + ready))
                    ++ready;
                if (dev_ok && ready < ahead_min && (c = pool.claim.claim_chunk()) >= 0) {
                    dev = true;
                    break;
                }
                if (ready) {
                    c = (int64_t)host_next++;
                    break;
                }
                std::this_thread::yield();
            }
        } else if (e < nchunks) {
            c = (int64_t)e;
            uint64_t backlog = 0;  // released host items not decoded yet
            for (uint64_t q = 0; q < nchunks && q * per_chunk < released; ++q)
                if (!pool.on_dev[q]) backlog += items_in(q) - pool.done[q].load(std::memory_order_acquire);
            dev = dev_ok && (dev_mode == 2 || backlog > backlog_max);
        }
        if (c < 0) break;
        pool.on_dev[c].store(dev ? 1 : 0, std::memory_order_release);
        slot_chunk[k] = c;
        uint8_t *d = ctx->d_ring + k * slot, *d_non = d + off_non, *d_st = d + off_st;
        qgcm_desc *d_desc = reinterpret_cast<qgcm_desc *>(d + off_desc);
        uint32_t *d_lens = reinterpret_cast<uint32_t *>(d + off_lens);
        qgcm_desc *hd = ctx->h_desc + k * cpk;
        uint32_t *hl = ctx->h_lens + (uint64_t)k * cpk;
        const uint64_t c0 = c * cpk, cn = (n - c0) < cpk ? (n - c0) : cpk;
        uint8_t *h = h_arena + c0 * stride;
        // Only the bytes a slot uses cross PCIe: a host chunk's rows are copied 2-D, each as wide as
        // the chunk's longest record (AAD, packet, tag||nonce) instead of the whole slot stride --
        // compressed packets fill ~60% of a 1472-B Payload.Raw.  A device chunk's output lengths are
        // not known when its copies are queued, so its slots travel whole both ways (the bytes past a
        // packet come back as they went: untouched, as compression.go's copy leaves them).
        uint64_t width = 4;
        uint32_t max_in = 0;
        for (uint64_t i = 0; i < cn; ++i) {
            const uint32_t L = lens[c0 + i];
            if (seal && dev) {
                max_in = std::max(max_in, L);
                continue;
            }
            const bool ok = !seal || codec[c0 + i];
            hd[i] = qgcm_desc{i * stride, ok ? L : QGCM_MAX_PAYLOAD, key_idx};
            if (ok) width = std::max<uint64_t>(width, 4ull + L + (seal ? QGCM_OVERHEAD : 0));
            if (!seal) max_in = std::max(max_in, L >= QGCM_OVERHEAD ? L - (uint32_t)QGCM_OVERHEAD : 0u);
        }
        if (dev) width = stride;
        max_in = std::min<uint32_t>(max_in, max_plain);  // seal: longer packets fail, as on the host
        auto copy = [&](void *dst, const void *src, uint64_t w, hipMemcpyKind kind) {
            w = std::min<uint64_t>(stride, (w + 3) & ~3ull);
            return w * 10 >= stride * 9 ? hipMemcpyAsync(dst, src, cn * stride, kind, s)
                                        : hipMemcpy2DAsync(dst, stride, src, stride, w, cn, kind, s);
        };
        if (dev) {
            memcpy(hl, lens + c0, 4 * cn);
            if (hipMemcpyAsync(d_lens, hl, 4 * cn, hipMemcpyHostToDevice, s) != hipSuccess) rc = QGCM_E_HIP;
        }
        if (rc == QGCM_OK &&
            (copy(d, h, width, hipMemcpyHostToDevice) != hipSuccess ||
             (!(seal && dev) &&
              hipMemcpyAsync(d_desc, hd, cn * sizeof(qgcm_desc), hipMemcpyHostToDevice, s) != hipSuccess) ||
             (non && hipMemcpyAsync(d_non, h_nonces + 12 * c0, 12 * cn, hipMemcpyHostToDevice, s) != hipSuccess)))
            rc = QGCM_E_HIP;
        if (rc == QGCM_OK && seal && dev)  // compress in place; failures get the sentinel length (seal skips them)
            rc = run_snappy(ctx, true, d, stride, (uint32_t)cn, d_lens, max_in, max_plain, nullptr, nullptr, d_desc,
                            key_idx, 0, s);
        if (rc == QGCM_OK) rc = run_descs(ctx, seal, d, d_desc, (uint32_t)cn, non ? d_non : nullptr, aad_len, d_st, s);
        if (rc == QGCM_OK && !seal && dev)  // authentic packets only; a failed decode clears the status
            rc = run_snappy(ctx, false, d, stride, (uint32_t)cn, d_lens, max_in, (uint32_t)(stride - 4), d_st, d_st,
                            nullptr, 0, QGCM_OVERHEAD, s);
        if (rc == QGCM_OK && (copy(h, d, width, hipMemcpyDeviceToHost) != hipSuccess ||
                              hipMemcpyAsync(ctx->h_stat + c0, d_st, cn, hipMemcpyDeviceToHost, s) != hipSuccess ||
                              (dev && hipMemcpyAsync(hl, d_lens, 4 * cn, hipMemcpyDeviceToHost, s) != hipSuccess)))
            rc = QGCM_E_HIP;
    }
    for (int k = 0; k < nslots; ++k)
        if (hipStreamSynchronize(stream_of(k)) != hipSuccess) rc = QGCM_E_HIP;
    if (rc != QGCM_OK) {
        pool.join();
        return rc;
    }
    for (int k = 0; k < nslots; ++k) finalize(k);
    if (!seal) pool.limit.store(total_items, std::memory_order_release);
    for (uint64_t c = 0; c < nchunks; ++c)
        if (!(seal && pool.on_dev[c])) pool.wait_chunk(c, items_in(c));
    pool.join();
    int bad = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const bool ok = ctx->h_stat[i] == 1 && codec[i];
        if (seal && ok) lens[i] += QGCM_OVERHEAD;
        bad += !ok;
        if (h_status) h_status[i] = ok ? 1 : 0;
    }
    return bad;
}

// Device snappy batch (snappy_kernels.hip): LDS layout per wave, workgroup size and grid from the
// longest packet the call admits.
static int run_snappy(qgcm_ctx *ctx, bool compress, uint8_t *d_arena, uint64_t stride, uint32_t n, uint32_t *d_lens,
                      uint32_t max_in, uint32_t limit, uint8_t *d_status, const uint8_t *d_status_in,
                      qgcm_desc *d_descs, uint32_t key_idx, uint32_t sub, hipStream_t s) {
    // compress: inputs up to kSnapDevMax; uncompress: outputs up to kSnapDevMax, inputs up to the longest
    // stream such an output can have
    const uint64_t in_max = compress ? kSnapDevMax : qgcm_snappy_max_compressed_length(kSnapDevMax);
    if (!ctx || (n && (!d_arena || !d_lens)) || (stride & 3) || stride < 4 || max_in > in_max ||
        max_in > stride - 4 || limit > stride - 4 || (!compress && limit > kSnapDevMax))
        return QGCM_E_ARG;
    if (n == 0) return QGCM_OK;
    auto a16 = [](uint32_t x) { return (x + 15u) & ~15u; };
    SnapArgs a{};
    a.arena = d_arena;
    a.stride = stride;
    a.n = n;
    a.lens = d_lens;
    a.status = d_status;
    a.status_in = d_status_in;
    a.descs = d_descs;
    a.key_idx = key_idx;
    a.max_in = max_in;
    a.limit = limit;
    a.sub = sub;
    uint32_t tab = 0;
    if (compress) {
        uint32_t bits = 8;
        while (bits < 14 && (1u << bits) < max_in) ++bits;
        tab = 2u << bits;
    }
    a.off_in = tab;
    a.off_out = a.off_in + a16(max_in + 24);  // + the 16-B chunks' overhang and stage_in's slack dwords
    a.off_sink = a.off_out + a16((compress ? (uint32_t)qgcm_snappy_max_compressed_length(max_in) : limit) + 8);
    // the codec (QGCM_SNAPPY_GROUP at qgcm_create, A/B knob): 1 (default) = four packets per wave --
    // the encoder's output straight into the slot (the region: table + the input staged up to max(len,
    // limit) bytes, the restore copy), the decoder's region [input | output | lane scratch]; 0 = one
    // wave per packet.  Packets past ~5 KiB (encoder) or whose regions pass 16 KiB (decoder) need more
    // LDS than four regions per wave can have, and limit 0 fails every packet: one wave per packet.
    bool group = compress && limit > 0 && ctx->snappy_group;
    bool gdec = !compress && ctx->snappy_group;  // the four-packets-per-wave decoder
    uint32_t gregion = 0;
    if (gdec) {  // [staged input | output | 64 B of lane scratch] per packet, four per wave
        a.off_in = 0;
        a.off_out = a16(max_in + 24);
        a.off_sink = a.off_out + a16(limit + 8);
        gregion = a.off_sink + 64;
        if (kSnapGroup * gregion > 64u * 1024u) {  // back to the wave decoder's layout
            gdec = false;
            a.off_out = a.off_in + a16(max_in + 24);
            a.off_sink = a.off_out + a16(limit + 8);
        }
    }
    if (group) {
        a.off_out = a.off_in + a16(std::max(max_in, limit) + 24);
        a.off_sink = a.off_out;
        if (kSnapGroup * a.off_sink > 160u * 1024u) {  // back to the wave encoder's layout
            group = false;
            a.off_out = a.off_in + a16(max_in + 24);
            a.off_sink = a.off_out + a16((uint32_t)qgcm_snappy_max_compressed_length(max_in) + 8);
        }
    }
    a.wave_bytes = group ? kSnapGroup * a.off_sink : gdec ? kSnapGroup * gregion : a.off_sink + 256;
    const uint32_t per_wave = group || gdec ? kSnapGroup : 1;
    int waves = group ? 1 : 4;
    while (waves > 1 && (size_t)waves * a.wave_bytes > 64u * 1024u) --waves;
    int per_cu = (int)((160u * 1024u) / ((uint32_t)waves * a.wave_bytes));
    per_cu = std::max(1, std::min(per_cu, 8));
    if (ctx->snappy_per_cu) per_cu = std::min(per_cu, std::max(1, ctx->snappy_per_cu / waves));
    const uint64_t need = (n + (uint64_t)waves * per_wave - 1) / ((uint64_t)waves * per_wave);
    const int grid = (int)std::min<uint64_t>(need, (uint64_t)ctx->num_cus * per_cu);
    if (hipSetDevice(ctx->device) != hipSuccess) return QGCM_E_HIP;
    ctx->count(compress ? QGCM_KERNEL_SNAPPY_ENC : QGCM_KERNEL_SNAPPY_DEC);
    return hip_fail(launch_snappy(compress, a, waves, grid, s, group ? 1 : gdec ? 2 : 0));
}

int qgcm_snappy_compress_batch(qgcm_ctx *ctx, uint8_t *d_arena, uint64_t stride, uint32_t n, uint32_t *d_lens,
                               uint32_t max_len, uint32_t limit, uint8_t *d_status, qgcm_desc *d_descs_out,
                               uint32_t key_idx, void *stream) {
    return run_snappy(ctx, true, d_arena, stride, n, d_lens, max_len, limit, d_status, nullptr, d_descs_out, key_idx,
                      0, (hipStream_t)stream);
}

int qgcm_snappy_uncompress_batch(qgcm_ctx *ctx, uint8_t *d_arena, uint64_t stride, uint32_t n, uint32_t *d_lens,
                                 uint32_t max_len, uint32_t cap, uint8_t *d_status, void *stream) {
    return run_snappy(ctx, false, d_arena, stride, n, d_lens, max_len, cap, d_status, nullptr, nullptr, 0, 0,
                      (hipStream_t)stream);
}

int qgcm_chain_codec(qgcm_ctx *ctx, int mode) {
    if (!ctx || mode < -1 || mode > 2) return QGCM_E_ARG;
    return mode < 0 ? ctx->chain_codec.load() : ctx->chain_codec.exchange(mode);
}

int qgcm_compress_seal_host(qgcm_ctx *ctx, uint8_t *h_arena, uint64_t stride, uint32_t n, uint32_t *lens,
                            uint32_t key_idx, const uint8_t *h_nonces, uint32_t aad_len, int threads,
                            uint8_t *h_status) {
    return run_host_chain(ctx, true, h_arena, stride, n, lens, key_idx, h_nonces, aad_len, threads, h_status);
}

int qgcm_open_uncompress_host(qgcm_ctx *ctx, uint8_t *h_arena, uint64_t stride, uint32_t n, uint32_t *lens,
                              uint32_t key_idx, uint32_t aad_len, int threads, uint8_t *h_status) {
    return run_host_chain(ctx, false, h_arena, stride, n, lens, key_idx, nullptr, aad_len, threads, h_status);
}

void *qgcm_host_alloc(size_t bytes) {
    void *p = nullptr;
    if (bytes == 0 || hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void qgcm_host_free(void *p) {
    if (p) hipHostFree(p);
}

int qgcm_seal_host(qgcm_ctx *ctx, uint8_t *h_arena, uint64_t stride, uint32_t n, uint32_t len, uint32_t key_idx,
                   const uint8_t *h_nonces, uint32_t aad_len, uint8_t *h_status) {
    return run_host(ctx, true, h_arena, stride, n, len, key_idx, h_nonces, aad_len, h_status);
}

int qgcm_open_host(qgcm_ctx *ctx, uint8_t *h_arena, uint64_t stride, uint32_t n, uint32_t len, uint32_t key_idx,
                   uint32_t aad_len, uint8_t *h_status) {
    return run_host(ctx, false, h_arena, stride, n, len, key_idx, nullptr, aad_len, h_status);
}

int qgcm_random_nonces(uint8_t *h_out, uint32_t n) {
    if (!h_out && n) return QGCM_E_ARG;
    size_t left = 12ull * n;
    uint8_t *p = h_out;
    while (left) {
        const ssize_t r = getrandom(p, left > 33554431 ? 33554431 : left, 0);
        if (r < 0 && errno == EINTR) continue;  // large requests can be interrupted by a signal
        if (r <= 0) return QGCM_E_ARG;
        p += r;
        left -= (size_t)r;
    }
    return QGCM_OK;
}

int qgcm_fill_uniform(uint8_t *d_arena, uint64_t stride, uint32_t n, uint32_t len, uint32_t aad_word,
                      uint64_t seed_payload, uint8_t *d_nonces, uint64_t seed_nonce, void *stream) {
    if ((n && !d_arena) || (n && stride < (uint64_t)len + 4)) return QGCM_E_ARG;
    return hip_fail(launch_fill_uniform(d_arena, stride, n, len, aad_word, seed_payload, d_nonces, seed_nonce,
                                        (hipStream_t)stream));
}

int qgcm_resident_stop(qgcm_ctx *ctx) {
    if (!ctx) return QGCM_E_ARG;
    return resident_quiesce(ctx->res.load(std::memory_order_acquire));
}

int qgcm_resident_stats(const qgcm_ctx *ctx, uint64_t *out, int n) {
    if (!ctx || n < 0 || (n && !out)) return -1;
    uint64_t v[kResStats];
    resident_stats(ctx->res.load(std::memory_order_acquire), v);
    const int m = n < kResStats ? n : kResStats;
    for (int i = 0; i < m; ++i) out[i] = v[i];
    return m;
}

int qgcm_launch_counts(const qgcm_ctx *ctx, uint64_t *out, int n) {
    if (!ctx || n < 0 || (n && !out)) return -1;
    const int m = n < QGCM_KERNEL_COUNTERS ? n : QGCM_KERNEL_COUNTERS;
    for (int i = 0; i < m; ++i) out[i] = ctx->launches[i].load(std::memory_order_relaxed);
    return m;
}

int qgcm_stream_copy(qgcm_ctx *ctx, void *d_dst, const void *d_src, uint64_t bytes, void *stream) {
    if (!ctx || (bytes && (!d_dst || !d_src)) || (bytes & 15) || ((uintptr_t)d_dst & 15) || ((uintptr_t)d_src & 15))
        return QGCM_E_ARG;
    if (hipSetDevice(ctx->device) != hipSuccess) return QGCM_E_HIP;
    return hip_fail(launch_stream_copy(d_dst, d_src, bytes, ctx->num_cus, (hipStream_t)stream));
}

}  // extern "C"
