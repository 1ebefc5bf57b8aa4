// group.cpp -- several GPUs behind one process: keyed host batches hash-sharded over device contexts.
//
// quantum is ONE process (main.go:29-114) whose NumWorkers outgoing/incoming workers
// (main.go:72-75) all call the same Encryption plugin.  On an 8 x MI355X node the drop-in therefore
// drives every GPU from that one process: a group holds one qgcm_ctx per
// member (one per GPU; several members may share a device, which is how the 1-GPU tests run G = 2).
//
// Partitioning: packet i goes to member hash(key_idx) mod G, the hash of
// quantum_amd/shard.py key_shard -- (key_idx * 0x9E3779B97F4A7C15 mod 2^64) >> 32.  A peer's packets
// stay on one GPU (in order), and a member only holds the keys of its own peers:
// qgcm_group_set_keys installs key k on member shard(k) only.  Packets are independent GCM
// instances, so there is no collective and no GPU-to-GPU traffic.
//
// One host thread and one stream pair per member for the duration of a call.  Its packets are
// gathered from the caller's arena into pinned staging chunks of up to kChunk bytes (records
// 16-B aligned, with the descriptors and nonces of the chunk behind them), copied in, sealed/opened
// by the member's descriptor batch (qgcm_seal_batch / qgcm_open_batch: sorted quad tiles), copied
// back, and scattered into the caller's slots, which keep their input order.  Two staging slots per
// member alternate, so the gather of chunk c + 1 overlaps chunk c on the device.
//
// NUMA: each member's thread runs on the CPUs local to its GPU (the PCI device's
// local_cpulist in sysfs, intersected with the process's allowed CPUs), and it allocates that
// member's pinned staging itself, so the gather/scatter copies and the DMA stay on the GPU's socket.
//
// The gather and the scatter are record-by-record memcpy (a peer's packets are scattered over the
// caller's arena): one thread moved ~8 GB/s each way and bound the call (7.8 GiB/s seal+open for
// 2^20 x 1350 B on one member, against 41 for qgcm_seal_host's contiguous pipeline).  Each member
// therefore has a pool of copy threads (QGCM_GROUP_THREADS per member, default 4, the member thread
// included, pinned like it) that split every chunk's gather and scatter by record.
//
// Zero-copy path: when the caller's arena (and nonce array) is pinned, device-accessible host memory
// (qgcm_host_alloc / hipHostMalloc / hipHostRegister) and every record lies inside that allocation,
// the member's GPU gathers the records itself (move_records_kernel: one wave per record, reads over
// PCIe into device staging), runs the descriptor batch there and scatters the results back into the
// slots -- the host only builds the per-record move lists (24 B per record).  QGCM_GROUP_ZEROCOPY=0
// forces the CPU path.
//
// DMA-run path (the default when it applies): when a member's packets lie in the arena as long runs of
// adjacent records -- the caller laid the batch out grouped by member (qgcm_group_order), or the group
// has one member -- nothing is gathered at all.  Each run (records of consecutive input packets, gaps
// of at most kRunGap bytes between them) is copied to device staging with one hipMemcpyAsync, the
// descriptor batch runs on the staging with rebased offsets, and the run is copied back whole; a
// record's gap bytes and untouched fields go back as they came.  Three streams per member (copy-in,
// kernels, copy-out) ordered by per-slot events over kDmaSlots staging slots, as qgcm_seal_host's
// pipeline does, so each PCIe direction sees a steady queue of large copies: the SDMA engines move the
// bytes (shader-driven zero-copy reached ~25 GB/s each way; DMA ~45).  QGCM_GROUP_DMA=0 disables it.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <ctype.h>
#include <sched.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "gcm_internal.h"

namespace {

constexpr uint64_t kChunk = 32ull << 20;    // staged slot bytes per chunk, copy path (pinned staging)
constexpr uint64_t kZcChunk = 256ull << 20; // zero-copy path (device staging): enough wave tiles per
                                            // chunk to fill the GPU (a 32-MB chunk is ~1500 tiles)
constexpr int kSlots = 2;                 // staging slots per member (double buffer)
constexpr int kCopyThreads = 4;           // gather/scatter threads per member (QGCM_GROUP_THREADS)
constexpr uint64_t kDmaChunk = 64ull << 20; // DMA-run path: staged bytes per chunk (QGCM_GROUP_DMA_CHUNK_MB)
// DMA-run path: staging slots in flight per member (QGCM_GROUP_DMA_SLOTS).  Three, not more: config 3
// from pinned host memory at 64-MiB chunks read 41.4 GiB/s with 3 slots, 25.7 with 4, 15.7 with 8 and
// 13.2 with 16 (profiles/r4_dma: with more slots every S-th chunk's copy-out stalls 4-5 ms, by the
// per-chunk timing events), and 34.2 with 2.
constexpr int kDmaSlots = 3;
constexpr uint64_t kRunGap = 256;         // largest gap between two records that still joins them in a run
constexpr uint64_t kMinRun = 64ull << 10; // DMA-run path only when runs average at least this many bytes

struct Stage {
    uint8_t *h = nullptr, *d = nullptr;  // pinned host / device: [records][descs][nonces][status]
    size_t cap = 0;
    hipStream_t s = nullptr;
    // the chunk currently in flight in this slot (scattered back once it has landed)
    std::vector<uint32_t> pk;  // caller packet indices
    std::vector<uint64_t> at;  // record offset of each packet in the staging area
    uint64_t status_off = 0;
    bool busy = false;
};

// A fixed set of copy threads; run(f) calls f(0) on the caller and f(1..n-1) on the pool, and returns
// once all have finished.  One run at a time (the member thread).
class CopyPool {
  public:
    CopyPool(int n, cpu_set_t cpus, int ncpus) : n_(n < 1 ? 1 : n) {
        for (int i = 1; i < n_; ++i)
            th_.emplace_back([this, i, cpus, ncpus] {
                if (ncpus > 0) pthread_setaffinity_np(pthread_self(), sizeof(cpu_set_t), &cpus);
                loop(i);
            });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int size() const { return n_; }
    void run(const std::function<void(int)> &f) {
        if (n_ == 1) {
            f(0);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            pending_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0; });
        job_ = nullptr;
    }

  private:
    void loop(int i) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)> *f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                f = job_;
            }
            (*f)(i);
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
};

// zero-copy path state of a member (grow-only): host move lists / staging descriptors (pinned), their
// device copies, device staging and the batch's status bytes
struct ZC {
    qgcm::RecMove *h_moves = nullptr, *d_moves = nullptr;  // [gather: m records + m nonces][scatter: m]
    qgcm_desc *h_descs = nullptr, *d_descs = nullptr;
    uint8_t *d_stage[kSlots] = {nullptr, nullptr};  // records then nonces, per slot
    uint8_t *d_status = nullptr, *h_status = nullptr;
    size_t cap = 0;         // records the lists are sized for
    uint64_t stage_cap = 0;  // bytes per staging slot
};

// DMA-run path state of a member (grow-only)
struct DmaState {
    std::vector<hipEvent_t> ev_in, ev_k, ev_out;  // per staging slot
    std::vector<uint8_t *> d_stage;  // [records][descs][nonces] of one chunk, stage_cap bytes each
    std::vector<uint8_t *> h_side;   // pinned [descs][nonces] of one chunk, side_cap bytes each
    uint64_t stage_cap = 0, side_cap = 0;
    uint8_t *d_stat = nullptr, *h_stat = nullptr;  // the member's statuses, all chunks (device, pinned)
    size_t stat_cap = 0;
};

struct Member {
    qgcm_ctx *ctx = nullptr;
    int device = 0;
    int num_cus = 0;
    Stage st[kSlots];
    ZC zc;
    DmaState dma;
    int last_path = 0;  // 0 copy, 1 zero-copy, 2 DMA runs, 3 direct (qgcm_group_last_path)
    cpu_set_t cpus;  // the GPU's local CPUs allowed to this process (empty: the thread is not pinned)
    int ncpus = 0;
    std::unique_ptr<CopyPool> pool;  // gather/scatter threads (created with the member)
};

// [lo, hi) of n records for pool slice i of k
inline void slice(size_t n, int i, int k, size_t &lo, size_t &hi) {
    lo = n * (size_t)i / (size_t)k;
    hi = n * (size_t)(i + 1) / (size_t)k;
}

using qgcm::gpu_local_cpus;

inline uint64_t rec_bytes(bool seal, uint32_t len) {  // AAD word + packet (+ tag || nonce), 16-B aligned
    return (4ull + len + (seal ? QGCM_OVERHEAD : 0) + 15) & ~15ull;
}

}  // namespace

struct qgcm_group {
    std::vector<Member> m;
    uint32_t max_keys = 0;
    bool zerocopy = true;  // QGCM_GROUP_ZEROCOPY=0: always gather/scatter on the CPU
    bool dma = true;       // QGCM_GROUP_DMA=0: never the DMA-run path
    int last_zc = 0;       // the last call took the zero-copy path (qgcm_group_last_zerocopy)
    uint64_t zc_chunk = kZcChunk;  // zero-copy staging chunk bytes (QGCM_GROUP_ZC_CHUNK_MB, tuning)
    // A/B and diagnostic knobs, read once at qgcm_group_create like the ones above (a getenv per call
    // would race a setenv from another thread)
    bool direct = true;             // QGCM_GROUP_DIRECT=0: worker-sized batches copy by DMA as larger ones
    int dma_slots = kDmaSlots;      // QGCM_GROUP_DMA_SLOTS: staging slots (chunks in flight) per member
    uint64_t dma_chunk = kDmaChunk; // QGCM_GROUP_DMA_CHUNK_MB: staged bytes per DMA chunk
    bool dma_timeline = false;      // QGCM_GROUP_DMA_TIMELINE=1: per-chunk timing events to stderr
    std::mutex call_mu;  // one batch call at a time (members' staging is reused per call)
};

namespace {

int grow(Stage &s, int device, size_t bytes) {
    if (bytes <= s.cap) return QGCM_OK;
    if (s.h) hipHostFree(s.h);
    if (s.d) hipFree(s.d);
    s.h = nullptr;
    s.d = nullptr;
    s.cap = 0;
    if (hipSetDevice(device) != hipSuccess) return QGCM_E_HIP;
    if (hipHostMalloc(&s.h, bytes, hipHostMallocDefault) != hipSuccess) return QGCM_E_NOMEM;
    if (hipMalloc(&s.d, bytes) != hipSuccess) return QGCM_E_NOMEM;
    s.cap = bytes;
    return QGCM_OK;
}

// Copies the results of the chunk in flight in `s` back into the caller's slots (after its stream
// has drained).  Seal: a sealed record comes back whole (ct, tag, nonce); a rejected one (no key on
// this member) was left untouched.  Open: the payload region comes back -- plaintext, or zeros after
// an authentication failure (Go 1.9 gcm Open), or the unchanged bytes of a rejected packet; Open
// never writes the tag or the nonce.
int land(Stage &s, CopyPool &pool, bool seal, uint8_t *h_arena, const qgcm_desc *descs, uint8_t *h_status, int &bad) {
    if (!s.busy) return QGCM_OK;
    s.busy = false;
    if (hipStreamSynchronize(s.s) != hipSuccess) return QGCM_E_HIP;
    const uint8_t *st = s.h + s.status_off;
    const int k = pool.size();
    pool.run([&](int t) {
        size_t lo, hi;
        slice(s.pk.size(), t, k, lo, hi);
        for (size_t j = lo; j < hi; ++j) {
            const qgcm_desc &d = descs[s.pk[j]];
            if (seal) {
                if (st[j] == 1) memcpy(h_arena + d.offset + 4, s.h + s.at[j] + 4, (size_t)d.len + QGCM_OVERHEAD);
            } else {
                memcpy(h_arena + d.offset + 4, s.h + s.at[j] + 4, (size_t)d.len - QGCM_OVERHEAD);
            }
        }
    });
    for (size_t j = 0; j < s.pk.size(); ++j) {
        bad += st[j] != 1;
        if (h_status) h_status[s.pk[j]] = st[j];
    }
    return QGCM_OK;
}

int run_member(Member &mb, bool seal, uint8_t *h_arena, const qgcm_desc *descs, const uint32_t *idx, size_t m,
               const uint8_t *h_nonces, uint32_t aad_len, uint8_t *h_status, int *bad_out) {
    int bad = 0, rc = QGCM_OK;
    // a fresh thread per call: pin it before it allocates or touches staging (first touch = local pages)
    if (mb.ncpus > 0) pthread_setaffinity_np(pthread_self(), sizeof(mb.cpus), &mb.cpus);
    if (hipSetDevice(mb.device) != hipSuccess) return QGCM_E_HIP;
    for (Stage &s : mb.st)
        if (!s.s && hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking) != hipSuccess) return QGCM_E_HIP;
    size_t next = 0;
    int k = 0;
    while (next < m && rc == QGCM_OK) {
        Stage &s = mb.st[k];
        k = (k + 1) % kSlots;
        if ((rc = land(s, *mb.pool, seal, h_arena, descs, h_status, bad)) != QGCM_OK) break;
        // chunk [next, end): records up to kChunk bytes (at least one packet)
        size_t end = next;
        uint64_t bytes = 0;
        while (end < m) {
            const uint64_t r = rec_bytes(seal, descs[idx[end]].len);
            if (end > next && bytes + r > kChunk) break;
            bytes += r;
            ++end;
        }
        const size_t cn = end - next;
        const uint64_t off_desc = bytes, off_non = off_desc + ((16ull * cn + 255) & ~255ull);
        const uint64_t off_st = off_non + (seal && h_nonces ? (12ull * cn + 255) & ~255ull : 0);
        const uint64_t total = off_st + ((cn + 255) & ~255ull);
        if ((rc = grow(s, mb.device, std::max<uint64_t>(total, 1ull << 20))) != QGCM_OK) break;
        s.pk.assign(idx + next, idx + end);
        s.at.resize(cn);
        s.status_off = off_st;
        qgcm_desc *ld = reinterpret_cast<qgcm_desc *>(s.h + off_desc);
        uint64_t pos = 0;
        for (size_t j = 0; j < cn; ++j) {  // record offsets in the staging area
            s.at[j] = pos;
            pos += rec_bytes(seal, descs[s.pk[j]].len);
        }
        const int kk = mb.pool->size();
        mb.pool->run([&](int t) {  // gather, split by record over the member's copy threads
            size_t lo, hi;
            slice(cn, t, kk, lo, hi);
            for (size_t j = lo; j < hi; ++j) {
                const qgcm_desc &d = descs[s.pk[j]];
                // seal: AAD, payload and the slot's tag/nonce area (the nonce may already be there); open:
                // the sealed record is len bytes after the AAD
                const uint64_t in = 4ull + d.len + (seal ? QGCM_OVERHEAD : 0);
                memcpy(s.h + s.at[j], h_arena + d.offset, in);
                ld[j] = qgcm_desc{s.at[j], d.len, d.key_idx};
                if (seal && h_nonces) memcpy(s.h + off_non + 12 * j, h_nonces + 12ull * s.pk[j], 12);
            }
        });
        const uint64_t in_bytes = off_st;  // records, descriptors, nonces
        if (hipMemcpyAsync(s.d, s.h, in_bytes, hipMemcpyHostToDevice, s.s) != hipSuccess) {
            rc = QGCM_E_HIP;
            break;
        }
        const qgcm_desc *dd = reinterpret_cast<const qgcm_desc *>(s.d + off_desc);
        rc = seal ? qgcm_seal_batch(mb.ctx, s.d, dd, (uint32_t)cn, h_nonces ? s.d + off_non : nullptr, aad_len,
                                    s.d + off_st, s.s)
                  : qgcm_open_batch(mb.ctx, s.d, dd, (uint32_t)cn, aad_len, s.d + off_st, s.s);
        if (rc != QGCM_OK) break;
        if (hipMemcpyAsync(s.h, s.d, bytes, hipMemcpyDeviceToHost, s.s) != hipSuccess ||
            hipMemcpyAsync(s.h + off_st, s.d + off_st, cn, hipMemcpyDeviceToHost, s.s) != hipSuccess) {
            rc = QGCM_E_HIP;
            break;
        }
        s.busy = true;
        next = end;
    }
    for (Stage &s : mb.st) {
        const int r = land(s, *mb.pool, seal, h_arena, descs, h_status, bad);
        if (rc == QGCM_OK) rc = r;
    }
    *bad_out = bad;
    return rc;
}

template <typename T>
bool grow_pinned(T *&h, T *&d, size_t count) {
    if (h) hipHostFree(h);
    if (d) hipFree(d);
    h = nullptr;
    d = nullptr;
    return hipHostMalloc(reinterpret_cast<void **>(&h), sizeof(T) * count, hipHostMallocDefault) == hipSuccess &&
           hipMalloc(reinterpret_cast<void **>(&d), sizeof(T) * count) == hipSuccess;
}

using qgcm::pinned_view;

// Zero-copy form of run_member: the member's GPU gathers its records from the pinned arena itself.
// v_arena / v_nonces: the arena's and nonces' device views resolved on this member's device.
int run_member_zc(Member &mb, bool seal, uint64_t v_arena, const qgcm_desc *descs, const uint32_t *idx, size_t m,
                  uint64_t v_nonces, uint32_t aad_len, uint8_t *h_status, int *bad_out, uint64_t chunk) {
    ZC &z = mb.zc;
    for (Stage &s : mb.st)
        if (!s.s && hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking) != hipSuccess) return QGCM_E_HIP;
    if (m > z.cap) {
        const size_t cap = std::max<size_t>(m, 4096);
        if (!grow_pinned(z.h_moves, z.d_moves, 3 * cap) || !grow_pinned(z.h_descs, z.d_descs, cap) ||
            !grow_pinned(z.h_status, z.d_status, cap))
            return QGCM_E_NOMEM;
        z.cap = cap;
    }
    // staging slot: a chunk's records (up to `chunk` bytes, or one larger record) + 256-B pad + their nonces
    uint64_t need = chunk;
    for (size_t j = 0; j < m; ++j) need = std::max<uint64_t>(need, rec_bytes(seal, descs[idx[j]].len));
    need += 256 + 12ull * (chunk / 32 + 1);  // records are >= 32 B: at most chunk / 32 + 1 per chunk
    if (need > z.stage_cap) {
        for (auto &st : z.d_stage) {
            if (st) hipFree(st);
            st = nullptr;
        }
        z.stage_cap = 0;
        for (auto &st : z.d_stage)
            if (hipMalloc(&st, need) != hipSuccess) return QGCM_E_NOMEM;
        z.stage_cap = need;
    }
    qgcm::RecMove *gm = z.h_moves, *nm = z.h_moves + m, *sm = z.h_moves + 2 * m;
    int rc = QGCM_OK;
    size_t next = 0;
    for (int c = 0; next < m && rc == QGCM_OK; ++c) {
        const int k = c % kSlots;
        hipStream_t s = mb.st[k].s;
        uint8_t *stage = z.d_stage[k];
        size_t end = next;
        uint64_t bytes = 0;
        while (end < m) {
            const uint64_t r = rec_bytes(seal, descs[idx[end]].len);
            if (end > next && bytes + r > chunk) break;
            bytes += r;
            ++end;
        }
        const size_t cn = end - next;
        const uint64_t non_off = (bytes + 255) & ~255ull;
        const bool with_nonces = seal && v_nonces;
        uint64_t pos = 0;
        for (size_t j = next; j < end; ++j) {
            const qgcm_desc &d = descs[idx[j]];
            const uint64_t in = 4ull + d.len + (seal ? QGCM_OVERHEAD : 0);
            const uint64_t dst = reinterpret_cast<uint64_t>(stage) + pos;
            gm[j] = qgcm::RecMove{v_arena + d.offset, dst, (uint32_t)in, 0};
            if (with_nonces)
                nm[j] = qgcm::RecMove{v_nonces + 12ull * idx[j],
                                      reinterpret_cast<uint64_t>(stage) + non_off + 12ull * (j - next), 12u, 0};
            const uint32_t out = seal ? d.len + QGCM_OVERHEAD : d.len - QGCM_OVERHEAD;
            sm[j] = qgcm::RecMove{dst + 4, v_arena + d.offset + 4, out, (uint32_t)(j - next)};
            z.h_descs[j] = qgcm_desc{pos, d.len, d.key_idx};
            pos += rec_bytes(seal, d.len);
        }
        // this chunk's lists -> device (stream-ordered before the kernels that read them)
        const size_t a = next;
        if (hipMemcpyAsync(z.d_moves + a, gm + a, sizeof(qgcm::RecMove) * cn, hipMemcpyHostToDevice, s) != hipSuccess ||
            (with_nonces &&
             hipMemcpyAsync(z.d_moves + m + a, nm + a, sizeof(qgcm::RecMove) * cn, hipMemcpyHostToDevice, s) !=
                 hipSuccess) ||
            hipMemcpyAsync(z.d_moves + 2 * m + a, sm + a, sizeof(qgcm::RecMove) * cn, hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            hipMemcpyAsync(z.d_descs + a, z.h_descs + a, sizeof(qgcm_desc) * cn, hipMemcpyHostToDevice, s) != hipSuccess) {
            rc = QGCM_E_HIP;
            break;
        }
        if (qgcm::launch_move_records(z.d_moves + a, (uint32_t)cn, nullptr, false, mb.num_cus, s) != hipSuccess ||
            (with_nonces &&
             qgcm::launch_move_records(z.d_moves + m + a, (uint32_t)cn, nullptr, false, mb.num_cus, s) != hipSuccess)) {
            rc = QGCM_E_HIP;
            break;
        }
        rc = seal ? qgcm_seal_batch(mb.ctx, stage, z.d_descs + a, (uint32_t)cn, with_nonces ? stage + non_off : nullptr,
                                    aad_len, z.d_status + a, s)
                  : qgcm_open_batch(mb.ctx, stage, z.d_descs + a, (uint32_t)cn, aad_len, z.d_status + a, s);
        if (rc != QGCM_OK) break;
        // scatter: a failed seal leaves the slot untouched; open writes plaintext or zeros
        if (qgcm::launch_move_records(z.d_moves + 2 * m + a, (uint32_t)cn, seal ? z.d_status + a : nullptr, true,
                                      mb.num_cus, s) != hipSuccess ||
            hipMemcpyAsync(z.h_status + a, z.d_status + a, cn, hipMemcpyDeviceToHost, s) != hipSuccess) {
            rc = QGCM_E_HIP;
            break;
        }
        next = end;
    }
    for (Stage &st : mb.st)
        if (hipStreamSynchronize(st.s) != hipSuccess && rc == QGCM_OK) rc = QGCM_E_HIP;
    int bad = 0;
    for (size_t j = 0; j < next; ++j) {
        bad += z.h_status[j] != 1;
        if (h_status) h_status[idx[j]] = z.h_status[j];
    }
    *bad_out = bad;
    return rc;
}

// ---- DMA-run path ----
struct Piece {
    uint64_t src, dst, bytes;  // arena offset, offset in the chunk's staging, length
};
struct DmaChunk {
    size_t p0, p1, j0, j1;  // pieces [p0, p1), member packets [j0, j1)
    uint64_t bytes;         // staging bytes the records occupy
};
struct DmaPlan {
    std::vector<Piece> pieces;
    std::vector<DmaChunk> chunks;
    std::vector<uint64_t> at;  // staging offset of member packet j within its chunk
    uint64_t piece_bytes = 0, max_bytes = 0;
    size_t max_pk = 0;
};

inline uint64_t rec_in(bool seal, uint32_t len) {  // bytes of a slot the call reads and may write
    return 4ull + len + (seal ? QGCM_OVERHEAD : 0);
}

// Runs of member packets idx[0..m) (input order, offsets nondecreasing over the whole batch): packet
// idx[j] joins the run of idx[j-1] when it is the next input packet and its record starts at most
// kRunGap bytes after the previous record ends.  Runs are cut into chunks of up to `chunk` staging
// bytes at record boundaries; each piece keeps its host address mod 256 (`mis` = the arena's) in
// staging: the payloads keep their alignment, and a piece's host and staging ends share 256-B boundaries.
void plan_dma(bool seal, const qgcm_desc *descs, const uint32_t *idx, size_t m, uint64_t chunk, uint32_t mis,
              DmaPlan &pl) {
    pl = DmaPlan{};
    pl.at.resize(m);
    uint64_t prev_end = 0;
    size_t j0 = 0, p0 = 0;
    for (size_t j = 0; j < m; ++j) {
        const qgcm_desc &d = descs[idx[j]];
        const uint64_t r0 = d.offset, r1 = r0 + rec_in(seal, d.len);
        bool joined = false;
        if (j > j0 && idx[j] == idx[j - 1] + 1 && r0 >= prev_end && r0 - prev_end <= kRunGap) {
            Piece &pc = pl.pieces.back();
            if (pc.dst + (r1 - pc.src) <= chunk) {
                pc.bytes = r1 - pc.src;
                joined = true;
            }
        }
        if (!joined) {
            uint64_t pos = pl.pieces.size() > p0 ? pl.pieces.back().dst + pl.pieces.back().bytes : 0;
            pos += (r0 + mis - pos) & 255;
            if (j > j0 && pos + (r1 - r0) > chunk) {  // close the chunk
                pl.chunks.push_back(DmaChunk{p0, pl.pieces.size(), j0, j, pos});
                j0 = j;
                p0 = pl.pieces.size();
                pos = (r0 + mis) & 255;
            }
            pl.pieces.push_back(Piece{r0, pos, r1 - r0});
        }
        const Piece &pc = pl.pieces.back();
        pl.at[j] = pc.dst + (r0 - pc.src);
        prev_end = r1;
    }
    if (m) {
        const Piece &pc = pl.pieces.back();
        pl.chunks.push_back(DmaChunk{p0, pl.pieces.size(), j0, m, pc.dst + pc.bytes});
    }
    for (const Piece &pc : pl.pieces) pl.piece_bytes += pc.bytes;
    for (DmaChunk &c : pl.chunks) {
        c.bytes = (pl.pieces[c.p1 - 1].dst + pl.pieces[c.p1 - 1].bytes + 255) & ~255ull;
        pl.max_bytes = std::max(pl.max_bytes, c.bytes);
        pl.max_pk = std::max(pl.max_pk, c.j1 - c.j0);
    }
}

int dma_ready(DmaState &z, uint64_t stage, uint64_t side, size_t slots, size_t m) {
    if (m > z.stat_cap) {
        if (z.d_stat) hipFree(z.d_stat);
        if (z.h_stat) hipHostFree(z.h_stat);
        z.d_stat = z.h_stat = nullptr;
        z.stat_cap = 0;
        if (hipMalloc(&z.d_stat, m) != hipSuccess || hipHostMalloc(&z.h_stat, m, hipHostMallocDefault) != hipSuccess)
            return QGCM_E_NOMEM;
        z.stat_cap = m;
    }
    while (z.ev_in.size() < slots) {
        hipEvent_t e[3] = {};
        for (hipEvent_t &x : e)
            if (hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess) {
                for (hipEvent_t y : e)
                    if (y) hipEventDestroy(y);
                return QGCM_E_HIP;
            }
        z.ev_in.push_back(e[0]);
        z.ev_k.push_back(e[1]);
        z.ev_out.push_back(e[2]);
    }
    if (stage + side > z.stage_cap) {
        for (uint8_t *p : z.d_stage) hipFree(p);
        z.d_stage.clear();
        z.stage_cap = stage + side;
    }
    while (z.d_stage.size() < slots) {
        uint8_t *p = nullptr;
        if (hipMalloc(&p, z.stage_cap) != hipSuccess) return QGCM_E_NOMEM;
        z.d_stage.push_back(p);
    }
    if (side > z.side_cap) {
        for (uint8_t *p : z.h_side) hipHostFree(p);
        z.h_side.clear();
        z.side_cap = side;
    }
    while (z.h_side.size() < slots) {
        uint8_t *p = nullptr;
        if (hipHostMalloc(&p, z.side_cap, hipHostMallocDefault) != hipSuccess) return QGCM_E_NOMEM;
        z.h_side.push_back(p);
    }
    return QGCM_OK;
}

// Direct: a member's worker-sized batch (at most direct_max packets and kDirectMaxBytes) whose
// records all start 16-B aligned in a pinned arena that holds each record's 16-B-rounded area runs one
// workgroup per packet on the records in place, over PCIe: no copies and one launch.  The kernel
// writes each record's whole 16-B-rounded area back, so `allowed` (run_group) is false unless EVERY
// record of the batch -- any member's, rejected ones included -- starts 16-B aligned: then no record
// begins inside another's rounded area, and members interleaved in one arena each seal their own in
// place at once without one member's write-back overwriting another's results.  Descriptors, nonces
// and statuses stay in pinned host memory as well.  Returns 1 when it ran (rc in *rc), 0 when the
// batch does not qualify (nothing done).
int run_member_direct(Member &mb, bool allowed, bool seal, uint8_t *h_arena, const qgcm_desc *descs,
                      const uint32_t *idx, size_t m, const uint8_t *h_nonces, uint32_t aad_len, uint8_t *h_status,
                      int *bad_out, int *rc) {
    if (!allowed || !m || m > qgcm::direct_max(mb.ctx)) return 0;
    uint64_t ext = 0;
    for (size_t j = 0; j < m; ++j) {
        const qgcm_desc &d = descs[idx[j]];
        const uint64_t area = (rec_in(seal, d.len) + 15) & ~15ull;
        if (((uintptr_t)(h_arena + d.offset) & 15) || area > qgcm::kOneCap - 16) return 0;
        ext = std::max(ext, d.offset + area);
    }
    uint64_t bytes = 0;  // the records' rounded areas: past kDirectMaxBytes the DMA pipeline is faster
    for (size_t j = 0; j < m; ++j) bytes += (rec_in(seal, descs[idx[j]].len) + 15) & ~15ull;
    if (bytes > qgcm::kDirectMaxBytes) return 0;
    const uint64_t va = pinned_view(h_arena, ext);
    if (!va || (va & 15)) return 0;
    DmaState &z = mb.dma;
    const bool non = seal && h_nonces;
    const uint64_t off_non = (16ull * m + 255) & ~255ull;
    const uint64_t side = off_non + (non ? (12ull * m + 255) & ~255ull : 0);  // [descs][nonces]
    *rc = dma_ready(z, 0, side, 1, m);
    if (*rc != QGCM_OK) return 1;
    uint8_t *hs = z.h_side[0];
    const uint64_t vs = pinned_view(hs, side), vst = pinned_view(z.h_stat, m);
    if (!vs || !vst) return 0;
    qgcm_desc *hd = reinterpret_cast<qgcm_desc *>(hs);
    for (size_t j = 0; j < m; ++j) {
        hd[j] = descs[idx[j]];
        if (non) memcpy(hs + off_non + 12 * j, h_nonces + 12ull * idx[j], 12);
    }
    std::lock_guard<std::mutex> io(qgcm::ctx_io_mu(mb.ctx));
    hipStream_t s = qgcm::ctx_pipe(mb.ctx, 0);
    *rc = qgcm::run_descs_one(mb.ctx, seal, reinterpret_cast<uint8_t *>(va), reinterpret_cast<const qgcm_desc *>(vs),
                              (uint32_t)m, non ? reinterpret_cast<const uint8_t *>(vs + off_non) : nullptr, aad_len,
                              reinterpret_cast<uint8_t *>(vst), s);
    if (hipStreamSynchronize(s) != hipSuccess && *rc == QGCM_OK) *rc = QGCM_E_HIP;
    int bad = 0;
    if (*rc == QGCM_OK)
        for (size_t j = 0; j < m; ++j) {
            bad += z.h_stat[j] != 1;
            if (h_status) h_status[idx[j]] = z.h_stat[j];
        }
    *bad_out = bad;
    mb.last_path = 3;
    return 1;
}

int run_member_dma(const qgcm_group *g, Member &mb, bool direct_ok, bool seal, uint8_t *h_arena,
                   const qgcm_desc *descs, const uint32_t *idx, const DmaPlan &pl, const uint8_t *h_nonces,
                   uint32_t aad_len, uint8_t *h_status, int *bad_out) {
    {
        int rc = QGCM_OK;
        if (run_member_direct(mb, direct_ok, seal, h_arena, descs, idx, pl.at.size(), h_nonces, aad_len, h_status,
                              bad_out, &rc))
            return rc;
    }
    DmaState &z = mb.dma;
    const bool non = seal && h_nonces;
    const uint64_t pk = pl.max_pk;
    const uint64_t off_non = (16ull * pk + 255) & ~255ull;
    const uint64_t side = off_non + (non ? (12ull * pk + 255) & ~255ull : 0);  // [descs][nonces]
    const size_t nc = pl.chunks.size();
    const size_t S = std::min<size_t>(nc, (size_t)g->dma_slots);
    const size_t m = pl.at.size();
    int rc = dma_ready(z, pl.max_bytes, side, S, m);
    if (rc != QGCM_OK) return rc;
    // the member context's own pipeline streams, those qgcm_seal_host moves 46 GB/s each way with
    // (streams of the group's own measured the same, profiles/r4_s6)
    // one chunk (a worker-sized batch) has nothing to overlap: one stream, no events, one synchronize
    std::lock_guard<std::mutex> io(qgcm::ctx_io_mu(mb.ctx));
    const bool one = nc == 1;
    const uint32_t one_max = qgcm::descs_one_max(mb.ctx);
    hipStream_t s_in = qgcm::ctx_pipe(mb.ctx, 0);
    hipStream_t s_k = one ? s_in : qgcm::ctx_pipe(mb.ctx, 1), s_out = one ? s_in : qgcm::ctx_pipe(mb.ctx, 2);
    // QGCM_GROUP_DMA_TIMELINE=1 (diagnostics): timing events after each chunk's copy-in, kernels and
    // copy-out, printed to stderr as ms since the call's first copy-in was queued (no profiler attached)
    std::vector<hipEvent_t> tl;
    hipEvent_t tl0 = nullptr;
    if (g->dma_timeline) {
        tl.assign(3 * nc, nullptr);
        for (hipEvent_t &e : tl) hipEventCreate(&e);
        hipEventCreate(&tl0);
        hipEventRecord(tl0, s_in);
    }
    // Statuses go to one member-wide device array and come back in ONE copy after the last kernel (a
    // small copy-out per chunk would cost a copy setup each).
    size_t c = 0;
    for (; c < nc && rc == QGCM_OK; ++c) {
        const int k = (int)(c % S);
        const DmaChunk &ch = pl.chunks[c];
        // slot k is reused: the copy-out of its previous chunk must have landed.  The host waits for it
        // (which also covers the side area's copy-in) rather than leaving the wait to the copy-in
        // stream: a copy-in queued behind a GPU-side wait for the copy-out stream's blit kernels took
        // the keyed host batch from 25.8 to 13.0 GiB/s at 64-MiB chunks (profiles/r4_s16)
        const size_t e = (size_t)k;  // the slot's events
        if (c >= S && hipEventSynchronize(z.ev_out[e]) != hipSuccess) {
            rc = QGCM_E_HIP;
            break;
        }
        uint8_t *hs = z.h_side[k], *ds = z.d_stage[k];
        const uint64_t dside = pl.max_bytes;  // descs / nonces behind the records
        const size_t cn = ch.j1 - ch.j0;
        qgcm_desc *hd = reinterpret_cast<qgcm_desc *>(hs);
        // a worker-sized chunk whose records all sit at 16-B-aligned staging offsets runs one workgroup
        // per packet (no worklist sort, every CU busy); staging keeps the host layout, so a record's
        // 16-B-rounded area holds no other record, and the chunk's staging bytes are 256-B rounded
        bool one_ok = cn <= one_max;
        for (size_t j = ch.j0; j < ch.j1; ++j) {
            const qgcm_desc &d = descs[idx[j]];
            hd[j - ch.j0] = qgcm_desc{pl.at[j], d.len, d.key_idx};
            if (non) memcpy(hs + off_non + 12 * (j - ch.j0), h_nonces + 12ull * idx[j], 12);
            one_ok = one_ok && !(pl.at[j] & 15) && ((rec_in(seal, d.len) + 15) & ~15ull) <= qgcm::kOneCap - 16;
        }
        for (size_t p = ch.p0; p < ch.p1 && rc == QGCM_OK; ++p) {
            const Piece &pc = pl.pieces[p];
            if (hipMemcpyAsync(ds + pc.dst, h_arena + pc.src, pc.bytes, hipMemcpyHostToDevice, s_in) != hipSuccess)
                rc = QGCM_E_HIP;
        }
        if (rc == QGCM_OK &&
            (hipMemcpyAsync(ds + dside, hs, side, hipMemcpyHostToDevice, s_in) != hipSuccess ||
             (!one && (hipEventRecord(z.ev_in[e], s_in) != hipSuccess ||
                       hipStreamWaitEvent(s_k, z.ev_in[e], 0) != hipSuccess))))
            rc = QGCM_E_HIP;
        if (rc != QGCM_OK) break;
        if (!tl.empty()) hipEventRecord(tl[3 * c], s_in);
        const qgcm_desc *dd = reinterpret_cast<const qgcm_desc *>(ds + dside);
        if (one_ok)
            rc = qgcm::run_descs_one(mb.ctx, seal, ds, dd, (uint32_t)cn, non ? ds + dside + off_non : nullptr, aad_len,
                                     z.d_stat + ch.j0, s_k);
        else
            rc = seal ? qgcm_seal_batch(mb.ctx, ds, dd, (uint32_t)cn, non ? ds + dside + off_non : nullptr, aad_len,
                                        z.d_stat + ch.j0, s_k)
                      : qgcm_open_batch(mb.ctx, ds, dd, (uint32_t)cn, aad_len, z.d_stat + ch.j0, s_k);
        if (rc != QGCM_OK) break;
        if (!tl.empty()) hipEventRecord(tl[3 * c + 1], s_k);
        if (!one && (hipEventRecord(z.ev_k[e], s_k) != hipSuccess || hipStreamWaitEvent(s_out, z.ev_k[e], 0) != hipSuccess))
            rc = QGCM_E_HIP;
        for (size_t p = ch.p0; p < ch.p1 && rc == QGCM_OK; ++p) {
            const Piece &pc = pl.pieces[p];
            if (hipMemcpyAsync(h_arena + pc.src, ds + pc.dst, pc.bytes, hipMemcpyDeviceToHost, s_out) != hipSuccess)
                rc = QGCM_E_HIP;
        }
        if (rc == QGCM_OK && !one && hipEventRecord(z.ev_out[e], s_out) != hipSuccess) rc = QGCM_E_HIP;
        if (!tl.empty()) hipEventRecord(tl[3 * c + 2], s_out);
    }
    // every kernel has run when s_k gets here
    if (rc == QGCM_OK && hipMemcpyAsync(z.h_stat, z.d_stat, m, hipMemcpyDeviceToHost, s_k) != hipSuccess)
        rc = QGCM_E_HIP;
    for (hipStream_t x : {s_in, s_k, s_out}) {
        if (one && x != s_in) continue;
        if (hipStreamSynchronize(x) != hipSuccess && rc == QGCM_OK) rc = QGCM_E_HIP;
    }
    if (!tl.empty()) {
        std::string line = "{\"dma_timeline_ms\": [";
        for (size_t q = 0; q < c; ++q) {
            float t[3] = {};
            for (int i = 0; i < 3; ++i) hipEventElapsedTime(&t[i], tl0, tl[3 * q + i]);
            char buf[96];
            snprintf(buf, sizeof buf, "%s[%.2f, %.2f, %.2f]", q ? ", " : "", t[0], t[1], t[2]);
            line += buf;
        }
        line += "]}\n";
        fputs(line.c_str(), stderr);
        for (hipEvent_t e : tl) hipEventDestroy(e);
        hipEventDestroy(tl0);
    }
    int bad = 0;
    if (rc == QGCM_OK)
        for (size_t j = 0; j < m; ++j) {
            bad += z.h_stat[j] != 1;
            if (h_status) h_status[idx[j]] = z.h_stat[j];
        }
    *bad_out = bad;
    return rc;
}

int run_group(qgcm_group *g, bool seal, uint8_t *h_arena, const qgcm_desc *descs, uint32_t n,
              const uint8_t *h_nonces, uint32_t aad_len, uint8_t *h_status) {
    if (!g || (n && (!h_arena || !descs)) || aad_len > 4 || n > QGCM_MAX_BATCH) return QGCM_E_ARG;
    if (n == 0) return 0;
    std::lock_guard<std::mutex> lk(g->call_mu);
    const int G = (int)g->m.size();
    std::vector<std::vector<uint32_t>> part(G);
    int pre_bad = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const qgcm_desc &d = descs[i];
        const bool ok = d.key_idx < g->max_keys && (seal ? d.len < QGCM_MAX_PAYLOAD
                                                          : d.len >= QGCM_OVERHEAD && d.len - QGCM_OVERHEAD < QGCM_MAX_PAYLOAD);
        if (!ok) {  // rejected as the device batch would: status 0, slot untouched
            if (h_status) h_status[i] = 0;
            ++pre_bad;
            continue;
        }
        part[qgcm_group_shard(g, d.key_idx)].push_back(i);
    }
    // zero-copy when the arena (and nonces) are pinned and hold every record, and every record starts
    // on a 4-B boundary (the record moves are dword-wise; other batches take the copy path, which
    // re-aligns records in staging).  Each member resolves the device view on its own device.
    bool zc = g->zerocopy;
    uint64_t extent = 0;
    for (uint32_t i = 0; zc && i < n; ++i) {
        extent = std::max<uint64_t>(extent, descs[i].offset + 4ull + descs[i].len + (seal ? QGCM_OVERHEAD : 0));
        zc = !(descs[i].offset & 3);
    }
    zc = zc && !((uintptr_t)h_arena & 3) && !(seal && h_nonces && ((uintptr_t)h_nonces & 3));
    // DMA runs need the input in arena order (a run is consecutive input packets) and 4-B record offsets
    bool sorted = g->dma;
    for (uint32_t i = 1; sorted && i < n; ++i) sorted = descs[i].offset >= descs[i - 1].offset;
    for (uint32_t i = 0; sorted && i < n; ++i) sorted = !(descs[i].offset & 3);
    sorted = sorted && !((uintptr_t)h_arena & 3);
    std::vector<DmaPlan> plan(G);
    // worker-sized batches from a pinned arena may go direct (run_member_direct checks the rest), so a
    // run under kMinRun still takes the DMA branch for them.  Direct writes whole 16-B-rounded areas
    // back, so it needs every record of the batch 16-B aligned (run_member_direct)
    bool all16 = g->direct;
    for (uint32_t i = 0; all16 && i < n; ++i) all16 = !(((uintptr_t)h_arena + descs[i].offset) & 15);
    const bool pinned_arena = all16 && pinned_view(h_arena, 1) != 0;
    const bool pinned = sorted && pinned_arena;
    auto dma_pays = [&](int k) {
        const DmaPlan &pl = plan[k];
        if (pl.piece_bytes >= kMinRun * pl.pieces.size()) return true;
        if (!pinned || pl.at.size() > qgcm::direct_max(g->m[k].ctx) || pl.piece_bytes > qgcm::kDirectMaxBytes)
            return false;
        return std::all_of(pl.at.begin(), pl.at.end(), [](uint64_t a) { return !(a & 15); });
    };
    const uint64_t dma_chunk = g->dma_chunk;
    std::vector<int> rc(G, QGCM_OK), bad(G, 0), used_zc(G, 1);
    std::vector<std::thread> thr;
    int active = 0;
    for (int k = 0; k < G; ++k) active += part[k].empty() ? 0 : 1;
    // A batch for one member whose records move by DMA runs on the calling thread: a thread per call
    // costs tens of microseconds, a worker-sized batch's whole budget.  (Other paths keep the member
    // thread: it is pinned to the GPU's NUMA node before it allocates or touches host staging.)
    const bool inline_one = active == 1 && sorted;
    for (int k = 0; k < G; ++k) {
        if (part[k].empty()) continue;
        auto work = [&, k](bool pin) {
            Member &mb = g->m[k];
            if (pin && mb.ncpus > 0) pthread_setaffinity_np(pthread_self(), sizeof(mb.cpus), &mb.cpus);
            if (hipSetDevice(mb.device) != hipSuccess) {
                rc[k] = QGCM_E_HIP;
                return;
            }
            if (sorted) {
                const size_t m = part[k].size();
                plan_dma(seal, descs, part[k].data(), m, dma_chunk, (uint32_t)((uintptr_t)h_arena & 255), plan[k]);
                if (dma_pays(k)) {
                    mb.last_path = 2;
                    used_zc[k] = 0;
                    rc[k] = run_member_dma(g, mb, pinned_arena, seal, h_arena, descs, part[k].data(), plan[k],
                                           h_nonces, aad_len, h_status, &bad[k]);
                    return;
                }
            }
            {  // a worker-sized share of an interleaved batch: in place, as by DMA runs above
                int drc = QGCM_OK;
                if (run_member_direct(mb, pinned_arena, seal, h_arena, descs, part[k].data(), part[k].size(),
                                      h_nonces, aad_len, h_status, &bad[k], &drc)) {
                    used_zc[k] = 0;
                    rc[k] = drc;
                    return;
                }
            }
            uint64_t va = 0, vn = 0;
            if (zc) {
                va = pinned_view(h_arena, extent);
                if (va && seal && h_nonces && !(vn = pinned_view(h_nonces, 12ull * n))) va = 0;
                if ((va | vn) & 3) va = 0;
            }
            used_zc[k] = va ? 1 : 0;
            mb.last_path = va ? 1 : 0;
            rc[k] = va ? run_member_zc(mb, seal, va, descs, part[k].data(), part[k].size(), vn, aad_len, h_status,
                                       &bad[k], g->zc_chunk)
                       : run_member(mb, seal, h_arena, descs, part[k].data(), part[k].size(), h_nonces, aad_len,
                                    h_status, &bad[k]);
        };
        if (!inline_one) {
            thr.emplace_back(work, true);
            continue;
        }
        // inline: the DMA plan decides first; a member that would take another path gets its thread
        const size_t m = part[k].size();
        plan_dma(seal, descs, part[k].data(), m, dma_chunk, (uint32_t)((uintptr_t)h_arena & 255), plan[k]);
        if (!dma_pays(k)) {
            thr.emplace_back(work, true);
            continue;
        }
        int dev0 = 0;
        const bool had = hipGetDevice(&dev0) == hipSuccess;
        Member &mb = g->m[k];
        if (hipSetDevice(mb.device) != hipSuccess) {
            rc[k] = QGCM_E_HIP;
        } else {
            mb.last_path = 2;
            used_zc[k] = 0;
            rc[k] = run_member_dma(g, mb, pinned_arena, seal, h_arena, descs, part[k].data(), plan[k], h_nonces,
                                   aad_len, h_status, &bad[k]);
        }
        if (had) hipSetDevice(dev0);  // the caller's current device, as it was
    }
    for (auto &t : thr) t.join();
    g->last_zc = zc && std::all_of(used_zc.begin(), used_zc.end(), [](int u) { return u == 1; }) ? 1 : 0;
    int total_bad = pre_bad;
    for (int k = 0; k < G; ++k) {
        if (rc[k] != QGCM_OK) return rc[k];
        total_bad += bad[k];
    }
    return total_bad;
}

}  // namespace

extern "C" {

qgcm_group *qgcm_group_create(const int *devices, int count, uint32_t max_keys, char *err, int errlen) {
    if (!devices || count < 1 || count > 64) {
        if (err && errlen > 0) snprintf(err, (size_t)errlen, "need 1..64 member devices");
        return nullptr;
    }
    auto g = std::make_unique<qgcm_group>();
    g->max_keys = max_keys;
    int threads = kCopyThreads;
    if (const char *v = getenv("QGCM_GROUP_THREADS")) threads = std::max(1, std::min(64, atoi(v)));
    if (const char *v = getenv("QGCM_GROUP_ZEROCOPY")) g->zerocopy = atoi(v) != 0;
    if (const char *v = getenv("QGCM_GROUP_DMA")) g->dma = atoi(v) != 0;
    if (const char *v = getenv("QGCM_GROUP_ZC_CHUNK_MB")) g->zc_chunk = (uint64_t)std::max(1, atoi(v)) << 20;
    if (const char *v = getenv("QGCM_GROUP_DIRECT")) g->direct = strcmp(v, "0") != 0;
    if (const char *v = getenv("QGCM_GROUP_DMA_SLOTS"); v && *v) g->dma_slots = std::max(2, std::min(64, atoi(v)));
    if (const char *v = getenv("QGCM_GROUP_DMA_CHUNK_MB"); v && *v)
        g->dma_chunk = (uint64_t)std::max(1, std::min(4096, atoi(v))) << 20;
    if (const char *v = getenv("QGCM_GROUP_DMA_TIMELINE")) g->dma_timeline = atoi(v) != 0;
    for (int k = 0; k < count; ++k) {
        Member mb;
        mb.device = devices[k];
        mb.ncpus = gpu_local_cpus(devices[k], &mb.cpus);
        hipDeviceGetAttribute(&mb.num_cus, hipDeviceAttributeMultiprocessorCount, devices[k]);
        mb.ctx = qgcm_create(devices[k], max_keys, err, errlen);
        if (mb.ctx) mb.pool = std::make_unique<CopyPool>(threads, mb.cpus, mb.ncpus);
        if (!mb.ctx) {
            for (Member &x : g->m) qgcm_destroy(x.ctx);
            return nullptr;
        }
        g->m.push_back(std::move(mb));
    }
    return g.release();
}

void qgcm_group_destroy(qgcm_group *g) {
    if (!g) return;
    for (Member &mb : g->m) {
        hipSetDevice(mb.device);
        for (Stage &s : mb.st) {
            if (s.s) {
                hipStreamSynchronize(s.s);
                hipStreamDestroy(s.s);
            }
            if (s.h) hipHostFree(s.h);
            if (s.d) hipFree(s.d);
        }
        ZC &z = mb.zc;
        if (z.h_moves) hipHostFree(z.h_moves);
        if (z.h_descs) hipHostFree(z.h_descs);
        if (z.h_status) hipHostFree(z.h_status);
        hipFree(z.d_moves);
        hipFree(z.d_descs);
        hipFree(z.d_status);
        for (uint8_t *st : z.d_stage) hipFree(st);
        DmaState &dm = mb.dma;
        for (size_t k = 0; k < dm.ev_in.size(); ++k)
            for (hipEvent_t e : {dm.ev_in[k], dm.ev_k[k], dm.ev_out[k]}) hipEventDestroy(e);
        for (uint8_t *p : dm.d_stage) hipFree(p);
        for (uint8_t *p : dm.h_side) hipHostFree(p);
        if (dm.d_stat) hipFree(dm.d_stat);
        if (dm.h_stat) hipHostFree(dm.h_stat);
        qgcm_destroy(mb.ctx);
    }
    delete g;
}

int qgcm_group_size(const qgcm_group *g) { return g ? (int)g->m.size() : 0; }

int qgcm_group_last_zerocopy(const qgcm_group *g) { return g ? g->last_zc : QGCM_E_ARG; }

int qgcm_group_last_path(const qgcm_group *g, int member) {
    return g && member >= 0 && member < (int)g->m.size() ? g->m[member].last_path : QGCM_E_ARG;
}

int qgcm_group_order(const qgcm_group *g, const uint32_t *key_idx, uint32_t n, uint32_t *order,
                     uint32_t *member_counts) {
    if (!g || g->m.empty() || (n && (!key_idx || !order))) return QGCM_E_ARG;
    const int G = (int)g->m.size();
    std::vector<uint64_t> start(G + 1, 0);
    std::vector<int> owner(n);
    for (uint32_t i = 0; i < n; ++i) {
        owner[i] = qgcm_group_shard(g, key_idx[i]);
        ++start[owner[i] + 1];
    }
    for (int k = 0; k < G; ++k) {
        if (member_counts) member_counts[k] = (uint32_t)start[k + 1];
        start[k + 1] += start[k];
    }
    for (uint32_t i = 0; i < n; ++i) order[start[owner[i]]++] = i;  // stable within a member
    return QGCM_OK;
}

int qgcm_group_member_cpus(const qgcm_group *g, int member) {
    return g && member >= 0 && member < (int)g->m.size() ? g->m[member].ncpus : QGCM_E_ARG;
}

qgcm_ctx *qgcm_group_ctx(qgcm_group *g, int member) {
    return g && member >= 0 && member < (int)g->m.size() ? g->m[member].ctx : nullptr;
}

int qgcm_group_shard(const qgcm_group *g, uint32_t key_idx) {
    if (!g || g->m.empty()) return QGCM_E_ARG;
    const uint64_t h = ((uint64_t)key_idx * 0x9E3779B97F4A7C15ull) >> 32;
    return (int)(h % g->m.size());
}

int qgcm_group_set_keys(qgcm_group *g, uint32_t first_idx, uint32_t count, const uint8_t *keys) {
    if (!g || (count && !keys)) return QGCM_E_ARG;
    if ((uint64_t)first_idx + count > g->max_keys) return QGCM_E_KEY;
    // each member gets the keys it owns, in runs of consecutive indices
    for (uint32_t i = 0; i < count;) {
        const int k = qgcm_group_shard(g, first_idx + i);
        uint32_t j = i + 1;
        while (j < count && qgcm_group_shard(g, first_idx + j) == k) ++j;
        const int rc = qgcm_set_keys(g->m[k].ctx, first_idx + i, j - i, keys + 32ull * i);
        if (rc != QGCM_OK) return rc;
        i = j;
    }
    return QGCM_OK;
}

int qgcm_group_clear_keys(qgcm_group *g, uint32_t first_idx, uint32_t count) {
    if (!g) return QGCM_E_ARG;
    if ((uint64_t)first_idx + count > g->max_keys) return QGCM_E_KEY;
    for (uint32_t i = 0; i < count;) {
        const int k = qgcm_group_shard(g, first_idx + i);
        uint32_t j = i + 1;
        while (j < count && qgcm_group_shard(g, first_idx + j) == k) ++j;
        const int rc = qgcm_clear_keys(g->m[k].ctx, first_idx + i, j - i);
        if (rc != QGCM_OK) return rc;
        i = j;
    }
    return QGCM_OK;
}

int qgcm_group_seal_host(qgcm_group *g, uint8_t *h_arena, const qgcm_desc *h_descs, uint32_t n,
                         const uint8_t *h_nonces, uint32_t aad_len, uint8_t *h_status) {
    return run_group(g, true, h_arena, h_descs, n, h_nonces, aad_len, h_status);
}

int qgcm_group_open_host(qgcm_group *g, uint8_t *h_arena, const qgcm_desc *h_descs, uint32_t n, uint32_t aad_len,
                         uint8_t *h_status) {
    return run_group(g, false, h_arena, h_descs, n, nullptr, aad_len, h_status);
}

}  // extern "C"
