// Internal interface between the C ABI (qgcm_api.cpp) and the gfx950 kernels (gcm_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <sched.h>

#include <mutex>
#include <stdint.h>
#include <vector>

#include "../../include/qgcm.h"

namespace qgcm {

// LDS: Te0/Te1 replicated 32x, rows of 256 B (x<<8 | lane*4, Te1 at +128) = 64 KiB; 8 KiB per 4-bit
// GHASH comb table.
constexpr uint32_t kTeBytes = 65536;
constexpr uint32_t kGhBytes = 8192;
// Device key slot: 60 round-key words (+4 pad), their rot16 copies, and the 4-bit comb tables of
// H and H^4 (2 x 512 x 16 B).
constexpr uint32_t kRkWords = 128;  // [0,64): rk words, [64,128): rot16(rk)
// Per key: nine 4-bit comb tables of 512 x 16 B: H, H^4 (the Horner step of the quad kernel), then
// H^2, H^3, H^5 (the once-per-packet recombination multiplies, read from global memory), then
// H^8, H^16, H^32, H^64 (the latency kernel's 64-way GHASH; the batch kernels never read them).
constexpr uint32_t kGhEntries = 4608;
constexpr uint32_t kGhH = 0, kGhH4 = 512, kGhH2 = 1024, kGhH3 = 1536, kGhH5 = 2048;
constexpr uint32_t kGhH8 = 2560, kGhH16 = 3072, kGhH32 = 3584, kGhH64 = 4096;

struct Batch {
    uint8_t *arena;
    const qgcm_desc *descs;     // NULL -> uniform
    const uint32_t *worklist;   // descriptor kernels: n_items entries, 0xffffffff = padding
    const uint8_t *nonces;      // seal only; NULL -> nonce already in slot
    uint8_t *status;            // may be NULL
    const uint32_t *rk_table;   // [max_keys][kRkWords]
    const uint4 *gh_table;      // [max_keys][kGhEntries]
    const uint32_t *te;         // [512] Te0 then Te1
    const uint8_t *key_valid;   // [max_keys]: 1 once qgcm_set_key(s) filled the slot (descriptor batches
                                // skip packets whose key slot was never set: status 0, slot untouched)
    uint64_t stride;
    uint32_t uniform_len;
    uint32_t uniform_key;
    uint32_t n;
    uint32_t n_items;           // multiple of 64
    uint32_t aad_len;           // 0 or 4
    uint32_t max_keys;
    uint32_t *tile_counter;     // descriptor quad kernels: dynamic tile index (zeroed per launch)
    const uint32_t *tile_keys;  // descriptor quad kernels: key of each 16-entry tile (all ones: padding,
                                // only after the last key run)
    const uint2 *runs;          // segmented kernel: the key runs of the worklist (QuadWorklist)
    uint32_t *run_next;
    const uint32_t *nruns;
    const uint32_t *tile_list;  // per-wave descriptor kernels: NULL = every tile of the worklist, else
    const uint32_t *n_list;     // only these tiles (*n_list of them; the segmented kernel's short keys)
    uint8_t *done;              // gcm_one_kernel (a per-packet call): set to 1 after the slot is written
                                // back and made system-visible (the host polls it instead of the stream)
    const uint4 *pw_table;      // latency engine: [pw_keys][kPwPowers][kPwEntries] kPwBits-bit comb tables of
    uint32_t pw_keys;           // H^1..H^kPwPowers (NULL / 0: the Horner + Estrin GHASH for every packet)
    uint32_t *pool;             // uniform kernel (QGCM_TILE_POOL=4, the default): this launch's pool set
                                // (zeroed; NULL: every tile through the workgroups' LDS counters)
    uint32_t *pool_done;        // pinned word: the grid's last wave stores pool_gen there once the set is
    uint32_t pool_gen;          // zeroed again
};
// Pool set of the uniform kernel's shared tail (words): [0] the tail's tile counter, [kPoolDoneWord] the
// grid's finished-workgroup count.  Zero between launches (the grid's last wave zeroes it, then posts
// the launch's generation to Batch::pool_done).
constexpr uint32_t kPoolDoneWord = 32;
constexpr uint32_t kPoolSetWords = 64;
constexpr uint32_t kPoolSets = 4096;  // sets in a context's ring (1 MiB; QGCM_POOL_SETS at qgcm_create: fewer, for tests)
bool quad_pool_global();            // the uniform kernel takes b.pool (QGCM_TILE_POOL=4)
constexpr uint32_t kPwPowers = 128;    // flat GHASH up to d + 2 = 128 exponents (payloads up to 2016 B)
constexpr uint32_t kPwBits = 6;                                  // comb window of the flat GHASH tables
constexpr uint32_t kPwWin = (128 + kPwBits - 1) / kPwBits;       // windows per block (22)
constexpr uint32_t kPwEntries = kPwWin << kPwBits;               // entries per power (1408: 22 KiB)
constexpr uint32_t kPwLaneWins = (kPwWin + 7) / 8;               // windows per lane of an 8-lane chain

// kernel variant ids (QGCM_VARIANT / QGCM_DESC_VARIANT; the numbers the A/B logs under profiles/ use)
constexpr int kVariantUniform = 12;  // single-key (uniform) batches: quad kernel (Tab2F), 32 waves/CU
constexpr int kVariantDescWave = 13;  // descriptor batches, per-wave 4-bit tables (Tab2), 12 waves/CU
constexpr int kVariantDescQuad = 14;  // default for descriptor batches: segmented Tab2F kernel (+ 13 for short keys)
hipError_t init_kernels();
bool variant_valid(int variant);
int variant_waves(int variant);
int variant_wgs_per_cu(int variant);
bool variant_desc(int variant);
int variant_complement(int variant);  // kernel for the short keys of a segmented variant (-1: none)
// sorted, 16-packet key-uniform worklist for the descriptor quad kernels (worklist.hip)
size_t quad_worklist_bytes(uint32_t n, uint32_t max_keys, uint32_t *n_items_out);
// Keys with fewer tiles than this are left to a per-wave kernel after the segmented kernel (one
// 16-wave workgroup on a run of one or two tiles per wave would mostly wait at its barrier).
constexpr uint32_t kSegMinTiles = 48;
struct QuadWorklist {
    uint32_t *worklist;      // n_items packet indices, 0xffffffff = padding
    uint32_t *tile_keys;     // key of each 16-entry tile
    uint2 *runs;             // [nruns]: tiles [begin, end) of each present key, in key order
    uint32_t *run_next;      // [nruns]: next tile to hand out of each run, relative (zeroed)
    uint32_t *nruns;         // device word
    uint32_t *short_tiles;   // [nshort]: the tiles of keys with fewer than kSegMinTiles tiles
    uint32_t *nshort;        // device word
    uint32_t *tile_counter;  // zeroed
    uint32_t n_items;
};
// status (may be NULL): the batch's status bytes; the one-workgroup path for small batches zeroes them
// itself (small_worklist(n)), the caller fills them otherwise
hipError_t launch_quad_worklist(const qgcm_desc *descs, uint32_t n, uint32_t max_keys, const uint8_t *key_valid,
                                bool seal, void *ws, size_t ws_bytes, QuadWorklist *out, hipStream_t s,
                                uint8_t *status, bool small);
// a batch of n packets builds its worklist in one workgroup (on: the context's QGCM_SMALL_WORKLIST
// setting); computed once per batch and passed to launch_quad_worklist, so the status fill and the
// worklist build always agree
bool small_worklist(uint32_t n, bool on);
hipError_t launch_packets(bool seal, int variant, const Batch &b, int grid, hipStream_t s);
// One packet, one 512-thread workgroup (qgcm_seal_one / qgcm_open_one): the slot (b.stride bytes,
// a multiple of 16, at most kOneCap - 16) is staged in LDS; b.n must be 1.
constexpr uint32_t kOneCap = 32768;
hipError_t launch_one(bool seal, const Batch &b, hipStream_t s);

// Resident per-packet service (resident.cpp): `workers` 512-thread workgroups of gcm_one_kernel's
// engine stay on the GPU and serve requests the host posts, so a per-packet call costs no launch.
// Slot s belongs to worker s / per_worker.  Requests travel in DEVICE memory (fine-grained, which the
// host CPU writes through the BAR: posted writes, and the GPU polls and reads its own HBM); results
// travel in pinned host memory (the GPU's posted writes, which the host reads from its cache).
// Host -> device: the slot's input bytes into in[s], then req[s].y..w = {op (1 seal, 0 open) |
// aad_len << 1, len, key_idx}, then req[s].x = seq (31-bit, +1 per request), each step fenced
// (sfence: the write-combined stores land in that order).  stop[16 w] != 0 ends worker w.
// Device -> host: the result bytes into out[s], then done[s] = seq << 1 | verdict.  Every access of
// memory the other side writes goes around the GPU caches (16-B sc0 sc1 buffer accesses, system-scope
// atomics for the words).  An instance ends on the host's stop words, or when worker 0 sees no request
// served for idle_ticks or the instance is life_ticks old (100 MHz clock): it raises the device
// shutdown word, every worker serves what its records hold and leaves, and the last one writes
// *over = gen.
constexpr uint32_t kResSlotBytes = 16384;  // request slot: [aad 4][payload][tag 16][nonce 12], 16-B rounded
constexpr uint32_t kResMaxPerWorker = 64;
constexpr size_t kResDevBytes = 64;        // device control words: [0] last activity, [1] shutdown, [2] left
struct ResArgs {
    const uint4 *req;       // device (host-written): [S] request records
    const uint32_t *stop;   // device (host-written): worker w's stop word at 16 w
    const uint8_t *in;      // device (host-written): [S][kResSlotBytes] request bytes
    uint8_t *out;           // host: [S][kResSlotBytes] result bytes
    uint32_t *done;         // host: [S]
    uint32_t *over;         // host: generation of the last instance that ended
    uint32_t *hits;         // host: worker w's count of seals served from a keystream ahead, at 16 w
    uint8_t *dev;           // device control words (kResDevBytes), zeroed per launch
    uint32_t workers, per_worker, gen, pad;
    uint64_t idle_ticks, life_ticks;
};
hipError_t launch_resident(const Batch &b, const ResArgs &a, hipStream_t s);
struct Resident;
// the service's settings, read from the QGCM_RESIDENT_* environment when the context is created (like
// every other QGCM_* knob), not when the service is first started by a per-packet call
struct ResidentConfig {
    uint64_t workers, slots, spin_us, spinners, idle_us, life_us, fail_after;
    bool ahead;  // QGCM_RESIDENT_AHEAD: draw the next nonce and keystream ahead (default on)
};
ResidentConfig resident_config_from_env();
Resident *resident_create(int device, const Batch &base, int num_cus, const ResidentConfig &cfg);  // nullptr: not available
void resident_destroy(Resident *r);
int resident_quiesce(Resident *r);
int resident_workers_running(const Resident *r);
// served, launches, slots, workers running, ahead hits, callers asleep, callers spinning, broken
constexpr int kResStats = 8;
void resident_stats(const Resident *r, uint64_t out[kResStats]);
int resident_pause(Resident *r);  // quiesce and hold new instances back (qgcm_set_keys) ...
void resident_resume(Resident *r);  // ... until this
constexpr long kResNotServed = -1000;  // resident_call: the request does not fit; take the launch path
bool random_nonce(uint8_t out[12]);   // getrandom, buffered per thread, fork-safe (resident.cpp)
long resident_call(Resident *r, bool seal, uint32_t key, uint8_t *data, long len, const uint8_t *aad,
                   uint32_t aad_len, const uint8_t *nonce);
constexpr uint32_t kOneUniformMax = 2048;    // measured cross-over with the quad kernel: 2048-4096 packets
// keyed batches of up to this many packets run one workgroup per packet when their records allow it:
// against the worklist + per-wave kernel it wins up to 8192 (1395 vs 1442 us a seal+open pair at 8192,
// 754 vs 921 at 4096: profiles/r4_s46_s51); the uniform kernel's cross-over is lower
constexpr uint32_t kDescOneMax = 8192;
// a batch sealed in place in pinned host memory (group.cpp run_member_direct, qgcm_seal_host) takes
// that kernel up to this many packets and kDirectMaxBytes of slots: keyed 1.57-1.65 ms a pair at 16384
// against 2.38 by DMA runs, 3.11 against 4.28 at 32768, 6.28-6.30 against 7.23 at 65536, but 12.3
// against 11.7 at 131072; uniform 5.92-5.97 against 6.30 at 65536 (profiles/r4_s52_s54, r4_s55_s56,
// r4_s62)
constexpr uint32_t kDirectMax = 65536;
constexpr uint64_t kDirectMaxBytes = 128ull << 20;
constexpr uint32_t kLaunchChunk = 1u << 20;  // packets per quad-kernel launch of a uniform batch
constexpr uint32_t kDescChunk = 0;           // packets per sorted chunk of a descriptor batch (0 = all)
bool ctx_one_kernel(const qgcm_ctx *ctx);
// the context's host-pipeline streams (0 copy-in, 1 kernels, 2 copy-out) and the mutex that guards them
// (group.cpp's DMA runs use them, as qgcm_seal_host does)
hipStream_t ctx_pipe(qgcm_ctx *ctx, int k);
std::mutex &ctx_io_mu(qgcm_ctx *ctx);
// Small keyed batches whose records the caller has checked (group.cpp's DMA staging): one workgroup
// per descriptor (gcm_one_kernel), no worklist.  descs_one_max: the largest batch that takes it (0:
// off; kDescOneMax, QGCM_DESC_ONE_MAX at qgcm_create; QGCM_VARIANT and QGCM_ONE_KERNEL turn it off as
// for uniform batches, and so does QGCM_DESC_ONE=0 at qgcm_create).  run_descs_one needs every record 16-B aligned in
// device memory, no other record inside its 16-B-rounded area (4 + len (+ 28 on seal), rounded up),
// and that area at most kOneCap - 16 bytes; keys, short opens and statuses behave as in the batch
// kernels.
uint32_t descs_one_max(const qgcm_ctx *ctx);
uint32_t direct_max(const qgcm_ctx *ctx);  // kDirectMax (QGCM_DIRECT_MAX at qgcm_create), 0 when the above is off
// Device-accessible address of pinned host memory [p, p + bytes) inside one allocation, or 0.
uint64_t pinned_view(const void *p, uint64_t bytes);
int run_descs_one(qgcm_ctx *ctx, bool seal, uint8_t *d_arena, const qgcm_desc *d_descs, uint32_t n,
                  const uint8_t *d_nonces, uint32_t aad_len, uint8_t *d_status, hipStream_t s);
hipError_t launch_stream_copy(void *dst, const void *src, uint64_t bytes, int num_cus, hipStream_t s);
// one record move of the group dispatcher's zero-copy path: src/dst device-accessible addresses
// (pinned host or device), 4-B aligned; status_idx: the record's status byte (scatter only)
struct RecMove {
    uint64_t src, dst;
    uint32_t bytes, status_idx;
};
// exact = false (gather): whole dwords, the last may extend past `bytes`; exact = true (scatter):
// exactly `bytes`, and only moves whose status byte is 1 when d_status is given
hipError_t launch_move_records(const RecMove *d_moves, uint32_t n, const uint8_t *d_status, bool exact, int num_cus,
                               hipStream_t s);
// Device snappy codec (snappy_kernels.hip): one wave per Payload.Raw slot at i * stride.
// LDS per wave: [hash table | staged input at off_in | output at off_out | lane scratch at off_sink],
// wave_bytes in all.
constexpr uint32_t kSnapDevMax = 16384;  // longest packet (in and out) the device codec takes
struct SnapArgs {
    uint8_t *arena;
    uint64_t stride;
    uint32_t n;
    uint32_t *lens;             // packet lengths, updated on success
    uint8_t *status;            // 1 ok / 0 failed, may be NULL
    const uint8_t *status_in;   // uncompress: only packets whose status_in is 1 (NULL: all)
    qgcm_desc *descs;           // compress: seal descriptors out {i * stride, len or QGCM_MAX_PAYLOAD, key}
    uint32_t key_idx;
    uint32_t max_in;            // packets longer than this fail
    uint32_t limit;             // compress: longest output kept; uncompress: output capacity
    uint32_t sub;               // uncompress: lens[i] - sub is the compressed length (28 after an open)
    uint32_t off_in, off_out, off_sink, wave_bytes;  // off_sink: 256 B of per-lane scratch
};
// group (compress only): true = snappy_compress_group_kernel, four packets per wave (a.wave_bytes = four
// packet regions of a.off_sink bytes); false = one wave per packet
constexpr uint32_t kSnapGroup = 4;
hipError_t launch_snappy(bool compress, const SnapArgs &a, int waves_per_wg, int grid, hipStream_t s, int group);

// Host worker placement (cpu_topo.cpp): the device's NUMA-local CPUs this process may use (count; 0 when
// sysfs has no answer), one CPU per physical core ordered preferred-first then least busy over a
// sample_ms window, and pinning the calling thread to one CPU.
int gpu_local_cpus(int device, cpu_set_t *out);
std::vector<int> spread_cpus(const cpu_set_t *prefer, int sample_ms);
void pin_to_cpu(int cpu);

hipError_t launch_pw_setup(uint32_t first, uint32_t count, const uint4 *gh_table, uint4 *pw, uint32_t pw_keys,
                           hipStream_t s);
hipError_t launch_key_setup(const uint8_t *d_keys, uint32_t first, uint32_t count, uint32_t *rk_table,
                            uint4 *gh_table, const uint8_t *d_sbox, hipStream_t s);
hipError_t launch_fill_uniform(uint8_t *arena, uint64_t stride, uint32_t n, uint32_t len, uint32_t aad_word,
                               uint64_t seed_payload, uint8_t *nonces, uint64_t seed_nonce, hipStream_t s);

}  // namespace qgcm
