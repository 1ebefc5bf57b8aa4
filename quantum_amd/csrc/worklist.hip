// worklist.hip -- descriptor batches -> key-uniform 16-packet tiles for the quad kernel.
//
// A batch of qgcm_desc (any key mix, any lengths; BASELINE config 3) is ordered by
// (key_idx, length descending) with a device radix sort, then each key's run is padded to a multiple
// of 16 entries so that every 16-packet wave tile uses ONE key (round keys in SGPRs, one GHASH table
// per wave) and holds packets of similar length (the 4-lane quads of a wave finish together).
// Packets that cannot be processed (key index out of range or naming a key slot that was never set,
// open with len < 28, payload of QGCM_MAX_PAYLOAD or more) are left out: their status stays 0 and
// their slot is untouched.  Excluded entries sort last under the all-ones key, which no valid packet
// can produce: key indices stay below QGCM_MAX_KEYS = 2^20 - 1 (qgcm_create caps max_keys).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gcm_internal.h"

namespace qgcm {

constexpr uint32_t kLenBits = 12;  // length rank bits of the sort key; key index in the top 20 bits

// the largest valid key index, QGCM_MAX_KEYS - 1, must sort below the all-ones excluded marker
static_assert(QGCM_MAX_KEYS - 1u < (1u << (32 - kLenBits)) - 1u, "key index would collide with the excluded marker");

__global__ void qwl_keys_kernel(const qgcm_desc *descs, uint32_t n, uint32_t max_keys, const uint8_t *key_valid,
                                bool seal, uint32_t *sort_keys, uint32_t *vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const qgcm_desc d = descs[i];
    uint32_t sk = 0xffffffffu;
    const bool ok = d.key_idx < max_keys && key_valid[d.key_idx] && (seal || d.len >= (uint32_t)QGCM_OVERHEAD) &&
                    d.len - (seal ? 0u : (uint32_t)QGCM_OVERHEAD) < QGCM_MAX_PAYLOAD;
    if (ok) {
        const uint32_t L = seal ? d.len : d.len - QGCM_OVERHEAD;
        const uint32_t nb = min((L + 15u) >> 4, (1u << kLenBits) - 1u);
        sk = (d.key_idx << kLenBits) | ((1u << kLenBits) - 1u - nb);  // longest first within a key
    }
    sort_keys[i] = sk;
    vals[i] = i;
}

// Per-key packet counts from the sorted keys (no atomics: 1M packets on 1024 keys made a
// histogram kernel contention-bound at ~0.2 ms): the first entry of a key run records its start,
// the last one its count.
__global__ void qwl_first_kernel(const uint32_t *sk, uint32_t n, uint32_t *first) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n || sk[j] == 0xffffffffu) return;
    const uint32_t k = sk[j] >> kLenBits;
    if (j == 0 || (sk[j - 1] >> kLenBits) != k) first[k] = j;
}

__global__ void qwl_count_kernel(const uint32_t *sk, uint32_t n, const uint32_t *first, uint32_t *counts) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n || sk[j] == 0xffffffffu) return;
    const uint32_t k = sk[j] >> kLenBits;
    if (j == n - 1 || sk[j + 1] == 0xffffffffu || (sk[j + 1] >> kLenBits) != k) counts[k] = j + 1 - first[k];
}

// Single workgroup: counts -> start (unpadded, sorted order), pstart (padded to 16, worklist), and
// for the segmented kernel the run table (runs[r] = the tiles [begin, end) of the r-th key with at
// least kSegMinTiles tiles) and the list of the other keys' tiles (short_tiles, for the per-wave
// kernel that runs after it).
__global__ void __launch_bounds__(1024) qwl_scan_kernel(const uint32_t *counts, uint32_t max_keys, uint32_t *start,
                                                        uint32_t *pstart, uint2 *runs, uint32_t *short_tiles,
                                                        uint32_t *nruns_nshort) {
    __shared__ uint32_t pu[1024], pp[1024], pr[1024], ps[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (max_keys + 1023) / 1024;
    const uint32_t lo = t * per, hi = min(lo + per, max_keys);
    uint32_t su = 0, sp = 0, sr = 0, ss = 0;
    for (uint32_t k = lo; k < hi; ++k) {
        const uint32_t nt = (counts[k] + 15u) >> 4;
        su += counts[k];
        sp += nt << 4;
        sr += nt >= kSegMinTiles ? 1u : 0u;
        ss += nt < kSegMinTiles ? nt : 0u;
    }
    pu[t] = su;
    pp[t] = sp;
    pr[t] = sr;
    ps[t] = ss;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint32_t a = t >= d ? pu[t - d] : 0, b = t >= d ? pp[t - d] : 0, c = t >= d ? pr[t - d] : 0,
                       e = t >= d ? ps[t - d] : 0;
        __syncthreads();
        pu[t] += a;
        pp[t] += b;
        pr[t] += c;
        ps[t] += e;
        __syncthreads();
    }
    uint32_t ru = pu[t] - su, rp = pp[t] - sp, rr = pr[t] - sr, rs = ps[t] - ss;
    for (uint32_t k = lo; k < hi; ++k) {
        start[k] = ru;
        pstart[k] = rp;
        const uint32_t nt = (counts[k] + 15u) >> 4;
        if (nt >= kSegMinTiles) {
            runs[rr++] = uint2{rp >> 4, (rp >> 4) + nt};
        } else {
            for (uint32_t j = 0; j < nt; ++j) short_tiles[rs++] = (rp >> 4) + j;
        }
        ru += counts[k];
        rp += nt << 4;
    }
    if (t == 1023) {
        nruns_nshort[0] = pr[1023];
        nruns_nshort[1] = ps[1023];
    }
}

// also the key of every tile (the first entry of each 16-entry tile of a key run)
__global__ void qwl_scatter_kernel(const uint32_t *sorted_keys, const uint32_t *sorted_vals, uint32_t n,
                                   const uint32_t *start, const uint32_t *pstart, uint32_t *worklist,
                                   uint32_t *tile_keys) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t sk = sorted_keys[j];
    if (sk == 0xffffffffu) return;
    const uint32_t k = sk >> kLenBits;
    const uint32_t w = pstart[k] + (j - start[k]);
    worklist[w] = sorted_vals[j];
    if ((w & 15u) == 0) tile_keys[w >> 4] = k;
}

// ---- small batches (n <= kSmallWl): the whole worklist in ONE workgroup ----
// A worker-sized batch (a recvmmsg batch, a few thousand packets) spent ~0.15 ms in the ~15 launches
// of the path below (keys, radix sort, per-key counts, scan, scatter, their fills), more than its
// kernels.  Here one 1024-thread workgroup sorts (sort key, index) pairs in LDS (bitonic, so ties keep
// arena order: the key's packets in input order within a length rank, as the stable radix sort leaves
// them), finds each key's segment, and writes the same worklist, tile keys, run table, short-tile list
// and counters the multi-launch path does.
constexpr uint32_t kSmallWl = 4096;
constexpr uint32_t kSmallThreads = 1024;

// exclusive scan of v[0..m) in place (m <= 4 * kSmallThreads); returns the total.  part: kSmallThreads words
__device__ uint32_t wg_exclusive_scan(uint32_t *v, uint32_t m, uint32_t *part) {
    const uint32_t t = threadIdx.x, per = (m + kSmallThreads - 1) / kSmallThreads;
    const uint32_t lo = min(t * per, m), hi = min(lo + per, m);
    uint32_t sum = 0;
    for (uint32_t k = lo; k < hi; ++k) sum += v[k];
    part[t] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < kSmallThreads; d <<= 1) {
        const uint32_t a = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += a;
        __syncthreads();
    }
    uint32_t run = part[t] - sum;
    const uint32_t total = part[kSmallThreads - 1];
    for (uint32_t k = lo; k < hi; ++k) {
        const uint32_t c = v[k];
        v[k] = run;
        run += c;
    }
    __syncthreads();
    return total;
}

__global__ void __launch_bounds__(kSmallThreads)
qwl_small_kernel(const qgcm_desc *descs, uint32_t n, uint32_t max_keys, const uint8_t *key_valid, bool seal,
                 uint32_t items, uint32_t *worklist, uint32_t *tile_keys, uint2 *runs, uint32_t *run_next,
                 uint32_t *short_tiles, uint32_t *counter, uint8_t *status) {
    __shared__ uint64_t e[kSmallWl];                   // (sort key << 32 | index), sorted ascending
    __shared__ uint32_t seg[kSmallWl], aux[kSmallWl];  // per entry, then per segment
    __shared__ uint32_t part[kSmallThreads];
    __shared__ uint32_t nvalid_s;
    const uint32_t t = threadIdx.x;
    uint32_t P = 64;
    while (P < n) P <<= 1;
    for (uint32_t i = t; i < P; i += kSmallThreads) {
        uint32_t sk = 0xffffffffu;
        if (i < n) {
            const qgcm_desc d = descs[i];
            const bool ok = d.key_idx < max_keys && key_valid[d.key_idx] && (seal || d.len >= (uint32_t)QGCM_OVERHEAD) &&
                            d.len - (seal ? 0u : (uint32_t)QGCM_OVERHEAD) < QGCM_MAX_PAYLOAD;
            if (ok) {
                const uint32_t L = seal ? d.len : d.len - QGCM_OVERHEAD;
                const uint32_t nb = min((L + 15u) >> 4, (1u << kLenBits) - 1u);
                sk = (d.key_idx << kLenBits) | ((1u << kLenBits) - 1u - nb);
            }
        }
        e[i] = ((uint64_t)sk << 32) | (i < n ? i : 0xffffffffu);
    }
    for (uint32_t i = t; i < items; i += kSmallThreads) worklist[i] = 0xffffffffu;  // padding entries
    if (status)  // the batch's statuses start at 0 (excluded packets keep it), in place of a separate fill
        for (uint32_t i = t; i < n; i += kSmallThreads) status[i] = 0;
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1)  // bitonic sort, ascending
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = t; i < P; i += kSmallThreads) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint64_t a = e[i], b = e[l];
                    if (((i & k) == 0) == (a > b)) {
                        e[i] = b;
                        e[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    // valid entries (sort key != all ones) come first; a segment starts where the key index changes
    for (uint32_t i = t; i < P; i += kSmallThreads) {
        const uint32_t sk = (uint32_t)(e[i] >> 32);
        const bool valid = sk != 0xffffffffu;
        if (valid && (i + 1 == P || (uint32_t)(e[i + 1] >> 32) == 0xffffffffu)) nvalid_s = i + 1;
        seg[i] = valid && (i == 0 || (uint32_t)(e[i - 1] >> 32) >> kLenBits != sk >> kLenBits) ? 1u : 0u;
    }
    if (t == 0 && (uint32_t)(e[0] >> 32) == 0xffffffffu) nvalid_s = 0;
    __syncthreads();
    const uint32_t nv = nvalid_s;
    const uint32_t S = wg_exclusive_scan(seg, nv, part);  // seg[i]: segment ordinal of i's segment start
    // per segment: start entry (aux), then tiles; entries keep their segment via seg[] after this pass
    for (uint32_t i = t; i < nv; i += kSmallThreads) {
        const bool start = i == 0 || (uint32_t)(e[i - 1] >> 32) >> kLenBits != (uint32_t)(e[i] >> 32) >> kLenBits;
        if (start) aux[seg[i]] = i;
    }
    __syncthreads();
    for (uint32_t i = t; i < nv; i += kSmallThreads) {  // seg[i] = the segment of entry i (its start's ordinal)
        const bool start = i == 0 || (uint32_t)(e[i - 1] >> 32) >> kLenBits != (uint32_t)(e[i] >> 32) >> kLenBits;
        if (!start) {
            uint32_t lo = 0, hi = S;  // the last segment whose start is <= i
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (aux[mid] <= i) lo = mid; else hi = mid;
            }
            seg[i] = lo;
        }
    }
    __syncthreads();
    // segment s: count = next start - start, tiles = ceil(count / 16); tile bases by an exclusive scan
    __shared__ uint32_t tiles[kSmallWl], rflag[kSmallWl], sflag[kSmallWl];
    for (uint32_t q = t; q < S; q += kSmallThreads) {
        const uint32_t cnt = (q + 1 < S ? aux[q + 1] : nv) - aux[q];
        const uint32_t nt = (cnt + 15u) >> 4;
        tiles[q] = nt;
        rflag[q] = nt >= kSegMinTiles ? 1u : 0u;
        sflag[q] = nt >= kSegMinTiles ? 0u : nt;
    }
    __syncthreads();
    // keep the counts: rflag / sflag are scanned in place, tiles too (copied first for the run ends)
    __shared__ uint32_t ntile[kSmallWl];
    for (uint32_t q = t; q < S; q += kSmallThreads) ntile[q] = tiles[q];
    __syncthreads();
    wg_exclusive_scan(tiles, S, part);
    const uint32_t nruns = wg_exclusive_scan(rflag, S, part);
    const uint32_t nshort = wg_exclusive_scan(sflag, S, part);
    for (uint32_t q = t; q < S; q += kSmallThreads) {
        const uint32_t base = tiles[q], nt = ntile[q];
        if (nt >= kSegMinTiles) {
            runs[rflag[q]] = uint2{base, base + nt};
            run_next[rflag[q]] = 0u;
        } else {
            for (uint32_t j = 0; j < nt; ++j) short_tiles[sflag[q] + j] = base + j;
        }
    }
    for (uint32_t i = t; i < nv; i += kSmallThreads) {
        const uint32_t q = seg[i];
        const uint32_t w = tiles[q] * 16u + (i - aux[q]);
        worklist[w] = (uint32_t)e[i];
        if ((w & 15u) == 0) tile_keys[w >> 4] = (uint32_t)(e[i] >> 32) >> kLenBits;
    }
    if (t == 0) {
        counter[0] = 0u;
        counter[1] = nruns;
        counter[2] = nshort;
        counter[3] = 0u;
    }
}

// rocprim's radix sort takes its merge-sort path up to 2^20 items by default (a block sort and ~20
// merge launches, ~150 us for a 2^20-packet batch); Onesweep (a histogram, a scan and one pass per
// 8-bit digit) is used for every size here.
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                              rocprim::default_config, 0>;

static hipError_t sort_pairs(void *tmp, size_t &bytes, const uint32_t *k_in, uint32_t *k_out, const uint32_t *v_in,
                             uint32_t *v_out, uint32_t n, int end_bit, hipStream_t s) {
    return rocprim::radix_sort_pairs<SortConfig>(tmp, bytes, k_in, k_out, v_in, v_out, (size_t)n, 0, end_bit, s);
}

size_t quad_worklist_bytes(uint32_t n, uint32_t max_keys, uint32_t *n_items_out) {
    const uint64_t cap = (uint64_t)n + 16ull * (n < max_keys ? n : max_keys);
    const uint32_t items = (uint32_t)((cap + 15) & ~15ull);
    size_t cub = 0;
    sort_pairs(nullptr, cub, nullptr, nullptr, nullptr, nullptr, n, 32, 0);
    if (n_items_out) *n_items_out = items;
    // keys in/out, vals in/out, counts, start, pstart, run counters, runs, worklist, tile keys, short
    // tiles, tile counter + run count + short count, sort temp (256-B aligned pieces)
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    return 4 * al(4ull * n) + 4 * al(4ull * max_keys) + al(8ull * max_keys) + al(4ull * items) + 2 * al(items / 4) +
           al(16) + al(cub);
}

bool small_worklist(uint32_t n, bool on) { return on && n && n <= kSmallWl; }

hipError_t launch_quad_worklist(const qgcm_desc *descs, uint32_t n, uint32_t max_keys, const uint8_t *key_valid,
                                bool seal, void *ws, size_t ws_bytes, QuadWorklist *out, hipStream_t s,
                                uint8_t *status, bool small) {
    uint32_t items = 0;
    const size_t need = quad_worklist_bytes(n, max_keys, &items);
    if (ws_bytes < need) return hipErrorInvalidValue;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    char *p = static_cast<char *>(ws);
    uint32_t *k_in = (uint32_t *)p;  p += al(4ull * n);
    uint32_t *k_out = (uint32_t *)p; p += al(4ull * n);
    uint32_t *v_in = (uint32_t *)p;  p += al(4ull * n);
    uint32_t *v_out = (uint32_t *)p; p += al(4ull * n);
    // zeroed together: counts, run counters, tile counter + run count + short count
    char *zero0 = p;
    uint32_t *counts = (uint32_t *)p; p += al(4ull * max_keys);
    uint32_t *run_next = (uint32_t *)p; p += al(4ull * max_keys);
    uint32_t *counter = (uint32_t *)p;  p += al(16);  // [0] tile counter, [1] run count, [2] short tiles
    const size_t zero_bytes = (size_t)(p - zero0);
    // all ones together: worklist (padding entries) and tile keys
    char *ones0 = p;
    uint32_t *worklist = (uint32_t *)p; p += al(4ull * items);
    uint32_t *tile_keys = (uint32_t *)p; p += al(items / 4);
    const size_t ones_bytes = (size_t)(p - ones0);
    uint32_t *start = (uint32_t *)p;  p += al(4ull * max_keys);
    uint32_t *pstart = (uint32_t *)p; p += al(4ull * max_keys);
    uint2 *runs = (uint2 *)p; p += al(8ull * max_keys);
    uint32_t *short_tiles = (uint32_t *)p; p += al(items / 4);
    void *cub_tmp = p;
    size_t cub_bytes = need - (size_t)(p - static_cast<char *>(ws));
    hipError_t e;
    if (small) {
        hipLaunchKernelGGL(qwl_small_kernel, dim3(1), dim3(kSmallThreads), 0, s, descs, n, max_keys, key_valid, seal,
                           items, worklist, tile_keys, runs, run_next, short_tiles, counter, status);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        out->worklist = worklist;
        out->tile_keys = tile_keys;
        out->runs = runs;
        out->run_next = run_next;
        out->nruns = counter + 1;
        out->short_tiles = short_tiles;
        out->nshort = counter + 2;
        out->tile_counter = counter;
        out->n_items = items;
        return hipSuccess;
    }
    if ((e = hipMemsetAsync(zero0, 0, zero_bytes, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(ones0, 0xff, ones_bytes, s)) != hipSuccess) return e;
    const int bs = 256, g = (int)((n + bs - 1) / bs);
    if (n) hipLaunchKernelGGL(qwl_keys_kernel, dim3(g), dim3(bs), 0, s, descs, n, max_keys, key_valid, seal, k_in,
                                 v_in);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // only the bits a valid key can use, plus one so that excluded entries (all ones) sort last
    int end_bit = kLenBits + 1;
    while (end_bit < 32 && (1ull << (end_bit - kLenBits - 1)) < max_keys) ++end_bit;
    if ((e = sort_pairs(cub_tmp, cub_bytes, k_in, k_out, v_in, v_out, n, end_bit, s)) != hipSuccess) return e;
    if (n) {
        hipLaunchKernelGGL(qwl_first_kernel, dim3(g), dim3(bs), 0, s, k_out, n, start);
        hipLaunchKernelGGL(qwl_count_kernel, dim3(g), dim3(bs), 0, s, k_out, n, start, counts);
    }
    hipLaunchKernelGGL(qwl_scan_kernel, dim3(1), dim3(1024), 0, s, counts, max_keys, start, pstart, runs,
                       short_tiles, counter + 1);
    if (n) hipLaunchKernelGGL(qwl_scatter_kernel, dim3(g), dim3(bs), 0, s, k_out, v_out, n, start, pstart, worklist,
                                 tile_keys);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    out->worklist = worklist;
    out->tile_keys = tile_keys;
    out->runs = runs;
    out->run_next = run_next;
    out->nruns = counter + 1;
    out->short_tiles = short_tiles;
    out->nshort = counter + 2;
    out->tile_counter = counter;
    out->n_items = items;
    return hipGetLastError();
}

}  // namespace qgcm
