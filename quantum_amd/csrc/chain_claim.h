// chain_claim.h -- the codec work split of the chained snappy + GCM host calls (qgcm_api.cpp
// run_host_chain): host codec workers claim 256-packet items from the FRONT of a
// batch, the device takes whole chunks from the BACK, and neither takes what the other started.
// One 64-bit atomic word holds both ends: front item << 32 | first device chunk.  Header-only (std C++),
// so tests/cpp/san_driver.cpp races it under TSan.
#pragma once
#include <stdint.h>

#include <atomic>

namespace qgcm {

struct ChunkClaims {
    std::atomic<uint64_t> word{0};
    uint64_t total_items = 0;
    uint64_t per_chunk = 1;  // items per chunk (the last chunk may have fewer)

    void reset(uint64_t nchunks, uint64_t items, uint64_t items_per_chunk) {
        total_items = items;
        per_chunk = items_per_chunk;
        word.store(nchunks);  // front item 0, no device chunk yet
    }
    // host worker: the next front item, or -1 once the front reaches the end or a device chunk
    int64_t claim_item() {
        uint64_t st = word.load();
        for (;;) {
            const uint64_t f = st >> 32, dlo = st & 0xffffffffull;
            if (f >= total_items || f / per_chunk >= dlo) return -1;
            if (word.compare_exchange_weak(st, st + (1ull << 32))) return (int64_t)f;
        }
    }
    // device: the last chunk no worker has started, or -1
    int64_t claim_chunk() {
        uint64_t st = word.load();
        for (;;) {
            const uint64_t f = st >> 32, dlo = st & 0xffffffffull;
            if (dlo == 0 || (dlo - 1) * per_chunk < f) return -1;
            if (word.compare_exchange_weak(st, (f << 32) | (dlo - 1))) return (int64_t)(dlo - 1);
        }
    }
    // chunks [device_from(), nchunks) belong to the device
    uint64_t device_from() const { return word.load() & 0xffffffffull; }
};

}  // namespace qgcm
