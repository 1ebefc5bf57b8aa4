// Host-code sanitizer driver ("use TSan/ASan on host lib tests").  Built by
// tests/test_host_sanitizers.py together with the host-only sources of libqgcm (snappy codec,
// key math) under -fsanitize=address,undefined or -fsanitize=thread; no GPU code is involved.
//   snappy: round trips of structured/random inputs; decoding of random and corrupted streams into
//           EXACT-size heap buffers (an overrun is an ASan report); the multi-threaded slot
//           compress/uncompress (TSan).
//   keymath: PBKDF2-HMAC-SHA512 and X25519 on a fixed vector (UB / overruns).
//   chain_claim.h: host workers claiming items from the front while the device claims chunks from
//           the back (TSan): every item is taken exactly once, by one side, and a device chunk by
//           no worker.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <random>
#include <thread>
#include <vector>

#include "../../quantum_amd/csrc/chain_claim.h"
#include "qgcm.h"

static int fail(const char *what) {
    fprintf(stderr, "FAIL: %s\n", what);
    return 1;
}

int main(int argc, char **argv) {
    const bool threads_only = argc > 1 && !strcmp(argv[1], "threads");
    std::mt19937_64 rng(12345);
    if (!threads_only) {
        // round trips
        for (int it = 0; it < 300; ++it) {
            const size_t n = (it % 7 == 0) ? rng() % 70000 : rng() % 3000;
            std::vector<uint8_t> src(n);
            const int mode = it % 3;
            for (size_t i = 0; i < n; ++i)
                src[i] = mode == 0 ? (uint8_t)rng() : mode == 1 ? (uint8_t)("quantum "[i % 8]) : (uint8_t)(i / 97);
            std::vector<uint8_t> comp(qgcm_snappy_max_compressed_length(n));
            const long c = qgcm_snappy_compress(src.data(), n, comp.data(), comp.size());
            if (c < 0) return fail("compress");
            std::vector<uint8_t> exact(c);  // exact-size input buffer: any over-read is reported
            memcpy(exact.data(), comp.data(), (size_t)c);
            if (qgcm_snappy_uncompressed_length(exact.data(), exact.size()) != (long)n) return fail("length");
            std::vector<uint8_t> out(n ? n : 1);
            if (qgcm_snappy_uncompress(exact.data(), exact.size(), out.data(), n) != (long)n) return fail("uncompress");
            if (n && memcmp(out.data(), src.data(), n)) return fail("round trip");
        }
        // malformed streams into exact-size buffers
        for (int it = 0; it < 20000; ++it) {
            const size_t m = 1 + rng() % 64;
            std::vector<uint8_t> junk(m);
            for (auto &b : junk) b = (uint8_t)rng();
            if (it % 2) junk[0] = (uint8_t)(rng() % 64);  // plausible small preamble
            const long want = qgcm_snappy_uncompressed_length(junk.data(), junk.size());
            if (want < 0 || want > 4096) continue;
            std::vector<uint8_t> out(want ? want : 1);
            const long got = qgcm_snappy_uncompress(junk.data(), junk.size(), out.data(), (size_t)want);
            if (got >= 0 && got != want) return fail("decoded length differs from the preamble");
        }
        // key math
        uint8_t key[32], pub[32], sec[32], priv[32];
        for (int i = 0; i < 32; ++i) priv[i] = (uint8_t)(i * 9 + 1);
        if (qgcm_derive_key((const uint8_t *)"AES256Key-32Characters1234567890", 32, (const uint8_t *)"salt", 4, key))
            return fail("pbkdf2");
        static const uint8_t want_key[4] = {0xed, 0x4f, 0x3d, 0xcd};  // SURVEY.md §8c vector prefix
        if (memcmp(key, want_key, 4)) return fail("pbkdf2 vector");
        if (qgcm_x25519_base(pub, priv) || qgcm_x25519(sec, priv, pub)) return fail("x25519");
    }
    // threaded slot codec (TSan)
    const uint32_t n = 4096;
    const uint64_t stride = 1472;
    std::vector<uint8_t> arena(n * stride), plain;
    std::vector<uint32_t> lens(n);
    for (uint32_t i = 0; i < n; ++i) {
        lens[i] = 64 + (uint32_t)(rng() % 1300);
        for (uint32_t j = 0; j < lens[i]; ++j) arena[i * stride + 4 + j] = (uint8_t)((j % 5 == 0) ? rng() : j);
    }
    plain = arena;
    std::vector<uint32_t> orig = lens;
    if (qgcm_snappy_compress_slots(arena.data(), stride, n, lens.data(), 8) != 0) return fail("compress_slots");
    std::vector<uint8_t> st(n);
    if (qgcm_snappy_uncompress_slots(arena.data(), stride, n, lens.data(), st.data(), 8) != 0)
        return fail("uncompress_slots");
    for (uint32_t i = 0; i < n; ++i)
        if (lens[i] != orig[i] || memcmp(&arena[i * stride + 4], &plain[i * stride + 4], orig[i]))
            return fail("slot round trip");
    // the chained codec's front/back claims (chain_claim.h) from 8 worker threads and a device thread
    for (int round = 0; round < 200; ++round) {
        const uint64_t per = 1 + rng() % 40, nchunks = 1 + rng() % 24;
        const uint64_t items = (nchunks - 1) * per + 1 + rng() % per;  // a short last chunk
        qgcm::ChunkClaims cl;
        cl.reset(nchunks, items, per);
        std::vector<std::atomic<int>> owner(items);
        for (auto &o : owner) o = 0;
        std::vector<std::atomic<int>> dev_chunk(nchunks);
        for (auto &d : dev_chunk) d = 0;
        std::vector<std::thread> ws;
        for (int t = 0; t < 8; ++t)
            ws.emplace_back([&] {
                for (int64_t it; (it = cl.claim_item()) >= 0;) owner[it].fetch_add(1);
            });
        std::thread dev([&] {
            for (int64_t c; (c = cl.claim_chunk()) >= 0;) {
                dev_chunk[c].fetch_add(1);
                for (uint64_t it = c * per; it < items && it < (c + 1) * per; ++it) owner[it].fetch_add(100);
                std::this_thread::yield();
            }
        });
        for (auto &w : ws) w.join();
        dev.join();
        const uint64_t dlo = cl.device_from();
        for (uint64_t it = 0; it < items; ++it) {
            const int o = owner[it].load();
            if (o != (it / per >= dlo ? 100 : 1)) return fail("chain claims: an item taken twice, by both sides or never");
        }
        for (uint64_t c = 0; c < nchunks; ++c)
            if (dev_chunk[c].load() != (c >= dlo ? 1 : 0)) return fail("chain claims: device chunks");
    }
    printf("sanitizer driver ok\n");
    return 0;
}
