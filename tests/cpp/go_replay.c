/*
 * go_replay.c -- replays, through include/qgcm.h, the exact C call sequence go/crypto/aes_gpu.go makes
 * when `go test -tags gpu ./crypto` runs the package's own crypto_test.go TestAES plus
 * go/crypto/aes_gpu_test.go (no Go toolchain exists in this image or on the GPU box, so the cgo shim is
 * exercised by its calls, not by cgo).  TEST INFRASTRUCTURE: links the oracle
 * (oracle/_build/liboracle.so) to check every sealed buffer: the nonce the library drew is in the
 * output, so oracle_aesgo_encrypt(key, plaintext, L, aad, that nonce) must reproduce it exactly.
 *
 * The process-wide device set of aes_gpu.go (Devices): created by the first NewAES, from QGCM_DEVICES
 * (aes_gpu_test.go's TestMain sets "0,0": two members on device 0) and QGCM_MAX_PEERS ("64"):
 * qgcm_device_count (only when QGCM_DEVICES is empty) + qgcm_group_create.  NewAES takes a free key slot
 * (recycled ones first), finds its owner (qgcm_group_shard + qgcm_group_ctx) and installs the key there
 * (qgcm_derive_key + qgcm_set_key); Encrypt / Decrypt are qgcm_seal_one / qgcm_open_one on the owner.
 *
 *   TestAES            crypto/crypto_test.go:54-101 TestAES, unchanged, through NewAES: 1472 x 0x01 in a
 *                      1500-B buffer, nil additional data (bytePtr(nil) = NULL, aad_len 0)
 *   TestAESEdges       the shim's guards: no room for tag/nonce (never reaches C), empty payload, Decrypt
 *                      of 0/5/11/12/27 bytes (errOpen before C below 28; libqgcm also returns -1 and
 *                      leaves the bytes untouched), tamper -> zeroed plaintext, an unset slot fails
 *   TestAESConcurrentGoroutines 16 threads x 200 packets through one key, 4-B AAD
 *   TestNewAESAcrossMembers 6 peers' keys spread over both members; each seals on its owner, the other
 *                      member (which never got the key) refuses it, a peer's packet fails under another's key
 *   TestSlotsRecycled  4 x QGCM_MAX_PEERS NewAES calls, every earlier AES collected (its finalizer marks the
 *                      slot's key unset and frees the slot: the stale index then fails both ways): the same
 *                      slots are re-keyed with new keys, each checked against the oracle
 *   TestGPUGroupBatch  NewGPUGroup({0,0}) + GPUGroup.NewAES / Order / NewArena / SealBatch / OpenBatch:
 *                      600 packets of 8 peers (one key slot never set) in Order's order in a pinned arena;
 *                      sealed against the oracle, opened back, a tampered packet zeroed, the unset key's
 *                      packets untouched
 *   TestCreateError    qgcm_create on a device that does not exist: NULL + a message (cError)
 * Usage: go_replay [TestName ...] (default: all).  Prints "--- PASS: Name" per test.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qgcm.h"

/* oracle/gcm_oracle.c (test infrastructure) */
long oracle_aesgo_encrypt(const uint8_t key[32], uint8_t *data, long length, const uint8_t *aad, long aad_len,
                          const uint8_t nonce[12]);

static int failures = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                       \
            return;                                                           \
        }                                                                     \
    } while (0)

static const char kSecret[] = "AES256Key-32Characters1234567890";

/* the sealed buffer data[0:L+28] equals the oracle's seal of `plain` under the nonce it carries */
static int matches_oracle(const uint8_t key[32], const uint8_t *plain, long L, const uint8_t *aad, long aad_len,
                          const uint8_t *sealed) {
    uint8_t *buf = malloc((size_t)L + 28 + 1), nonce[12];
    memcpy(nonce, sealed + L + 16, 12);
    memcpy(buf, plain, (size_t)L);
    int ok = oracle_aesgo_encrypt(key, buf, L, aad, aad_len, nonce) == L + 28 && !memcmp(buf, sealed, (size_t)L + 28);
    free(buf);
    return ok;
}

/* ---- aes_gpu.go's GPUGroup / AES, as C state ---- */
enum { kMaxSlots = 1024 };
struct group {
    qgcm_group *g;
    uint32_t next, max, nfree;
    uint32_t free[kMaxSlots];
    pthread_mutex_t mu;
};
struct aes { /* type AES struct { g, ctx, idx, salt } */
    struct group *g;
    qgcm_ctx *ctx;
    uint32_t idx;
    uint8_t key[32]; /* kept for the oracle only; the Go object holds no key bytes */
};

/* NewGPUGroup */
static struct group *new_group(const int *devs, int n, uint32_t max) {
    char err[QGCM_ERRLEN];
    struct group *gg = calloc(1, sizeof *gg);
    gg->g = qgcm_group_create(devs, n, max, err, sizeof err);
    if (!gg->g) {
        fprintf(stderr, "qgcm_group_create: %s\n", err);
        free(gg);
        return NULL;
    }
    gg->max = max;
    pthread_mutex_init(&gg->mu, NULL);
    return gg;
}

static void release_slot(struct group *gg, uint32_t idx) { /* the AES finalizer: GPUGroup.release */
    qgcm_group_clear_keys(gg->g, idx, 1);
    pthread_mutex_lock(&gg->mu);
    gg->free[gg->nfree++] = idx;
    pthread_mutex_unlock(&gg->mu);
}

/* GPUGroup.NewAES: a free slot (recycled first), its owner, qgcm_derive_key + qgcm_set_key there */
static int group_new_aes(struct group *gg, const uint8_t *secret, size_t slen, const uint8_t *salt, size_t saltlen,
                         struct aes *out) {
    pthread_mutex_lock(&gg->mu);
    uint32_t idx;
    if (gg->nfree) {
        idx = gg->free[--gg->nfree];
    } else if (gg->next < gg->max) {
        idx = gg->next++;
    } else {
        pthread_mutex_unlock(&gg->mu);
        return -1; /* errSlots */
    }
    pthread_mutex_unlock(&gg->mu);
    const int owner = qgcm_group_shard(gg->g, idx);
    qgcm_ctx *ctx = qgcm_group_ctx(gg->g, owner);
    if (!ctx || qgcm_derive_key(secret, slen, salt, saltlen, out->key) != QGCM_OK ||
        qgcm_set_key(ctx, idx, out->key) != QGCM_OK) {
        release_slot(gg, idx);
        return -1;
    }
    out->g = gg;
    out->ctx = ctx;
    out->idx = idx;
    return 0;
}

/* Devices(): the process-wide set, once */
static struct group *g_process;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void devices_once(void) {
    const char *spec = getenv("QGCM_DEVICES");
    int devs[64], n = 0;
    if (!spec || !*spec) {
        n = qgcm_device_count();
        for (int i = 0; i < n && i < 64; ++i) devs[i] = i;
    } else {
        for (const char *p = spec; *p && n < 64;) {
            devs[n++] = atoi(p);
            while (*p && *p != ',') ++p;
            if (*p == ',') ++p;
        }
    }
    const char *mp = getenv("QGCM_MAX_PEERS");
    const uint32_t max = mp && *mp ? (uint32_t)atoi(mp) : 4096u;
    if (n > 0 && max > 0 && max <= kMaxSlots) g_process = new_group(devs, n, max);
}
static struct group *devices(void) {
    pthread_once(&g_once, devices_once);
    return g_process;
}

/* NewAES(secret, salt) */
static int new_aes(const uint8_t *secret, size_t slen, const uint8_t *salt, size_t saltlen, struct aes *out) {
    struct group *gg = devices();
    return gg ? group_new_aes(gg, secret, slen, salt, saltlen, out) : -1;
}

/* AES.Encrypt / AES.Decrypt (the shim's guards, then the C call on the owner) */
static long aes_encrypt(const struct aes *a, uint8_t *data, long cap, long length, const uint8_t *ad, long adlen) {
    if (length < 0 || length + QGCM_OVERHEAD > cap || adlen > 4) return -1;
    return qgcm_seal_one(a->ctx, a->idx, data, length, adlen ? ad : NULL, (uint32_t)adlen, NULL);
}
static long aes_decrypt(const struct aes *a, uint8_t *data, long len, const uint8_t *ad, long adlen) {
    if (len < QGCM_OVERHEAD || adlen > 4) return -1; /* errOpen */
    return qgcm_open_one(a->ctx, a->idx, len ? data : NULL, len, adlen ? ad : NULL, (uint32_t)adlen);
}

static void TestAES(void) {
    uint8_t salt[QGCM_SALT_BYTES];
    for (int i = 0; i < 32; ++i) salt[i] = (uint8_t)(i * 37 + 1); /* TestAES: rand.Read(salt) */
    struct aes a;
    CHECK(new_aes((const uint8_t *)kSecret, 32, salt, 32, &a) == 0);
    enum { bufLen = 1500, dataLen = bufLen - 28 };
    uint8_t buf[bufLen], expected[dataLen];
    memset(buf, 0, sizeof buf);
    memset(buf, 1, dataLen); /* fillSlice(buf[:dataLen]) */
    memset(expected, 1, dataLen);
    long n = aes_encrypt(&a, buf, bufLen, dataLen, NULL, 0); /* aes.Encrypt(buf, dataLen, nil) */
    CHECK(n == bufLen);
    CHECK(memcmp(buf, expected, dataLen) != 0);
    CHECK(matches_oracle(a.key, expected, dataLen, NULL, 0, buf));
    n = aes_decrypt(&a, buf, bufLen, NULL, 0); /* aes.Decrypt(buf, nil) */
    CHECK(n == dataLen);
    CHECK(memcmp(buf, expected, dataLen) == 0);
    printf("--- PASS: TestAES\n");
}

static void TestAESEdges(void) {
    uint8_t salt[32] = {0};
    struct aes a;
    CHECK(new_aes((const uint8_t *)kSecret, 32, salt, 32, &a) == 0);
    const uint8_t ip[4] = {10, 99, 0, 1};
    uint8_t small[27];
    CHECK(aes_encrypt(&a, small, sizeof small, 0, ip, 4) == -1); /* no room for tag and nonce */
    uint8_t empty[28];
    memset(empty, 0xAA, sizeof empty);
    CHECK(aes_encrypt(&a, empty, 28, 0, ip, 4) == 28);
    CHECK(matches_oracle(a.key, empty, 0, ip, 4, empty));
    CHECK(aes_decrypt(&a, empty, 28, ip, 4) == 0);
    const long shorts[] = {0, 5, 11, 12, 27};
    for (unsigned k = 0; k < sizeof shorts / sizeof shorts[0]; ++k) {
        uint8_t s[28], before[28];
        for (int i = 0; i < 28; ++i) s[i] = before[i] = (uint8_t)(i + k);
        CHECK(aes_decrypt(&a, s, shorts[k], ip, 4) == -1); /* the shim answers errOpen */
        /* ... and libqgcm agrees when called directly, leaving the bytes */
        CHECK(qgcm_open_one(a.ctx, a.idx, shorts[k] ? s : NULL, shorts[k], ip, 4) == -1);
        CHECK(memcmp(s, before, sizeof s) == 0);
    }
    uint8_t data[1350 + 28], plain[1350];
    for (int i = 0; i < 1350; ++i) plain[i] = data[i] = 1; /* fillSlice(data[:1350]) */
    CHECK(aes_encrypt(&a, data, sizeof data, 1350, ip, 4) == 1350 + 28);
    CHECK(matches_oracle(a.key, plain, 1350, ip, 4, data));
    uint8_t tail[28];
    memcpy(tail, data + 1350, 28);
    data[7] ^= 1;
    CHECK(aes_decrypt(&a, data, sizeof data, ip, 4) == -1);
    for (int i = 0; i < 1350; ++i) CHECK(data[i] == 0);
    CHECK(memcmp(data + 1350, tail, 28) == 0);
    /* a slot no NewAES filled (a Mapping whose AES was never created) fails, untouched */
    struct aes unset = a;
    unset.idx = a.g->max - 1;
    uint8_t z[64 + 28] = {0};
    if (unset.idx != a.idx) {
        CHECK(aes_encrypt(&unset, z, sizeof z, 64, ip, 4) == -1);
        for (unsigned i = 0; i < sizeof z; ++i) CHECK(z[i] == 0);
    }
    printf("--- PASS: TestAESEdges\n");
}

struct worker {
    const struct aes *a;
    int w, ok;
};

static void *concurrent_worker(void *p) {
    struct worker *k = p;
    uint8_t buf[1472], plain[1472];
    const uint8_t ip[4] = {10, 99, 0, (uint8_t)k->w};
    k->ok = 1;
    for (int i = 0; i < 200 && k->ok; ++i) {
        const long l = (k->w * 131 + i * 17) % 1433;
        for (long j = 0; j < l; ++j) plain[j] = buf[4 + j] = (uint8_t)(k->w + i + j);
        const long n = aes_encrypt(k->a, buf + 4, 1468, l, ip, 4);
        if (n != l + 28 || !matches_oracle(k->a->key, plain, l, ip, 4, buf + 4)) k->ok = 0;
        const long m = aes_decrypt(k->a, buf + 4, n, ip, 4);
        if (m != l || memcmp(buf + 4, plain, (size_t)l)) k->ok = 0;
    }
    return NULL;
}

static void TestAESConcurrentGoroutines(void) {
    uint8_t salt[32] = {0};
    struct aes a;
    CHECK(new_aes((const uint8_t *)kSecret, 32, salt, 32, &a) == 0);
    pthread_t th[16];
    struct worker w[16];
    for (int i = 0; i < 16; ++i) {
        w[i] = (struct worker){&a, i, 0};
        pthread_create(&th[i], NULL, concurrent_worker, &w[i]);
    }
    int ok = 1;
    for (int i = 0; i < 16; ++i) {
        pthread_join(th[i], NULL);
        ok &= w[i].ok;
    }
    CHECK(ok);
    printf("--- PASS: TestAESConcurrentGoroutines\n");
}

static void TestNewAESAcrossMembers(void) {
    struct group *gg = devices();
    CHECK(gg != NULL);
    struct aes peers[6];
    int seen[64] = {0}, members = 0;
    for (int k = 0; k < 6; ++k) {
        uint8_t salt[32];
        memset(salt, 0x70 + k, sizeof salt);
        CHECK(group_new_aes(gg, (const uint8_t *)kSecret, 32, salt, 32, &peers[k]) == 0);
        const int m = qgcm_group_shard(gg->g, peers[k].idx);
        members += !seen[m];
        seen[m] = 1;
    }
    const int size = qgcm_group_size(gg->g);
    CHECK(size < 2 || members >= 2);
    const uint8_t ip[4] = {10, 99, 0, 9};
    for (int k = 0; k < 6; ++k) {
        uint8_t data[500 + 28], plain[500], wrong[500 + 28];
        for (int j = 0; j < 500; ++j) plain[j] = data[j] = (uint8_t)(j + k);
        CHECK(aes_encrypt(&peers[k], data, sizeof data, 500, ip, 4) == 528);
        CHECK(matches_oracle(peers[k].key, plain, 500, ip, 4, data));
        /* another member never got this key: it refuses the slot and leaves the buffer */
        if (size > 1) {
            const int owner = qgcm_group_shard(gg->g, peers[k].idx);
            qgcm_ctx *other = qgcm_group_ctx(gg->g, (owner + 1) % size);
            memcpy(wrong, data, sizeof data);
            CHECK(qgcm_open_one(other, peers[k].idx, wrong, sizeof wrong, ip, 4) == -1);
            CHECK(memcmp(wrong, data, sizeof data) == 0);
        }
        /* another peer's key does not open it */
        memcpy(wrong, data, sizeof data);
        CHECK(aes_decrypt(&peers[(k + 1) % 6], wrong, sizeof wrong, ip, 4) == -1);
        CHECK(aes_decrypt(&peers[k], data, sizeof data, ip, 4) == 500);
        CHECK(memcmp(data, plain, 500) == 0);
    }
    printf("--- PASS: TestNewAESAcrossMembers\n");
}

static void TestSlotsRecycled(void) {
    struct group *gg = devices();
    CHECK(gg != NULL);
    struct aes prev = {0};
    int have_prev = 0;
    for (uint32_t i = 0; i < 4 * gg->max; ++i) {
        if (have_prev) {
            release_slot(gg, prev.idx); /* runtime.GC(): the previous AES was collected */
            /* a KeyIndex kept past its AES (a batch Desc) now fails, in both directions, bytes untouched */
            uint8_t z[64 + 28], zb[64 + 28];
            for (int j = 0; j < 64 + 28; ++j) z[j] = zb[j] = (uint8_t)(j * 3 + i);
            CHECK(qgcm_seal_one(prev.ctx, prev.idx, z, 64, NULL, 0, NULL) == -1);
            CHECK(qgcm_open_one(prev.ctx, prev.idx, z, 64 + 28, NULL, 0) == -1);
            CHECK(memcmp(z, zb, sizeof z) == 0);
        }
        uint8_t salt[32];
        memset(salt, (int)(i * 13 + 5), sizeof salt); /* every NewAES a different key */
        struct aes a;
        CHECK(new_aes((const uint8_t *)kSecret, 32, salt, 32, &a) == 0);
        uint8_t buf[64 + 28], plain[64];
        for (int j = 0; j < 64; ++j) plain[j] = buf[j] = (uint8_t)(i + j);
        CHECK(aes_encrypt(&a, buf, sizeof buf, 64, NULL, 0) == 92);
        CHECK(matches_oracle(a.key, plain, 64, NULL, 0, buf)); /* the slot's NEW key, not a cached one */
        CHECK(aes_decrypt(&a, buf, sizeof buf, NULL, 0) == 64);
        CHECK(memcmp(buf, plain, 64) == 0);
        prev = a;
        have_prev = 1;
    }
    printf("--- PASS: TestSlotsRecycled\n");
}

static void TestGPUGroupBatch(void) {
    const int devs[2] = {0, 0}; /* NewGPUGroup([]int{0, 0}, 16) */
    struct group *gg = new_group(devs, 2, 16);
    CHECK(gg != NULL);
    enum { kPeers = 8, kN = 600 };
    struct aes peers[kPeers];
    uint32_t keyOf[kPeers];
    for (uint32_t k = 0; k < kPeers - 1; ++k) { /* GPUGroup.NewAES; slot 7 is never set */
        uint8_t salt[32];
        memset(salt, (int)(0x40 + k), sizeof salt);
        CHECK(group_new_aes(gg, (const uint8_t *)kSecret, 32, salt, 32, &peers[k]) == 0);
        keyOf[k] = peers[k].idx;
    }
    keyOf[kPeers - 1] = kPeers - 1;
    uint32_t peer[kN], order[kN], counts[2];
    for (uint32_t i = 0; i < kN; ++i) peer[i] = keyOf[(i * 7 + i / 5) % kPeers];
    CHECK(qgcm_group_order(gg->g, peer, kN, order, counts) == QGCM_OK); /* GPUGroup.Order */
    CHECK(counts[0] + counts[1] == kN);
    qgcm_desc d[kN];
    uint64_t off = 0;
    for (uint32_t j = 0; j < kN; ++j) {
        const uint32_t i = order[j], L = 1 + (i * 37) % 1400;
        d[j] = (qgcm_desc){off, L, peer[i]};
        off += (4 + L + 28 + 15) & ~15ull;
    }
    uint8_t *arena = qgcm_host_alloc(off), *plain = malloc(off), *nonces = qgcm_host_alloc(12 * kN); /* NewArena */
    uint8_t status[kN];
    CHECK(arena && plain && nonces);
    for (uint64_t b = 0; b < off; ++b) arena[b] = (uint8_t)(b * 131 + 7);
    memcpy(plain, arena, off);
    int ok = qgcm_random_nonces(nonces, kN) == QGCM_OK; /* SealBatch */
    int unset = 0;
    for (uint32_t j = 0; j < kN; ++j) unset += d[j].key_idx == kPeers - 1;
    ok &= qgcm_group_seal_host(gg->g, arena, d, kN, nonces, 4, status) == unset;
    for (uint32_t j = 0; j < kN && ok; ++j) {
        const uint8_t *slot = arena + d[j].offset, *pslot = plain + d[j].offset;
        if (d[j].key_idx == kPeers - 1) {
            ok &= status[j] == 0 && !memcmp(slot, pslot, 4 + d[j].len + 28);
        } else {
            const struct aes *a = NULL;
            for (int k = 0; k < kPeers - 1; ++k)
                if (peers[k].idx == d[j].key_idx) a = &peers[k];
            ok &= a != NULL && status[j] == 1 && !memcmp(slot + 4 + d[j].len + 16, nonces + 12 * j, 12);
            ok &= a != NULL && matches_oracle(a->key, pslot + 4, d[j].len, pslot, 4, slot + 4);
        }
    }
    uint32_t victim = 0;
    while (d[victim].key_idx == kPeers - 1) ++victim;
    arena[d[victim].offset + 4] ^= 1; /* tamper with one ciphertext */
    for (uint32_t j = 0; j < kN; ++j) d[j].len += 28; /* OpenBatch: sealed lengths */
    ok &= qgcm_group_open_host(gg->g, arena, d, kN, 4, status) == unset + 1;
    for (uint32_t j = 0; j < kN && ok; ++j) {
        const uint32_t L = d[j].len - 28;
        const uint8_t *slot = arena + d[j].offset, *pslot = plain + d[j].offset;
        if (d[j].key_idx == kPeers - 1) {
            ok &= status[j] == 0 && !memcmp(slot, pslot, 4 + L + 28);
            continue;
        }
        if (j == victim) {
            ok &= status[j] == 0;
            for (uint32_t b = 0; b < L; ++b) ok &= slot[4 + b] == 0;
        } else {
            ok &= status[j] == 1 && !memcmp(slot, pslot, 4 + L);
        }
    }
    qgcm_host_free(arena);
    qgcm_host_free(nonces);
    free(plain);
    qgcm_group_destroy(gg->g); /* GPUGroup.Close */
    free(gg);
    CHECK(ok);
    printf("--- PASS: TestGPUGroupBatch\n");
}

static void TestCreateError(void) {
    char err[QGCM_ERRLEN] = {0};
    CHECK(qgcm_create(4096, 16, err, sizeof err) == NULL);
    CHECK(err[0] != 0);
    printf("--- PASS: TestCreateError\n");
}

static int want(int argc, char **argv, const char *name) {
    if (argc < 2) return 1;
    for (int i = 1; i < argc; ++i)
        if (!strcmp(argv[i], name)) return 1;
    return 0;
}

int main(int argc, char **argv) {
    /* aes_gpu_test.go TestMain */
    if (!getenv("QGCM_DEVICES") || !*getenv("QGCM_DEVICES")) setenv("QGCM_DEVICES", "0,0", 1);
    if (!getenv("QGCM_MAX_PEERS") || !*getenv("QGCM_MAX_PEERS")) setenv("QGCM_MAX_PEERS", "64", 1);
    if (want(argc, argv, "TestAES")) TestAES();
    if (want(argc, argv, "TestAESEdges")) TestAESEdges();
    if (want(argc, argv, "TestAESConcurrentGoroutines")) TestAESConcurrentGoroutines();
    if (want(argc, argv, "TestNewAESAcrossMembers")) TestNewAESAcrossMembers();
    if (want(argc, argv, "TestSlotsRecycled")) TestSlotsRecycled();
    if (want(argc, argv, "TestGPUGroupBatch")) TestGPUGroupBatch();
    if (want(argc, argv, "TestCreateError")) TestCreateError();
    if (g_process) {
        qgcm_group_destroy(g_process->g);
        free(g_process);
    }
    return failures ? 1 : 0;
}
