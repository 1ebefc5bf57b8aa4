/*
 * go_replay.c -- replays, through include/qgcm.h, the exact C call sequence go/crypto/gpu_aes.go
 * makes when go/crypto/gpu_aes_test.go runs (no Go toolchain exists in this image or on the GPU box,
 * so the cgo shim is exercised by its calls, not by cgo).  TEST INFRASTRUCTURE: links the oracle
 * (oracle/_build/liboracle.so) to check every sealed buffer: the nonce the library drew is in the
 * output, so oracle_aesgo_encrypt(key, plaintext, L, aad, that nonce) must reproduce it exactly.
 *
 *   TestGPUAES        crypto/crypto_test.go:54-101 TestAES: 1472 x 0x01 in a 1500-B buffer, nil
 *                     additional data (bytePtr(nil) = NULL, aad_len 0), Encrypt -> 1500, Decrypt -> 1472
 *   TestGPUAESEdges   the shim's guards: no room for tag/nonce (never reaches C), empty payload,
 *                     Decrypt of 0/5/11/12/27 bytes (-> errOpen before C below 28; libqgcm also
 *                     returns -1 and leaves the bytes untouched when called), tamper -> zeroed plaintext
 *   TestGPUAESConcurrent 16 threads x 200 packets through one key with qgcm_seal_one/open_one, 4-B AAD
 *   TestGPUGroup      NewGPUGroup + NewGPUAES: key installed on the owning member only, calls on it
 *   TestGPUGroupBatch GPUGroup.Order / NewArena / SealBatch / OpenBatch: 600 packets of 8 peers (one key
 *                     slot never set) laid out in Order's order in a pinned arena; sealed against the
 *                     oracle, opened back, a tampered packet zeroed, the unset key's packets untouched
 *   TestCreateError   qgcm_create on a device that does not exist: NULL + a message (cError)
 * Usage: go_replay [TestName ...] (default: all).  Prints "--- PASS: Name" per test.
 */
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

/* installKey: qgcm_derive_key + qgcm_set_key, returning the key for the oracle */
static int install_key(qgcm_ctx *ctx, uint32_t idx, const uint8_t *salt, uint8_t key[32]) {
    if (qgcm_derive_key((const uint8_t *)kSecret, 32, salt, 32, key) != QGCM_OK) return -1;
    return qgcm_set_key(ctx, idx, key);
}

/* the sealed buffer data[0:L+28] equals the oracle's seal of `plain` under the nonce it carries */
static int matches_oracle(const uint8_t key[32], const uint8_t *plain, long L, const uint8_t *aad, long aad_len,
                          const uint8_t *sealed) {
    uint8_t *buf = malloc((size_t)L + 28), nonce[12];
    memcpy(nonce, sealed + L + 16, 12);
    memcpy(buf, plain, (size_t)L);
    int ok = oracle_aesgo_encrypt(key, buf, L, aad, aad_len, nonce) == L + 28 && !memcmp(buf, sealed, (size_t)L + 28);
    free(buf);
    return ok;
}

static void TestGPUAES(qgcm_ctx *ctx) {
    uint8_t salt[32], key[32];
    for (int i = 0; i < 32; ++i) salt[i] = (uint8_t)(i * 37 + 1); /* TestAES: a random salt */
    CHECK(install_key(ctx, 0, salt, key) == QGCM_OK);
    enum { bufLen = 1500, dataLen = bufLen - 28 };
    uint8_t buf[bufLen], expected[dataLen];
    memset(buf, 0, sizeof buf);
    memset(buf, 1, dataLen); /* fillSlice(buf[:dataLen]) */
    memset(expected, 1, dataLen);
    /* aes.Encrypt(buf, dataLen, nil): bytePtr(nil) = NULL, len 0; seal_one with nonce NULL (getrandom) */
    long n = qgcm_seal_one(ctx, 0, buf, dataLen, NULL, 0, NULL);
    CHECK(n == bufLen);
    CHECK(memcmp(buf, expected, dataLen) != 0);
    CHECK(matches_oracle(key, expected, dataLen, NULL, 0, buf));
    n = qgcm_open_one(ctx, 0, buf, bufLen, NULL, 0); /* aes.Decrypt(buf, nil) */
    CHECK(n == dataLen);
    CHECK(memcmp(buf, expected, dataLen) == 0);
    printf("--- PASS: TestGPUAES\n");
}

static void TestGPUAESEdges(qgcm_ctx *ctx) {
    uint8_t salt[32] = {0}, key[32];
    CHECK(install_key(ctx, 1, salt, key) == QGCM_OK);
    const uint8_t ip[4] = {10, 99, 0, 1};
    /* empty payload: Encrypt(make([]byte, 28), 0, ip) -> 28, Decrypt -> 0 */
    uint8_t empty[28];
    memset(empty, 0xAA, sizeof empty);
    CHECK(qgcm_seal_one(ctx, 1, empty, 0, ip, 4, NULL) == 28);
    CHECK(matches_oracle(key, empty, 0, ip, 4, empty));
    CHECK(qgcm_open_one(ctx, 1, empty, 28, ip, 4) == 0);
    /* short Decrypt inputs: the shim answers errOpen itself below 28; the C call agrees and leaves them */
    const long shorts[] = {0, 5, 11, 12, 27};
    for (unsigned k = 0; k < sizeof shorts / sizeof shorts[0]; ++k) {
        uint8_t s[28], before[28];
        for (int i = 0; i < 28; ++i) s[i] = before[i] = (uint8_t)(i + k);
        CHECK(qgcm_open_one(ctx, 1, shorts[k] ? s : NULL, shorts[k], ip, 4) == -1);
        CHECK(memcmp(s, before, sizeof s) == 0);
    }
    /* tamper: Decrypt fails with the plaintext zeroed, tag and nonce untouched */
    uint8_t data[1350 + 28], plain[1350];
    for (int i = 0; i < 1350; ++i) plain[i] = data[i] = (uint8_t)(i * 7);
    CHECK(qgcm_seal_one(ctx, 1, data, 1350, ip, 4, NULL) == 1350 + 28);
    CHECK(matches_oracle(key, plain, 1350, ip, 4, data));
    uint8_t tail[28];
    memcpy(tail, data + 1350, 28);
    data[7] ^= 1;
    CHECK(qgcm_open_one(ctx, 1, data, sizeof data, ip, 4) == -1);
    for (int i = 0; i < 1350; ++i) CHECK(data[i] == 0);
    CHECK(memcmp(data + 1350, tail, 28) == 0);
    /* an unset key slot (a Mapping whose AES was never created) fails, untouched */
    uint8_t z[64 + 28] = {0};
    CHECK(qgcm_seal_one(ctx, 63, z, 64, ip, 4, NULL) == -1);
    for (unsigned i = 0; i < sizeof z; ++i) CHECK(z[i] == 0);
    printf("--- PASS: TestGPUAESEdges\n");
}

struct worker {
    qgcm_ctx *ctx;
    const uint8_t *key;
    int w, ok;
};

static void *concurrent_worker(void *p) {
    struct worker *a = p;
    uint8_t buf[1472], plain[1472];
    const uint8_t ip[4] = {10, 99, 0, (uint8_t)a->w};
    a->ok = 1;
    for (int i = 0; i < 200 && a->ok; ++i) {
        const long l = (a->w * 131 + i * 17) % 1433;
        for (long j = 0; j < l; ++j) plain[j] = buf[4 + j] = (uint8_t)(a->w + i + j);
        const long n = qgcm_seal_one(a->ctx, 2, buf + 4, l, ip, 4, NULL);
        if (n != l + 28 || !matches_oracle(a->key, plain, l, ip, 4, buf + 4)) a->ok = 0;
        const long m = qgcm_open_one(a->ctx, 2, buf + 4, n, ip, 4);
        if (m != l || memcmp(buf + 4, plain, (size_t)l)) a->ok = 0;
    }
    return NULL;
}

static void TestGPUAESConcurrent(qgcm_ctx *ctx) {
    uint8_t salt[32], key[32];
    for (int i = 0; i < 32; ++i) salt[i] = (uint8_t)(255 - i);
    CHECK(install_key(ctx, 2, salt, key) == QGCM_OK);
    pthread_t th[16];
    struct worker a[16];
    for (int w = 0; w < 16; ++w) {
        a[w] = (struct worker){ctx, key, w, 0};
        pthread_create(&th[w], NULL, concurrent_worker, &a[w]);
    }
    int ok = 1;
    for (int w = 0; w < 16; ++w) {
        pthread_join(th[w], NULL);
        ok &= a[w].ok;
    }
    CHECK(ok);
    printf("--- PASS: TestGPUAESConcurrent\n");
}

static void TestGPUGroup(void) {
    const int devs[2] = {0, 0}; /* a node's GPUs, stood in for by two contexts on device 0 */
    char err[QGCM_ERRLEN];
    qgcm_group *g = qgcm_group_create(devs, 2, 16, err, sizeof err);
    CHECK(g != NULL);
    CHECK(qgcm_group_size(g) == 2);
    int ok = 1;
    for (uint32_t idx = 0; idx < 6 && ok; ++idx) { /* GPUGroup.NewGPUAES */
        const int owner = qgcm_group_shard(g, idx);
        qgcm_ctx *c = qgcm_group_ctx(g, owner), *other = qgcm_group_ctx(g, 1 - owner);
        uint8_t salt[32], key[32];
        memset(salt, (int)idx, sizeof salt);
        ok &= install_key(c, idx, salt, key) == QGCM_OK;
        uint8_t data[100 + 28], plain[100];
        for (int i = 0; i < 100; ++i) plain[i] = data[i] = (uint8_t)(i ^ idx);
        ok &= qgcm_seal_one(c, idx, data, 100, NULL, 0, NULL) == 128 && matches_oracle(key, plain, 100, NULL, 0, data);
        ok &= qgcm_open_one(other, idx, data, 128, NULL, 0) == -1; /* the key lives on its owner only */
        ok &= memcmp(data, plain, 100) != 0;                         /* ... and was left untouched */
        ok &= qgcm_open_one(c, idx, data, 128, NULL, 0) == 100 && !memcmp(data, plain, 100);
    }
    qgcm_group_destroy(g);
    CHECK(ok);
    printf("--- PASS: TestGPUGroup\n");
}

static void TestGPUGroupBatch(void) {
    const int devs[2] = {0, 0};
    char err[QGCM_ERRLEN];
    qgcm_group *g = qgcm_group_create(devs, 2, 16, err, sizeof err);
    CHECK(g != NULL);
    enum { kPeers = 8, kN = 600 };
    uint8_t keys[kPeers][32];
    for (uint32_t k = 0; k < kPeers - 1; ++k) { /* NewGPUAES on the owner; slot 7 is never set */
        uint8_t salt[32];
        memset(salt, (int)(0x40 + k), sizeof salt);
        CHECK(install_key(qgcm_group_ctx(g, qgcm_group_shard(g, k)), k, salt, keys[k]) == QGCM_OK);
    }
    uint32_t peer[kN], order[kN], counts[2];
    for (uint32_t i = 0; i < kN; ++i) peer[i] = (i * 7 + i / 5) % kPeers;
    CHECK(qgcm_group_order(g, peer, kN, order, counts) == QGCM_OK); /* GPUGroup.Order */
    CHECK(counts[0] + counts[1] == kN);
    /* NewArena: slot j (the order[j]-th packet) = [AAD 4][L payload][28], 16-B aligned slots */
    qgcm_desc d[kN];
    uint64_t off = 0;
    for (uint32_t j = 0; j < kN; ++j) {
        const uint32_t i = order[j], L = 1 + (i * 37) % 1400;
        d[j] = (qgcm_desc){off, L, peer[i]};
        off += (4 + L + 28 + 15) & ~15ull;
    }
    uint8_t *arena = qgcm_host_alloc(off), *plain = malloc(off), *nonces = qgcm_host_alloc(12 * kN);
    uint8_t status[kN];
    CHECK(arena && plain && nonces);
    for (uint64_t b = 0; b < off; ++b) arena[b] = (uint8_t)(b * 131 + 7);
    memcpy(plain, arena, off);
    int ok = qgcm_random_nonces(nonces, kN) == QGCM_OK; /* SealBatch */
    int unset = 0;
    for (uint32_t j = 0; j < kN; ++j) unset += d[j].key_idx == kPeers - 1;
    ok &= qgcm_group_seal_host(g, arena, d, kN, nonces, 4, status) == unset;
    for (uint32_t j = 0; j < kN && ok; ++j) {
        const uint8_t *slot = arena + d[j].offset, *pslot = plain + d[j].offset;
        if (d[j].key_idx == kPeers - 1) {
            ok &= status[j] == 0 && !memcmp(slot, pslot, 4 + d[j].len + 28);
        } else {
            ok &= status[j] == 1 && !memcmp(slot + 4 + d[j].len + 16, nonces + 12 * j, 12);
            ok &= matches_oracle(keys[d[j].key_idx], pslot + 4, d[j].len, pslot, 4, slot + 4);
        }
    }
    uint32_t victim = 0;
    while (d[victim].key_idx == kPeers - 1) ++victim;
    arena[d[victim].offset + 4] ^= 1; /* tamper with one ciphertext */
    for (uint32_t j = 0; j < kN; ++j) d[j].len += 28; /* OpenBatch: sealed lengths */
    ok &= qgcm_group_open_host(g, arena, d, kN, 4, status) == unset + 1;
    for (uint32_t j = 0; j < kN && ok; ++j) {
        const uint32_t L = d[j].len - 28;
        const uint8_t *slot = arena + d[j].offset, *pslot = plain + d[j].offset;
        if (d[j].key_idx == kPeers - 1) { /* never set: status 0, the slot still as it came */
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
    qgcm_group_destroy(g);
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
    char err[QGCM_ERRLEN];
    qgcm_ctx *ctx = NULL;
    if (want(argc, argv, "TestGPUAES") || want(argc, argv, "TestGPUAESEdges") ||
        want(argc, argv, "TestGPUAESConcurrent")) {
        ctx = qgcm_create(0, 64, err, sizeof err); /* NewGPUContext(0, 64) */
        if (!ctx) {
            fprintf(stderr, "qgcm_create: %s\n", err);
            return 1;
        }
    }
    if (want(argc, argv, "TestGPUAES")) TestGPUAES(ctx);
    if (want(argc, argv, "TestGPUAESEdges")) TestGPUAESEdges(ctx);
    if (want(argc, argv, "TestGPUAESConcurrent")) TestGPUAESConcurrent(ctx);
    if (want(argc, argv, "TestGPUGroup")) TestGPUGroup();
    if (want(argc, argv, "TestGPUGroupBatch")) TestGPUGroupBatch();
    if (want(argc, argv, "TestCreateError")) TestCreateError();
    if (ctx) qgcm_destroy(ctx);
    return failures ? 1 : 0;
}
