/*
 * oracle/ossl_check.c -- TEST INFRASTRUCTURE ONLY.
 *
 * An independent third-party implementation of the same standards the reference's
 * Go 1.9 stdlib implements (OpenSSL 3 libcrypto: EVP_aes_256_gcm, PKCS5_PBKDF2_HMAC
 * with SHA-512, X25519).  Used for two things only:
 *   1. cross-checking the plain-C restatement (gcm_oracle.c) and generating golden
 *      fixtures (tests/golden/, script tests/golden/make_golden.py);
 *   2. the CPU baseline leg of bench.py: crypto/aes.go semantics (crypto/aes.go:41-62:
 *      per-packet 12-B getrandom nonce, Seal in place, ct||tag||nonce, 4-B AAD) on
 *      OpenSSL's AES-NI/VPCLMULQDQ GCM -- the same instruction class as Go's
 *      gcm_amd64.s -- over common.Payload framing, one worker thread per core the way
 *      quantum runs NumWorkers pinned goroutines (worker/outgoing.go:83-93).
 * Never linked into the product path.
 */
#include <openssl/evp.h>
#include <openssl/rand.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>
#include <time.h>

int ossl_gcm_seal(const uint8_t key[32], const uint8_t iv[12], const uint8_t *aad, int aad_len,
                  const uint8_t *pt, int len, uint8_t *ct, uint8_t tag[16]) {
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    int out = 0, ok = 1;
    ok &= EVP_EncryptInit_ex(c, EVP_aes_256_gcm(), NULL, key, iv);
    if (aad_len) ok &= EVP_EncryptUpdate(c, NULL, &out, aad, aad_len);
    if (len) ok &= EVP_EncryptUpdate(c, ct, &out, pt, len);
    ok &= EVP_EncryptFinal_ex(c, ct + len, &out);
    ok &= EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, tag);
    EVP_CIPHER_CTX_free(c);
    return ok ? 0 : -1;
}

int ossl_gcm_open(const uint8_t key[32], const uint8_t iv[12], const uint8_t *aad, int aad_len,
                  const uint8_t *ct, int len, const uint8_t tag[16], uint8_t *pt) {
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    int out = 0, ok = 1;
    ok &= EVP_DecryptInit_ex(c, EVP_aes_256_gcm(), NULL, key, iv);
    if (aad_len) ok &= EVP_DecryptUpdate(c, NULL, &out, aad, aad_len);
    if (len) ok &= EVP_DecryptUpdate(c, pt, &out, ct, len);
    ok &= EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_TAG, 16, (void *)tag);
    int fin = EVP_DecryptFinal_ex(c, pt + len, &out);
    EVP_CIPHER_CTX_free(c);
    return (ok && fin > 0) ? 0 : -1;
}

int ossl_pbkdf2_sha512(const uint8_t *secret, int secret_len, const uint8_t *salt, int salt_len,
                       int iters, uint8_t *out, int out_len) {
    return PKCS5_PBKDF2_HMAC((const char *)secret, secret_len, salt, salt_len, iters, EVP_sha512(),
                             out_len, out) == 1 ? 0 : -1;
}

/* X25519(scalar, u): out = scalar * point (RFC 7748), as curve25519.ScalarMult. */
int ossl_x25519(uint8_t out[32], const uint8_t scalar[32], const uint8_t point[32]) {
    EVP_PKEY *priv = EVP_PKEY_new_raw_private_key(EVP_PKEY_X25519, NULL, scalar, 32);
    EVP_PKEY *peer = EVP_PKEY_new_raw_public_key(EVP_PKEY_X25519, NULL, point, 32);
    int rc = -1;
    if (priv && peer) {
        EVP_PKEY_CTX *ctx = EVP_PKEY_CTX_new(priv, NULL);
        size_t len = 32;
        if (ctx && EVP_PKEY_derive_init(ctx) == 1 && EVP_PKEY_derive_set_peer(ctx, peer) == 1 &&
            EVP_PKEY_derive(ctx, out, &len) == 1 && len == 32)
            rc = 0;
        EVP_PKEY_CTX_free(ctx);
    }
    EVP_PKEY_free(priv);
    EVP_PKEY_free(peer);
    return rc;
}

/* X25519(scalar, 9): curve25519.ScalarBaseMult (crypto/ecdh.go:17). */
int ossl_x25519_base(uint8_t out[32], const uint8_t scalar[32]) {
    EVP_PKEY *priv = EVP_PKEY_new_raw_private_key(EVP_PKEY_X25519, NULL, scalar, 32);
    size_t len = 32;
    int rc = (priv && EVP_PKEY_get_raw_public_key(priv, out, &len) == 1 && len == 32) ? 0 : -1;
    EVP_PKEY_free(priv);
    return rc;
}

/* Seal a uniform Raw-slot batch: slot i at arena + i*stride = [aad][payload L][tag][nonce]. */
int ossl_seal_uniform(const uint8_t key[32], uint8_t *arena, long stride, long n, int L, int aad_len,
                      const uint8_t *nonces) {
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    int out = 0, ok = EVP_EncryptInit_ex(c, EVP_aes_256_gcm(), NULL, key, NULL);
    for (long i = 0; i < n && ok; i++) {
        uint8_t *raw = arena + i * stride, *data = raw + 4;
        const uint8_t *iv = nonces + 12 * i;
        ok &= EVP_EncryptInit_ex(c, NULL, NULL, NULL, iv);
        if (aad_len) ok &= EVP_EncryptUpdate(c, NULL, &out, raw, aad_len);
        ok &= EVP_EncryptUpdate(c, data, &out, data, L);
        ok &= EVP_EncryptFinal_ex(c, data + L, &out);
        ok &= EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, data + L);
        memcpy(data + L + 16, iv, 12);
    }
    EVP_CIPHER_CTX_free(c);
    return ok ? 0 : -1;
}

/* Descriptor batch (config 3), as oracle_aesgo_seal_descs: packet i at arena + offs[i] = [aad 4][L],
 * key keys + 32 * kidx[i], nonce nonces + 12 i; packets [lo, hi).  For the golden digests. */
int ossl_seal_descs(const uint8_t *keys, uint8_t *arena, const uint64_t *offs, const uint32_t *lens,
                    const uint32_t *kidx, const uint8_t *nonces, int aad_len, long lo, long hi) {
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    int ok = c != NULL, out = 0;
    long cur = -1;
    for (long i = lo; i < hi && ok; i++) {
        if ((long)kidx[i] != cur) {
            cur = kidx[i];
            ok &= EVP_EncryptInit_ex(c, EVP_aes_256_gcm(), NULL, keys + 32 * (size_t)cur, NULL);
        }
        uint8_t *raw = arena + offs[i], *data = raw + 4;
        const int L = (int)lens[i];
        const uint8_t *iv = nonces + 12 * (size_t)i;
        ok &= EVP_EncryptInit_ex(c, NULL, NULL, NULL, iv);
        if (aad_len) ok &= EVP_EncryptUpdate(c, NULL, &out, raw, aad_len);
        ok &= EVP_EncryptUpdate(c, data, &out, data, L);
        ok &= EVP_EncryptFinal_ex(c, data + L, &out);
        ok &= EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, data + L);
        memcpy(data + L + 16, iv, 12);
    }
    if (c) EVP_CIPHER_CTX_free(c);
    return ok ? 0 : -1;
}

/* ---------------- CPU baseline: crypto/aes.go semantics, one worker per thread ---------------- */

typedef struct {
    const uint8_t *key;
    long packets;
    int L;
    int mode; /* 0: getrandom nonce per packet (crypto/aes.go:44); 1: counter nonce (no syscall) */
    int ok;
    double seconds;
} worker_arg;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *baseline_worker(void *p) {
    worker_arg *a = (worker_arg *)p;
    /* one 1472-B Raw buffer per worker, reused (worker/outgoing.go:88) */
    uint8_t raw[1472 + 9000];
    uint8_t aad[4] = {10, 99, 0, 1};
    int out = 0, ok = 1;
    for (int i = 0; i < a->L; i++) raw[4 + i] = (uint8_t)(i * 131 + 7);
    memcpy(raw, aad, 4);
    EVP_CIPHER_CTX *e = EVP_CIPHER_CTX_new(), *d = EVP_CIPHER_CTX_new();
    ok &= EVP_EncryptInit_ex(e, EVP_aes_256_gcm(), NULL, a->key, NULL);
    ok &= EVP_DecryptInit_ex(d, EVP_aes_256_gcm(), NULL, a->key, NULL);
    double t0 = now_s();
    for (long i = 0; i < a->packets && ok; i++) {
        uint8_t *data = raw + 4;
        int L = a->L;
        /* Encrypt: crypto/aes.go:41-52 -- fresh nonce from the kernel RNG per packet */
        uint8_t nonce[12];
        if (a->mode == 0) {
            if (getrandom(nonce, 12, 0) != 12) { ok = 0; break; }
        } else {
            memset(nonce, 0, 12);
            memcpy(nonce, &i, sizeof i);
        }
        ok &= EVP_EncryptInit_ex(e, NULL, NULL, NULL, nonce);
        ok &= EVP_EncryptUpdate(e, NULL, &out, raw, 4);
        ok &= EVP_EncryptUpdate(e, data, &out, data, L);
        ok &= EVP_EncryptFinal_ex(e, data + L, &out);
        ok &= EVP_CIPHER_CTX_ctrl(e, EVP_CTRL_GCM_GET_TAG, 16, data + L);
        memcpy(data + L + 16, nonce, 12);
        /* Decrypt: crypto/aes.go:57-62 */
        int length = L + 28 - 12;
        ok &= EVP_DecryptInit_ex(d, NULL, NULL, NULL, data + length);
        ok &= EVP_DecryptUpdate(d, NULL, &out, raw, 4);
        ok &= EVP_DecryptUpdate(d, data, &out, data, length - 16);
        ok &= EVP_CIPHER_CTX_ctrl(d, EVP_CTRL_GCM_SET_TAG, 16, data + length - 16);
        ok &= EVP_DecryptFinal_ex(d, data + L, &out) > 0;
    }
    a->seconds = now_s() - t0;
    a->ok = ok;
    EVP_CIPHER_CTX_free(e);
    EVP_CIPHER_CTX_free(d);
    return NULL;
}

/* Runs `threads` workers, each sealing+opening `packets_per_thread` packets of L bytes.
 * Returns wall seconds (max over workers), or -1 on failure. */
double ossl_cpu_baseline_mode(const uint8_t key[32], int threads, long packets_per_thread, int L, int mode) {
    if (threads < 1 || threads > 1024 || L < 0 || L > 9000) return -1;
    pthread_t *tid = calloc((size_t)threads, sizeof(pthread_t));
    worker_arg *args = calloc((size_t)threads, sizeof(worker_arg));
    double t0 = now_s();
    for (int t = 0; t < threads; t++) {
        args[t].key = key;
        args[t].packets = packets_per_thread;
        args[t].L = L;
        args[t].mode = mode;
        pthread_create(&tid[t], NULL, baseline_worker, &args[t]);
    }
    int ok = 1;
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        ok &= args[t].ok;
    }
    double wall = now_s() - t0;
    free(tid);
    free(args);
    return ok ? wall : -1.0;
}

double ossl_cpu_baseline(const uint8_t key[32], int threads, long packets_per_thread, int L) {
    return ossl_cpu_baseline_mode(key, threads, packets_per_thread, L, 0);
}
