/*
 * qgcm.h -- C ABI of the MI355X-native AES-256-GCM packet sealer (libqgcm.so).
 *
 * This is the drop-in boundary for quantum's Encryption plugin path.  Every entry point
 * names the reference interface it replaces (paths relative to the quantum tree):
 *
 *   crypto/aes.go:22-26   type AES {block, aead, salt}        -> qgcm_ctx + key slot (key_idx)
 *   crypto/aes.go:65-83   NewAES(secret, salt)                -> qgcm_derive_key + qgcm_set_key
 *   crypto/aes.go:41-52   (*AES).Encrypt(data, length, aad)   -> qgcm_seal_one / qgcm_seal_batch
 *   crypto/aes.go:57-62   (*AES).Decrypt(data, aad)           -> qgcm_open_one / qgcm_open_batch
 *   crypto/aes.go:29-36   EncryptedSize / DecryptedSize       -> QGCM_OVERHEAD (= 16 + 12)
 *   crypto/ecdh.go:13-31  GenerateECKeyPair / GenerateSharedSecret -> qgcm_x25519*
 *   plugin/encryption.go:16-40 Encryption.Apply calls Encrypt/Decrypt per packet (qgcm_seal_one /
 *                         qgcm_open_one); workers that batch their packets call the host or device
 *                         batch entry points instead.
 *
 * Error convention follows the reference's own cgo layer (crypto/dtls.go:37-40, dtls.h:43-48):
 * constructors return NULL and fill a caller-supplied error buffer; everything else returns
 * a negative QGCM_E* code (see qgcm_strerror) or, for the per-packet calls, -1 exactly where the
 * Go method returns an error.  All functions are thread-safe unless stated otherwise.
 *
 * Packet slot layout (common/payload.go:7-45, common/common.go:16-38): a slot is one
 * common.Payload.Raw buffer: [0:4) sender private IPv4 = the GCM additional data,
 * [4:4+L) payload.  Sealing writes ct over the payload, then tag (16 B) and nonce (12 B):
 * [4:4+L) ct, [4+L:4+L+16) tag, [4+L+16:4+L+28) nonce -- exactly crypto/aes.go:49-51.
 * Slot offsets must be multiples of 4; slots need capacity 4+L+28 bytes.
 *
 * Device pointers are HIP device pointers on the context's device; `stream` is a hipStream_t
 * (NULL = the null stream).  Batch calls are asynchronous with respect to the host.
 */
#ifndef QGCM_H
#define QGCM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QGCM_KEY_BYTES 32    /* crypto/crypto.go:7 keyLength */
#define QGCM_SALT_BYTES 32   /* crypto/aes.go:17 SaltLength */
#define QGCM_NONCE_BYTES 12  /* cipher.NewGCM standard nonce */
#define QGCM_TAG_BYTES 16    /* cipher.NewGCM standard tag (aead.Overhead()) */
#define QGCM_OVERHEAD 28     /* EncryptedSize - len = Overhead + NonceSize, crypto/aes.go:29-36 */
#define QGCM_PBKDF2_ITERS 10000 /* crypto/aes.go:18 */
#define QGCM_MAX_PAYLOAD (1u << 28) /* largest plaintext per packet (GCM allows 2^36-32; packets are <= 9000) */
#define QGCM_ERRLEN 120      /* crypto/dtls.go:23 errorLen */
#define QGCM_MAX_BATCH (1u << 31) /* packets per batch call (tile indices stay 32-bit); more -> QGCM_E_ARG */
/* largest max_keys of a context: the descriptor sort key is key_idx << 12 | length rank, 32 bits, and
 * its all-ones value marks excluded packets, so key index 2^20 - 1 is reserved */
#define QGCM_MAX_KEYS ((1u << 20) - 1)

/* status codes */
#define QGCM_OK 0
#define QGCM_E_ARG -1       /* bad argument / size */
#define QGCM_E_HIP -2       /* HIP runtime error */
#define QGCM_E_KEY -3       /* key index not set or out of range */
#define QGCM_E_AUTH -4      /* message authentication failed (errOpen) */
#define QGCM_E_NOMEM -5

typedef struct qgcm_ctx qgcm_ctx;

/* One packet descriptor of a device batch.  For seal, len = payload length L
 * (Encrypt's `length`); for open, len = sealed length L+28 (len(Payload.Packet) as
 * passed to Decrypt).  offset = byte offset of the slot (the Raw buffer) in the arena. */
typedef struct qgcm_desc {
    uint64_t offset;
    uint32_t len;
    uint32_t key_idx;
} qgcm_desc;

/* ---- context (replaces the per-process Go AEAD objects) ---- */
/* max_keys in [1, QGCM_MAX_KEYS].  Key slots start unset: a packet naming an unset slot fails (status 0,
 * slot untouched; QGCM_E_KEY / -1 from the uniform and per-packet calls), as Apply would on a peer
 * whose Mapping.AES is nil (common/mapping.go:94-99 leaves it nil when the peer published no keys). */
qgcm_ctx *qgcm_create(int device, uint32_t max_keys, char *err, int errlen);
void qgcm_destroy(qgcm_ctx *ctx);
const char *qgcm_strerror(int code);
const char *qgcm_version(void);
/* HIP devices this process sees (0 when there are none or the runtime fails).  The Go drop-in's
 * process-wide device set (go/crypto/aes_gpu.go, QGCM_DEVICES unset) is every one of them. */
int qgcm_device_count(void);

/* ---- key setup: crypto/aes.go:65-83 NewAES, common/mapping.go:90-99 ---- */
/* key = PBKDF2-HMAC-SHA512(secret, salt, 10000, 32)  (crypto/aes.go:66) -- host */
int qgcm_derive_key(const uint8_t *secret, size_t secret_len, const uint8_t *salt, size_t salt_len,
                    uint8_t key[QGCM_KEY_BYTES]);
/* Batched: keys[i] = PBKDF2(secrets[i], salts[i]) for count peers, multithreaded host. */
int qgcm_derive_keys(const uint8_t *secrets, const uint8_t *salts, uint32_t count, uint8_t *keys);
/* aes.NewCipher + cipher.NewGCM (crypto/aes.go:68-76): expands round keys and the GHASH
 * tables on the device for slot key_idx.  Synchronous. */
int qgcm_set_key(qgcm_ctx *ctx, uint32_t key_idx, const uint8_t key[QGCM_KEY_BYTES]);
int qgcm_set_keys(qgcm_ctx *ctx, uint32_t first_idx, uint32_t count, const uint8_t *keys);
/* Marks key slots [first_idx, first_idx + count) unset (the slot's AES was released: go/crypto/aes_gpu.go's
 * finalizer, crypto::DeviceSet::Release).  Afterwards every call naming one of them fails as for a key never
 * set (per-packet calls -1 / QGCM_E_KEY, descriptor batches status 0) until qgcm_set_key(s) installs a new
 * key there, so a stale key index never seals or opens under the slot's next peer.  Synchronous; ends the
 * resident instance like qgcm_set_keys. */
int qgcm_clear_keys(qgcm_ctx *ctx, uint32_t first_idx, uint32_t count);
/* X25519 (crypto/ecdh.go:13-31): pub = X25519(priv, 9); secret = X25519(priv, peer_pub). */
int qgcm_x25519_base(uint8_t pub[32], const uint8_t priv[32]);
int qgcm_x25519(uint8_t secret[32], const uint8_t priv[32], const uint8_t peer_pub[32]);

/* ---- device batches (the throughput path) ---- */
/* Seal n packets in place.  nonces: device array of n*12 bytes (nonce i for packet i, written
 * into the slot like crypto/aes.go:50), or NULL to use the nonce already present at
 * [4+L+16, 4+L+28) of each slot.  aad_len: 0 (nil additional) or 4 (the Payload IP header).
 * status (device, n bytes, may be NULL): 1 = sealed, 0 = rejected (key index out of range or never set,
 * payload of QGCM_MAX_PAYLOAD or more; the slot is untouched). */
int qgcm_seal_batch(qgcm_ctx *ctx, uint8_t *d_arena, const qgcm_desc *d_descs, uint32_t n,
                    const uint8_t *d_nonces, uint32_t aad_len, uint8_t *d_status, void *stream);
/* Open n packets in place.  status[i] = 1 if authentic (plaintext at [4, 4+len-28)),
 * 0 on errOpen (tag mismatch: plaintext region zeroed as Go 1.9 gcm.Open does;
 * len < 28: slot untouched). */
int qgcm_open_batch(qgcm_ctx *ctx, uint8_t *d_arena, const qgcm_desc *d_descs, uint32_t n,
                    uint32_t aad_len, uint8_t *d_status, void *stream);
/* Uniform batches: slot i at i*stride, same length and key for all packets (no descriptor
 * traffic).  seal: len = L; open: len = L + 28. */
int qgcm_seal_uniform(qgcm_ctx *ctx, uint8_t *d_arena, uint64_t stride, uint32_t n, uint32_t len,
                      uint32_t key_idx, const uint8_t *d_nonces, uint32_t aad_len,
                      uint8_t *d_status, void *stream);
int qgcm_open_uniform(qgcm_ctx *ctx, uint8_t *d_arena, uint64_t stride, uint32_t n, uint32_t len,
                      uint32_t key_idx, uint32_t aad_len, uint8_t *d_status, void *stream);

/* ---- per-packet host calls, the exact Encrypt/Decrypt contract ---- */
/* crypto/aes.go:41-52: seals data[0:length] in place, appends tag and nonce; data must have
 * capacity length+28.  nonce NULL -> 12 fresh bytes from getrandom(2) as crypto/rand does.
 * aad may be NULL (aad_len 0).  Returns length+28, or -1. */
long qgcm_seal_one(qgcm_ctx *ctx, uint32_t key_idx, uint8_t *data, long length, const uint8_t *aad,
                   uint32_t aad_len, const uint8_t *nonce);
/* crypto/aes.go:57-62: opens data[0:len] in place.  Returns len-28, or -1 (errOpen; data[0:len-28]
 * zeroed on tag mismatch; len < 28 leaves data untouched -- the reference panics below 12). */
long qgcm_open_one(qgcm_ctx *ctx, uint32_t key_idx, uint8_t *data, long len, const uint8_t *aad,
                   uint32_t aad_len);

/* Per-packet calls are served by a RESIDENT kernel (16 workgroups by default, QGCM_RESIDENT_WORKERS;
 * 16 request slots each, QGCM_RESIDENT_SLOTS), so a call costs no launch: the caller writes its packet and
 * a 16-B request record into fine-grained DEVICE memory through the PCIe BAR (the CPU agent is granted
 * access with hsa_amd_agents_allow_access), the workers poll those records in their own HBM, and write
 * the result and a done word into pinned host memory that the caller watches.  Without CPU access to that
 * memory (or QGCM_RESIDENT=0), and for payloads past ~16 KiB, every call takes a gcm_one_kernel launch
 * instead; qgcm_resident_stats says which served (requests served, instances launched).
 * The kernel is started by the first call and ends by itself after QGCM_RESIDENT_IDLE_US (2000) without
 * a request or QGCM_RESIDENT_LIFE_US (8000) of life, after serving what is pending (the next call starts
 * it again): work queued behind it on a shared hardware queue, or a device-wide synchronize, waits that
 * long at most.  qgcm_set_key(s) and qgcm_destroy end it too (it caches key tables).
 * Per-packet calls of up to 2016 B hash with per-key tables of H^1..H^128 (6-bit combs, 2.75 MiB of
 * device memory per key slot, built by qgcm_set_key(s)) for the first QGCM_FLAT_GHASH_KEYS slots
 * (default min(max_keys, 256); 0 = off: every packet takes the slower chained GHASH).
 * A seal without a caller's nonce draws the nonce of its slot's NEXT seal too and hands it to the worker,
 * which computes that nonce's counter blocks while idle (QGCM_RESIDENT_AHEAD=0: off); the next seal
 * on the slot uses that nonce (drawn from getrandom like any other, used once) and skips the counter
 * blocks.  qgcm_resident_stop ends it now; qgcm_resident_stats writes {requests served, instances
 * launched, request slots, workers running now, seals served from a keystream computed ahead, callers
 * asleep now, callers spinning now, 1 if the resident path has failed and every call takes the launch
 * path} (min(n, 8) values, returns that number or -1).  qgcm_set_key(s) ends the instance before it
 * changes the key tables and holds the next one back until the new keys are published; a per-packet call
 * racing it waits (or, if the context's resident service was not started yet, starts it). */
int qgcm_resident_stop(qgcm_ctx *ctx);
int qgcm_resident_stats(const qgcm_ctx *ctx, uint64_t *out, int n);

/* ---- host batches (end-to-end incl. PCIe) ---- */
/* Slots in host memory at i*stride; copies in, runs the device batch, copies back, synchronously.
 * Pipelined in 64 MiB chunks over 3 streams (H2D of chunk c+1 || kernel c || D2H of chunk c-1);
 * h_arena from qgcm_host_alloc (pinned) is DMA'd in place, pageable memory is staged by HIP.  A pinned
 * batch of up to 65536 packets (128 MiB) with 16-B-aligned slots (stride a multiple of 16) is sealed in place
 * instead: one kernel on the arena's device view, no copies (QGCM_HOST_DIRECT=0 disables it).
 * Returns the number of packets that failed (0 = all ok) or a negative error.  status may be NULL.
 * Replaces the per-packet Apply loop of worker/outgoing.go:55-93 / worker/incoming.go:54-92 for a
 * batch of packets a worker has collected. */
int qgcm_seal_host(qgcm_ctx *ctx, uint8_t *h_arena, uint64_t stride, uint32_t n, uint32_t len,
                   uint32_t key_idx, const uint8_t *h_nonces, uint32_t aad_len, uint8_t *h_status);
int qgcm_open_host(qgcm_ctx *ctx, uint8_t *h_arena, uint64_t stride, uint32_t n, uint32_t len,
                   uint32_t key_idx, uint32_t aad_len, uint8_t *h_status);

/* ---- several GPUs behind one process (quantum is one process: main.go:29-114, 72-75) ---- */
/* A group of `count` member contexts, member k on devices[k] (members may share a device, but then share
 * its hardware queues and PCIe link: one member per GPU is the intended layout).  Keyed
 * traffic is hash-sharded: key index k belongs to member qgcm_group_shard(k) = ((k * 0x9E3779B97F4A7C15)
 * mod 2^64 >> 32) mod count (quantum_amd/shard.py key_shard), so a peer's packets stay on
 * one GPU and each member holds only its peers' keys.  No collective, no GPU-to-GPU traffic.
 * NULL + err on failure. */
typedef struct qgcm_group qgcm_group;
qgcm_group *qgcm_group_create(const int *devices, int count, uint32_t max_keys, char *err, int errlen);
void qgcm_group_destroy(qgcm_group *g);
int qgcm_group_size(const qgcm_group *g);
qgcm_ctx *qgcm_group_ctx(qgcm_group *g, int member);  /* member's context (device batches on it) */
/* Number of CPUs member's host thread is pinned to: its GPU's NUMA-local CPUs (sysfs local_cpulist of
 * the PCI device) that the process may use; 0 = not pinned (no sysfs answer). */
int qgcm_group_member_cpus(const qgcm_group *g, int member);
int qgcm_group_shard(const qgcm_group *g, uint32_t key_idx);
/* Installs keys[i] as key first_idx + i on its owning member only (qgcm_set_keys there). */
int qgcm_group_set_keys(qgcm_group *g, uint32_t first_idx, uint32_t count, const uint8_t *keys);
/* qgcm_clear_keys on the owning member of each key index. */
int qgcm_group_clear_keys(qgcm_group *g, uint32_t first_idx, uint32_t count);
/* Host batches over the group: packet i is the Raw slot at h_arena + h_descs[i].offset (seal: len = L,
 * capacity 4 + L + 28; open: len = L + 28), any key mix.  Packets are split by owner; one host thread and
 * one stream set per member gathers its packets into pinned staging, copies them to its device, runs the
 * descriptor batch, copies back and writes the results into the same slots (input order kept).
 * h_nonces: n * 12 B (seal; NULL = nonce already in the slot).  h_status[i] (may be NULL): 1 ok, 0 failed
 * (as qgcm_seal_batch / qgcm_open_batch).  Returns the number of failed packets or a negative error.
 * One call at a time per group (calls are serialized).  When h_arena (and h_nonces) is pinned host memory
 * (qgcm_host_alloc, hipHostMalloc, hipHostRegister) holding every record, the members' GPUs gather and
 * scatter the records themselves over PCIe (zero-copy); otherwise host threads copy them through pinned
 * staging (QGCM_GROUP_THREADS per member); so does a batch with a record offset that is not a multiple of
 * 4.  QGCM_GROUP_ZEROCOPY=0 forces the copy path. */
int qgcm_group_seal_host(qgcm_group *g, uint8_t *h_arena, const qgcm_desc *h_descs, uint32_t n,
                         const uint8_t *h_nonces, uint32_t aad_len, uint8_t *h_status);
int qgcm_group_open_host(qgcm_group *g, uint8_t *h_arena, const qgcm_desc *h_descs, uint32_t n, uint32_t aad_len,
                         uint8_t *h_status);
/* 1 if the last qgcm_group_seal_host / open_host call took the zero-copy path on every member, else 0. */
int qgcm_group_last_zerocopy(const qgcm_group *g);
/* DMA runs: when the descriptors are in arena order (offsets nondecreasing, multiples of 4) and a member's
 * packets form runs of adjacent records (consecutive packets, at most 256 B between one record's end and
 * the next one's start) averaging 64 KiB or more, that member copies each run to and from its device with
 * one DMA each way (64 MiB chunks, three staging slots, three streams), with no gather, scatter or
 * shader-driven PCIe traffic;
 * the gap bytes inside a run go back unchanged.  A batch laid out in qgcm_group_order's order, or any batch
 * of a one-member group, takes it.  A chunk of at most 8192 packets whose records all start 16-B aligned
 * runs one workgroup per packet instead of the sorted worklist (QGCM_DESC_ONE=0 disables that).
 * Direct: a member's share of up to 65536 packets (128 MiB) whose records all start 16-B aligned, in a
 * pinned arena that also holds each record's 16-B-rounded area, is sealed in place by that kernel over
 * PCIe with no copies, whether the members' records are adjacent or interleaved (QGCM_GROUP_DIRECT=0
 * disables it).
 * QGCM_GROUP_DMA=0 disables the DMA runs.  qgcm_group_last_path: the path member
 * took in the last call (0 host copies, 1 zero-copy, 2 DMA runs, 3 direct) or QGCM_E_ARG. */
int qgcm_group_last_path(const qgcm_group *g, int member);
/* The order in which to lay out a keyed batch so that each member's packets are contiguous (a stable
 * counting sort by qgcm_group_shard): order[0..n) = input indices, member by member; member_counts
 * (may be NULL) receives each member's packet count.  A caller that assembles its batch in this order
 * gets the DMA-run path.  Returns QGCM_OK or QGCM_E_ARG. */
int qgcm_group_order(const qgcm_group *g, const uint32_t *key_idx, uint32_t n, uint32_t *order,
                     uint32_t *member_counts);

/* Pinned (page-locked) host memory for arenas handed to the *_host calls; NULL on failure. */
void *qgcm_host_alloc(size_t bytes);
void qgcm_host_free(void *p);

/* ---- nonce source for production seals (crypto/aes.go:42-47 draws per packet) ---- */
/* Fills n*12 bytes of host memory from getrandom(2). */
int qgcm_random_nonces(uint8_t *h_out, uint32_t n);

/* ---- snappy block format: the compression plugin (plugin/compression.go) ---- */
/* Host codec (C++; golang/snappy is not in the reference).  Encode restates golang/snappy's block
 * encoder (compression.go:17 snappy.Encode), the same bytes as libsnappy 1.1.8 (tests/golden/
 * snappy.json); Decode accepts every valid stream and returns -1 on malformed input
 * (compression.go:22-25 decode error). */
size_t qgcm_snappy_max_compressed_length(size_t n);
long qgcm_snappy_compress(const uint8_t *src, size_t n, uint8_t *dst, size_t cap);
long qgcm_snappy_uncompressed_length(const uint8_t *src, size_t n);
long qgcm_snappy_uncompress(const uint8_t *src, size_t n, uint8_t *dst, size_t cap);
/* Payload.Raw slots at i*stride: packet i = lens[i] bytes at slot+4, (de)compressed in place,
 * lens[i] updated (compression.go Apply, Outgoing / Incoming), `threads` host workers.  Returns the
 * number of packets that failed (untouched; status[i] = 0) or -1. */
int qgcm_snappy_compress_slots(uint8_t *arena, uint64_t stride, uint32_t n, uint32_t *lens, int threads);
/* As qgcm_snappy_compress_slots, but a packet also fails when its compressed form exceeds `limit`
 * bytes (room left for the seal's tag and nonce); status[i] = 1 ok / 0 failed (may be NULL). */
int qgcm_snappy_compress_slots_limit(uint8_t *arena, uint64_t stride, uint32_t n, uint32_t *lens, uint64_t limit,
                                     uint8_t *status, int threads);
int qgcm_snappy_uncompress_slots(uint8_t *arena, uint64_t stride, uint32_t n, uint32_t *lens,
                                 uint8_t *status, int threads);
/* Device codec (gfx950, one wave per packet), the same bytes as the host codec: Payload.Raw slots at
 * i*stride in device memory (stride a multiple of 4), packet i = d_lens[i] bytes at slot+4, replaced
 * in place (compression.go:39-51), d_lens[i] updated.  compress: packets longer than max_len, or
 * whose compressed form exceeds limit, fail; uncompress: packets longer than max_len, that do not
 * decode, or that decode to more than cap bytes fail.  A failed packet's slot and length are
 * untouched (d_status[i] = 0; 1 = ok; may be NULL).  All limits are at most stride - 4; compress's
 * max_len and uncompress's cap at most QGCM_SNAPPY_DEVICE_MAX, uncompress's max_len at most
 * qgcm_snappy_max_compressed_length(QGCM_SNAPPY_DEVICE_MAX).  compress also writes, when d_descs_out is
 * not NULL, the seal descriptor of each packet ({i*stride, compressed length, key_idx}; a failed packet
 * gets length QGCM_MAX_PAYLOAD, which the seal rejects), so qgcm_seal_batch can follow on the stream
 * (the chain main.go:50-51 sorts: compression, then encryption).  Asynchronous on stream. */
#define QGCM_SNAPPY_DEVICE_MAX 16384
int qgcm_snappy_compress_batch(qgcm_ctx *ctx, uint8_t *d_arena, uint64_t stride, uint32_t n, uint32_t *d_lens,
                               uint32_t max_len, uint32_t limit, uint8_t *d_status, qgcm_desc *d_descs_out,
                               uint32_t key_idx, void *stream);
int qgcm_snappy_uncompress_batch(qgcm_ctx *ctx, uint8_t *d_arena, uint64_t stride, uint32_t n, uint32_t *d_lens,
                                 uint32_t max_len, uint32_t cap, uint8_t *d_status, void *stream);

/* ---- Compression + Encryption chain (BASELINE config 5) ---- */
/* Host batches in the order main.go:50-51 sorts the plugins: outgoing compression.go then
 * encryption.go Apply, incoming the reverse.  Slot i at i*stride holds [aad 4][packet lens[i] B].
 * compress_seal: snappy-compress each packet in place, then seal it (lens[i] <- compressed + 28).
 * open_uncompress: open each sealed packet, then uncompress (lens[i] <- plaintext length).
 * Chunks pipeline the codec (`threads` host workers and/or the device codec, qgcm_chain_codec) with
 * PCIe copies and the device kernels.
 * Returns the number of failed packets (status 0: codec error, no room for the tag and nonce, or
 * failed authentication -- plaintext zeroed as in qgcm_open_batch), or a negative error. */
int qgcm_compress_seal_host(qgcm_ctx *ctx, uint8_t *h_arena, uint64_t stride, uint32_t n, uint32_t *lens,
                            uint32_t key_idx, const uint8_t *h_nonces, uint32_t aad_len, int threads,
                            uint8_t *h_status);
int qgcm_open_uncompress_host(qgcm_ctx *ctx, uint8_t *h_arena, uint64_t stride, uint32_t n, uint32_t *lens,
                              uint32_t key_idx, uint32_t aad_len, int threads, uint8_t *h_status);
/* Where the chained calls run the snappy codec: 0 = host workers only; 1 = split (default): the device
 * codec takes the chunks the host workers cannot keep up with (seal: the last untouched chunks when a
 * stream slot is free and fewer than two compressed host chunks are waiting; open: when the host decode
 * backlog exceeds two chunks); 2 = device only.  The bytes are the same either way.  Returns the previous mode
 * (mode -1: just read it) or QGCM_E_ARG.  QGCM_CHAIN_DEVICE sets the initial mode. */
int qgcm_chain_codec(qgcm_ctx *ctx, int mode);

/* ---- batched UDP I/O (socket/udp.go:35-70, one syscall per batch) ---- */
/* Datagram i is slot i's Raw[:lens[i]] (wire format [4-B IP][packet]), moved with recvmmsg/sendmmsg
 * straight into / out of a host arena (pinned from qgcm_host_alloc: then also the DMA source of
 * qgcm_*_host).  qgcm_udp_socket binds ip:port (port 0: any; bufbytes > 0 sizes SO_RCVBUF/SNDBUF)
 * and returns the fd or -1.  recv waits up to timeout_ms (-1 forever) for the first datagram and then
 * takes what is queued, up to max_n; returns the count (0 on timeout) or -1.  send returns the
 * number of datagrams sent or -1. */
int qgcm_udp_socket(const char *ip, int port, int bufbytes);
/* One queue of a multi-queue socket (socket/udp.go:55-70: one per worker on the same address):
 * SO_REUSEPORT, so the kernel spreads incoming flows over the queues of the group. */
int qgcm_udp_queue(const char *ip, int port, int bufbytes);
int qgcm_udp_port(int fd);
int qgcm_udp_close(int fd);
int qgcm_udp_recv_slots(int fd, uint8_t *arena, uint64_t stride, uint32_t max_n, uint32_t *lens, int timeout_ms);
int qgcm_udp_send_slots(int fd, const uint8_t *arena, uint64_t stride, uint32_t n, const uint32_t *lens,
                        const char *ip, int port);

/* ---- batched TUN I/O (device/tun.go:51-118) ---- */
/* qgcm_tun_open: device/tun.go:97-118 (createTUN) for `queues` queues of one multi-queue TUN device
 * (IFF_TUN | IFF_NO_PI | IFF_MULTI_QUEUE), fds[i] = queue i; the kernel's device name goes to
 * ifname_out.  qgcm_tun_up: device/tun.go:121-150 (initTun): up, MTU, address/prefix.  Both return 0
 * or -errno.  read_slots: device/tun.go:51-57 batched -- waits up to timeout_ms for the first packet,
 * then drains what the queue holds (up to max_n) into Raw[4:] of slots 0, 1, ... (lens[i] = packet
 * length); returns the count (0 on timeout) or -1.  write_slots: device/tun.go:60-63 batched --
 * writes Raw[4 : 4 + lens[i]]; returns the number written or -1. */
int qgcm_tun_open(const char *name, int queues, int *fds, char *ifname_out, size_t ifname_len);
int qgcm_tun_up(const char *ifname, const char *ip, int prefix, int mtu);
int qgcm_tun_read_slots(int fd, uint8_t *arena, uint64_t stride, uint32_t max_n, uint32_t *lens, int timeout_ms);
int qgcm_tun_write_slots(int fd, const uint8_t *arena, uint64_t stride, uint32_t n, const uint32_t *lens);
int qgcm_tun_close(int fd);

/* ---- introspection: which kernels served this context's calls ---- */
/* Launch counts per kernel family since qgcm_create (uniform batches launch in chunks of 2^19
 * packets; a descriptor batch launches the segmented kernel and then the per-wave kernel for its
 * short keys; gcm_one_kernel serves per-packet calls the resident kernel does not take and uniform
 * batches of up to 2048 packets).  Writes min(n, QGCM_KERNEL_COUNTERS) counters, returns that number or -1. */
#define QGCM_KERNEL_QUAD 0      /* gcm_quad_kernel, single-key (uniform) batches */
#define QGCM_KERNEL_SEGMENTED 1 /* gcm_seg_kernel, descriptor batches (long key runs) */
#define QGCM_KERNEL_PER_WAVE 2  /* gcm_quad_kernel, descriptor batches (short key runs) */
#define QGCM_KERNEL_ONE 3       /* gcm_one_kernel, one workgroup per packet */
#define QGCM_KERNEL_RESIDENT 4  /* per-packet calls served by the resident kernel (requests, not launches) */
#define QGCM_KERNEL_SNAPPY_ENC 5 /* snappy_compress_kernel (device codec; chained calls: one per device chunk) */
#define QGCM_KERNEL_SNAPPY_DEC 6 /* snappy_uncompress_kernel */
#define QGCM_KERNEL_TAIL_WAITS 7 /* uniform launches that waited, on their stream, for their shared-tail counter
                                    set's previous launch (the context's ring came round; not a launch) */
#define QGCM_KERNEL_COUNTERS 8
int qgcm_launch_counts(const qgcm_ctx *ctx, uint64_t *out, int n);

/* ---- measurement: achievable HBM copy rate (reads + writes bytes) for the roofline ---- */
/* 16-B aligned device buffers, bytes a multiple of 16.  Asynchronous on stream. */
int qgcm_stream_copy(qgcm_ctx *ctx, void *d_dst, const void *d_src, uint64_t bytes, void *stream);

/* ---- synthetic workload generator (bench/tests; BASELINE.json configs) ---- */
/* Slot i at i*stride: [aad_word LE][payload L bytes of the splitmix64(seed_payload) stream at
 * byte offset i*L]; nonces[i*12..] = splitmix64(seed_nonce) stream at byte offset i*12. */
int qgcm_fill_uniform(uint8_t *d_arena, uint64_t stride, uint32_t n, uint32_t len, uint32_t aad_word,
                      uint64_t seed_payload, uint8_t *d_nonces, uint64_t seed_nonce, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* QGCM_H */
