// Copyright (c) 2026. Licensed under the MPL-2.0 like the quantum tree it is added to.

// +build gpu

// aes_gpu.go -- the MI355X drop-in for quantum's crypto.AES (crypto/aes.go), over libqgcm's C ABI
// (include/qgcm.h).  A maintainer copies this file into quantum's crypto/ directory, adds the line
// `// +build !gpu` to crypto/aes.go, and builds with `go build -tags gpu`.  Nothing else changes:
// this file defines the same package-level names crypto/aes.go does -- SaltLength, type AES with
// EncryptedSize / DecryptedSize / Encrypt / Decrypt, and NewAES(secret, salt) (*AES, error) with the
// signatures of crypto/aes.go:15-83 -- so common.Mapping.AES (*crypto.AES, common/mapping.go:54),
// ParseMapping (common/mapping.go:90-99) and plugin.Encryption.Apply (plugin/encryption.go:16-40)
// compile and run unchanged, and crypto_test.go's own TestAES / BenchmarkAES (crypto/crypto_test.go:54-131)
// exercise the GPU path.  Without the tag the package builds exactly as before.  The cgo preamble, the
// prebuilt-library LDFLAGS and the "NULL plus a 120-byte error string" convention follow
// crypto/dtls.go:6-40, the reference's own cgo layer.
//
// Device state is process-wide, created by the first NewAES (quantum is one process per node,
// main.go:29-114, and every Mapping's AES of that process shares it):
//   - QGCM_DEVICES: the GPUs to use, e.g. "0,1,2,3,4,5,6,7" (default: every device the process sees);
//   - QGCM_MAX_PEERS: key slots (default 4096; a slot is recycled when its AES is garbage-collected).
// The set is a qgcm_group of one member context per device (one member on a 1-GPU box); NewAES installs
// a peer's key on member hash(key slot) mod G only, where that peer's Encrypt / Decrypt calls then run
// (SURVEY.md s8e: packets are independent, no GPU-to-GPU traffic).
//
// Encrypt / Decrypt are one packet per call (worker/outgoing.go:83-93 calls Apply per packet), served
// by libqgcm's resident kernel with no launch per call.  Batched workers use the extra API below
// (Devices, GPUGroup.Order / SealBatch / OpenBatch, Arena, Desc; INTEGRATION.md s2).
//
// Differences from crypto/aes.go, all where the reference would panic:
//   - Encrypt with length < 0 or len(data) < length + 28 returns (-1, errShortBuffer);
//   - Decrypt of fewer than 28 bytes returns errOpen (the reference panics below 12 bytes,
//     crypto/aes.go:58-59, and returns errOpen from 12 to 27);
//   - additional data longer than 4 bytes (the Payload IP header; quantum never passes more) is refused.
// nil or empty `additional` (crypto/crypto_test.go TestAES passes nil) and empty slices never have
// their first element addressed: bytePtr returns nil for them.
package crypto

/*
#cgo CFLAGS: -I${SRCDIR}/../vendor/qgcm/include
#cgo LDFLAGS: -L${SRCDIR}/../vendor/qgcm/lib -lqgcm -Wl,-rpath,${SRCDIR}/../vendor/qgcm/lib
#include <stdlib.h>
#include <qgcm.h>
*/
import "C"

import (
	"errors"
	"fmt"
	"os"
	"runtime"
	"strconv"
	"strings"
	"sync"
	"unsafe"
)

const (
	// SaltLength is the length that the passed in salt slice should be for AES objects (crypto/aes.go:16-17).
	SaltLength = 32
	iterations = C.QGCM_PBKDF2_ITERS // crypto/aes.go:18, applied by qgcm_derive_key
)

var (
	// errOpen is the error cipher.AEAD.Open returns on a tag mismatch (crypto/cipher gcm.go).
	errOpen        = errors.New("cipher: message authentication failed")
	errShortBuffer = errors.New("qgcm: data buffer shorter than length + 28")
	errAdditional  = errors.New("qgcm: additional data longer than 4 bytes")
	errSlots       = errors.New("qgcm: out of key slots (QGCM_MAX_PEERS)")
	errBatch       = errors.New("qgcm: batch record outside the arena, or status shorter than the batch")
)

const overhead = C.QGCM_OVERHEAD // tag (16) + nonce (12): aead.Overhead() + aead.NonceSize()

// bytePtr is &b[0] as a C pointer, or nil for an empty (or nil) slice, which cgo cannot address.
func bytePtr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// cError turns a C error buffer into a Go error (crypto/dtls.go:37-40).
func cError(buf *C.char) error { return errors.New(C.GoString(buf)) }

// AES represents an aes-256-gcm AEAD cipher object (crypto/aes.go:22-26): one key slot of the
// process's GPU set.  The slot holds the expanded key schedule and GHASH tables on the GPU that owns it.
type AES struct {
	g    *GPUGroup
	ctx  *C.qgcm_ctx // the member context that holds the key
	idx  uint32
	salt []byte
}

// EncryptedSize returns the minimum size of the data buffer for encryption, which includes the gcm
// tag size + nonce size (crypto/aes.go:29-31).
func (crypt *AES) EncryptedSize(data []byte) int { return len(data) + overhead }

// DecryptedSize returns the size of the data once decrypted (crypto/aes.go:34-36).
func (crypt *AES) DecryptedSize(data []byte) int { return len(data) - overhead }

// Encrypt takes the data buffer and encrypts up to length bytes in place, while injecting the nonce and
// gcm tag at the end and signing the additional data (crypto/aes.go:41-52): data[:length] becomes the
// ciphertext, then the 16-byte tag and the 12-byte nonce (drawn by libqgcm from getrandom(2),
// crypto/rand's source); returns length + 28.
//
// additional may be nil.
func (crypt *AES) Encrypt(data []byte, length int, additional []byte) (int, error) {
	if length < 0 || length+overhead > len(data) {
		return -1, errShortBuffer
	}
	if len(additional) > 4 {
		return -1, errAdditional
	}
	n := C.qgcm_seal_one(crypt.ctx, C.uint32_t(crypt.idx), bytePtr(data), C.long(length), bytePtr(additional),
		C.uint32_t(len(additional)), nil)
	runtime.KeepAlive(crypt) // the slot is not recycled while a call on it runs
	if n < 0 {
		return -1, errors.New("qgcm: seal failed")
	}
	return int(n), nil
}

// Decrypt takes the data buffer and decrypts it and verifies the additional data (crypto/aes.go:57-62):
// the nonce is the last 12 bytes, the tag the 16 before; returns len(data) - 28.  On a tag mismatch the
// plaintext region is zeroed, as Go 1.9's gcm Open does, and errOpen is returned.
//
// additional and data must be the same buffers passed to Encrypt.
func (crypt *AES) Decrypt(data []byte, additional []byte) (int, error) {
	if len(data) < overhead || len(additional) > 4 {
		return crypt.DecryptedSize(data), errOpen
	}
	n := C.qgcm_open_one(crypt.ctx, C.uint32_t(crypt.idx), bytePtr(data), C.long(len(data)), bytePtr(additional),
		C.uint32_t(len(additional)))
	runtime.KeepAlive(crypt)
	if n < 0 {
		return crypt.DecryptedSize(data), errOpen
	}
	return int(n), nil
}

// KeyIndex is this peer's key slot: the Key field of its packets' Descs in a batch (extra API).  Keep
// the AES reachable while batches name its slot: the slot is recycled once the AES is collected.
func (crypt *AES) KeyIndex() uint32 { return crypt.idx }

// Member is the index of the group member (GPU) that holds this peer's key and serves its calls.
func (crypt *AES) Member() int { return int(C.qgcm_group_shard(crypt.g.grp, C.uint32_t(crypt.idx))) }

// NewAES returns a new AEAD based cipher object based on the passed in secret and salt
// (crypto/aes.go:65-83): PBKDF2-HMAC-SHA512(secret, salt, 10000, 32) on the host (qgcm_derive_key),
// then aes.NewCipher + cipher.NewGCM as a device key schedule and GHASH tables (qgcm_set_key) on the GPU
// that owns the new key slot.  The first call creates the process's device set (Devices).
func NewAES(secret, salt []byte) (*AES, error) {
	gg, err := Devices()
	if err != nil {
		return nil, err
	}
	return gg.NewAES(secret, salt)
}

var process struct {
	once sync.Once
	g    *GPUGroup
	err  error
}

// Devices returns the process-wide GPU set every NewAES installs its key in, created on first use
// from QGCM_DEVICES and QGCM_MAX_PEERS (see the file comment).  Batched workers seal and open through it.
func Devices() (*GPUGroup, error) {
	process.once.Do(func() {
		devs, err := deviceList(os.Getenv("QGCM_DEVICES"), int(C.qgcm_device_count()))
		if err != nil {
			process.err = err
			return
		}
		peers := uint32(4096)
		if v := os.Getenv("QGCM_MAX_PEERS"); v != "" {
			p, err := strconv.ParseUint(v, 10, 32)
			if err != nil || p == 0 || p > uint64(C.QGCM_MAX_KEYS) {
				process.err = fmt.Errorf("qgcm: QGCM_MAX_PEERS=%q", v)
				return
			}
			peers = uint32(p)
		}
		process.g, process.err = NewGPUGroup(devs, peers)
	})
	return process.g, process.err
}

// deviceList parses QGCM_DEVICES ("0,1,2,3"; empty: devices 0..visible-1).
func deviceList(spec string, visible int) ([]int, error) {
	if strings.TrimSpace(spec) == "" {
		if visible < 1 {
			return nil, errors.New("qgcm: no HIP device visible")
		}
		out := make([]int, visible)
		for i := range out {
			out[i] = i
		}
		return out, nil
	}
	var out []int
	for _, f := range strings.Split(spec, ",") {
		d, err := strconv.Atoi(strings.TrimSpace(f))
		if err != nil || d < 0 {
			return nil, fmt.Errorf("qgcm: QGCM_DEVICES=%q", spec)
		}
		out = append(out, d)
	}
	return out, nil
}

// GPUGroup drives every GPU of a node from quantum's one process (qgcm_group_*): a peer's key lives on
// GPU hash(key slot) mod G, and that peer's per-packet calls go to that GPU (SURVEY.md s8e).
type GPUGroup struct {
	grp  *C.qgcm_group
	mu   sync.Mutex
	next uint32
	max  uint32
	free []uint32 // key slots of garbage-collected AES objects, reused first

	bmu    sync.Mutex     // one batch at a time (qgcm_group_seal_host serializes calls anyway)
	nonces unsafe.Pointer // pinned nonce buffer of the last SealBatch (qgcm_host_alloc), 12 B per packet
	ncap   int
}

// NewGPUGroup opens one context per device in `devices` (a device may repeat).
func NewGPUGroup(devices []int, maxKeys uint32) (*GPUGroup, error) {
	if len(devices) == 0 {
		return nil, errors.New("qgcm: no devices")
	}
	devs := make([]C.int, len(devices))
	for i, d := range devices {
		devs[i] = C.int(d)
	}
	buf := (*C.char)(C.malloc(C.QGCM_ERRLEN))
	defer C.free(unsafe.Pointer(buf))
	grp := C.qgcm_group_create(&devs[0], C.int(len(devs)), C.uint32_t(maxKeys), buf, C.QGCM_ERRLEN)
	if grp == nil {
		return nil, cError(buf)
	}
	return &GPUGroup{grp: grp, max: maxKeys}, nil
}

// NewAES derives the key (crypto/aes.go:66) and installs it on the GPU that owns the next free key
// slot only; the returned object seals and opens there.  quantum's datastore watch calls ParseMapping,
// and with it NewAES, again on every mapping update (datastore/etcdv2.go:236-276), so a slot whose AES
// has become unreachable is returned to the group by a finalizer and reused.
func (gg *GPUGroup) NewAES(secret, salt []byte) (*AES, error) {
	gg.mu.Lock()
	var idx uint32
	switch {
	case len(gg.free) > 0:
		idx = gg.free[len(gg.free)-1]
		gg.free = gg.free[:len(gg.free)-1]
	case gg.next < gg.max:
		idx = gg.next
		gg.next++
	default:
		gg.mu.Unlock()
		return nil, errSlots
	}
	gg.mu.Unlock()
	owner := C.qgcm_group_shard(gg.grp, C.uint32_t(idx))
	ctx := C.qgcm_group_ctx(gg.grp, owner)
	if ctx == nil {
		gg.release(idx)
		return nil, errors.New("qgcm: no owner context")
	}
	if err := installKey(ctx, idx, secret, salt); err != nil {
		gg.release(idx)
		return nil, err
	}
	a := &AES{g: gg, ctx: ctx, idx: idx, salt: salt}
	runtime.SetFinalizer(a, func(a *AES) { a.g.release(a.idx) })
	return a, nil
}

// release marks the slot's key unset on its owner before the slot is reused, so a KeyIndex kept in a
// batch Desc after its AES was dropped fails that packet's status instead of sealing or opening under
// whichever peer gets the slot next.
func (gg *GPUGroup) release(idx uint32) {
	C.qgcm_group_clear_keys(gg.grp, C.uint32_t(idx), 1)
	gg.mu.Lock()
	gg.free = append(gg.free, idx)
	gg.mu.Unlock()
}

func installKey(ctx *C.qgcm_ctx, idx uint32, secret, salt []byte) error {
	var key [C.QGCM_KEY_BYTES]C.uint8_t
	if rc := C.qgcm_derive_key(bytePtr(secret), C.size_t(len(secret)), bytePtr(salt), C.size_t(len(salt)),
		&key[0]); rc != C.QGCM_OK {
		return errors.New(C.GoString(C.qgcm_strerror(rc)))
	}
	if rc := C.qgcm_set_key(ctx, C.uint32_t(idx), &key[0]); rc != C.QGCM_OK {
		return errors.New(C.GoString(C.qgcm_strerror(rc)))
	}
	return nil
}

// Size is the number of members (one context per listed device).
func (gg *GPUGroup) Size() int { return int(C.qgcm_group_size(gg.grp)) }

// Close releases every member context (no call may be in flight; the process-wide set is never closed).
func (gg *GPUGroup) Close() {
	if gg.grp != nil {
		C.qgcm_group_destroy(gg.grp)
		gg.grp = nil
	}
	if gg.nonces != nil {
		C.qgcm_host_free(gg.nonces)
		gg.nonces = nil
	}
}

// ---- batched workers (INTEGRATION.md s2, s2b) ----
// A worker that has read a batch of packets (recvmmsg / TUN reads) into one pinned Payload.Raw arena
// seals or opens the whole batch with one call instead of one Encrypt / Decrypt per packet
// (worker/outgoing.go:55-93, worker/incoming.go:54-92 loop over packets).  Laid out in Order's order,
// each GPU's packets are adjacent and move by DMA (qgcm_group_last_path 2); a worker-sized batch (up to
// 65536 packets and 128 MiB) whose slots all start 16-B aligned, e.g. the 1472-B MaxPacketLength
// stride, is sealed in place in the arena instead (qgcm_group_last_path 3).

// Arena is pinned host memory for a batch of Payload.Raw slots (qgcm_host_alloc), copied by DMA in
// place.  Bytes aliases it until Free.
type Arena struct {
	Bytes []byte
	p     unsafe.Pointer
}

// NewArena allocates size bytes of pinned host memory.
func NewArena(size int) (*Arena, error) {
	if size <= 0 || size > 1<<40 {
		return nil, errors.New("qgcm: arena size out of range")
	}
	p := C.qgcm_host_alloc(C.size_t(size))
	if p == nil {
		return nil, errors.New("qgcm: pinned allocation failed")
	}
	return &Arena{Bytes: (*[1 << 40]byte)(p)[:size:size], p: p}, nil
}

// Free releases the arena (no batch call may be using it).
func (a *Arena) Free() {
	if a.p != nil {
		C.qgcm_host_free(a.p)
		a.p, a.Bytes = nil, nil
	}
}

// Desc is one packet of a batch, laid out as qgcm_desc: the offset of its Payload.Raw slot in the
// arena, its length (SealBatch: the payload length L; OpenBatch: the sealed length L+28) and its
// peer's key slot (AES.KeyIndex).  The slot is [4-B AAD (the IP header, Payload.Raw[0:4])][packet] with
// room for the 28-B tag and nonce after a payload to be sealed.
type Desc struct {
	Offset uint64
	Len    uint32
	Key    uint32
}

// Desc and qgcm_desc have the same size (the two array lengths are non-negative only if equal).
var _ [unsafe.Sizeof(Desc{}) - unsafe.Sizeof(C.qgcm_desc{})]byte
var _ [unsafe.Sizeof(C.qgcm_desc{}) - unsafe.Sizeof(Desc{})]byte

// Order returns the order in which to lay out a batch whose packet i belongs to peer keys[i] so that
// each GPU's packets are adjacent (qgcm_group_order: stable, GPU by GPU), and each GPU's count.
func (gg *GPUGroup) Order(keys []uint32) ([]uint32, []int, error) {
	order := make([]uint32, len(keys))
	counts := make([]C.uint32_t, int(C.qgcm_group_size(gg.grp)))
	if len(keys) > 0 {
		rc := C.qgcm_group_order(gg.grp, (*C.uint32_t)(unsafe.Pointer(&keys[0])), C.uint32_t(len(keys)),
			(*C.uint32_t)(unsafe.Pointer(&order[0])), &counts[0])
		if rc != C.QGCM_OK {
			return nil, nil, errors.New(C.GoString(C.qgcm_strerror(rc)))
		}
	}
	out := make([]int, len(counts))
	for i, c := range counts {
		out[i] = int(c)
	}
	return order, out, nil
}

func checkBatch(arena *Arena, descs []Desc, status []byte, seal bool) error {
	if arena == nil || arena.p == nil || (status != nil && len(status) < len(descs)) {
		return errBatch
	}
	extra := uint64(4)
	if seal {
		extra += overhead
	}
	for i := range descs {
		if descs[i].Offset+extra+uint64(descs[i].Len) > uint64(len(arena.Bytes)) {
			return errBatch
		}
	}
	return nil
}

// SealBatch seals every packet of the batch in place, as Encrypt does one (crypto/aes.go:41-52):
// slot [AAD][payload L] becomes [AAD][ciphertext L][tag 16][nonce 12], each nonce drawn from
// getrandom(2).  status[i] (nil, or at least len(descs) bytes) is 1 for a sealed packet and 0 for one
// that failed (a key slot that was never set, a length out of range), whose slot is left untouched.
// Returns the number of failed packets.
func (gg *GPUGroup) SealBatch(arena *Arena, descs []Desc, status []byte) (int, error) {
	if err := checkBatch(arena, descs, status, true); err != nil {
		return 0, err
	}
	n := len(descs)
	if n == 0 {
		return 0, nil
	}
	gg.bmu.Lock()
	defer gg.bmu.Unlock()
	if 12*n > gg.ncap {
		if gg.nonces != nil {
			C.qgcm_host_free(gg.nonces)
		}
		gg.nonces, gg.ncap = C.qgcm_host_alloc(C.size_t(12*n)), 12*n
		if gg.nonces == nil {
			gg.ncap = 0
			return 0, errors.New("qgcm: pinned allocation failed")
		}
	}
	if rc := C.qgcm_random_nonces((*C.uint8_t)(gg.nonces), C.uint32_t(n)); rc != C.QGCM_OK {
		return 0, errors.New(C.GoString(C.qgcm_strerror(rc)))
	}
	rc := C.qgcm_group_seal_host(gg.grp, (*C.uint8_t)(arena.p), (*C.qgcm_desc)(unsafe.Pointer(&descs[0])),
		C.uint32_t(n), (*C.uint8_t)(gg.nonces), 4, bytePtr(status))
	if rc < 0 {
		return 0, fmt.Errorf("qgcm: group seal: %s", C.GoString(C.qgcm_strerror(rc)))
	}
	return int(rc), nil
}

// OpenBatch opens every packet of the batch in place, as Decrypt does one (crypto/aes.go:57-62):
// slot [AAD][ciphertext][tag][nonce] (Len = L+28) becomes [AAD][plaintext L]...; a packet whose tag
// does not verify gets status 0 and its plaintext region zeroed, as Go's gcm Open leaves it.
// Returns the number of failed packets.
func (gg *GPUGroup) OpenBatch(arena *Arena, descs []Desc, status []byte) (int, error) {
	if err := checkBatch(arena, descs, status, false); err != nil {
		return 0, err
	}
	if len(descs) == 0 {
		return 0, nil
	}
	gg.bmu.Lock()
	defer gg.bmu.Unlock()
	rc := C.qgcm_group_open_host(gg.grp, (*C.uint8_t)(arena.p), (*C.qgcm_desc)(unsafe.Pointer(&descs[0])),
		C.uint32_t(len(descs)), 4, bytePtr(status))
	if rc < 0 {
		return 0, fmt.Errorf("qgcm: group open: %s", C.GoString(C.qgcm_strerror(rc)))
	}
	return int(rc), nil
}
