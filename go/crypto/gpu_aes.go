// Copyright (c) 2026. Licensed under the MPL-2.0 like the quantum tree it is added to.

// +build gpu

// gpu_aes.go -- the MI355X drop-in for quantum's crypto.AES (crypto/aes.go), over libqgcm's C ABI
// (include/qgcm.h).  A maintainer copies this file into quantum's crypto/ directory and builds with
// `go build -tags gpu`; without the tag the package builds exactly as before.  The cgo preamble,
// the prebuilt-library LDFLAGS and the "NULL plus a 120-byte error string" convention follow
// crypto/dtls.go:6-40, the reference's own cgo layer.
//
// GPUAES has crypto.AES's method set -- EncryptedSize, DecryptedSize, Encrypt, Decrypt
// (crypto/aes.go:29-62) -- with the same sizes, buffer layout (ct || tag || nonce, in place) and errors,
// so plugin/encryption.go:16-40 calls it unchanged once common.Mapping.AES (common/mapping.go:54) is
// typed by that method set (INTEGRATION.md s1).  Differences, all where the reference would panic:
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
	"sync"
	"unsafe"
)

var (
	// errOpen is the error cipher.AEAD.Open returns on a tag mismatch (crypto/cipher gcm.go).
	errOpen        = errors.New("cipher: message authentication failed")
	errShortBuffer = errors.New("qgcm: data buffer shorter than length + 28")
	errAdditional  = errors.New("qgcm: additional data longer than 4 bytes")
	errSlots       = errors.New("qgcm: out of key slots")
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

// GPUContext owns one MI355X device's key tables (qgcm_ctx): the device-side state of every
// crypto.AES object of the process.
type GPUContext struct {
	ctx  *C.qgcm_ctx
	mu   sync.Mutex
	next uint32
	max  uint32
}

// NewGPUContext opens device `device` with room for maxKeys peer keys.
func NewGPUContext(device int, maxKeys uint32) (*GPUContext, error) {
	buf := (*C.char)(C.malloc(C.QGCM_ERRLEN))
	defer C.free(unsafe.Pointer(buf))
	ctx := C.qgcm_create(C.int(device), C.uint32_t(maxKeys), buf, C.QGCM_ERRLEN)
	if ctx == nil {
		return nil, cError(buf)
	}
	return &GPUContext{ctx: ctx, max: maxKeys}, nil
}

// Close releases the device context (no call may be in flight).
func (g *GPUContext) Close() {
	if g.ctx != nil {
		C.qgcm_destroy(g.ctx)
		g.ctx = nil
	}
}

// GPUAES is a drop-in for *crypto.AES (crypto/aes.go:22-26): one key slot of a GPUContext.
type GPUAES struct {
	g    *GPUContext
	ctx  *C.qgcm_ctx // the context that holds the key (a group member's, see GPUGroup)
	idx  uint32
	salt []byte
}

// NewGPUAES replaces NewAES (crypto/aes.go:65-83): PBKDF2-HMAC-SHA512(secret, salt, 10000, 32) on
// the host (qgcm_derive_key), then aes.NewCipher + cipher.NewGCM as a device key schedule and GHASH
// tables (qgcm_set_key).
func (g *GPUContext) NewGPUAES(secret, salt []byte) (*GPUAES, error) {
	g.mu.Lock()
	idx := g.next
	if idx >= g.max {
		g.mu.Unlock()
		return nil, errSlots
	}
	g.next++
	g.mu.Unlock()
	if err := installKey(g.ctx, idx, secret, salt); err != nil {
		return nil, err
	}
	return &GPUAES{g: g, ctx: g.ctx, idx: idx, salt: salt}, nil
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

// EncryptedSize == crypto/aes.go:29-31.
func (a *GPUAES) EncryptedSize(data []byte) int { return len(data) + overhead }

// DecryptedSize == crypto/aes.go:34-36.
func (a *GPUAES) DecryptedSize(data []byte) int { return len(data) - overhead }

// Encrypt == crypto/aes.go:41-52: seals data[:length] in place, then the 16-byte tag and the 12-byte
// nonce (drawn by libqgcm from getrandom(2), crypto/rand's source); returns length + 28.
func (a *GPUAES) Encrypt(data []byte, length int, additional []byte) (int, error) {
	if length < 0 || length+overhead > len(data) {
		return -1, errShortBuffer
	}
	if len(additional) > 4 {
		return -1, errAdditional
	}
	// one packet per call, served by libqgcm's resident kernel (no launch per call)
	n := C.qgcm_seal_one(a.ctx, C.uint32_t(a.idx), bytePtr(data), C.long(length), bytePtr(additional),
		C.uint32_t(len(additional)), nil)
	if n < 0 {
		return -1, errors.New("qgcm: seal failed")
	}
	return int(n), nil
}

// Decrypt == crypto/aes.go:57-62: opens data in place (nonce = the last 12 bytes, tag the 16 before);
// returns len(data) - 28.  On a tag mismatch the plaintext region is zeroed, as Go 1.9's gcm Open does.
func (a *GPUAES) Decrypt(data []byte, additional []byte) (int, error) {
	if len(data) < overhead || len(additional) > 4 {
		return a.DecryptedSize(data), errOpen
	}
	n := C.qgcm_open_one(a.ctx, C.uint32_t(a.idx), bytePtr(data), C.long(len(data)), bytePtr(additional),
		C.uint32_t(len(additional)))
	if n < 0 {
		return a.DecryptedSize(data), errOpen
	}
	return int(n), nil
}

// GPUGroup drives every GPU of a node from quantum's one process (qgcm_group_*): a peer's key lives on
// GPU hash(key index) mod G, and that peer's per-packet calls go to that GPU (SURVEY.md s8e).
type GPUGroup struct {
	grp  *C.qgcm_group
	mu   sync.Mutex
	next uint32
	max  uint32

	bmu    sync.Mutex     // one batch at a time (qgcm_group_seal_host serializes calls anyway)
	nonces unsafe.Pointer // pinned nonce buffer of the last SealBatch (qgcm_host_alloc), 12 B per packet
	ncap   int
}

// NewGPUGroup opens one context per device in `devices`.
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

// NewGPUAES derives the key and installs it on its owning GPU only; the returned object seals and
// opens there.
func (gg *GPUGroup) NewGPUAES(secret, salt []byte) (*GPUAES, error) {
	gg.mu.Lock()
	idx := gg.next
	if idx >= gg.max {
		gg.mu.Unlock()
		return nil, errSlots
	}
	gg.next++
	gg.mu.Unlock()
	owner := C.qgcm_group_shard(gg.grp, C.uint32_t(idx))
	ctx := C.qgcm_group_ctx(gg.grp, owner)
	if ctx == nil {
		return nil, errors.New("qgcm: no owner context")
	}
	if err := installKey(ctx, idx, secret, salt); err != nil {
		return nil, err
	}
	return &GPUAES{ctx: ctx, idx: idx, salt: salt}, nil
}

// Close releases every member context.
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
// 65536 packets and 128 MiB) whose slots start 16-B aligned, e.g. the 1472-B MaxPacketLength
// stride, is sealed in place in the arena instead (qgcm_group_last_path 3).

// KeyIndex is the key slot of this peer: the Key field of its packets' Descs.
func (a *GPUAES) KeyIndex() uint32 { return a.idx }

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
// peer's key slot (KeyIndex).  The slot is [4-B AAD (the IP header, Payload.Raw[0:4])][packet] with
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
