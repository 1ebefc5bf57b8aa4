// +build gpu

// aes_gpu_test.go -- with `go test -tags gpu ./crypto` on a machine with an MI355X, the package's own
// crypto_test.go TestAES and BenchmarkAES (crypto_test.go:54-131) run unchanged against the GPU-backed
// AES of aes_gpu.go (NewAES is the same call).  This file adds what they do not cover: the edges the shim
// guards (nil additional data, short buffers, tampering), many goroutines on one AES, keys spread over
// the members of the process-wide device set, slot recycling, and a batched worker's round trip.
// TestMain makes the process-wide set two members on device 0 unless QGCM_DEVICES says otherwise, so the
// multi-member paths run on a 1-GPU box too.  tests/cpp/go_replay.c replays the same C call sequence
// from C, which this image can build and the GPU box can run (there is no Go toolchain in either).
package crypto

import (
	"os"
	"runtime"
	"sync"
	"testing"
	"time"
)

func TestMain(m *testing.M) {
	if os.Getenv("QGCM_DEVICES") == "" {
		os.Setenv("QGCM_DEVICES", "0,0")
	}
	if os.Getenv("QGCM_MAX_PEERS") == "" {
		os.Setenv("QGCM_MAX_PEERS", "64")
	}
	os.Exit(m.Run())
}

func TestAESEdges(t *testing.T) {
	aes, err := NewAES([]byte("AES256Key-32Characters1234567890"), make([]byte, SaltLength))
	if err != nil {
		t.Fatal(err)
	}
	ip := []byte{10, 99, 0, 1}
	if n, err := aes.Encrypt(make([]byte, 27), 0, ip); err == nil || n != -1 {
		t.Fatal("Encrypt into a buffer without room for tag and nonce must fail")
	}
	empty := make([]byte, 28)
	if n, err := aes.Encrypt(empty, 0, ip); err != nil || n != 28 {
		t.Fatalf("Encrypt of an empty payload: %d %v", n, err)
	}
	if n, err := aes.Decrypt(empty, ip); err != nil || n != 0 {
		t.Fatalf("Decrypt of an empty payload: %d %v", n, err)
	}
	for _, l := range []int{0, 5, 11, 12, 27} { // the reference panics below 12, errOpen up to 27
		short := make([]byte, l)
		if _, err := aes.Decrypt(short, ip); err != errOpen {
			t.Fatalf("Decrypt of %d bytes: %v", l, err)
		}
	}
	data := make([]byte, 1350+28)
	fillSlice(data[:1350])
	if _, err := aes.Encrypt(data, 1350, ip); err != nil {
		t.Fatal(err)
	}
	data[7] ^= 1
	if _, err := aes.Decrypt(data, ip); err != errOpen {
		t.Fatal("a tampered packet must fail")
	}
	for _, b := range data[:1350] {
		if b != 0 {
			t.Fatal("the plaintext of a failed Open must be zeroed (Go 1.9 gcm Open)")
		}
	}
}

// TestAESConcurrentGoroutines: quantum's 2 x NumWorkers locked worker threads (main.go:72-75) call one
// peer's AES at once, each with its own 1472-B buffer (worker/outgoing.go:88).
func TestAESConcurrentGoroutines(t *testing.T) {
	aes, err := NewAES([]byte("AES256Key-32Characters1234567890"), make([]byte, SaltLength))
	if err != nil {
		t.Fatal(err)
	}
	var wg sync.WaitGroup
	fail := make(chan string, 16)
	for w := 0; w < 16; w++ {
		wg.Add(1)
		go func(w int) {
			defer wg.Done()
			runtime.LockOSThread() // worker/outgoing.go:86
			buf := make([]byte, 1472)
			ip := []byte{10, 99, 0, byte(w)}
			for i := 0; i < 200; i++ {
				l := (w*131 + i*17) % 1433
				for j := 0; j < l; j++ {
					buf[4+j] = byte(w + i + j)
				}
				n, err := aes.Encrypt(buf[4:], l, ip)
				if err != nil || n != l+28 {
					fail <- "encrypt"
					return
				}
				if m, err := aes.Decrypt(buf[4:4+n], ip); err != nil || m != l {
					fail <- "decrypt"
					return
				}
				for j := 0; j < l; j++ {
					if buf[4+j] != byte(w+i+j) {
						fail <- "roundtrip"
						return
					}
				}
			}
		}(w)
	}
	wg.Wait()
	close(fail)
	for f := range fail {
		t.Fatal(f)
	}
}

// TestNewAESAcrossMembers: peers' keys land on different members of the process-wide set (hash of the
// key slot), each peer's packets seal and open on its member, and two peers derived from different
// salts do not open each other's packets.
func TestNewAESAcrossMembers(t *testing.T) {
	gg, err := Devices()
	if err != nil {
		t.Fatal(err)
	}
	members := map[int]bool{}
	var peers []*AES
	for k := 0; k < 6; k++ {
		salt := make([]byte, SaltLength)
		for i := range salt {
			salt[i] = byte(0x70 + k)
		}
		a, err := gg.NewAES([]byte("AES256Key-32Characters1234567890"), salt)
		if err != nil {
			t.Fatal(err)
		}
		members[a.Member()] = true
		peers = append(peers, a)
	}
	if n := gg.Size(); n > 1 && len(members) < 2 {
		t.Fatalf("6 peers on %d members all landed on one", n)
	}
	ip := []byte{10, 99, 0, 9}
	for k, a := range peers {
		data := make([]byte, 500+28)
		for j := range data[:500] {
			data[j] = byte(j + k)
		}
		if n, err := a.Encrypt(data, 500, ip); err != nil || n != 528 {
			t.Fatalf("peer %d Encrypt: %d %v", k, n, err)
		}
		other := peers[(k+1)%len(peers)]
		wrong := append([]byte(nil), data...)
		if _, err := other.Decrypt(wrong, ip); err != errOpen {
			t.Fatalf("peer %d's packet opened under peer %d's key", k, (k+1)%len(peers))
		}
		if n, err := a.Decrypt(data, ip); err != nil || n != 500 {
			t.Fatalf("peer %d Decrypt: %d %v", k, n, err)
		}
		for j := range data[:500] {
			if data[j] != byte(j+k) {
				t.Fatalf("peer %d did not round-trip", k)
			}
		}
	}
}

// TestSlotsRecycled: ParseMapping runs again on every mapping update (datastore/etcdv2.go:236-276), so
// NewAES is called far more often than there are peers; unreachable AES objects give their slots back.
func TestSlotsRecycled(t *testing.T) {
	gg, err := Devices()
	if err != nil {
		t.Fatal(err)
	}
	for i := 0; i < 4*int(gg.max); i++ {
		a, err := NewAES([]byte("AES256Key-32Characters1234567890"), make([]byte, SaltLength))
		for tries := 0; err == errSlots && tries < 50; tries++ {
			runtime.GC() // the finalizers of collected AES objects return their slots
			time.Sleep(10 * time.Millisecond)
			a, err = NewAES([]byte("AES256Key-32Characters1234567890"), make([]byte, SaltLength))
		}
		if err != nil {
			t.Fatalf("NewAES #%d: %v", i, err)
		}
		buf := make([]byte, 64+28)
		if n, err := a.Encrypt(buf, 64, nil); err != nil || n != 92 {
			t.Fatalf("Encrypt on recycled slot %d: %d %v", a.KeyIndex(), n, err)
		}
		if n, err := a.Decrypt(buf, nil); err != nil || n != 64 {
			t.Fatalf("Decrypt on recycled slot %d: %d %v", a.KeyIndex(), n, err)
		}
	}
}

// TestGPUGroupBatch: a batched worker's round trip over a two-member group: 600 packets of 8 peers
// laid out in Order's order in a pinned arena, SealBatch, then OpenBatch restores every payload; a
// tampered packet fails with its plaintext zeroed, and a slot no NewAES filled fails with its slot
// untouched.  tests/cpp/go_replay.c TestGPUGroupBatch replays the same calls against the oracle.
func TestGPUGroupBatch(t *testing.T) {
	gg, err := NewGPUGroup([]int{0, 0}, 16)
	if err != nil {
		t.Fatal(err)
	}
	defer gg.Close()
	const peers, n = 8, 600
	var keyOf [peers]uint32
	live := make([]*AES, 0, peers)
	for k := 0; k < peers-1; k++ {
		salt := make([]byte, SaltLength)
		for i := range salt {
			salt[i] = byte(0x40 + k)
		}
		a, err := gg.NewAES([]byte("AES256Key-32Characters1234567890"), salt)
		if err != nil {
			t.Fatal(err)
		}
		keyOf[k] = a.KeyIndex()
		live = append(live, a)
	}
	keyOf[peers-1] = peers - 1 // a slot no NewAES filled
	peer := make([]uint32, n)
	for i := range peer {
		peer[i] = keyOf[(i*7+i/5)%peers]
	}
	order, counts, err := gg.Order(peer)
	if err != nil || counts[0]+counts[1] != n {
		t.Fatalf("Order: %v %v", counts, err)
	}
	descs := make([]Desc, n)
	off := 0
	for j, i := range order {
		l := 1 + (int(i)*37)%1400
		descs[j] = Desc{Offset: uint64(off), Len: uint32(l), Key: peer[i]}
		off += (4 + l + 28 + 15) &^ 15
	}
	arena, err := NewArena(off)
	if err != nil {
		t.Fatal(err)
	}
	defer arena.Free()
	for b := range arena.Bytes {
		arena.Bytes[b] = byte(b*131 + 7)
	}
	plain := append([]byte(nil), arena.Bytes...)
	status := make([]byte, n)
	unset := 0
	for _, d := range descs {
		if d.Key == peers-1 {
			unset++
		}
	}
	if bad, err := gg.SealBatch(arena, descs, status); err != nil || bad != unset {
		t.Fatalf("SealBatch: %d failed (want %d), %v", bad, unset, err)
	}
	victim := 0
	for descs[victim].Key == peers-1 {
		victim++
	}
	arena.Bytes[descs[victim].Offset+4] ^= 1
	for j := range descs {
		descs[j].Len += 28
	}
	if bad, err := gg.OpenBatch(arena, descs, status); err != nil || bad != unset+1 {
		t.Fatalf("OpenBatch: %d failed (want %d), %v", bad, unset+1, err)
	}
	for j, d := range descs {
		o, l := int(d.Offset), int(d.Len)-28
		switch {
		case d.Key == peers-1:
			if status[j] != 0 || string(arena.Bytes[o:o+4+l+28]) != string(plain[o:o+4+l+28]) {
				t.Fatalf("packet %d of the unset key was touched", j)
			}
		case j == victim:
			for _, b := range arena.Bytes[o+4 : o+4+l] {
				if status[j] != 0 || b != 0 {
					t.Fatal("the tampered packet must fail with its plaintext zeroed")
				}
			}
		default:
			if status[j] != 1 || string(arena.Bytes[o:o+4+l]) != string(plain[o:o+4+l]) {
				t.Fatalf("packet %d did not round-trip", j)
			}
		}
	}
	runtime.KeepAlive(live) // their slots are named by the batch's Descs
}
