// +build gpu

// gpu_aes_test.go -- crypto/crypto_test.go's TestAES and BenchmarkAES (crypto_test.go:54-131) run on
// GPUAES, plus the edges the shim guards (nil additional data, short buffers, tampering, many
// goroutines calling one GPUAES at once) and a batched worker's round trip over a GPUGroup.  `go test -tags gpu ./crypto` on a machine with an MI355X.
// tests/cpp/go_replay.c replays the same C call sequence from C, which this image can build and the
// GPU box can run (there is no Go toolchain in either).
package crypto

import (
	"crypto/rand"
	"sync"
	"testing"
)

func newGPUContext(t testing.TB) *GPUContext {
	g, err := NewGPUContext(0, 64)
	if err != nil {
		t.Fatalf("NewGPUContext: %s", err)
	}
	return g
}

func TestGPUAES(t *testing.T) {
	g := newGPUContext(t)
	defer g.Close()
	key := []byte("AES256Key-32Characters1234567890")
	salt := make([]byte, SaltLength)
	if _, err := rand.Read(salt); err != nil {
		t.Fatalf("Unable to random salt: %s", err)
	}
	aes, err := g.NewGPUAES(key, salt)
	if err != nil {
		t.Fatalf("Unable to create the AES object: %s", err)
	}
	buf := make([]byte, bufLen)
	expected := make([]byte, dataLen)
	fillSlice(buf[:dataLen])
	fillSlice(expected)
	if aes.EncryptedSize(buf) != len(buf)+tagLen+nonceLen {
		t.Fatal("The AES minimum size is incorrect")
	}
	length, err := aes.Encrypt(buf, dataLen, nil) // nil additional data, as TestAES
	if err != nil || length != aes.EncryptedSize(buf[:dataLen]) {
		t.Fatalf("Encrypt: %d %v", length, err)
	}
	if testEq(buf[:dataLen], expected) {
		t.Fatal("Encrypted output matches plaintext.")
	}
	length, err = aes.Decrypt(buf, nil)
	if err != nil || length != dataLen || !testEq(buf[:dataLen], expected) {
		t.Fatalf("Decrypt: %d %v", length, err)
	}
}

func TestGPUAESEdges(t *testing.T) {
	g := newGPUContext(t)
	defer g.Close()
	aes, err := g.NewGPUAES([]byte("AES256Key-32Characters1234567890"), make([]byte, SaltLength))
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

func TestGPUAESConcurrentGoroutines(t *testing.T) {
	g := newGPUContext(t)
	defer g.Close()
	aes, err := g.NewGPUAES([]byte("AES256Key-32Characters1234567890"), make([]byte, SaltLength))
	if err != nil {
		t.Fatal(err)
	}
	var wg sync.WaitGroup
	fail := make(chan string, 16)
	for w := 0; w < 16; w++ {
		wg.Add(1)
		go func(w int) {
			defer wg.Done()
			buf := make([]byte, 1472) // worker/outgoing.go:88, one buffer per worker
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

func BenchmarkGPUAES(b *testing.B) {
	g := newGPUContext(b)
	defer g.Close()
	aes, err := g.NewGPUAES([]byte("AES256Key-32Characters1234567890"), make([]byte, SaltLength))
	if err != nil {
		b.Fatal(err)
	}
	buf := make([]byte, bufLen)
	fillSlice(buf[:dataLen])
	b.SetBytes(dataLen)
	b.ResetTimer()
	for i := 0; i < b.N; i++ {
		n, _ := aes.Encrypt(buf, dataLen, nil)
		aes.Decrypt(buf[:n], nil)
	}
}

// TestGPUGroupBatch: a batched worker's round trip over a two-member group (both on device 0 here):
// 600 packets of 8 peers laid out in Order's order in a pinned arena, SealBatch, then OpenBatch
// restores every payload; a tampered packet fails with its plaintext zeroed, and a peer whose key was
// never installed fails with its slot untouched.  tests/cpp/go_replay.c TestGPUGroupBatch replays the
// same calls and checks each sealed slot against the oracle.
func TestGPUGroupBatch(t *testing.T) {
	gg, err := NewGPUGroup([]int{0, 0}, 16)
	if err != nil {
		t.Fatal(err)
	}
	defer gg.Close()
	const peers, n = 8, 600
	var keyOf [peers]uint32
	for k := 0; k < peers-1; k++ {
		salt := make([]byte, SaltLength)
		for i := range salt {
			salt[i] = byte(0x40 + k)
		}
		a, err := gg.NewGPUAES([]byte("AES256Key-32Characters1234567890"), salt)
		if err != nil {
			t.Fatal(err)
		}
		keyOf[k] = a.KeyIndex()
	}
	keyOf[peers-1] = peers - 1 // a slot no NewGPUAES filled
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
}
