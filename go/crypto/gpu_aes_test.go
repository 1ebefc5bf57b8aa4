// +build gpu

// gpu_aes_test.go -- crypto/crypto_test.go's TestAES and BenchmarkAES (crypto_test.go:54-131) run on
// GPUAES, plus the edges the shim guards (nil additional data, short buffers, tampering, many
// goroutines calling one GPUAES at once).  `go test -tags gpu ./crypto` on a machine with an MI355X.
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
