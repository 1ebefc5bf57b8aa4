// cpu_chain.cpp -- BASELINE config 1, the reference's CPU configuration, as bench.py's cpu_baseline
// (TEST / BASELINE INFRASTRUCTURE: never part of the product path).
//
// The reference's plugin chain over common.Payload (plugin/plugin_test.go:163-216 TestMulti with the
// worker pipelines' framing, worker/outgoing.go:55-80 and worker/incoming.go:54-79): per packet,
// NewTunPayload(Raw, L), the sorted plugins' Apply(Outgoing) -- Encryption (plugin/encryption.go:16-40)
// then Mock (plugin/mock.go) -- then NewSockPayload(Raw, Length) and the reverse-sorted plugins'
// Apply(Incoming).  The chain is this repo's C++ mirror of the Go code (include/quantum.hpp, compiled
// into libqgcm.so; no device call is made here); the AES under it is OpenSSL EVP aes-256-gcm with
// crypto/aes.go:41-62 semantics (a getrandom nonce per Encrypt, in place, nonce appended; Decrypt
// takes the last 12 bytes as the nonce) standing in for Go 1.9's crypto/cipher GCM (AES-NI +
// PCLMULQDQ assembly), which is not in this image.
//
// Usage: cpu_chain <threads> <payloads per thread> <L> <seconds> [nonces]
// Each thread owns `payloads` Payload.Raw buffers (1472 B, common.MaxPacketLength) and loops over
// them for `seconds`; the clock starts once every thread has built its buffers (set-up is not
// throughput).  nonces: "syscall" (default) -- one getrandom(2) per Encrypt, as Go 1.9's crypto/rand
// does for crypto/aes.go:44 -- or "buffered": 4 KiB of getrandom output per thread, 341 nonces a
// syscall (what libqgcm's per-packet path does), to separate the kernel's RNG from the cipher when
// threads do not scale.  Prints one JSON line: packets sealed and opened per second, GiB/s (each
// payload byte counted once sealed and once opened), the process's user / system CPU seconds over the
// timed part, and whether every payload came back intact.  QGCM_CHAIN_CPUS="a,b,c": thread t runs
// pinned on the t-th listed CPU (mod the list), e.g. one CPU per physical core (bench.py's sweep).
#include <openssl/evp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <sched.h>
#include <sys/random.h>
#include <sys/resource.h>

#include <atomic>
#include <chrono>
#include <memory>
#include <thread>
#include <vector>

#include "../include/quantum.hpp"

using namespace quantum;

namespace {

bool g_buffered = false;

bool draw_nonce(uint8_t nonce[12]) {
    if (!g_buffered) return getrandom(nonce, 12, 0) == 12;
    thread_local uint8_t buf[4092];
    thread_local size_t left = 0;
    if (left < 12) {
        if (getrandom(buf, sizeof buf, 0) != (ssize_t)sizeof buf) return false;
        left = sizeof buf;
    }
    memcpy(nonce, buf + sizeof buf - left, 12);
    left -= 12;
    return true;
}

double cpu_seconds(bool sys) {
    rusage ru{};
    getrusage(RUSAGE_SELF, &ru);
    const timeval &t = sys ? ru.ru_stime : ru.ru_utime;
    return t.tv_sec + t.tv_usec * 1e-6;
}

class OsslAES : public crypto::AES {
  public:
    explicit OsslAES(const uint8_t key[32]) {
        e_ = EVP_CIPHER_CTX_new();
        d_ = EVP_CIPHER_CTX_new();
        EVP_EncryptInit_ex(e_, EVP_aes_256_gcm(), nullptr, key, nullptr);
        EVP_DecryptInit_ex(d_, EVP_aes_256_gcm(), nullptr, key, nullptr);
    }
    ~OsslAES() override {
        EVP_CIPHER_CTX_free(e_);
        EVP_CIPHER_CTX_free(d_);
    }
    // crypto/aes.go:41-52
    std::pair<int, Error> Encrypt(common::Slice data, int length, common::Slice additional) const override {
        uint8_t nonce[12];
        if (!draw_nonce(nonce)) return {-1, Error{"rand"}};
        if ((size_t)length + 28 > data.cap) return {-1, Error{"short buffer"}};
        int out = 0, ok = 1;
        ok &= EVP_EncryptInit_ex(e_, nullptr, nullptr, nullptr, nonce);
        if (additional.len) ok &= EVP_EncryptUpdate(e_, nullptr, &out, additional.data, (int)additional.len);
        ok &= EVP_EncryptUpdate(e_, data.data, &out, data.data, length);
        ok &= EVP_EncryptFinal_ex(e_, data.data + length, &out);
        ok &= EVP_CIPHER_CTX_ctrl(e_, EVP_CTRL_GCM_GET_TAG, 16, data.data + length);
        memcpy(data.data + length + 16, nonce, 12);
        if (!ok) return {-1, Error{"seal"}};
        return {length + 28, Error{}};
    }
    // crypto/aes.go:57-62
    std::pair<int, Error> Decrypt(common::Slice data, common::Slice additional) const override {
        if (data.len < 28) return {-1, Error{"short"}};
        const int length = (int)data.len - 12, L = length - 16;
        int out = 0, ok = 1;
        ok &= EVP_DecryptInit_ex(d_, nullptr, nullptr, nullptr, data.data + length);
        if (additional.len) ok &= EVP_DecryptUpdate(d_, nullptr, &out, additional.data, (int)additional.len);
        ok &= EVP_DecryptUpdate(d_, data.data, &out, data.data, L);
        ok &= EVP_CIPHER_CTX_ctrl(d_, EVP_CTRL_GCM_SET_TAG, 16, data.data + L);
        ok &= EVP_DecryptFinal_ex(d_, data.data + L, &out) > 0;
        if (!ok) {
            memset(data.data, 0, (size_t)L);
            return {L, Error{"cipher: message authentication failed"}};
        }
        return {L, Error{}};
    }

  private:
    EVP_CIPHER_CTX *e_ = nullptr, *d_ = nullptr;
};

}  // namespace

int main(int argc, char **argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 1;
    const int payloads = argc > 2 ? atoi(argv[2]) : 10000;
    const int L = argc > 3 ? atoi(argv[3]) : 1350;
    const double seconds = argc > 4 ? atof(argv[4]) : 2.0;
    g_buffered = argc > 5 && !strcmp(argv[5], "buffered");
    std::vector<int> pin;
    if (const char *cl = getenv("QGCM_CHAIN_CPUS"))
        for (const char *p = cl; *p;) {
            pin.push_back(atoi(p));
            while (*p && *p != ',') ++p;
            if (*p == ',') ++p;
        }
    if (threads < 1 || payloads < 1 || L < 0 || L + 4 + 28 > common::MaxPacketLength) return 2;
    uint8_t key[32];
    const char *secret = "AES256Key-32Characters1234567890";
    uint8_t salt[32];
    for (int i = 0; i < 32; ++i) salt[i] = (uint8_t)i;
    if (qgcm_derive_key((const uint8_t *)secret, 32, salt, 32, key) != QGCM_OK) return 2;  // crypto/aes.go:66
    std::atomic<long> done{0};
    std::atomic<int> bad{0};
    std::atomic<bool> stop{false}, go{false};
    std::atomic<int> ready{0};
    std::vector<std::thread> ths;
    for (int t = 0; t < threads; ++t) {
        ths.emplace_back([&, t] {
            if (!pin.empty()) {
                cpu_set_t one;
                CPU_ZERO(&one);
                CPU_SET(pin[t % pin.size()], &one);
                pthread_setaffinity_np(pthread_self(), sizeof one, &one);
            }
            // one Encryption and one Mock plugin per worker, sorted as main.go:50-51 does
            auto enc = plugin::New(plugin::EncryptionPlugin).first;
            auto mock = plugin::New(plugin::MockPlugin).first;
            std::vector<plugin::Plugin *> out = {mock.get(), enc.get()}, in = out;
            plugin::Sort(out);
            plugin::Sort(in, true);
            common::Mapping mapping;
            mapping.SupportedPlugins = {plugin::EncryptionPlugin};
            mapping.AES = std::make_shared<OsslAES>(key);
            std::vector<std::vector<uint8_t>> bufs(payloads, std::vector<uint8_t>(common::MaxPacketLength));
            std::vector<uint8_t> ref(L);
            for (int i = 0; i < L; ++i) ref[i] = (uint8_t)(i * 131 + t);
            for (auto &b : bufs) {
                const uint8_t ip[4] = {10, 99, 0, (uint8_t)t};
                memcpy(b.data(), ip, 4);
                memcpy(b.data() + 4, ref.data(), L);
            }
            ++ready;
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            long n = 0;
            for (bool first = true; first || !stop.load(std::memory_order_relaxed); first = false) {
                for (auto &b : bufs) {
                    common::Slice raw = common::MakeSlice(b);
                    common::Payload p = common::NewTunPayload(raw, L);  // worker/outgoing.go:58
                    common::Payload *pp = &p;
                    common::Mapping *mp = &mapping;
                    bool ok = true;
                    for (plugin::Plugin *pl : out) {  // worker/outgoing.go:66-72
                        auto r = pl->Apply(plugin::Outgoing, pp, mp);
                        pp = r.payload;
                        ok &= r.ok;
                    }
                    common::Payload q = common::NewSockPayload(raw, pp->Length);  // worker/incoming.go:58
                    pp = &q;
                    for (plugin::Plugin *pl : in) {  // worker/incoming.go:66-72
                        auto r = pl->Apply(plugin::Incoming, pp, mp);
                        pp = r.payload;
                        ok &= r.ok;
                    }
                    if (first && (!ok || pp->Length != L + 4 || memcmp(b.data() + 4, ref.data(), L) != 0)) ++bad;
                    ++n;
                }
            }
            done += n;
        });
    }
    while (ready.load() < threads) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    const double u0 = cpu_seconds(false), s0 = cpu_seconds(true);
    const auto t0 = std::chrono::steady_clock::now();
    go.store(true, std::memory_order_release);
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    stop = true;
    for (auto &th : ths) th.join();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double us = cpu_seconds(false) - u0, ss = cpu_seconds(true) - s0;
    const double pps = done.load() / dt;
    printf("{\"threads\": %d, \"payloads_per_thread\": %d, \"payload_len\": %d, \"nonces\": \"%s\", "
           "\"pinned\": %s, \"seconds\": %.3f, \"packets_per_s\": %.0f, \"GiB_s\": %.4f, \"user_s\": %.3f, \"sys_s\": %.3f, "
           "\"cpus_busy\": %.2f, \"intact\": %s}\n",
           threads, payloads, L, g_buffered ? "buffered" : "syscall", pin.empty() ? "false" : "true", dt, pps, 2.0 * pps * L / (1 << 30), us, ss,
           (us + ss) / dt, bad.load() ? "false" : "true");
    return bad.load() ? 1 : 0;
}
