// udp_e2e.cpp -- the whole outgoing + incoming path of one tunnel over loopback UDP, batched:
//   "TUN" packets (Payload.Raw slots) -> qgcm_seal_host (pinned H2D, gfx950 seal, D2H)
//   -> qgcm_udp_send_slots (sendmmsg) -> loopback -> qgcm_udp_recv_slots (recvmmsg)
//   -> qgcm_open_host -> plaintext checked against what was sent.
// worker/outgoing.go:55-80 and worker/incoming.go:54-79 with socket/udp.go:35-47, one batch per
// syscall and per device launch instead of one packet.  The receiver drains
// in its own thread; the sender keeps at most `window` datagrams unread so the default socket
// buffer (rmem_max, no privileges on the GPU box) never overflows -- a loss would be counted.
// Build: g++ -O2 -std=c++17 -Iinclude tools/udp_e2e.cpp -Lquantum_amd -lqgcm -Wl,-rpath,'$ORIGIN/../quantum_amd' -lpthread -o tools/udp_e2e
// Usage: tools/udp_e2e [batches] [packets_per_batch] [payload_len] [window] [datagrams_per_syscall]
// (datagrams_per_syscall 1 = the reference's one sendto / recvfrom per packet)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "qgcm.h"

using Clock = std::chrono::steady_clock;

int main(int argc, char **argv) {
    const uint32_t batches = argc > 1 ? atoi(argv[1]) : 64;
    const uint32_t B = argc > 2 ? atoi(argv[2]) : 16384;
    const uint32_t L = argc > 3 ? atoi(argv[3]) : 1350;
    const uint32_t window = argc > 4 ? atoi(argv[4]) : 96;
    const uint32_t per_call = argc > 5 ? (uint32_t)atoi(argv[5]) : 32;
    const uint64_t stride = 1472;  // common.MaxPacketLength
    if (L + 4 + QGCM_OVERHEAD > stride) {
        fprintf(stderr, "payload too long for a Raw slot\n");
        return 2;
    }
    char err[QGCM_ERRLEN];
    qgcm_ctx *ctx = qgcm_create(0, 4, err, sizeof err);
    if (!ctx) {
        fprintf(stderr, "qgcm_create: %s\n", err);
        return 1;
    }
    uint8_t key[32];
    const char *secret = "AES256Key-32Characters1234567890";
    uint8_t salt[32];
    for (int i = 0; i < 32; ++i) salt[i] = (uint8_t)i;
    qgcm_derive_key((const uint8_t *)secret, 32, salt, 32, key);
    qgcm_set_key(ctx, 0, key);

    uint8_t *tx = (uint8_t *)qgcm_host_alloc(B * stride), *rx = (uint8_t *)qgcm_host_alloc(B * stride);
    uint8_t *nonces = (uint8_t *)qgcm_host_alloc(12ull * B);
    std::vector<uint8_t> plain(B * stride);
    std::vector<uint32_t> tx_lens(B, L + 4 + QGCM_OVERHEAD), rx_lens(B);
    uint64_t x = 0x5EED0001;
    for (uint32_t i = 0; i < B; ++i) {
        uint8_t *s = plain.data() + i * stride;
        s[0] = 10, s[1] = 99, s[2] = 0, s[3] = 1;  // the sender's private IP: the AAD
        for (uint32_t j = 0; j < L; ++j) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            s[4 + j] = (uint8_t)(x >> 56);
        }
    }
    const int a = qgcm_udp_socket("127.0.0.1", 0, 1 << 22), b = qgcm_udp_socket("127.0.0.1", 0, 1 << 22);
    if (a < 0 || b < 0) {
        fprintf(stderr, "sockets\n");
        return 1;
    }
    const int port_b = qgcm_udp_port(b);

    std::atomic<uint64_t> rx_count{0};
    std::atomic<bool> rx_fail{false};
    double t_open = 0, t_recv = 0;
    uint64_t bad_bytes = 0, lost = 0;
    std::thread receiver([&] {
        for (uint32_t k = 0; k < batches; ++k) {
            uint32_t got = 0;
            const auto t0 = Clock::now();
            while (got < B) {
                const int r = qgcm_udp_recv_slots(b, rx + (uint64_t)got * stride, stride,
                                                  std::min<uint32_t>(B - got, per_call), &rx_lens[got], 2000);
                if (r <= 0) break;  // timeout: datagrams lost
                got += (uint32_t)r;
                rx_count += (uint64_t)r;
            }
            const auto t1 = Clock::now();
            lost += B - got;
            // incoming.go:60-67: the decrypt step of the chain, on the whole received batch
            const int bad = qgcm_open_host(ctx, rx, stride, got, L + QGCM_OVERHEAD, 0, 4, nullptr);
            const auto t2 = Clock::now();
            if (bad != 0) rx_fail = true;
            for (uint32_t i = 0; i < got; ++i)
                if (rx_lens[i] != L + 4 + QGCM_OVERHEAD || memcmp(rx + i * stride, plain.data() + i * stride, 4 + L))
                    ++bad_bytes;
            t_recv += std::chrono::duration<double>(t1 - t0).count();
            t_open += std::chrono::duration<double>(t2 - t1).count();
        }
    });

    double t_seal = 0, t_send = 0;
    uint64_t sent_total = 0;
    const auto start = Clock::now();
    for (uint32_t k = 0; k < batches; ++k) {
        memcpy(tx, plain.data(), B * stride);  // the TUN reads of this batch
        qgcm_random_nonces(nonces, B);          // crypto/aes.go:42-47, one getrandom per batch
        const auto t0 = Clock::now();
        if (qgcm_seal_host(ctx, tx, stride, B, L, 0, nonces, 4, nullptr) != 0) {
            fprintf(stderr, "seal_host failed\n");
            return 1;
        }
        const auto t1 = Clock::now();
        for (uint32_t i = 0; i < B;) {
            while (sent_total - rx_count.load() > window) std::this_thread::yield();
            const uint32_t n = std::min<uint32_t>(B - i, per_call);
            const int r = qgcm_udp_send_slots(a, tx + (uint64_t)i * stride, stride, n, &tx_lens[i], "127.0.0.1", port_b);
            if (r <= 0) {
                fprintf(stderr, "send failed\n");
                return 1;
            }
            i += (uint32_t)r;
            sent_total += (uint64_t)r;
        }
        const auto t2 = Clock::now();
        t_seal += std::chrono::duration<double>(t1 - t0).count();
        t_send += std::chrono::duration<double>(t2 - t1).count();
    }
    receiver.join();
    const double wall = std::chrono::duration<double>(Clock::now() - start).count();
    const double pkts = (double)batches * B;
    printf("{\"config\": \"udp_loopback_e2e\", \"batches\": %u, \"packets_per_batch\": %u, \"payload_len\": %u, "
           "\"window\": %u, \"datagrams_per_syscall\": %u, \"wall_s\": %.4f, \"packets_per_s\": %.0f, \"payload_GiBps\": %.3f, "
           "\"seal_host_s\": %.4f, \"send_s\": %.4f, \"recv_s\": %.4f, \"open_host_s\": %.4f, "
           "\"lost\": %lu, \"bad\": %lu, \"auth_ok\": %s}\n",
           batches, B, L, window, per_call, wall, pkts / wall, pkts * L / wall / (1 << 30), t_seal, t_send, t_recv, t_open,
           (unsigned long)lost, (unsigned long)bad_bytes, rx_fail ? "false" : "true");
    qgcm_udp_close(a);
    qgcm_udp_close(b);
    qgcm_host_free(tx);
    qgcm_host_free(rx);
    qgcm_host_free(nonces);
    qgcm_destroy(ctx);
    return (lost || bad_bytes || rx_fail) ? 3 : 0;
}
