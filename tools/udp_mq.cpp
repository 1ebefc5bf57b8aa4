// udp_mq.cpp -- the tunnel of udp_e2e.cpp with quantum's multi-queue socket layout: Q worker pairs
// (worker/outgoing.go + worker/incoming.go, one per queue, main.go:72-75), each outgoing worker with
// its own socket (its own flow), the incoming side Q SO_REUSEPORT queues on one port
// (qgcm_udp_queue, socket/udp.go:55-70) that the kernel spreads the flows over.  Outgoing: "TUN"
// slots -> qgcm_seal_host -> sendmmsg.  Incoming: recvmmsg on its queue -> qgcm_open_host on whatever
// arrived -> each plaintext checked against the packet its first 4 payload bytes name.  All workers
// share one device context.  Flow control: at most `window` unread datagrams per outgoing worker.
// Build: g++ -O2 -std=c++17 -Iinclude tools/udp_mq.cpp -Lquantum_amd -lqgcm -Wl,-rpath,'$ORIGIN/../../quantum_amd' -lpthread -o tools/bin/udp_mq
// Usage: tools/bin/udp_mq [queues] [batches_per_worker] [packets_per_batch] [payload_len] [window]
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
    const int Q = argc > 1 ? atoi(argv[1]) : 4;
    const uint32_t batches = argc > 2 ? atoi(argv[2]) : 16;
    const uint32_t B = argc > 3 ? atoi(argv[3]) : 8192;
    const uint32_t L = argc > 4 ? atoi(argv[4]) : 1350;
    const uint32_t window = argc > 5 ? atoi(argv[5]) : 64;
    const uint32_t per_call = 32;
    const uint64_t stride = 1472;  // common.MaxPacketLength
    if (Q < 1 || Q > 64 || L < 4 || L + 4 + QGCM_OVERHEAD > stride) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    char err[QGCM_ERRLEN];
    qgcm_ctx *ctx = qgcm_create(0, 4, err, sizeof err);
    if (!ctx) {
        fprintf(stderr, "qgcm_create: %s\n", err);
        return 1;
    }
    uint8_t key[32], salt[32];
    for (int i = 0; i < 32; ++i) salt[i] = (uint8_t)i;
    qgcm_derive_key((const uint8_t *)"AES256Key-32Characters1234567890", 32, salt, 32, key);
    qgcm_set_key(ctx, 0, key);

    // the packets every outgoing worker sends: slot i's payload starts with i (LE)
    std::vector<uint8_t> plain(B * stride);
    uint64_t x = 0x5EED0001;
    for (uint32_t i = 0; i < B; ++i) {
        uint8_t *s = plain.data() + i * stride;
        s[0] = 10, s[1] = 99, s[2] = 0, s[3] = 1;
        for (uint32_t j = 0; j < L; ++j) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            s[4 + j] = (uint8_t)(x >> 56);
        }
        memcpy(s + 4, &i, 4);
    }
    std::vector<int> rxq(Q), txs(Q);
    rxq[0] = qgcm_udp_queue("127.0.0.1", 0, 1 << 22);
    const int port = rxq[0] >= 0 ? qgcm_udp_port(rxq[0]) : -1;
    for (int q = 1; q < Q; ++q) rxq[q] = qgcm_udp_queue("127.0.0.1", port, 1 << 22);
    for (int q = 0; q < Q; ++q) txs[q] = qgcm_udp_socket("127.0.0.1", 0, 1 << 22);
    for (int q = 0; q < Q; ++q)
        if (rxq[q] < 0 || txs[q] < 0) {
            fprintf(stderr, "sockets\n");
            return 1;
        }

    const uint64_t total = (uint64_t)Q * batches * B;
    std::atomic<uint64_t> dequeued{0}, received{0}, bad{0}, auth_fail{0};
    std::vector<std::atomic<uint64_t>> sent(Q);
    for (auto &s : sent) s = 0;
    std::atomic<int> senders_done{0};
    std::vector<uint64_t> per_queue(Q, 0);

    auto incoming = [&](int q) {  // worker/incoming.go on queue q
        uint8_t *rx = (uint8_t *)qgcm_host_alloc(B * stride);
        std::vector<uint32_t> lens(B);
        std::vector<uint8_t> st(B);
        for (;;) {
            uint32_t got = 0;
            while (got < B) {
                const int r = qgcm_udp_recv_slots(rxq[q], rx + (uint64_t)got * stride, stride,
                                                  std::min<uint32_t>(B - got, per_call), &lens[got], got ? 2 : 20);
                if (r <= 0) break;  // nothing for 20 ms: open what arrived
                got += (uint32_t)r;
                dequeued += (uint64_t)r;  // the senders' flow control counts datagrams off the socket
            }
            if (got) {
                const int nbad = qgcm_open_host(ctx, rx, stride, got, L + QGCM_OVERHEAD, 0, 4, st.data());
                if (nbad != 0) auth_fail += nbad > 0 ? (uint64_t)nbad : got;
                for (uint32_t i = 0; i < got; ++i) {
                    uint32_t idx;
                    memcpy(&idx, rx + i * stride + 4, 4);
                    if (lens[i] != L + 4 + QGCM_OVERHEAD || idx >= B ||
                        memcmp(rx + i * stride, plain.data() + (uint64_t)idx * stride, 4 + L))
                        ++bad;
                }
                per_queue[q] += got;
                received += got;
            } else if (senders_done.load() == Q) {
                break;  // senders finished and the queue stayed empty
            }
        }
        qgcm_host_free(rx);
    };
    auto outgoing = [&](int q) {  // worker/outgoing.go on its own flow
        uint8_t *tx = (uint8_t *)qgcm_host_alloc(B * stride);
        uint8_t *nonces = (uint8_t *)qgcm_host_alloc(12ull * B);
        std::vector<uint32_t> lens(B, L + 4 + QGCM_OVERHEAD);
        for (uint32_t k = 0; k < batches; ++k) {
            memcpy(tx, plain.data(), B * stride);  // this batch's TUN reads
            qgcm_random_nonces(nonces, B);
            if (qgcm_seal_host(ctx, tx, stride, B, L, 0, nonces, 4, nullptr) != 0) {
                bad += B;
                continue;
            }
            for (uint32_t i = 0; i < B;) {
                // at most `window` of this worker's datagrams unread (shared receive count, so a
                // conservative per-flow bound: every worker's share of what is in flight)
                uint64_t mine = 0;
                for (int j = 0; j < Q; ++j) mine += sent[j].load();
                if (mine - dequeued.load() > (uint64_t)window * Q) {
                    std::this_thread::yield();
                    continue;
                }
                const uint32_t n = std::min<uint32_t>(B - i, per_call);
                const int r = qgcm_udp_send_slots(txs[q], tx + (uint64_t)i * stride, stride, n, &lens[i], "127.0.0.1",
                                                  port);
                if (r <= 0) {
                    ++bad;
                    break;
                }
                i += (uint32_t)r;
                sent[q] += (uint64_t)r;
            }
        }
        qgcm_host_free(tx);
        qgcm_host_free(nonces);
        ++senders_done;
    };
    const auto t0 = Clock::now();
    std::vector<std::thread> th;
    for (int q = 0; q < Q; ++q) th.emplace_back(incoming, q);
    for (int q = 0; q < Q; ++q) th.emplace_back(outgoing, q);
    for (auto &t : th) t.join();
    // the receivers' last 20 ms idle poll is not traffic: take it off the wall time
    const double wall = std::chrono::duration<double>(Clock::now() - t0).count() - 0.02;
    const uint64_t got = received.load();
    printf("{\"config\": \"udp_loopback_multiqueue\", \"queues\": %d, \"packets\": %lu, \"payload_len\": %u, "
           "\"wall_s\": %.4f, \"packets_per_s\": %.0f, \"payload_GiBps\": %.3f, \"lost\": %lu, \"bad\": %lu, "
           "\"auth_fail\": %lu, \"per_queue\": [",
           Q, (unsigned long)total, L, wall, got / wall, (double)got * L / wall / (1 << 30), (unsigned long)(total - got),
           (unsigned long)bad.load(), (unsigned long)auth_fail.load());
    for (int q = 0; q < Q; ++q) printf("%s%lu", q ? ", " : "", (unsigned long)per_queue[q]);
    printf("]}\n");
    for (int q = 0; q < Q; ++q) {
        qgcm_udp_close(rxq[q]);
        qgcm_udp_close(txs[q]);
    }
    qgcm_destroy(ctx);
    return (total != got || bad || auth_fail) ? 3 : 0;
}
