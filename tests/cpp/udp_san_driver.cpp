// udp_san_driver.cpp -- quantum_amd/csrc/udp_batch.cpp (recvmmsg / sendmmsg straight into and out of
// Payload.Raw slots) under AddressSanitizer / UBSan, built by tests/test_host_sanitizers.py.  Over
// loopback: 2000 datagrams of 1..1472 bytes sent in batches of up to 64, received in batches of at
// most 48 into a 48-slot arena (so receives stop with datagrams still queued), every one back byte
// for byte and in order; empty and zero-slot calls, and a queue pair (SO_REUSEPORT) bound to one port.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <random>
#include <vector>

#include "qgcm.h"

namespace {
constexpr uint64_t kStride = 1472;
int fail(const char *what) {
    fprintf(stderr, "udp driver: %s\n", what);
    return 1;
}
}  // namespace

int main() {
    const int a = qgcm_udp_socket("127.0.0.1", 0, 1 << 23), b = qgcm_udp_socket("127.0.0.1", 0, 1 << 23);
    if (a < 0 || b < 0) return fail("socket");
    const int port = qgcm_udp_port(b);
    std::mt19937 rng(0x5EED);
    const uint32_t total = 2000;
    std::vector<std::vector<uint8_t>> sent;
    std::vector<uint8_t> out(64 * kStride), in(48 * kStride);
    std::vector<uint32_t> olens(64), ilens(48);
    uint32_t got = 0;
    for (uint32_t done = 0; done < total;) {
        const uint32_t n = std::min<uint32_t>(1 + rng() % 64, total - done);
        for (uint32_t i = 0; i < n; ++i) {
            olens[i] = 1 + rng() % kStride;
            std::vector<uint8_t> m(olens[i]);
            for (auto &x : m) x = (uint8_t)rng();
            memcpy(out.data() + i * kStride, m.data(), m.size());
            sent.push_back(std::move(m));
        }
        if (qgcm_udp_send_slots(a, out.data(), kStride, n, olens.data(), "127.0.0.1", port) != (int)n) return fail("send");
        done += n;
        // drain what has arrived, in 48-slot batches
        for (;;) {
            const int r = qgcm_udp_recv_slots(b, in.data(), kStride, 48, ilens.data(), got < done ? 200 : 0);
            if (r < 0) return fail("recv");
            if (r == 0) break;
            for (int i = 0; i < r; ++i, ++got) {
                if (got >= sent.size() || ilens[i] != sent[got].size() ||
                    memcmp(in.data() + (uint64_t)i * kStride, sent[got].data(), ilens[i]) != 0)
                    return fail("datagram lost, reordered or altered");
            }
            if (got == done) break;
        }
    }
    if (got != total) return fail("count");
    if (qgcm_udp_recv_slots(b, in.data(), kStride, 0, ilens.data(), 0) != 0) return fail("zero-slot recv");
    if (qgcm_udp_recv_slots(b, in.data(), kStride, 48, ilens.data(), 10) != 0) return fail("empty recv");
    if (qgcm_udp_send_slots(a, out.data(), kStride, 0, olens.data(), "127.0.0.1", port) != 0) return fail("zero send");
    const int q0 = qgcm_udp_queue("127.0.0.1", 0, 0);
    if (q0 < 0) return fail("queue");
    const int q1 = qgcm_udp_queue("127.0.0.1", qgcm_udp_port(q0), 0);
    if (q1 < 0 || qgcm_udp_port(q1) != qgcm_udp_port(q0)) return fail("second queue on the same port");
    for (int fd : {a, b, q0, q1}) qgcm_udp_close(fd);
    printf("udp driver ok: %u datagrams\n", got);
    return 0;
}
