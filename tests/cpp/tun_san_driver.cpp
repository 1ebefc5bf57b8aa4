// tun_san_driver.cpp -- quantum_amd/csrc/tun_batch.cpp (the batched TUN reads and writes) under
// AddressSanitizer / UBSan, built by tests/test_host_sanitizers.py.  The read form is the one
// QGCM_TUN_URING selects for this process (unset: preadv2; 1: io_uring; -1: poll + read).
//
// A two-queue TUN device is brought up on 10.213.9.1/24; UDP datagrams of varied lengths sent to
// 10.213.9.2 come out of the queues as IPv4 packets in Payload.Raw[4:] slots of a small arena (batches
// of at most 8 slots, so a drain fills the arena and stops with packets still queued); every datagram
// must be read exactly once with its payload intact.  Then a packet written to a queue must reach a
// local UDP socket.  Exit 0 and "tun driver ok" on success, 77 when the kernel refuses the device.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <map>
#include <vector>

#include "qgcm.h"

namespace {

constexpr uint64_t kStride = 1472;
const char *kHost = "10.213.9.1", *kPeer = "10.213.9.2";

int fail(const char *what) {
    fprintf(stderr, "tun driver: %s\n", what);
    return 1;
}

uint16_t csum(const uint8_t *p, size_t n) {
    uint32_t s = 0;
    for (size_t i = 0; i + 1 < n; i += 2) s += (uint32_t)(p[i] << 8 | p[i + 1]);
    if (n & 1) s += (uint32_t)p[n - 1] << 8;
    while (s >> 16) s = (s & 0xffff) + (s >> 16);
    return (uint16_t)~s;
}

}  // namespace

int main() {
    int fds[2];
    char name[16] = {0};
    if (qgcm_tun_open("qgcms%d", 2, fds, name, sizeof name) < 0) return 77;
    if (qgcm_tun_up(name, kHost, 24, 1433) < 0) {
        for (int fd : fds) qgcm_tun_close(fd);
        return 77;
    }
    int rc = 0;
    // send: flows f = 0..3, datagrams j = 0..39, payload [f, j, j, ...] of 20 + 31 * j bytes
    std::map<std::pair<int, int>, std::vector<uint8_t>> sent, got;
    {
        const int s = socket(AF_INET, SOCK_DGRAM, 0);
        sockaddr_in me{}, to{};
        me.sin_family = to.sin_family = AF_INET;
        inet_pton(AF_INET, kHost, &me.sin_addr);
        inet_pton(AF_INET, kPeer, &to.sin_addr);
        if (s < 0 || bind(s, reinterpret_cast<sockaddr *>(&me), sizeof me) != 0) return fail("socket");
        for (int f = 0; f < 4; ++f)
            for (int j = 0; j < 40; ++j) {
                std::vector<uint8_t> m(20 + 31 * j, (uint8_t)j);
                m[0] = (uint8_t)f;
                to.sin_port = htons((uint16_t)(9000 + f));
                if (sendto(s, m.data(), m.size(), 0, reinterpret_cast<sockaddr *>(&to), sizeof to) != (ssize_t)m.size())
                    return fail("sendto");
                sent[{f, j}] = m;
            }
        close(s);
    }
    std::vector<uint8_t> arena(8 * kStride);
    std::vector<uint32_t> lens(8);
    for (int round = 0; round < 400 && got.size() < sent.size(); ++round)
        for (int fd : fds) {
            const int n = qgcm_tun_read_slots(fd, arena.data(), kStride, 8, lens.data(), 5);
            if (n < 0) return fail("read");
            for (int i = 0; i < n; ++i) {
                const uint8_t *pkt = arena.data() + (uint64_t)i * kStride + 4;
                const uint32_t L = lens[i];
                if (L < 28 || (pkt[0] >> 4) != 4 || pkt[9] != 17) continue;  // not one of ours
                const uint32_t ihl = (pkt[0] & 15u) * 4;
                const int f = (pkt[ihl + 2] << 8 | pkt[ihl + 3]) - 9000;
                std::vector<uint8_t> data(pkt + ihl + 8, pkt + L);
                if (f < 0 || f > 3 || data.size() < 2) continue;
                const int j = data[1];
                if (got.count({f, j})) rc = fail("datagram read twice");
                got[{f, j}] = data;
            }
        }
    if (got != sent) return fail("datagrams lost or altered");
    // write: one IPv4/UDP packet from the peer to a bound local socket
    {
        const int rx = socket(AF_INET, SOCK_DGRAM, 0);
        sockaddr_in me{};
        me.sin_family = AF_INET;
        inet_pton(AF_INET, kHost, &me.sin_addr);
        socklen_t ml = sizeof me;
        if (rx < 0 || bind(rx, reinterpret_cast<sockaddr *>(&me), sizeof me) != 0 ||
            getsockname(rx, reinterpret_cast<sockaddr *>(&me), &ml) != 0)
            return fail("rx socket");
        std::vector<uint8_t> slot(kStride, 0);
        uint8_t *p = slot.data() + 4;
        const char msg[] = "written through a queue";
        const uint16_t ulen = (uint16_t)(8 + sizeof msg), tot = (uint16_t)(20 + ulen);
        p[0] = 0x45;
        p[2] = (uint8_t)(tot >> 8);
        p[3] = (uint8_t)tot;
        p[6] = 0x40;
        p[8] = 64;
        p[9] = 17;
        inet_pton(AF_INET, kPeer, p + 12);
        inet_pton(AF_INET, kHost, p + 16);
        const uint16_t c = csum(p, 20);
        p[10] = (uint8_t)(c >> 8);
        p[11] = (uint8_t)c;
        p[20] = 0x23;
        p[21] = 0x28;  // source port 9000
        memcpy(p + 22, &me.sin_port, 2);
        p[24] = (uint8_t)(ulen >> 8);
        p[25] = (uint8_t)ulen;
        memcpy(p + 28, msg, sizeof msg);
        const uint32_t L = tot;
        if (qgcm_tun_write_slots(fds[1], slot.data(), kStride, 1, &L) != 1) return fail("write");
        timeval tv{2, 0};
        setsockopt(rx, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
        char buf[64] = {0};
        if (recv(rx, buf, sizeof buf, 0) != (ssize_t)sizeof msg || memcmp(buf, msg, sizeof msg) != 0)
            return fail("written packet not delivered");
        close(rx);
    }
    for (int fd : fds) qgcm_tun_close(fd);
    if (rc == 0) printf("tun driver ok: %zu datagrams\n", got.size());
    return rc;
}
