// udp_batch.cpp -- socket/udp.go:35-47 batched.
//
// The reference moves one datagram per syscall: Read = recvfrom into the worker's Raw buffer then
// NewSockPayload(buf, n); Write = sendto(Raw[:Length], mapping.Sockaddr).  A GPU batch of thousands
// of packets needs the I/O batched too, or the path is syscall-bound long before it is crypto-bound.
// These calls move whole batches of Payload.Raw slots (slot i at arena + i*stride; the datagram IS
// Raw[:Length], wire format [4-B private IP][ct][tag][nonce]) with recvmmsg / sendmmsg, straight
// into / out of the (pinned) host arena that qgcm_seal_host / qgcm_open_host and the chained
// snappy paths consume, so the datagram bytes are never copied on the host.
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <vector>

#include "../../include/qgcm.h"

namespace {

constexpr unsigned kVlen = 1024;  // UIO_MAXIOV: most messages one recvmmsg/sendmmsg call takes

bool make_addr(const char *ip, int port, sockaddr_in *a) {
    memset(a, 0, sizeof *a);
    a->sin_family = AF_INET;
    a->sin_port = htons((uint16_t)port);
    return port >= 0 && port <= 65535 && inet_pton(AF_INET, ip, &a->sin_addr) == 1;
}

}  // namespace

extern "C" {

// socket/udp.go:49-70 (createUDPSocket): one queue.  rcvbuf_bytes > 0 also sizes SO_RCVBUF/SO_SNDBUF
// (a batch of packets must fit the kernel buffer between two recvmmsg calls).
int qgcm_udp_socket(const char *ip, int port, int bufbytes) {
    sockaddr_in a;
    if (!ip || !make_addr(ip, port, &a)) return -1;
    const int fd = socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0);
    if (fd < 0) return -1;
    const int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    if (bufbytes > 0) {
        setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &bufbytes, sizeof bufbytes);
        setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &bufbytes, sizeof bufbytes);
    }
    if (bind(fd, reinterpret_cast<sockaddr *>(&a), sizeof a) != 0) {
        close(fd);
        return -1;
    }
    return fd;
}

// One queue of a multi-queue UDP socket: socket/udp.go:55-70 (newUDP) opens cfg.NumWorkers sockets on
// the same ListenAddr, one per worker (socket.go:52-77 sets SO_REUSEADDR).  On Linux only SO_REUSEPORT
// spreads the incoming datagrams over such a group -- by a hash of the sender's address and port, so
// each flow stays on one queue and in order -- which is what the per-worker queues are for.  Every
// queue of a group must be opened by the same user; a port of 0 is resolved by the first queue
// (qgcm_udp_port) and passed to the others.
int qgcm_udp_queue(const char *ip, int port, int bufbytes) {
    sockaddr_in a;
    if (!ip || !make_addr(ip, port, &a)) return -1;
    const int fd = socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0);
    if (fd < 0) return -1;
    const int one = 1;
    if (setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one) != 0 ||
        setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one) != 0) {
        close(fd);
        return -1;
    }
    if (bufbytes > 0) {
        setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &bufbytes, sizeof bufbytes);
        setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &bufbytes, sizeof bufbytes);
    }
    if (bind(fd, reinterpret_cast<sockaddr *>(&a), sizeof a) != 0) {
        close(fd);
        return -1;
    }
    return fd;
}

int qgcm_udp_port(int fd) {
    sockaddr_in a;
    socklen_t n = sizeof a;
    if (getsockname(fd, reinterpret_cast<sockaddr *>(&a), &n) != 0) return -1;
    return ntohs(a.sin_port);
}

int qgcm_udp_close(int fd) { return close(fd) == 0 ? 0 : -1; }

// socket/udp.go:35-41, batched: waits up to timeout_ms (-1 = forever) for the first datagram, then
// takes every datagram already queued, up to max_n, into slots 0, 1, ... (lens[i] = its length, as
// NewSockPayload(buf, n)).  A datagram longer than the slot is truncated to `stride` bytes, as
// recvfrom into the worker's buffer truncates.  Returns the number received (0 on timeout) or -1.
int qgcm_udp_recv_slots(int fd, uint8_t *arena, uint64_t stride, uint32_t max_n, uint32_t *lens, int timeout_ms) {
    if (fd < 0 || (max_n && (!arena || !lens)) || stride == 0) return -1;
    if (max_n == 0) return 0;
    pollfd p{fd, POLLIN, 0};
    int pr;
    do {
        pr = poll(&p, 1, timeout_ms);
    } while (pr < 0 && errno == EINTR);
    if (pr < 0) return -1;
    if (pr == 0) return 0;
    std::vector<mmsghdr> msgs(std::min<uint32_t>(max_n, kVlen));
    std::vector<iovec> iov(msgs.size());
    uint32_t got = 0;
    while (got < max_n) {
        const unsigned k = (unsigned)std::min<uint64_t>(max_n - got, msgs.size());
        for (unsigned i = 0; i < k; ++i) {
            iov[i] = iovec{arena + (uint64_t)(got + i) * stride, (size_t)stride};
            msgs[i] = mmsghdr{};
            msgs[i].msg_hdr.msg_iov = &iov[i];
            msgs[i].msg_hdr.msg_iovlen = 1;
        }
        const int r = recvmmsg(fd, msgs.data(), k, MSG_DONTWAIT, nullptr);
        if (r < 0) {
            if (errno == EINTR) continue;
            if (errno == EAGAIN || errno == EWOULDBLOCK) break;
            return got ? (int)got : -1;
        }
        for (int i = 0; i < r; ++i) lens[got + i] = msgs[i].msg_len;
        got += (uint32_t)r;
        if ((unsigned)r < k) break;
    }
    return (int)got;
}

// socket/udp.go:43-47, batched: sends Raw[:lens[i]] of slots 0..n-1 to ip:port (one peer's batch,
// mapping.Sockaddr).  Blocks while the socket buffer is full, as sendto does.  Returns the number
// of datagrams sent (n on success) or -1 if none could be.
int qgcm_udp_send_slots(int fd, const uint8_t *arena, uint64_t stride, uint32_t n, const uint32_t *lens,
                        const char *ip, int port) {
    sockaddr_in dst;
    if (fd < 0 || (n && (!arena || !lens)) || !ip || !make_addr(ip, port, &dst)) return -1;
    std::vector<mmsghdr> msgs(std::min<uint32_t>(std::max<uint32_t>(n, 1), kVlen));
    std::vector<iovec> iov(msgs.size());
    uint32_t sent = 0;
    while (sent < n) {
        const unsigned k = (unsigned)std::min<uint64_t>(n - sent, msgs.size());
        for (unsigned i = 0; i < k; ++i) {
            iov[i] = iovec{const_cast<uint8_t *>(arena) + (uint64_t)(sent + i) * stride,
                           (size_t)std::min<uint64_t>(lens[sent + i], stride)};
            msgs[i] = mmsghdr{};
            msgs[i].msg_hdr.msg_name = &dst;
            msgs[i].msg_hdr.msg_namelen = sizeof dst;
            msgs[i].msg_hdr.msg_iov = &iov[i];
            msgs[i].msg_hdr.msg_iovlen = 1;
        }
        const int r = sendmmsg(fd, msgs.data(), k, 0);
        if (r < 0) {
            if (errno == EINTR) continue;
            return sent ? (int)sent : -1;
        }
        sent += (uint32_t)r;
    }
    return (int)sent;
}

}  // extern "C"
