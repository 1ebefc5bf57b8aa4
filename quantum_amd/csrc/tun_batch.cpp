// tun_batch.cpp -- device/tun.go batched (the TUN half of the host I/O).
//
// The reference opens one queue of a multi-queue TUN device per worker (device/tun.go:67-93
// newTUN, :97-118 createTUN: IFF_TUN | IFF_NO_PI | IFF_MULTI_QUEUE) and moves one packet per
// syscall: Read = read(queue, Raw[PacketStart:]) then NewTunPayload(buf, n) (:51-57); Write =
// write(queue, payload.Packet) (:60-63).  A TUN fd has no recvmmsg, so a batch here is "wait for
// the first packet, then drain what the queue already holds without blocking", straight into the
// Payload.Raw slots of a (pinned) host arena -- slot i at arena + i * stride, the packet at
// Raw[4:], the 4 leading bytes left for the private IP (common/payload.go:22-36) -- which is the
// layout qgcm_seal_host and qgcm_compress_seal_host consume.  The link set-up of initTun
// (device/tun.go:121-150: up, MTU, address + route by netlink) is done here with the classic
// interface ioctls; the route of the address's prefix comes with the address.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <linux/if.h>
#include <linux/if_tun.h>
#include <netinet/in.h>
#include <poll.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <unistd.h>

#include "../../include/qgcm.h"

namespace {

constexpr uint64_t kPacketStart = 4;  // common.PacketStart

void set_name(ifreq *r, const char *name) {
    memset(r, 0, sizeof *r);
    if (name) memcpy(r->ifr_name, name, strnlen(name, IFNAMSIZ - 1));  // stays NUL-terminated (memset above)
}

}  // namespace

extern "C" {

// device/tun.go:97-118 for `queues` queues of one device: fds[i] = queue i (O_RDWR | O_CLOEXEC,
// blocking, as the reference).  `name` may hold a %d pattern ("quantum%d") or be empty; the kernel's
// name is written to ifname_out.  Returns 0, or -errno with every queue opened so far closed.
int qgcm_tun_open(const char *name, int queues, int *fds, char *ifname_out, size_t ifname_len) {
    if (queues <= 0 || !fds) return -EINVAL;
    char dev[IFNAMSIZ] = {0};
    if (name) strncpy(dev, name, IFNAMSIZ - 1);
    for (int i = 0; i < queues; ++i) {
        const int fd = open("/dev/net/tun", O_RDWR | O_CLOEXEC);
        int err = fd < 0 ? errno : 0;
        if (fd >= 0) {
            ifreq r;
            set_name(&r, dev);
            r.ifr_flags = IFF_TUN | IFF_NO_PI | IFF_MULTI_QUEUE;
            if (ioctl(fd, TUNSETIFF, &r) != 0) {
                err = errno;
                close(fd);
            } else {
                memcpy(dev, r.ifr_name, IFNAMSIZ);  // later queues attach to the same device
                dev[IFNAMSIZ - 1] = 0;
                fds[i] = fd;
            }
        }
        if (err) {
            for (int j = 0; j < i; ++j) close(fds[j]);
            return -err;
        }
    }
    if (ifname_out && ifname_len) {
        strncpy(ifname_out, dev, ifname_len - 1);
        ifname_out[ifname_len - 1] = 0;
    }
    return 0;
}

// device/tun.go:121-150 (initTun): link up, MTU (common.MTU = 1433 in the reference), IPv4 address
// with a prefix of `prefix` bits (the kernel adds the prefix route).  Returns 0 or -errno.
int qgcm_tun_up(const char *ifname, const char *ip, int prefix, int mtu) {
    in_addr a;
    if (!ifname || !ip || prefix < 0 || prefix > 32 || inet_pton(AF_INET, ip, &a) != 1) return -EINVAL;
    const int s = socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0);
    if (s < 0) return -errno;
    int rc = 0;
    ifreq r;
    auto addr_req = [&](unsigned long req, uint32_t v) {
        set_name(&r, ifname);
        sockaddr_in sa{};
        sa.sin_family = AF_INET;
        sa.sin_addr.s_addr = v;
        memcpy(&r.ifr_addr, &sa, sizeof sa);
        return ioctl(s, req, &r) == 0 ? 0 : -errno;
    };
    const uint32_t mask = prefix ? htonl(0xffffffffu << (32 - prefix)) : 0u;
    rc = addr_req(SIOCSIFADDR, a.s_addr);
    if (rc == 0) rc = addr_req(SIOCSIFNETMASK, mask);
    if (rc == 0 && mtu > 0) {
        set_name(&r, ifname);
        r.ifr_mtu = mtu;
        if (ioctl(s, SIOCSIFMTU, &r) != 0) rc = -errno;
    }
    if (rc == 0) {
        set_name(&r, ifname);
        if (ioctl(s, SIOCGIFFLAGS, &r) != 0) {
            rc = -errno;
        } else {
            r.ifr_flags |= IFF_UP | IFF_RUNNING;
            if (ioctl(s, SIOCSIFFLAGS, &r) != 0) rc = -errno;
        }
    }
    close(s);
    return rc;
}

// device/tun.go:51-57, batched: waits up to timeout_ms (-1 = forever) for the first packet, then
// reads every packet the queue already holds, up to max_n, into Raw[4:] of slots 0, 1, ...;
// lens[i] = the packet length n (NewTunPayload(buf, n): Payload.Length = 4 + n).  A packet longer
// than stride - 4 is truncated, as read() into the worker's buffer truncates.  Returns the number
// read (0 on timeout) or -1.
int qgcm_tun_read_slots(int fd, uint8_t *arena, uint64_t stride, uint32_t max_n, uint32_t *lens, int timeout_ms) {
    if (fd < 0 || (max_n && (!arena || !lens)) || stride <= kPacketStart) return -1;
    if (max_n == 0) return 0;
    pollfd p{fd, POLLIN, 0};
    int pr;
    do {
        pr = poll(&p, 1, timeout_ms);
    } while (pr < 0 && errno == EINTR);
    if (pr < 0) return -1;
    if (pr == 0) return 0;
    uint32_t got = 0;
    while (got < max_n) {
        if (got) {  // drain without blocking: only what is already queued joins this batch
            p.revents = 0;
            do {
                pr = poll(&p, 1, 0);
            } while (pr < 0 && errno == EINTR);
            if (pr <= 0) break;
        }
        const ssize_t n = read(fd, arena + (uint64_t)got * stride + kPacketStart, (size_t)(stride - kPacketStart));
        if (n < 0) {
            if (errno == EINTR) continue;
            if (errno == EAGAIN || errno == EWOULDBLOCK) break;
            return got ? (int)got : -1;
        }
        lens[got++] = (uint32_t)n;
    }
    return (int)got;
}

// device/tun.go:60-63, batched: writes Raw[4 : 4 + lens[i]] of slots 0..n-1 (payload.Packet after
// Open / uncompress) to the queue.  Returns the number written (n on success) or -1 if none was.
// A packet the kernel rejects (e.g. not IPv4/IPv6) ends the batch there, as a failed Write drops it.
int qgcm_tun_write_slots(int fd, const uint8_t *arena, uint64_t stride, uint32_t n, const uint32_t *lens) {
    if (fd < 0 || (n && (!arena || !lens)) || stride <= kPacketStart) return -1;
    uint32_t done = 0;
    while (done < n) {
        const size_t len = (size_t)(lens[done] < stride - kPacketStart ? lens[done] : stride - kPacketStart);
        const ssize_t w = write(fd, arena + (uint64_t)done * stride + kPacketStart, len);
        if (w < 0) {
            if (errno == EINTR) continue;
            break;
        }
        ++done;
    }
    return done || n == 0 ? (int)done : -1;
}

int qgcm_tun_close(int fd) { return close(fd) == 0 ? 0 : -1; }

}  // extern "C"
