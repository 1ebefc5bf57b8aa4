// tun_batch.cpp -- device/tun.go batched (the TUN half of the host I/O).
//
// The reference opens one queue of a multi-queue TUN device per worker (device/tun.go:67-93
// newTUN, :97-118 createTUN: IFF_TUN | IFF_NO_PI | IFF_MULTI_QUEUE) and moves one packet per
// syscall: Read = read(queue, Raw[PacketStart:]) then NewTunPayload(buf, n) (:51-57); Write =
// write(queue, payload.Packet) (:60-63).  A TUN fd has no recvmmsg, so a batch here is "wait for
// the first packet, then drain what the queue already holds without blocking", straight into the
// Payload.Raw slots of a (pinned) host arena -- slot i at arena + i * stride, the packet at
// Raw[4:], the 4 leading bytes left for the private IP (common/payload.go:22-36) -- which is the
// layout qgcm_seal_host and qgcm_compress_seal_host consume.  After the poll for the first packet the
// drain is one preadv2(RWF_NOWAIT) per packet (the TUN driver honours IOCB_NOWAIT: a packet, or
// -EAGAIN once the queue is empty), one syscall per packet instead of a poll and a read.  One io_uring
// submission of RWF_NOWAIT reads per batch (QGCM_TUN_URING=1) was built and measured slower (read_mode
// below).  The link set-up of initTun
// (device/tun.go:121-150: up, MTU, address + route by netlink) is done here with the classic
// interface ioctls; the route of the address's prefix comes with the address.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <linux/if.h>
#include <linux/if_tun.h>
#include <netinet/in.h>
#include <poll.h>
#include <stdlib.h>
#include <string.h>
#include <linux/io_uring.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <sys/uio.h>
#include <unistd.h>

#include <atomic>

#include "../../include/qgcm.h"

namespace {

constexpr uint64_t kPacketStart = 4;  // common.PacketStart

// One io_uring per calling thread (a worker thread owns its queues, worker/outgoing.go:83-93), created
// on the first batched read; kRingEntries reads per submission.
constexpr unsigned kRingEntries = 256;

struct Ring {
    int fd = -1;
    unsigned *sq_head = nullptr, *sq_tail = nullptr, *sq_mask = nullptr, *sq_array = nullptr;
    unsigned *cq_head = nullptr, *cq_tail = nullptr, *cq_mask = nullptr;
    io_uring_sqe *sqes = nullptr;
    io_uring_cqe *cqes = nullptr;
    void *sq_ptr = nullptr, *cq_ptr = nullptr;
    size_t sq_len = 0, cq_len = 0, sqe_len = 0;
    bool broken = false;

    bool init() {
        io_uring_params p{};
        fd = (int)syscall(__NR_io_uring_setup, kRingEntries, &p);
        if (fd < 0) return false;
        sq_len = p.sq_off.array + p.sq_entries * sizeof(unsigned);
        cq_len = p.cq_off.cqes + p.cq_entries * sizeof(io_uring_cqe);
        const bool single = p.features & IORING_FEAT_SINGLE_MMAP;
        if (single) sq_len = cq_len = sq_len > cq_len ? sq_len : cq_len;
        sq_ptr = mmap(nullptr, sq_len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, IORING_OFF_SQ_RING);
        if (sq_ptr == MAP_FAILED) return fail();
        cq_ptr = single ? sq_ptr
                        : mmap(nullptr, cq_len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, IORING_OFF_CQ_RING);
        if (cq_ptr == MAP_FAILED) return fail();
        sqe_len = p.sq_entries * sizeof(io_uring_sqe);
        void *sq = mmap(nullptr, sqe_len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, IORING_OFF_SQES);
        if (sq == MAP_FAILED) return fail();
        sqes = static_cast<io_uring_sqe *>(sq);
        auto at = [](void *base, unsigned off) { return reinterpret_cast<unsigned *>(static_cast<char *>(base) + off); };
        sq_head = at(sq_ptr, p.sq_off.head);
        sq_tail = at(sq_ptr, p.sq_off.tail);
        sq_mask = at(sq_ptr, p.sq_off.ring_mask);
        sq_array = at(sq_ptr, p.sq_off.array);
        cq_head = at(cq_ptr, p.cq_off.head);
        cq_tail = at(cq_ptr, p.cq_off.tail);
        cq_mask = at(cq_ptr, p.cq_off.ring_mask);
        cqes = reinterpret_cast<io_uring_cqe *>(static_cast<char *>(cq_ptr) + p.cq_off.cqes);
        return true;
    }
    bool fail() {
        close(fd);
        fd = -1;
        return false;
    }
    ~Ring() {
        if (fd < 0) return;
        munmap(sqes, sqe_len);
        if (cq_ptr != sq_ptr) munmap(cq_ptr, cq_len);
        munmap(sq_ptr, sq_len);
        close(fd);
    }
};

thread_local Ring tl_ring;
thread_local int tl_ring_state = 0;  // 0 not tried, 1 ready, -1 unavailable
// The read path, fixed at the first batched read of the process: 0 preadv2(RWF_NOWAIT) per packet (the
// default), 1 one io_uring submission per batch (QGCM_TUN_URING=1), 2 poll + read per packet, the
// round-4 form (QGCM_TUN_URING=-1).  tools/tun_rate.py, 400 000 packets of 1378 B through a TUN queue,
// time inside the read calls per packet, three interleaved runs: preadv2 0.68 / 0.80 / 0.68 us,
// io_uring 0.83 / 0.91 / 1.11, poll + read 0.93 / 0.97 / 1.09 -- the kernel's per-packet work (the
// skb copy-out and free), not the syscall entry, is most of the cost, and io_uring's per-request
// set-up and completion cost more than the syscall it saves.
std::atomic<int> g_read_mode{-1};

int read_mode() {
    int m = g_read_mode.load(std::memory_order_relaxed);
    if (m < 0) {
        const char *v = getenv("QGCM_TUN_URING");
        m = !v ? 0 : !strcmp(v, "1") ? 1 : !strcmp(v, "-1") ? 2 : 0;
        g_read_mode.store(m, std::memory_order_relaxed);
    }
    return m;
}

Ring *ring() {
    if (read_mode() != 1) return nullptr;
    if (tl_ring_state == 0) tl_ring_state = tl_ring.init() ? 1 : -1;
    return tl_ring_state > 0 && !tl_ring.broken ? &tl_ring : nullptr;
}

// Up to k (<= kRingEntries) non-blocking reads into slots [first, first + k), one submission; the
// packets that were queued land in those slots, holes (a read that found the queue empty while a
// later one found a packet that had just arrived) are closed up.  Returns how many landed (lens set),
// or -1 when the ring took no read (nothing consumed: the caller falls back).  What was submitted is
// read off the kernel's SQ head, not the return value: an io_uring_enter interrupted while it waits
// for completions has still submitted its reads, and a partial submission leaves the rest queued.
int uring_drain(Ring &r, int fd, uint8_t *arena, uint64_t stride, uint32_t first, uint32_t k, uint32_t *lens) {
    const unsigned tail0 = *r.sq_tail;  // == the SQ head: every earlier entry was taken or withdrawn
    unsigned tail = tail0;
    for (uint32_t j = 0; j < k; ++j) {
        const unsigned idx = tail & *r.sq_mask;
        io_uring_sqe &e = r.sqes[idx];
        memset(&e, 0, sizeof e);
        e.opcode = IORING_OP_READ;
        e.fd = fd;
        e.addr = reinterpret_cast<uint64_t>(arena + (uint64_t)(first + j) * stride + kPacketStart);
        e.len = (uint32_t)(stride - kPacketStart);
        e.off = (uint64_t)-1;  // the file position (a character device: none)
        e.rw_flags = RWF_NOWAIT;
        e.user_data = j;
        r.sq_array[idx] = idx;
        ++tail;
    }
    __atomic_store_n(r.sq_tail, tail, __ATOMIC_RELEASE);
    int sub;
    do {
        sub = (int)syscall(__NR_io_uring_enter, r.fd, k, k, IORING_ENTER_GETEVENTS, nullptr, 0);
    } while (sub < 0 && errno == EINTR);
    const unsigned took = __atomic_load_n(r.sq_head, __ATOMIC_ACQUIRE) - tail0;
    if (took < k) __atomic_store_n(r.sq_tail, tail0 + took, __ATOMIC_RELEASE);  // withdraw the rest
    if (took == 0) return -1;
    // the taken reads (entries 0 .. took-1, in order) complete inline under RWF_NOWAIT: reap them all,
    // waiting if need be -- a completion left behind would be read as the next batch's
    static thread_local int32_t res[kRingEntries];
    for (uint32_t j = 0; j < took; ++j) res[j] = -EAGAIN;
    unsigned head = *r.cq_head, seen = 0;
    while (seen < took) {
        const unsigned ctail = __atomic_load_n(r.cq_tail, __ATOMIC_ACQUIRE);
        for (; head != ctail && seen < took; ++head, ++seen) {
            const io_uring_cqe &c = r.cqes[head & *r.cq_mask];
            if (c.user_data < kRingEntries) res[c.user_data] = c.res;
        }
        __atomic_store_n(r.cq_head, head, __ATOMIC_RELEASE);
        if (seen < took) {
            int w;
            do {
                w = (int)syscall(__NR_io_uring_enter, r.fd, 0, took - seen, IORING_ENTER_GETEVENTS, nullptr, 0);
            } while (w < 0 && errno == EINTR);
            if (w < 0) {  // cannot wait: keep what completed; the ring is not used again (late completions)
                r.broken = true;
                break;
            }
        }
    }
    uint32_t got = 0;
    for (uint32_t j = 0; j < took; ++j) {
        if (res[j] < 0) continue;
        if (got != j)
            memmove(arena + (uint64_t)(first + got) * stride + kPacketStart,
                    arena + (uint64_t)(first + j) * stride + kPacketStart, (size_t)res[j]);
        lens[first + got++] = (uint32_t)res[j];
    }
    return (int)got;
}

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
    if (Ring *r = ring()) {
        // one submission per kRingEntries slots; the next only while the queue kept every read busy
        while (got < max_n) {
            const uint32_t k = max_n - got < kRingEntries ? max_n - got : kRingEntries;
            const int n = uring_drain(*r, fd, arena, stride, got, k, lens);
            if (n < 0) break;  // the ring failed: the loop below takes over
            got += (uint32_t)n;
            if ((uint32_t)n < k) return (int)got;
        }
        if (got == max_n) return (int)got;
    }
    // no io_uring: one preadv2(RWF_NOWAIT) per packet (a poll + read where that is refused too, or
    // with QGCM_TUN_URING=-1: the round-4 form, for A/Bs)
    static std::atomic<int> nowait_ok{1};
    if (read_mode() == 2) nowait_ok.store(0, std::memory_order_relaxed);
    while (got < max_n && nowait_ok.load(std::memory_order_relaxed)) {
        iovec v{arena + (uint64_t)got * stride + kPacketStart, (size_t)(stride - kPacketStart)};
        const ssize_t n = preadv2(fd, &v, 1, -1, RWF_NOWAIT);
        if (n < 0) {
            if (errno == EINTR) continue;
            if (errno == EAGAIN || errno == EWOULDBLOCK) return (int)got;
            if (errno == EOPNOTSUPP || errno == EINVAL || errno == ENOSYS) {
                nowait_ok.store(0, std::memory_order_relaxed);
                break;
            }
            return got ? (int)got : -1;
        }
        lens[got++] = (uint32_t)n;
    }
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
