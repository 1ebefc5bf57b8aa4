// cpu_topo.cpp -- where libqgcm's host worker threads run.
//
// The GPU boxes are shared hosts (256 CPUs, this job a 16-CPU cgroup share): threads left to the
// scheduler land on SMT siblings of each other and of other tenants' busy threads.  bench.py's CPU
// sweep measured the reference's plugin chain at 5.9 GiB/s with 16 threads left to the scheduler and
// 17.5 with the same 16 threads pinned one per least-loaded physical core.  The chain's
// snappy workers (qgcm_compress_seal_host / qgcm_open_uncompress_host) are the same kind of work, so
// they are placed the same way: one per physical core, the GPU's NUMA-local cores first, the least
// busy first.
#include <hip/hip_runtime.h>
#include <ctype.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <utility>
#include <vector>

#include "gcm_internal.h"

namespace {

// "0-31,64-95" -> set bits (sysfs cpulist format)
void parse_cpulist(const char *txt, cpu_set_t *set) {
    CPU_ZERO(set);
    const char *p = txt;
    while (*p) {
        char *e;
        const long a = strtol(p, &e, 10);
        if (e == p) break;
        long b = a;
        p = e;
        if (*p == '-') {
            b = strtol(p + 1, &e, 10);
            p = e;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (c >= 0) CPU_SET((int)c, set);
        while (*p == ',' || *p == '\n' || *p == ' ') ++p;
    }
}

bool read_file(const char *path, char *buf, size_t cap) {
    FILE *f = fopen(path, "r");
    if (!f) return false;
    const size_t got = fread(buf, 1, cap - 1, f);
    fclose(f);
    buf[got] = 0;
    return got > 0;
}

// per-CPU (total, idle) jiffies from /proc/stat
std::vector<std::pair<unsigned long long, unsigned long long>> cpu_times() {
    std::vector<std::pair<unsigned long long, unsigned long long>> out;
    FILE *f = fopen("/proc/stat", "r");
    if (!f) return out;
    char line[512];
    while (fgets(line, sizeof line, f)) {
        if (strncmp(line, "cpu", 3) != 0 || !isdigit((unsigned char)line[3])) continue;
        int cpu = 0;
        unsigned long long v[10] = {0};
        const int k = sscanf(line, "cpu%d %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu", &cpu, &v[0], &v[1], &v[2],
                             &v[3], &v[4], &v[5], &v[6], &v[7], &v[8], &v[9]);
        if (k < 5 || cpu < 0) continue;
        unsigned long long tot = 0;
        for (int i = 0; i < k - 1; ++i) tot += v[i];
        if ((size_t)cpu >= out.size()) out.resize(cpu + 1, {0, 0});
        out[cpu] = {tot, v[3] + v[4]};
    }
    fclose(f);
    return out;
}

}  // namespace

// CPUs of the device's NUMA node that this process may run on; 0 when sysfs has no answer
int qgcm::gpu_local_cpus(int device, cpu_set_t *out) {
    CPU_ZERO(out);
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus), device) != hipSuccess) return 0;
    for (char *c = bus; *c; ++c) *c = (char)tolower(*c);
    char path[160];
    snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/local_cpulist", bus);
    char txt[4096];
    if (!read_file(path, txt, sizeof txt)) return 0;
    cpu_set_t local, allowed;
    parse_cpulist(txt, &local);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return 0;
    CPU_AND(out, &local, &allowed);
    return CPU_COUNT(out);
}

// One CPU per physical core this process may run on (the lowest allowed SMT sibling): the cores in
// `prefer` (may be null) first, then the rest; within each, the cores whose hardware threads were the
// least busy over a `sample_ms` window of /proc/stat first.
std::vector<int> qgcm::spread_cpus(const cpu_set_t *prefer, int sample_ms) {
    cpu_set_t allowed;
    std::vector<int> out;
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return out;
    const auto t0 = cpu_times();
    if (sample_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(sample_ms));
    const auto t1 = cpu_times();
    auto busy = [&](int c) {
        if ((size_t)c >= t0.size() || (size_t)c >= t1.size()) return 0.0;
        const double dt = (double)(t1[c].first - t0[c].first);
        return dt > 0 ? 1.0 - (double)(t1[c].second - t0[c].second) / dt : 0.0;
    };
    struct Core {
        int cpu;
        bool preferred;
        double load;
    };
    std::vector<Core> cores;
    std::vector<bool> seen(CPU_SETSIZE, false);
    for (int c = 0; c < CPU_SETSIZE; ++c) {
        if (!CPU_ISSET(c, &allowed) || seen[c]) continue;
        char path[128], txt[256];
        snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", c);
        cpu_set_t sib;
        if (read_file(path, txt, sizeof txt)) {
            parse_cpulist(txt, &sib);
        } else {
            CPU_ZERO(&sib);
            CPU_SET(c, &sib);
        }
        double load = 0;
        for (int s = 0; s < CPU_SETSIZE; ++s)
            if (CPU_ISSET(s, &sib)) {
                seen[s] = true;
                load = std::max(load, busy(s));
            }
        cores.push_back({c, prefer && CPU_ISSET(c, prefer), load});
    }
    std::stable_sort(cores.begin(), cores.end(), [](const Core &a, const Core &b) {
        if (a.preferred != b.preferred) return a.preferred;
        return a.load < b.load;
    });
    for (const Core &k : cores) out.push_back(k.cpu);
    return out;
}

void qgcm::pin_to_cpu(int cpu) {
    cpu_set_t one;
    CPU_ZERO(&one);
    CPU_SET(cpu, &one);
    (void)sched_setaffinity(0, sizeof one, &one);  // this thread (a tid of 0 is the caller)
}
