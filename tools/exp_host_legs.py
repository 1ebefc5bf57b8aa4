"""The PCIe-inclusive legs of bench.py, each in a fresh process, with where their pinned host memory
lives: e2e_pinned_host (config 2 through qgcm_seal_host / qgcm_open_host), config3_host (config 3
through qgcm_group_seal_host / open_host, DMA runs) and config5 (the snappy + GCM host chain).  For
each leg the NUMA nodes of a sample of its pinned arena's pages (move_pages(2) query) and the GPU's
NUMA node (sysfs) are printed, to tell a slow box from a remote-node arena.

    python3 tools/exp_host_legs.py [leg ...]      (default: e2e config3_host config5 e2e)

A leg written "config3_host+e2e" runs both legs in the same process, one after the other.
"""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import ctypes as C, json, os, sys
sys.path.insert(0, %(root)r)
import numpy as np
import bench
from quantum_amd import _lib

nodes_seen = []
real_alloc = _lib.lib().qgcm_host_alloc

def page_nodes(ptr, nbytes, samples=64):
    libc = C.CDLL(None, use_errno=True)
    page = 4096
    n = max(1, min(samples, nbytes // page))
    addrs = (C.c_void_p * n)(*[ptr + (nbytes // n) * i // page * page for i in range(n)])
    status = (C.c_int * n)()
    rc = libc.syscall(279, 0, C.c_ulong(n), addrs, None, status, 0)  # move_pages: query only
    return sorted(set(status)) if rc == 0 else ["move_pages rc %%d" %% rc]

class Probe:
    def __call__(self, nbytes):
        p = real_alloc(nbytes)
        if p and nbytes >= (64 << 20):
            nodes_seen.append({"bytes": nbytes, "nodes": page_nodes(p, nbytes)})
        return p

lib = _lib.lib()
probe = Probe()
class Shim:
    def __getattr__(self, k):
        return probe if k == "qgcm_host_alloc" else getattr(lib, k)
_lib.lib = lambda: Shim()
key = bench.derive_key(bench.SECRET, bench.SALT)
outs = []
for leg in %(leg)r.split("+"):  # legs joined by "+" run one after another in this one process
    nodes_seen.clear()
    if leg == "e2e":
        out = bench.extra_e2e(key)
    elif leg == "e2e_big":  # 4.5 M packets, 6.3 GB: past qgcm_seal_host's 4-GiB staging ring (rotating slots)
        out = bench.extra_e2e(key, reps=2, n=9 << 19)
    elif leg == "config3_host":
        out = bench.extra_config3_host(verify=False)
    elif leg == "config3_host2":  # two member contexts on this GPU, the batch in qgcm_group_order's order
        out = bench.extra_config3_host(verify=False, members=2)
    elif leg == "config5":
        out = bench.extra_config5(key, bench.host_cpus()["share"], verify=False)
    elif leg.startswith("sleep"):  # e.g. sleep20: idle this many seconds between legs
        import time
        time.sleep(float(leg[5:]))
        continue
    elif leg == "config4_one_gpu":  # device-resident (no pinned arena): what it leaves behind for the next leg
        out = bench.extra_config4_one_gpu(key)
    outs.append({"leg": leg, "value": out.get("value"), "pcie_GBps_each_way": out.get("pcie_GBps_each_way"),
                 "pinned_arena_numa_nodes": list(nodes_seen), "affinity_cpus": len(os.sched_getaffinity(0))})
print(json.dumps(outs if len(outs) > 1 else outs[0]))
'''


def gpu_numa() -> str:
    try:
        import glob
        for d in glob.glob("/sys/class/drm/card*/device/numa_node"):
            return open(d).read().strip()
    except OSError:
        pass
    return "?"


def main() -> None:
    legs = sys.argv[1:] or ["e2e", "config3_host", "config5", "e2e"]
    print(json.dumps({"gpu_numa_node": gpu_numa()}), flush=True)
    for leg in legs:
        r = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT, "leg": leg}], capture_output=True,
                           text=True, timeout=300)
        if r.returncode != 0:
            print(json.dumps({"leg": leg, "error": r.stderr[-500:]}), flush=True)
            sys.exit(1)
        print(r.stdout.strip().splitlines()[-1], flush=True)


if __name__ == "__main__":
    main()
