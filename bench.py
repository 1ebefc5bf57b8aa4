"""bench.py -- AES-256-GCM seal+unseal GiB/s on device-resident packet batches (BASELINE.json).

Workload (BASELINE.json configs): at N = 1 GPU, config 2 -- 2^20 packets x 1350 B, one key
(NewAES("AES256Key-32Characters1234567890", salt 00..1f)), AAD = 4-B private IP, explicit seeded
nonces, slots laid out as Payload.Raw records of 1408 B with 64-B aligned payloads.  At N > 1, config
4 -- 64 x 2^20 packets x 1350 B sharded over the N GPUs (one process per GPU, each owning its
contiguous shard: packets are independent, no data-path collective), so the total work is fixed
("strong"); --workload config2 keeps 2^20 packets per GPU instead ("weak").  One step = seal every
packet, then unseal every packet (crypto/aes.go Encrypt then Decrypt), the reference's BenchmarkAES
loop body (crypto/crypto_test.go:103-131) over a batch.

Before the W warmup steps the GPU runs the same step for --settle-ms of wall time (clock settle,
DESIGN.md s5 "Clock ramp": after an idle start the clocks take ~70 ms of load to come up).

At N = 1, after the headline, the same process also times the other BASELINE configs into
`extra_configs` (never `value`): config 3 on the parity-checked workload (quantum_amd/workloads.py,
with its golden arena digests), config 2 from pinned host memory (PCIe included) and config 5.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

`--gpus N` with N > 1 and no launcher starts torch.distributed.run with N ranks itself; under a
launcher WORLD_SIZE must equal N (anything else exits non-zero).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from quantum_amd import batch, shard  # noqa: E402
from quantum_amd.crypto import Context, derive_key  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, MI355X_MICROARCH.md "Chip-level parameters"
COPY_GUIDE_GBS = 6290.0  # the same table's measured float4 copy (read + write)
# PMC passes of this command (tools/pmc_traffic.py), newest first
LAUNCH_CHUNK = 1 << 20  # quantum_amd/csrc/gcm_internal.h kLaunchChunk
TRAFFIC_JSONS = [os.path.join(ROOT, "profiles", d, "traffic.json") for d in ("r6_s26", "r6_s22", "r6_s12", "r6_s10", "r6_s3", "r5_s37", "r5_s7", "r4_s21", "r4_s3", "r3_s39", "r3_s15", "r3_s1")]
CONFIG4_PACKETS = 64 << 20  # BASELINE config 4: 64 M packets over the node's GPUs
SECRET = b"AES256Key-32Characters1234567890"
SALT = bytes(range(32))
AAD = bytes([10, 99, 0, 1])


def parse() -> argparse.Namespace:
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=500)  # ~1.7 s timed (the clocks ramp for ~70 ms after an idle gap)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workload", choices=["auto", "config2", "config4"], default="auto",
                   help="auto: config2 at 1 GPU, config4 (64 M packets sharded) at more")
    p.add_argument("--packets", type=int, default=0, help="packets per GPU (overrides the workload's)")
    p.add_argument("--settle-ms", type=float, default=500.0, help="clock settle before warmup (0 = none)")
    p.add_argument("--len", type=int, default=1350, help="payload bytes per packet")
    p.add_argument("--stride", type=int, default=0, help="slot stride (0 = smallest 64-B multiple)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extra", action="store_true", help="skip configs 3 / 5 and the host-memory rate (N=1)")
    p.add_argument("--no-verify", action="store_true", help="skip the golden arena digests of configs 3 and 5")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = the CPU share this job was given")
    p.add_argument("--dist-backend", default="nccl", help="nccl (RCCL, default) or gloo (rehearsal)")
    p.add_argument("--one-device", action="store_true",
                   help="every rank on cuda:0 (multi-rank rehearsal on a 1-GPU box, gloo only)")
    return p.parse_args()


def host_cpus() -> dict:
    """What the host has and what this job may use: nproc, the affinity mask, the cgroup CPU quota,
    the job's thread budget (OMP_NUM_THREADS, set to the box's share by the GPU pool), model, flags."""
    info = {"nproc": os.cpu_count() or 1}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = info["nproc"]
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    info["cgroup_quota_cpus"] = quota
    share = info["affinity"]
    if quota:
        share = min(share, max(1, int(quota)))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        share = min(share, int(omp))
    info["share"] = share
    model, flags = "", set()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name") and not model:
                model = line.split(":", 1)[1].strip()
            elif line.startswith("flags") and not flags:
                flags = set(line.split(":", 1)[1].split())
    except OSError:
        pass
    info["model"] = model
    info["crypto_flags"] = sorted(f for f in ("aes", "vaes", "pclmulqdq", "vpclmulqdq", "avx2", "avx512f")
                                  if f in flags)
    return info


def cgroup_cpu_stat() -> dict:
    """The job cgroup's CPU accounting (cgroup v2 cpu.stat): usage and throttling counters."""
    out = {}
    try:
        for ln in open("/sys/fs/cgroup/cpu.stat"):
            k, v = ln.split()
            out[k] = int(v)
    except (OSError, ValueError):
        pass
    return out


SWEEP_THREADS = (1, 2, 4, 8, 12, 15, 16)


def cpu_busy(sample_s: float = 0.25) -> dict[int, float]:
    """Busy fraction of every CPU of the host over `sample_s` (/proc/stat), i.e. what the GPU box's
    other tenants are running right now."""
    def snap():
        out = {}
        for ln in open("/proc/stat"):
            if ln.startswith("cpu") and ln[3:4].isdigit():
                f = ln.split()
                v = [int(x) for x in f[1:]]
                idle = v[3] + (v[4] if len(v) > 4 else 0)
                out[int(f[0][3:])] = (sum(v), idle)
        return out
    try:
        a = snap()
        time.sleep(sample_s)
        b = snap()
    except (OSError, ValueError):
        return {}
    busy = {}
    for c, (t1, i1) in b.items():
        t0, i0 = a.get(c, (t1, i1))
        dt = t1 - t0
        busy[c] = 1.0 - (i1 - i0) / dt if dt > 0 else 0.0
    return busy


def core_cpus(busy: dict[int, float] | None = None) -> list[int]:
    """One CPU per physical core of this process's affinity set (the lowest SMT sibling allowed), the
    cores whose hardware threads the host's other work uses least first (`busy`, cpu_busy()): the
    list the pinned sweep points place their threads on."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return []
    seen, cores = set(), []
    for c in allowed:
        try:
            sib = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
        except OSError:
            sib = str(c)
        if sib not in seen:
            seen.add(sib)
            sibs = []
            for part in sib.split(","):
                lo, _, hi = part.partition("-")
                sibs.extend(range(int(lo), int(hi or lo) + 1))
            load = max((busy or {}).get(x, 0.0) for x in sibs)
            cores.append((round(load, 2), c))
    return [c for _, c in sorted(cores)]


def cpu_baseline(key: bytes, L: int, threads: int, host: dict, seconds: float = 1.0) -> dict:
    """BASELINE config 1 on the host cores: the reference's plugin chain over common.Payload
    (Encryption + Mock, sorted; NewTunPayload -> Apply(Outgoing) -> NewSockPayload -> Apply(Incoming))
    on 10 000 x L-byte payloads per thread -- this repo's C++ mirror of the Go plugin code over OpenSSL
    EVP AES-256-GCM with crypto/aes.go semantics (oracle/cpu_chain.cpp).  Run by main() BEFORE anything
    touches the GPU, each point a fresh child process: a thread sweep up to `threads` (the CPU share
    the GPU pool grants this job), each point with the reference's nonce draw (one getrandom(2) per
    Encrypt, as Go's crypto/rand) left to the scheduler and pinned one thread per physical core, and
    with buffered nonces (341 per syscall, pinned); the cgroup's cpu.stat throttling counters are read
    around every point.  `value` is the best sustained point of the faithful (per-packet getrandom)
    chain, pinned or not; the per-thread efficiency at that point is stated.  Also the bare
    AES-GCM loop (oracle/ossl_check.c: one reused buffer, no plugin chain) on one thread."""
    import subprocess

    from oracle import oracle as O

    exe = os.path.join(ROOT, "oracle", "_build", "cpu_chain")

    busy = cpu_busy()
    cores = core_cpus(busy)

    def chain(t: int, nonces: str, pinned: bool) -> dict:
        env = dict(os.environ)
        env.pop("QGCM_CHAIN_CPUS", None)
        if pinned and cores:
            env["QGCM_CHAIN_CPUS"] = ",".join(map(str, cores))
        c0 = cgroup_cpu_stat()
        out = subprocess.run([exe, str(t), "10000", str(L), str(seconds), nonces], capture_output=True, text=True,
                             timeout=120, env=env)
        c1 = cgroup_cpu_stat()
        if out.returncode != 0:
            raise RuntimeError(f"cpu_chain failed: {out.stderr[-500:]}")
        d = json.loads(out.stdout.strip().splitlines()[-1])
        d["nr_throttled"] = c1.get("nr_throttled", 0) - c0.get("nr_throttled", 0) if c0 else None
        d["throttled_ms"] = round((c1.get("throttled_usec", 0) - c0.get("throttled_usec", 0)) / 1e3, 1) if c0 else None
        return d

    counts = sorted({t for t in SWEEP_THREADS if t <= threads} | {threads})
    sweep = []
    for t in counts:
        for mode, pinned in (("syscall", False), ("syscall", True), ("buffered", True)):
            d = chain(t, mode, pinned)
            sweep.append({k: d[k] for k in ("threads", "nonces", "pinned", "GiB_s", "packets_per_s", "cpus_busy",
                                            "user_s", "sys_s", "nr_throttled", "throttled_ms", "intact")})
    faithful = [p for p in sweep if p["nonces"] == "syscall"]
    one = max((p for p in faithful if p["threads"] == 1), key=lambda p: p["packets_per_s"])
    best = max(faithful, key=lambda p: p["GiB_s"])
    eff = best["packets_per_s"] / (best["threads"] * one["packets_per_s"])
    full = max((p for p in faithful if p["threads"] == counts[-1]), key=lambda p: p["packets_per_s"])
    full_buf = next(p for p in sweep if p["nonces"] == "buffered" and p["threads"] == counts[-1])
    # the bare AES-GCM loop (no plugin chain, one reused buffer), one thread, ~2 s
    n0 = 20000
    t0 = O.ossl_cpu_baseline(key, 1, n0, L)
    n1 = max(n0, int(n0 / t0 * 2.0))
    aes_only = 2 * n1 * L / O.ossl_cpu_baseline(key, 1, n1, L) / 2**30
    try:
        kernel = os.uname().release
    except AttributeError:
        kernel = ""
    return {"value": best["GiB_s"], "unit": "GiB/s", "cores": best["threads"], "kind": "port",
            "best_point_pinned": best["pinned"], "physical_cores_allowed": len(cores),
            "host_cpus_busy_before": {"over_50pct": sum(1 for v in busy.values() if v > 0.5),
                                      "sum": round(sum(busy.values()), 1), "sampled_s": 0.25},
            "one_core": one["GiB_s"], "nproc": host["nproc"],
            "per_thread_efficiency": round(eff, 3),
            "at_share": {"threads": full["threads"], "GiB_s": full["GiB_s"], "cpus_busy": full["cpus_busy"],
                         "pinned": full["pinned"],
                         "sys_share": round(full["sys_s"] / max(1e-9, full["user_s"] + full["sys_s"]), 3),
                         "buffered_nonces_GiB_s": full_buf["GiB_s"]},
            "throttled_ms": round(sum(p["throttled_ms"] or 0 for p in sweep), 1),
            "aes_gcm_only_one_core": round(aes_only, 3),
            "round_trips_per_s_best": best["packets_per_s"], "round_trips_per_s_one_thread": one["packets_per_s"],
            "best_cpus_busy": best["cpus_busy"],
            "best_cpu_us_per_pair": round(best["cpus_busy"] / best["packets_per_s"] * 1e6, 3),
            "intact": all(p["intact"] for p in sweep),
            "measured_before_gpu_init": True, "kernel": kernel,
            "sweep": sweep, "host": host,
            "sample": (f"config 1: the plugin chain (Encryption + Mock over common.Payload, both directions), "
                       f"10000 payloads x {L} B per thread looped {seconds} s per point, threads "
                       f"{'/'.join(map(str, counts))} (this job's CPU share of a {host['nproc']}-CPU host: "
                       f"{threads}), each point a fresh child process run before the GPU is initialised, "
                       f"threads left to the scheduler and pinned one per physical core (least-loaded cores "
                       f"first); "
                       f"C++ mirror of the Go plugins (oracle/cpu_chain.cpp) over OpenSSL EVP aes-256-gcm with "
                       f"crypto/aes.go semantics (getrandom nonce per packet, in place); value = best point "
                       f"({best['threads']} threads, {best['packets_per_s']:.0f} packets/s sealed and opened, "
                       f"per-thread efficiency {eff:.2f}); one thread {one['GiB_s']:.3f} GiB/s; the bare "
                       f"AES-GCM loop without the chain {aes_only:.3f} GiB/s on one thread")}


def stream_copy_gbs(ctx, nbytes: int, dev, stream, reps: int = 5) -> float:
    """Achievable HBM copy rate (read + write bytes / s) with libqgcm's in-repo stream kernel (one 16-B
    non-temporal load and store per lane, a 4-KiB tile per workgroup: the fastest of the shapes
    tools/microbench/copy.hip timed, profiles/r6_s2), on random bytes (a constant buffer runs at a
    higher clock)."""
    from quantum_amd import _lib

    nbytes &= ~15
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev)
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    h = stream.cuda_stream
    _lib.check(_lib.lib().qgcm_stream_copy(ctx.handle, dst.data_ptr(), src.data_ptr(), nbytes, h), "stream_copy")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        _lib.lib().qgcm_stream_copy(ctx.handle, dst.data_ptr(), src.data_ptr(), nbytes, h)
    e1.record(stream)
    torch.cuda.synchronize()
    return 2 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9


def pmc_traffic(kind: str, N: int, L: int, stride: int):
    """HBM bytes per launch and LDS-array busy fraction of the dominant kernel from the committed
    rocprofv3 PMC passes of this command (the newest profiles/*/traffic.json), or None when they are
    absent or for another workload."""
    for path in TRAFFIC_JSONS:
        try:
            t = json.load(open(path))
        except (OSError, ValueError):
            continue
        if t.get("workload") != {"packets": N, "payload_len": L, "slot_stride": stride} or kind not in t["kernels"]:
            continue
        k = t["kernels"][kind]
        return k["hbm_bytes"], k.get("lds_array_busy"), os.path.relpath(path, ROOT)
    return None, None, None


def _sha256_device(t) -> str:
    import hashlib

    h = hashlib.sha256()
    step = 1 << 28
    for i in range(0, t.numel(), step):
        h.update(memoryview(t[i:i + step].cpu().numpy()))
    return h.hexdigest()


def extra_config3(reps: int = 5, verify: bool = True) -> dict:
    """BASELINE config 3 on the parity-checked workload (quantum_amd/workloads.py, the one
    tests/test_gpu_config3.py compares with the oracle and tests/golden/config3_digest.json pins):
    2^20 packets of U{64..9000} B under 1024 X25519 + PBKDF2 peer keys, device-resident descriptor
    batches (qgcm_seal_batch / qgcm_open_batch: device worklist sort + segmented kernel).  Each call is
    timed with HIP events on its stream (sort included).  verify: the arena's SHA-256 after the timed
    seal/open pairs (the opened state) and after one more seal, against the golden digests."""
    from quantum_amd import workloads as W

    t0 = time.perf_counter()
    keys = W.peer_keys()
    t_keys = time.perf_counter() - t0
    ctx = Context(device=0, max_keys=W.NKEYS)
    ctx.set_keys(0, keys)
    lens, kidx = W.lengths(), W.key_indices()
    offs, size = W.layout(lens)
    arena = W.device_arena(torch, size, offs, kidx)
    nonces = torch.from_numpy(W.nonces()).cuda()
    status = torch.zeros(W.N, dtype=torch.uint8, device="cuda")
    d_seal = batch.make_descs(offs, lens, kidx, "cuda")
    d_open = batch.make_descs(offs, lens.astype(np.int64) + 28, kidx, "cuda")
    stream = torch.cuda.current_stream()
    ok = True
    for _ in range(2):
        batch.seal_batch(ctx, arena, d_seal, W.N, nonces, status=status, stream=stream)
        ok &= int(status.sum()) == W.N
        batch.open_batch(ctx, arena, d_open, W.N, status=status, stream=stream)
        ok &= int(status.sum()) == W.N
    ts, to = [], []
    for _ in range(reps):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record(stream)
        batch.seal_batch(ctx, arena, d_seal, W.N, nonces, status=status, stream=stream)
        e[1].record(stream)
        batch.open_batch(ctx, arena, d_open, W.N, status=status, stream=stream)
        e[2].record(stream)
        torch.cuda.synchronize()
        ok &= int(status.sum()) == W.N
        ts.append(e[0].elapsed_time(e[1]))
        to.append(e[1].elapsed_time(e[2]))
    seal_ms, open_ms = float(np.median(ts)), float(np.median(to))
    payload = int(lens.sum())
    out = {"workload": "config3: 2^20 x U{64..9000} B, 1024 peer keys (quantum_amd/workloads.py)",
           "packets": W.N, "keys": W.NKEYS, "payload_bytes": payload,
           "value": round(2 * payload / ((seal_ms + open_ms) * 1e-3) / 2**30, 2), "unit": "GiB/s",
           "seal_ms": round(seal_ms, 3), "open_ms": round(open_ms, 3), "reps": reps,
           "timing": "HIP events around each qgcm_seal_batch / qgcm_open_batch call (worklist sort included)",
           "frac_seal": round((2 * payload + 44 * W.N) / (seal_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "frac_open": round((2 * payload + 32 * W.N) / (open_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "status_ok": ok, "key_setup_host_s": round(t_keys, 3)}
    if verify:
        gold = json.load(open(os.path.join(ROOT, "tests", "golden", "config3_digest.json")))
        out["digest_opened_ok"] = _sha256_device(arena) == gold["sha256_opened"]
        batch.seal_batch(ctx, arena, d_seal, W.N, nonces, status=status, stream=stream)
        out["digest_sealed_ok"] = _sha256_device(arena) == gold["sha256_sealed"]
    del arena  # into torch's cache (config3_host reuses it; see the note there)
    ctx.close()
    return out


def extra_config3_host(reps: int = 3, verify: bool = True, members: int = 1) -> dict:
    """Config 3's keyed batch from pinned HOST memory through the multi-GPU drop-in's entry point
    (qgcm_group_seal_host / qgcm_group_open_host, one member on this GPU: the path quantum's multi-peer
    traffic takes, worker/outgoing.go:55-80 with common/mapping.go:90-99 keys): PCIe included.  The
    member's packets are one run of adjacent records, so they move by DMA in 64-MiB chunks (no gather).
    verify: the opened arena after the timed reps and the sealed arena of one more seal against
    tests/golden/config3_digest.json.  members > 1 (tools/exp_host_legs.py only): that many member
    contexts on this GPU, the batch laid out in qgcm_group_order's order (each member's packets one run;
    the digests then do not apply)."""
    from quantum_amd import _lib
    from quantum_amd import workloads as W
    import ctypes as C

    keys = W.peer_keys()
    lens, kidx = W.lengths(), W.key_indices()
    grp = shard.Group([0] * members, max_keys=W.NKEYS)
    grp.set_keys(0, keys)
    if members > 1:
        order = grp.order(kidx)[0]
        lens, kidx = lens[order], kidx[order]
        verify = False
    offs, size = W.layout(lens)
    Lb = _lib.lib()
    a_ptr, n_ptr = Lb.qgcm_host_alloc(size), Lb.qgcm_host_alloc(12 * W.N)
    host = np.frombuffer((C.c_uint8 * size).from_address(a_ptr), np.uint8)
    nons = np.frombuffer((C.c_uint8 * (12 * W.N)).from_address(n_ptr), np.uint8)
    dev = W.device_arena(torch, size, offs, kidx)
    host[:] = dev.cpu().numpy()
    # freed into torch's cache, not to the driver: HBM released to the driver is cleared in the
    # background, and while that runs concurrent H2D + D2H copies move at about half rate (a 90-GB free
    # measured 29 vs 48 GB/s each way for a few seconds, profiles/r4_s9), which would land in the timing
    del dev
    nons[:] = W.nonces()
    d_seal = shard.host_descs(offs, lens, kidx)
    d_open = shard.host_descs(offs, lens.astype(np.int64) + 28, kidx)
    status = np.zeros(W.N, np.uint8)
    bad = grp.seal_host(a_ptr, d_seal, W.N, n_ptr, 4, status.ctypes.data)  # warm-up pair (staging, streams)
    bad += grp.open_host(a_ptr, d_open, W.N, 4, status.ctypes.data)
    ts, to = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        bad += grp.seal_host(a_ptr, d_seal, W.N, n_ptr, 4, status.ctypes.data)
        t1 = time.perf_counter()
        bad += grp.open_host(a_ptr, d_open, W.N, 4, status.ctypes.data)
        t2 = time.perf_counter()
        ts.append(t1 - t0)
        to.append(t2 - t1)
    path = ",".join(grp.last_path(m) for m in range(members))
    out = {}
    if verify:
        gold = json.load(open(os.path.join(ROOT, "tests", "golden", "config3_digest.json")))
        out["digest_opened_ok"] = _sha256_host(host) == gold["sha256_opened"]
        bad += grp.seal_host(a_ptr, d_seal, W.N, n_ptr, 4, status.ctypes.data)
        out["digest_sealed_ok"] = _sha256_host(host) == gold["sha256_sealed"]
    s, o = float(np.median(ts)), float(np.median(to))
    payload = int(lens.sum())
    del host, nons
    Lb.qgcm_host_free(a_ptr)
    Lb.qgcm_host_free(n_ptr)
    grp.close()
    return {"workload": "config3 from pinned host memory: 2^20 x U{64..9000} B, 1024 peer keys, "
                        "qgcm_group_seal_host / open_host (one member), H2D + seal/open + D2H",
            "value": round(2 * payload / (s + o) / 2**30, 2), "unit": "GiB/s", "payload_bytes": payload,
            "seal_s": round(s, 4), "open_s": round(o, 4), "member_path": path,
            "pcie_GBps_each_way": round(size / ((s + o) / 2) / 1e9, 2), "status_ok": bad == 0, "reps": reps, **out}


def extra_e2e(key: bytes, reps: int = 3, n: int = 1 << 20) -> dict:
    """Config 2 from pinned HOST memory: qgcm_seal_host / qgcm_open_host (H2D + kernels + D2H,
    pipelined in 64 MiB chunks over three streams): the PCIe-inclusive rate (never `value`).  n: packets
    (tools/exp_host_legs.py runs batches past the 4-GiB staging ring, whose slots then rotate)."""
    from quantum_amd import _lib
    import ctypes as C

    N, L = n, 1350
    stride = batch.slot_stride(L, align=64)
    ctx = Context(device=0, max_keys=4)
    ctx.set_key(0, key)
    Lb = _lib.lib()
    dev = torch.zeros(N * stride, dtype=torch.uint8, device="cuda")
    non_d = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(dev, stride, N, L, int.from_bytes(AAD, "little"), 0x5EED0001, non_d, 0x5EED0002)
    a_ptr, n_ptr = Lb.qgcm_host_alloc(N * stride), Lb.qgcm_host_alloc(12 * N)
    host = np.frombuffer((C.c_uint8 * (N * stride)).from_address(a_ptr), np.uint8)
    nons = np.frombuffer((C.c_uint8 * (12 * N)).from_address(n_ptr), np.uint8)
    host[:] = dev.cpu().numpy()
    nons[:] = non_d.cpu().numpy()
    batch.seal_uniform(ctx, dev, stride, N, L, 0, non_d)  # the device path's result, for the check
    rc = Lb.qgcm_seal_host(ctx.handle, a_ptr, stride, N, L, 0, n_ptr, 4, None)
    same = bool(np.array_equal(host, dev.cpu().numpy()))
    del dev, non_d
    rc |= Lb.qgcm_open_host(ctx.handle, a_ptr, stride, N, L + 28, 0, 4, None)
    ts, to = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        rc |= Lb.qgcm_seal_host(ctx.handle, a_ptr, stride, N, L, 0, n_ptr, 4, None)
        t1 = time.perf_counter()
        rc |= Lb.qgcm_open_host(ctx.handle, a_ptr, stride, N, L + 28, 0, 4, None)
        t2 = time.perf_counter()
        ts.append(t1 - t0)
        to.append(t2 - t1)
    s, o = float(np.median(ts)), float(np.median(to))
    del host, nons
    Lb.qgcm_host_free(a_ptr)
    Lb.qgcm_host_free(n_ptr)
    ctx.close()
    torch.cuda.empty_cache()
    return {"workload": f"config2 from pinned host memory: {N} x {L} B, H2D + seal/open + D2H",
            "value": round(2 * N * L / (s + o) / 2**30, 2), "unit": "GiB/s", "seal_s": round(s, 4),
            "open_s": round(o, 4), "pcie_GBps_each_way": round(N * stride / ((s + o) / 2) / 1e9, 2),
            "matches_device_path": same, "status_ok": rc == 0, "reps": reps}


def extra_worker_batches(key: bytes, reps: int = 30, sizes=(64, 1024, 16384)) -> dict:
    """Worker-sized batches (a recvmmsg batch of Payload.Raw slots, 1350 B in 1472-B slots, pinned):
    median microseconds per seal + open pair through qgcm_seal_host (one peer) and through a one-member
    group (qgcm_group_seal_host, 8 peers, packet i of peer i % 8), both sealed in place.
    Checked in the run: the first host seal equals the device path's bytes (qgcm_seal_uniform), the
    first group seal the device descriptor batch's (qgcm_seal_batch); every open restores the plaintext."""
    from quantum_amd import _lib
    import ctypes as C

    L, stride, nmax = 1350, 1472, max(sizes)
    keys = b"".join(bytes((b + 7 * k) & 0xFF for b in key) for k in range(8))  # 8 distinct peer keys
    ctx = Context(device=0, max_keys=8)
    ctx.set_key(0, keys[:32])
    grp = shard.Group([0], max_keys=8)
    grp.set_keys(0, keys)
    dctx = Context(device=0, max_keys=8)
    for k in range(8):
        dctx.set_key(k, keys[32 * k:32 * k + 32])
    Lb = _lib.lib()
    a_ptr, n_ptr = Lb.qgcm_host_alloc(nmax * stride), Lb.qgcm_host_alloc(12 * nmax)
    host = np.frombuffer((C.c_uint8 * (nmax * stride)).from_address(a_ptr), np.uint8)
    nons = np.frombuffer((C.c_uint8 * (12 * nmax)).from_address(n_ptr), np.uint8)
    rng = np.random.default_rng(0x5EED0077)
    host[:] = rng.integers(0, 256, host.size, dtype=np.uint8)
    host.reshape(nmax, stride)[:, :4] = np.frombuffer(AAD, np.uint8)
    Lb.qgcm_random_nonces(n_ptr, nmax)
    plain = host.copy()
    out, ok = {}, True
    for n in sizes:
        offs = np.arange(n, dtype=np.uint64) * stride
        kidx = (np.arange(n) % 8).astype(np.uint32)
        d_seal = shard.host_descs(offs, np.full(n, L, np.uint32), kidx)
        d_open = shard.host_descs(offs, np.full(n, L + 28, np.uint32), kidx)
        row = {}
        for path in ("host", "group"):
            # the device path's bytes for this batch, from the same plaintext and nonces
            dev = torch.from_numpy(plain[:n * stride].copy()).cuda()
            dn = torch.from_numpy(nons[:12 * n].copy()).cuda()
            if path == "host":
                batch.seal_uniform(ctx, dev, stride, n, L, 0, dn)
            else:
                batch.seal_batch(dctx, dev, batch.make_descs(offs, [L] * n, kidx.tolist(), "cuda"), n, dn)
            want = dev.cpu().numpy()
            ts = []
            for r in range(reps + 1):
                t0 = time.perf_counter()
                if path == "host":
                    bad = Lb.qgcm_seal_host(ctx.handle, a_ptr, stride, n, L, 0, n_ptr, 4, None)
                    if r == 0:
                        ok &= bool(np.array_equal(host[:n * stride], want))
                    bad += Lb.qgcm_open_host(ctx.handle, a_ptr, stride, n, L + 28, 0, 4, None)
                else:
                    bad = grp.seal_host(a_ptr, d_seal, n, n_ptr, 4)
                    if r == 0:
                        ok &= bool(np.array_equal(host[:n * stride], want))
                    bad += grp.open_host(a_ptr, d_open, n, 4)
                if r:
                    ts.append(time.perf_counter() - t0)
                ok &= bad == 0
            ok &= bool(np.array_equal(host[:n * stride].reshape(n, stride)[:, :4 + L],
                                      plain[:n * stride].reshape(n, stride)[:, :4 + L]))
            row[f"{path}_pair_us"] = round(float(np.median(ts)) * 1e6, 1)
            row[f"{path}_path"] = "seal_host" if path == "host" else grp.last_path(0)
            del dev, dn
        out[str(n)] = row
    del host, nons
    Lb.qgcm_host_free(a_ptr)
    Lb.qgcm_host_free(n_ptr)
    grp.close()
    dctx.close()
    ctx.close()
    return {"workload": f"worker-sized batches from pinned host memory: {list(sizes)} x {L} B in {stride}-B slots, "
                        "seal + open pair, qgcm_seal_host (1 peer) and a one-member group (8 peers)",
            "value": out[str(sizes[0])]["group_pair_us"], "unit": f"us per seal+open pair of {sizes[0]} keyed packets",
            "higher_is_better": False, "by_packets": out, "matches_device_path": ok, "status_ok": ok, "reps": reps}


def _sha256_host(a: np.ndarray) -> str:
    import hashlib

    h = hashlib.sha256()
    flat = a.reshape(-1)
    for i in range(0, flat.size, 1 << 28):
        h.update(memoryview(flat[i:i + (1 << 28)]))
    return h.hexdigest()


def _config5_golden() -> dict:
    return json.load(open(os.path.join(ROOT, "tests", "golden", "config5_digest.json")))


def extra_config5(key: bytes, threads: int, reps: int = 3, verify: bool = True) -> dict:
    """BASELINE config 5: snappy compress -> seal, then open -> uncompress, 2^20 x 1350 B packets in
    pinned host memory (quantum_amd/workloads.py config5_*: each packet's first half seeded random bytes,
    second half a repeated HTTP request line), host codec workers overlapped with PCIe copies and the
    device (qgcm_compress_seal_host / qgcm_open_uncompress_host; copies included).  verify: after the timed
    reps of each codec mode, one more compress+seal whose whole arena and lengths must hash to
    tests/golden/config5_digest.json (libsnappy + OpenSSL), then open+uncompress back to the plaintext."""
    from quantum_amd import _lib
    from quantum_amd import workloads as W
    import ctypes as C

    N, L, stride = W.C5_N, W.C5_LEN, W.C5_STRIDE  # stride = common.MaxPacketLength (the Payload.Raw buffer)
    gold = _config5_golden() if verify else None
    ctx = Context(device=0, max_keys=4)
    ctx.set_key(0, key)
    Lb = _lib.lib()
    a_ptr, n_ptr = Lb.qgcm_host_alloc(N * stride), Lb.qgcm_host_alloc(12 * N)
    host = np.frombuffer((C.c_uint8 * (N * stride)).from_address(a_ptr), np.uint8).reshape(N, stride)
    nons = np.frombuffer((C.c_uint8 * (12 * N)).from_address(n_ptr), np.uint8)
    host[:] = W.config5_packets(N, L, stride)
    nons[:] = W.config5_nonces(N)
    plain = host[:, :4 + L].copy()
    lens = np.full(N, L, np.uint32)

    def run(mode: int) -> tuple[float, float, int, int, tuple[int, int], bool | None]:
        batch.chain_codec(ctx, mode)
        ts, to, bad, sealed = [], [], 0, 0
        c0 = ctx.launch_counts()
        for _ in range(reps):
            lens[:] = L
            t0 = time.perf_counter()
            bad += batch.compress_seal_host(ctx, a_ptr, stride, N, lens, 0, n_ptr, threads=threads)
            t1 = time.perf_counter()
            sealed = int(lens.sum())
            bad += batch.open_uncompress_host(ctx, a_ptr, stride, N, lens, 0, threads=threads)
            t2 = time.perf_counter()
            ts.append(t1 - t0)
            to.append(t2 - t1)
        c1 = ctx.launch_counts()
        dev = (c1["snappy_enc"] - c0["snappy_enc"]) // reps, (c1["snappy_dec"] - c0["snappy_dec"]) // reps
        digest_ok = None
        if gold is not None:  # untimed: the sealed state against the golden digest, then back
            lens[:] = L
            bad += batch.compress_seal_host(ctx, a_ptr, stride, N, lens, 0, n_ptr, threads=threads)
            digest_ok = (_sha256_host(host) == gold["sha256_sealed"] and
                         _sha256_host(lens.astype("<u4")) == gold["sha256_sealed_lens"])
            bad += batch.open_uncompress_host(ctx, a_ptr, stride, N, lens, 0, threads=threads)
        return float(np.median(ts)), float(np.median(to)), bad, sealed, dev, digest_ok

    modes = {}
    for mode, name in ((0, "host"), (2, "device"), (1, "split")):  # the default (split) last: the value
        s, o, bad, sealed, dev, digest_ok = run(mode)
        ok = bad == 0 and bool(np.array_equal(host[:, :4 + L], plain)) and bool((lens == L).all())
        modes[name] = {"value": round(2 * N * L / (s + o) / 2**30, 2), "compress_seal_s": round(s, 4),
                       "open_uncompress_s": round(o, 4), "device_chunks_seal_open": dev, "restored": ok,
                       "sealed_digest_ok": digest_ok}
    restored = all(m["restored"] for m in modes.values())
    digests = None if gold is None else all(m["sealed_digest_ok"] for m in modes.values())
    del host, nons, plain
    Lb.qgcm_host_free(a_ptr)
    Lb.qgcm_host_free(n_ptr)
    ctx.close()
    return {"workload": f"config5: snappy -> AES-256-GCM chain, {N} x {L} B host packets, copies included",
            "value": round(2 * N * L / (s + o) / 2**30, 2), "unit": "GiB/s of uncompressed payload",
            "compress_seal_s": round(s, 4), "open_uncompress_s": round(o, 4),
            "sealed_over_plain": round(sealed / (N * L), 4), "codec_threads": threads,
            "codec": "snappy block codec (golang/snappy's algorithm, libsnappy-exact bytes): host C++ workers "
                     "with the gfx950 device codec taking the chunks they cannot keep up with (qgcm_chain_codec 1)",
            "chunks": (N * stride + (32 << 20) - 1) // (32 << 20), "by_codec_mode": modes,
            "sealed_digest_ok": digests, "digest_source": "tests/golden/config5_digest.json",
            "status_ok": restored, "restored": restored, "reps": reps}


def extra_config5_resident(key: bytes, reps: int = 5, verify: bool = True) -> dict:
    """Config 5's chain with the codec on the GPU and the packets resident in HBM (no PCIe): device
    snappy compress (writing the seal descriptors) -> seal, then open -> device uncompress, on config
    5's packets and nonces; HIP events per stage, the arena checked against the plaintext after each rep.
    verify: the first rep's sealed arena and lengths against tests/golden/config5_digest.json."""
    from quantum_amd import workloads as W

    N, L, stride = W.C5_N, W.C5_LEN, W.C5_STRIDE
    gold = _config5_golden() if verify else None
    ctx = Context(device=0, max_keys=4)
    ctx.set_key(0, key)
    plain = torch.from_numpy(W.config5_packets(N, L, stride).reshape(-1)).cuda()
    arena = plain.clone()
    nonces = torch.from_numpy(W.config5_nonces(N)).cuda()
    lens = torch.empty(N, dtype=torch.int32, device="cuda")
    descs = torch.empty(16 * N, dtype=torch.uint8, device="cuda")
    status = torch.empty(N, dtype=torch.uint8, device="cuda")
    limit = stride - 4 - 28
    times = {k: [] for k in ("compress", "seal", "open", "uncompress")}
    ok, sealed, digest_ok = True, 0, None
    for r in range(reps + 1):
        arena.copy_(plain)
        lens.fill_(L)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        ev[0].record()
        batch.snappy_compress(ctx, arena, stride, N, lens, stride - 4, limit, status, descs_out=descs, key_idx=0)
        ev[1].record()
        batch.seal_batch(ctx, arena, descs, N, nonces, status=status)
        ev[2].record()
        torch.cuda.synchronize()
        ok &= bool((status == 1).all())
        clen = lens.clone()
        sealed = int(clen.sum()) + 28 * N
        if r == 0 and gold is not None:  # untimed warm-up rep
            digest_ok = (_sha256_device(arena) == gold["sha256_sealed"] and
                         _sha256_host(clen.cpu().numpy().astype("<u4") + np.uint32(28)) == gold["sha256_sealed_lens"])
        d = descs.view(torch.int32).view(N, 4)
        d[:, 2] += 28  # the receiver's descriptors: sealed lengths (outside the timed stages)
        ev[3].record()
        batch.open_batch(ctx, arena, descs, N, status=status)
        ev[4].record()
        batch.snappy_uncompress(ctx, arena, stride, N, clen, limit, stride - 4, status)
        ev[5].record()
        torch.cuda.synchronize()
        ok &= bool((status == 1).all()) and bool((clen == L).all())
        ok &= bool(torch.equal(arena.view(N, stride)[:, :4 + L], plain.view(N, stride)[:, :4 + L]))
        if r > 0:
            for k, (a, b) in zip(times, ((0, 1), (1, 2), (3, 4), (4, 5))):
                times[k].append(ev[a].elapsed_time(ev[b]))
    med = {k: float(np.median(v)) for k, v in times.items()}
    ctx.close()
    del arena, plain
    torch.cuda.empty_cache()
    total = sum(med.values())
    return {"workload": f"config5 on device-resident slots: device snappy -> AES-256-GCM and back, {N} x {L} B",
            "value": round(2 * N * L / (total * 1e-3) / 2**30, 2), "unit": "GiB/s of uncompressed payload (kernels only)",
            **{f"{k}_ms": round(v, 3) for k, v in med.items()},
            "compress_GBps": round(N * L / (med["compress"] * 1e-3) / 1e9, 1),
            "uncompress_GBps": round(N * L / (med["uncompress"] * 1e-3) / 1e9, 1),
            "sealed_over_plain": round(sealed / (N * L), 4), "status_ok_and_restored": ok,
            "sealed_digest_ok": digest_ok, "reps": reps}


def extra_two_streams(key: bytes, steps: int = 200, settle: int = 100) -> dict:
    """Config 2's batch as a deployment with two workers would run it: the arena's halves on two streams,
    each half sealed then opened by its own qgcm_seal_uniform / qgcm_open_uniform calls, the streams
    never joined inside the timed steps (tools/exp_streams.py "halves").  On one stream every launch waits
    for the previous one to drain; here one stream's launches fill the other's drain (profiles/r6_s6,
    r6_s7: +3.3% over one stream at ~5% fewer cycles).  Never `value`: the headline keeps bench.py's
    one-stream step, whose per-launch kernel times the roofline is quoted on.  The arena's digests after
    the timed steps are checked against tests/golden/rank_digest.json."""
    N, L = 1 << 20, 1350
    stride = batch.slot_stride(L, align=64)
    ctx = Context(device=0, max_keys=4)
    ctx.set_key(0, key)
    alloc = torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda")
    arena = alloc[60:]
    nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
    status = torch.zeros(N, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(arena, stride, N, L, int.from_bytes(AAD, "little"), 0x5EED0001, nonces, 0x5EED0002)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    h = N // 2
    halves = [(arena[k * h * stride:(k + 1) * h * stride], nonces[12 * k * h:12 * (k + 1) * h],
               status[k * h:(k + 1) * h]) for k in range(2)]

    def run(k):
        for _ in range(k):
            for s, (a, no, st) in zip(streams, halves):
                batch.seal_uniform(ctx, a, stride, h, L, 0, no, status=None, stream=s)
                batch.open_uniform(ctx, a, stride, h, L + 28, 0, status=st, stream=s)

    run(settle)
    torch.cuda.synchronize()
    tele = GpuTelemetry(0)
    tele.start()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tele.stop()
    clock = tele.summary()
    tele.close()
    ok = int(status.sum().item()) == N
    d = rank_digests(ctx, arena, nonces, status, stride, N, L, 0, torch.cuda.current_stream())
    ctx.close()
    del alloc, arena, nonces, status
    torch.cuda.empty_cache()
    ms = el * 1e3 / steps
    return {"workload": f"config2 as two workers: the halves of {N} x {L} B on two streams, each sealed then opened",
            "value": round(2 * N * L / (ms * 1e-3) / 2**30, 2), "unit": "GiB/s", "ms_per_step": round(ms, 4),
            "steps": steps, "algorithmic_GBps": round(N * (4 * L + 76) / (ms * 1e-3) / 1e9, 1),
            "frac_of_hbm_peak": round(N * (4 * L + 76) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "sclk_mhz_mean": clock["sclk_mhz_mean"], "power_w_mean": clock["power_w_mean"],
            "status_ok": ok, "sealed_digest_ok": d["sealed_digest_ok"], "opened_digest_ok": d["opened_digest_ok"],
            "note": "never `value`: the headline is the one-stream step"}


def extra_config4_one_gpu(key: bytes, steps: int = 3, warmup: int = 1, settle_ms: float = 300.0) -> dict:
    """BASELINE config 4's whole batch on ONE GPU: 64 x 2^20 x 1350 B (94.5 GB of 1408-B slots, one
    MI355X holds it), seal then unseal, so the N-GPU lines (config 4 sharded over N ranks) have a
    same-workload N = 1 anchor: per-GPU efficiency at N = value_N / (N x this value).  One step is the
    same pair of uniform calls the headline makes (2^20-packet launches), timed between synchronizes."""
    N, L = CONFIG4_PACKETS, 1350
    stride = batch.slot_stride(L, align=64)
    ctx = Context(device=0, max_keys=4)
    ctx.set_key(0, key)
    alloc = torch.empty(N * stride + 64, dtype=torch.uint8, device="cuda")
    arena = alloc[60:]
    nonces = torch.empty(12 * N, dtype=torch.uint8, device="cuda")
    status = torch.zeros(N, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(arena, stride, N, L, int.from_bytes(AAD, "little"), 0x5EED0001, nonces, 0x5EED0002)
    stream = torch.cuda.current_stream()

    def step():
        batch.seal_uniform(ctx, arena, stride, N, L, 0, nonces, status=None, stream=stream)
        batch.open_uniform(ctx, arena, stride, N, L + 28, 0, status=status, stream=stream)

    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < settle_ms:
        step()
        torch.cuda.synchronize()
    tele = GpuTelemetry(0)
    tele.start()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tele.stop()
    clock = tele.summary()
    tele.close()
    ok = int(status.sum().item()) == N
    del alloc, arena, nonces, status
    ctx.close()
    torch.cuda.empty_cache()
    return {"workload": f"config4 on one GPU: {N} x {L} B packets (the whole 8-GPU batch), seal then unseal, 1 key",
            "value": round(2 * N * L / (el / steps) / 2**30, 2), "unit": "GiB/s",
            "ms_per_step": round(el * 1e3 / steps, 2), "steps": steps, "packets": N, "slot_stride": stride,
            "arena_GB": round(N * stride / 1e9, 1), "status_ok": ok,
            "sclk_mhz_mean": clock["sclk_mhz_mean"], "power_w_mean": clock["power_w_mean"],
            "power_cap_w": clock["power_cap_w"], "gpu_clock_power": clock,
            "use": "N = 1 anchor of the config-4 scaling curve (bench.py --gpus N runs config 4 sharded)"}


def rank_digests(ctx, arena, nonces, status, stride: int, N: int, L: int, rank: int, stream,
                 verify: bool = True) -> dict:
    """After the timed loop (untimed), on every rank: the first P slots of this rank's arena against
    tests/golden/rank_digest.json (make_rank_golden.py: the C restatement over every packet of ranks 0-7,
    equal to OpenSSL; rank r's fill uses seeds 0x5EED0001 + r / 0x5EED0002 + r, and slot i's bytes depend
    only on i and the seeds, so one golden covers every N), P the largest of 2^20 / 2^18 / 2^16 that fits.
    Three states: what the timed steps left (sealed then opened K times: plaintext with each slot's
    tag || nonce), then one more seal of the prefix with the same calls (ciphertext, tag, nonce), then the
    open back.  At N = 1 and 2^20 packets the prefix is the whole headline arena (rank 0's 2^20 digests
    equal tests/golden/headline_digest.json).  Other layouts: the fields say why not."""
    if not verify:
        return {"sealed_digest_ok": None, "digest_skipped": "--no-verify"}
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "rank_digest.json")))
    fits = [p for p in gold["prefixes"] if p <= N]
    if (L, stride) != (gold["len"], gold["stride"]) or rank >= len(gold["ranks"]) or not fits:
        return {"sealed_digest_ok": None, "digest_skipped": "not the golden's layout"}
    P = max(fits)
    want = gold["ranks"][rank]["prefixes"][str(P)]
    a, st = arena[:P * stride], status[:P]  # the prefix's slots only
    torch.cuda.synchronize()
    timed_ok = _sha256_device(a) == want["sha256_opened"]
    batch.seal_uniform(ctx, a, stride, P, L, 0, nonces[:12 * P], status=None, stream=stream)
    torch.cuda.synchronize()
    sealed_ok = _sha256_device(a) == want["sha256_sealed"]
    batch.open_uniform(ctx, a, stride, P, L + 28, 0, status=st, stream=stream)
    torch.cuda.synchronize()
    opened_ok = _sha256_device(a) == want["sha256_opened"] and int(st.sum().item()) == P
    return {"sealed_digest_ok": sealed_ok, "opened_digest_ok": opened_ok and timed_ok, "digest_prefix": P,
            "digest_source": "tests/golden/rank_digest.json"}


class GpuTelemetry:
    """Clock and power of this rank's GPU while the timed steps run (DESIGN.md s5 "The clock and the power
    limit"): a background thread reads amdsmi's gpu_metrics of the PCI device torch calls cuda:<dev>
    every `period_s`, and the power cap once.  Reported: the mean of the per-XCD current GFX clocks, the
    mean socket power, the cap, and the share of the interval the SMU counted as power- (PPT) or
    thermally-limited (its residency accumulators, differenced over the interval).  When amdsmi is
    missing or refuses this process, `summary()` says so instead of a number."""

    def __init__(self, device: int, period_s: float = 0.01):
        import threading

        self.period, self.samples, self.err, self.h, self.smi = period_s, [], None, None, None
        self.first = self.last = None
        self.span = "the timed steps"
        self.started = False
        self._stop = threading.Event()
        self._th = None
        try:
            import amdsmi

            amdsmi.amdsmi_init()
            self.smi = amdsmi
            p = torch.cuda.get_device_properties(device)
            bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
            for h in amdsmi.amdsmi_get_processor_handles():
                if amdsmi.amdsmi_get_gpu_device_bdf(h).lower() == bdf.lower():
                    self.h = h
            if self.h is None:
                self.err = f"amdsmi has no device {bdf}"
        except Exception as e:  # noqa: BLE001 -- reported in the line, never fatal
            self.err = f"amdsmi: {type(e).__name__}: {e}"

    @staticmethod
    def _num(v):
        if isinstance(v, (int, float)) and v not in (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF):
            return float(v)
        return None

    def _read(self) -> dict | None:
        try:
            m = self.smi.amdsmi_get_gpu_metrics_info(self.h)
        except Exception as e:  # noqa: BLE001
            self.err = f"gpu_metrics: {type(e).__name__}: {e}"
            return None
        clk = m.get("current_gfxclks")
        clks = [self._num(c) for c in clk] if isinstance(clk, (list, tuple)) else [self._num(clk)]
        clks = [c for c in clks if c]
        if not clks:
            c = self._num(m.get("current_gfxclk")) or self._num(m.get("average_gfxclk_frequency"))
            clks = [c] if c else []
        power = self._num(m.get("current_socket_power")) or self._num(m.get("average_socket_power"))
        return {"t": time.perf_counter(), "sclk": sum(clks) / len(clks) if clks else None, "power": power,
                "xcd": clks if isinstance(clk, (list, tuple)) and len(clks) > 1 else None,
                "uclk": self._num(m.get("current_uclk")), "socclk": self._num(m.get("current_socclk")),
                "hotspot": self._num(m.get("temperature_hotspot")),
                "acc": {k: self._num(m.get(k)) for k in ("accumulation_counter", "ppt_residency_acc",
                                                           "socket_thm_residency_acc", "prochot_residency_acc")},
                "throttle": m.get("throttle_status")}

    def _loop(self) -> None:
        while not self._stop.wait(self.period):
            s = self._read()
            if s:
                self.samples.append(s)

    def start(self) -> None:
        self.started = True
        if self.h is None:
            return
        import threading

        self.first = self._read()
        self._th = threading.Thread(target=self._loop, daemon=True)
        self._th.start()

    def stop(self) -> None:
        if self._th is not None:
            self._stop.set()
            self._th.join()
            self.last = self._read()

    def _per_xcd(self):
        xs = [x["xcd"] for x in self.samples if x.get("xcd")]
        if not xs or len({len(x) for x in xs}) != 1:
            return None
        return [round(sum(c) / len(c), 1) for c in zip(*xs)]

    def summary(self) -> dict:
        if self.h is None or not self.samples:
            return {"sclk_mhz_mean": None, "power_w_mean": None, "power_cap_w": None,
                    "telemetry": self.err or "no samples"}
        clk = [s["sclk"] for s in self.samples if s["sclk"]]
        pw = [s["power"] for s in self.samples if s["power"]]
        cap = None
        try:
            c = self.smi.amdsmi_get_power_cap_info(self.h)
            cap = self._num(c.get("power_cap"))
            if cap and cap > 1e5:  # reported in microwatts by this amdsmi
                cap /= 1e6
        except Exception as e:  # noqa: BLE001
            self.err = f"power_cap: {type(e).__name__}: {e}"
        out = {"sclk_mhz_mean": round(sum(clk) / len(clk), 1) if clk else None,
               "sclk_mhz_min": min(clk) if clk else None, "sclk_mhz_max": max(clk) if clk else None,
               "power_w_mean": round(sum(pw) / len(pw), 1) if pw else None, "power_w_max": max(pw) if pw else None,
               "power_cap_w": cap, "samples": len(self.samples),
               # per-XCD GFX clocks (the XCDs run at different speeds: DESIGN.md 4.1, the shared tail)
               "sclk_mhz_mean_per_xcd": self._per_xcd(),
               **{f"{k}_mean": (round(sum(v) / len(v), 1) if v else None)
                  for k, v in (("uclk_mhz", [x["uclk"] for x in self.samples if x["uclk"]]),
                               ("socclk_mhz", [x["socclk"] for x in self.samples if x["socclk"]]),
                               ("hotspot_c", [x["hotspot"] for x in self.samples if x["hotspot"]]))},
               "telemetry": f"amdsmi gpu_metrics every {self.period * 1e3:.0f} ms over {self.span}"}
        a0, a1 = (self.first or {}).get("acc", {}), (self.last or {}).get("acc", {})
        ticks = (a1.get("accumulation_counter") or 0) - (a0.get("accumulation_counter") or 0)
        if ticks > 0:
            for k, name in (("ppt_residency_acc", "ppt_limited_frac"), ("socket_thm_residency_acc", "thermal_limited_frac"),
                            ("prochot_residency_acc", "prochot_frac")):
                if a0.get(k) is not None and a1.get(k) is not None:
                    out[name] = round((a1[k] - a0[k]) / ticks, 3)
        if self.err:
            out["telemetry_note"] = self.err
        return out

    def close(self) -> None:
        self.stop()
        if self.smi is not None:
            try:
                self.smi.amdsmi_shut_down()
            except Exception:  # noqa: BLE001
                pass


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args: argparse.Namespace) -> None:
    """`--gpus N` means N ranks.  Without a launcher around us (no WORLD_SIZE) and N > 1, start
    torch.distributed.run with N local ranks on this script -- as a child process, before anything
    here touches the GPU -- and exit with its status.  Under a launcher, WORLD_SIZE must equal N.
    quantum runs one process per node (main.go:72-75); here the unit of independence is a GPU, so the
    bench is one rank per GPU with no data-path collective."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
        return
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus == 1:
        return
    if not args.one_device:
        have = torch.cuda.device_count()  # does not initialise the GPU on this image
        if have < args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but only {have} GPU(s) are visible "
                             "(--one-device --dist-backend gloo rehearses N ranks on one GPU)")
    elif args.dist_backend == "nccl":
        raise SystemExit("--one-device needs --dist-backend gloo (RCCL allows one rank per GPU)")
    import subprocess

    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    rc = subprocess.run(cmd, env=env).returncode
    sys.exit(rc)


def extra_per_packet(seconds: float = 1.5) -> dict:
    """The per-call drop-in (qgcm_seal_one / qgcm_open_one, crypto/aes.go:41-62 from quantum's worker
    threads, worker/outgoing.go:83-93): tools/bin/per_packet_bench (built by __graft_entry__.build()),
    one 1350-B seal+open in flight per thread, through the resident kernel and through a kernel launch
    per call, 1 / 16 / 64 threads, and the resident kernel with every waiting caller asleep on a futex
    (QGCM_RESIDENT_SPINNERS=0) at 16 and 64.  Each point reports `cpu_us_per_pair`: the process's host CPU
    time per seal+open pair.  Run as child processes after the headline."""
    import subprocess

    exe = os.path.join(ROOT, "tools", "bin", "per_packet_bench")
    if not os.path.exists(exe):
        return {"skipped": "tools/bin/per_packet_bench not built (python -c 'import __graft_entry__ as g; g.build()')"}
    out = {"workload": "per-packet Encrypt/Decrypt calls, 1350 B, one packet in flight per thread",
           "unit": "seal+open round trips/s"}
    for threads, mode, spinners in ((1, "both", None), (16, "both", None), (64, "resident", None),
                                    (16, "resident", "0"), (64, "resident", "0")):
        env = dict(os.environ)
        env.pop("QGCM_RESIDENT_SPINNERS", None)
        if spinners is not None:
            env["QGCM_RESIDENT_SPINNERS"] = spinners
        r = subprocess.run([exe, str(threads), "1350", str(seconds), "0", mode], capture_output=True, text=True,
                           timeout=120, env=env)
        if r.returncode != 0:
            raise RuntimeError(f"per_packet_bench {threads}: rc {r.returncode}: {r.stderr[-300:]}")
        for ln in r.stdout.splitlines():
            d = json.loads(ln)
            name = f"{d['path']}_t{threads}" + ("" if spinners is None else f"_spinners{spinners}")
            out[name] = {k: d[k] for k in ("round_trips_per_s", "call_pair_p50_us", "call_pair_p99_us", "failures",
                                           "cpus_busy", "cpu_us_per_pair")}
    return out


def main() -> None:
    args = parse()
    launch_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    key = derive_key(SECRET, SALT)  # crypto/aes.go:66, host, once
    host = host_cpus()
    # the CPU baseline first, before anything initialises the GPU (no runtime threads, no GPU-side
    # host work in this cgroup while the CPU chain runs)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        print("[bench] cpu baseline sweep", file=sys.stderr, flush=True)
        cpu = cpu_baseline(key, args.len, args.cpu_threads or host["share"], host)
    dist = None
    if args.one_device and args.dist_backend == "nccl" and world > 1:
        raise SystemExit("--one-device needs --dist-backend gloo (RCCL allows one rank per GPU)")
    local = 0 if args.one_device else local
    torch.cuda.set_device(local)  # before the process group, so RCCL binds each rank to its GPU
    dev = torch.device("cuda", local)
    if world > 1 or "WORLD_SIZE" in os.environ:  # under a launcher: a process group even for one rank
        import torch.distributed as dist

        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", init_method="env://", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend, init_method="env://")

    workload = args.workload if args.workload != "auto" else ("config2" if world == 1 else "config4")
    if args.packets:
        N = args.packets
    elif workload == "config4":
        lo, hi = shard.packet_range(CONFIG4_PACKETS, world, rank)
        N = hi - lo
    else:
        N = 1 << 20
    L = args.len
    stride = args.stride or batch.slot_stride(L, align=64)
    ctx = Context(device=local, max_keys=16)
    ctx.set_key(0, key)

    # Slots are Payload.Raw records; the arena starts 60 B into a 64-B aligned allocation so every
    # payload (Raw[4:]) is 64-B aligned and each quad of lanes moves whole 64-B granules.
    arena_alloc = torch.zeros(N * stride + 64, dtype=torch.uint8, device=dev)
    arena = arena_alloc[60:]
    nonces = torch.zeros(12 * N, dtype=torch.uint8, device=dev)
    status = torch.zeros(N, dtype=torch.uint8, device=dev)
    aad_word = int.from_bytes(AAD, "little")
    batch.fill_uniform(arena, stride, N, L, aad_word, 0x5EED0001 + rank, nonces, 0x5EED0002 + rank)
    stream = torch.cuda.current_stream()

    # ev: (after the seal, after the open); the timed loop records one event before its first step, and
    # each step's last event is the next step's first, so the K steps carry 2K + 1 records (each record is
    # a packet in the stream between two launches: ~5 us, profiles/r6_s22)
    def step(ev=None):
        batch.seal_uniform(ctx, arena, stride, N, L, 0, nonces, status=None, stream=stream)
        if ev is not None:
            ev[0].record(stream)
        batch.open_uniform(ctx, arena, stride, N, L + 28, 0, status=status, stream=stream)
        if ev is not None:
            ev[1].record(stream)

    # clock settle: the same step back to back for settle_ms of wall time, so the timed steps run at
    # the clocks the chip holds under this load (not timed, not counted as warmup)
    # clock and power (GpuTelemetry): sampled from 100 ms into the settle loop (the clocks have come up
    # by then, DESIGN.md s5 "Clock ramp") through the timed steps -- the same step back to back all along,
    # so a short timed region (the driver's 20 steps are ~65 ms) still gets a few dozen samples
    tele = GpuTelemetry(local)
    tele.span = "the settle loop's last part, the warmup and the timed steps (the same step back to back)"
    settle = 0
    t_settle = time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
        step()
        settle += 1
        if settle % 8 == 0:
            torch.cuda.synchronize()  # bound the launch queue; the loop keeps the GPU busy
            if not tele.started and (time.perf_counter() - t_settle) * 1e3 >= min(100.0, args.settle_ms / 2):
                tele.start()
    if not tele.started:
        tele.span = "the warmup and the timed steps"
        tele.start()
    for _ in range(args.warmup):
        step()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.steps + 1)]

    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record(stream)
    for k in range(args.steps):
        step((evs[2 * k + 1], evs[2 * k + 2]))
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tele.stop()
    clock = tele.summary()
    tele.close()
    ok = int(status.sum().item()) == N  # the last timed open authenticated every packet
    # max over ranks, AND of the per-rank status (the only cross-rank traffic; no data collective)
    seal_ms = sum(evs[2 * k].elapsed_time(evs[2 * k + 1]) for k in range(args.steps)) / args.steps
    open_ms = sum(evs[2 * k + 1].elapsed_time(evs[2 * k + 2]) for k in range(args.steps)) / args.steps
    own_elapsed = elapsed
    coll_dev = dev if args.dist_backend == "nccl" else None
    elapsed, ok = shard.reduce_step_time(elapsed, ok, dist, coll_dev)
    # every rank checks its own arena against the golden (untimed, before anything else touches it)
    digests = rank_digests(ctx, arena, nonces, status, stride, N, L, rank, stream, verify=not args.no_verify)

    def flag(v):
        return -1.0 if v is None else float(bool(v))

    def num(v):
        return float("nan") if v is None else float(v)

    # every rank's own figures (after the timed region): per-GPU rates of the multi-GPU line
    per_rank = shard.gather_rank_stats([own_elapsed, seal_ms, open_ms, N, flag(digests["sealed_digest_ok"]),
                                        flag(digests.get("opened_digest_ok")), num(clock["sclk_mhz_mean"]),
                                        num(clock["power_w_mean"])], dist, coll_dev)
    ms_step = elapsed * 1e3 / args.steps
    total_packets = CONFIG4_PACKETS if workload == "config4" and not args.packets else world * N
    total_bytes = 2 * total_packets * L  # each payload byte counted once sealed and once unsealed
    value = total_bytes / (elapsed / args.steps) / 2**30

    # dominant kernel roofline: algorithmic bytes per launch: seal 2L+44, open 2L+32
    if seal_ms >= open_ms:
        kname, kms, per_pkt = "seal", seal_ms, 2 * L + 44
    else:
        kname, kms, per_pkt = "open", open_ms, 2 * L + 32
    achieved = N * per_pkt / (kms * 1e-3) / 1e9
    read_pkt = L + 16 if kname == "seal" else L + 32  # the HBM-read-only variant
    achieved_read = N * read_pkt / (kms * 1e-3) / 1e9
    traffic, lds_busy, traffic_src = pmc_traffic(kname, N, L, stride)
    # libqgcm launches a uniform batch in chunks of LAUNCH_CHUNK packets: kms spans them all
    chunk = int(os.environ.get("QGCM_LAUNCH_CHUNK", str(LAUNCH_CHUNK))) // 64 * 64 or N
    launches = -(-N // chunk)
    # after the timed region; an arena-sized buffer up to 4 GiB (past the 256-MiB Infinity Cache the rate
    # does not depend on the size: 6.52 / 6.47 TB/s at 1.48 / 8 GB, profiles/r6_s2)
    copy_gbs = stream_copy_gbs(ctx, min(N * stride, 4 << 30), dev, stream)

    if rank == 0:
        line = {
            "metric": "AES-256-GCM seal+unseal GiB/s (device-resident packets) at 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if workload == "config4" and world > 1 and not args.packets else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded splitmix64 payloads and nonces, one PBKDF2-derived key)",
            "config": {"workload": (f"config4: {total_packets} x {L} B packets sharded over {world} GPUs "
                                    f"({N} per GPU), seal then unseal, 1 key, AAD 4 B" if workload == "config4" else
                                    f"config2: {N} x {L} B packets per GPU, seal then unseal, 1 key, AAD 4 B"),
                       "packets_total": total_packets, "packets_per_gpu": N, "payload_len": L, "slot_stride": stride,
                       "payload_align": 64, "parallelism": f"shards x{world}, no collectives",
                       "clock_settle_steps": settle},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "frac_read": round(achieved_read / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "traffic_over_algorithmic": round(traffic / (N * per_pkt), 3) if traffic else None,
                         "bytes_per_packet": per_pkt, "kernel_ms": round(kms, 4),
                         "launches_per_call": launches, "packets_per_launch": min(chunk, N),
                         "launch_ms": round(kms / launches, 4),
                         "achieved_read_only": round(achieved_read, 1),
                         "read_bytes_per_packet": read_pkt,
                         "copy_achievable": round(copy_gbs, 1),
                         "copy_reference_guide": COPY_GUIDE_GBS,
                         # against the larger of this run's copy kernel and the guide's measured float4 copy
                         "frac_of_copy": round(achieved / max(copy_gbs, COPY_GUIDE_GBS), 4),
                         "binding_unit": "LDS (T-table AES + comb GHASH lookups, DESIGN.md 4.1)",
                         "lds_array_busy": lds_busy,
                         # the kernel's cycles per launch at the measured mean GFX clock: the box-independent
                         # figure (the kernel runs at the chip's power limit, so boxes differ by their clock)
                         "launch_mcycles_at_mean_sclk": (round(kms / launches * clock["sclk_mhz_mean"] / 1e3, 3)
                                                         if clock["sclk_mhz_mean"] else None)},
            "kernels_ms": {"seal": round(seal_ms, 4), "open": round(open_ms, 4)},
            "per_gpu": [{"rank": r, "packets": int(p[3]), "ms_per_step": round(p[0] * 1e3 / args.steps, 4),
                         "GiB_s": round(2 * p[3] * L / (p[0] / args.steps) / 2**30, 2),
                         "seal_ms": round(p[1], 4), "open_ms": round(p[2], 4),
                         "sealed_digest_ok": None if p[4] < 0 else bool(p[4]),
                         "opened_digest_ok": None if p[5] < 0 else bool(p[5]),
                         "sclk_mhz_mean": None if p[6] != p[6] else round(p[6], 1),
                         "power_w_mean": None if p[7] != p[7] else round(p[7], 1)} for r, p in enumerate(per_rank)],
            "dist_backend": args.dist_backend if dist is not None else None,
            "status_ok": ok,
            **digests,
            "sclk_mhz_mean": clock["sclk_mhz_mean"], "power_w_mean": clock["power_w_mean"],
            "power_cap_w": clock["power_cap_w"], "gpu_clock_power": clock,
        }
        # every rank's digests: the line's flags are the AND over ranks (a rank without a golden prefix: None)
        for k in ("sealed_digest_ok", "opened_digest_ok"):
            flags = [g[k] for g in line["per_gpu"]]
            line[k] = False if False in flags else (True if flags and all(flags) else None)
        if world > 1:
            line["digest_source"] = "tests/golden/rank_digest.json (each rank's own prefix)"
        rates = [g["GiB_s"] for g in line["per_gpu"]]
        line["per_gpu_GiB_s"] = {"min": min(rates), "max": max(rates), "mean": round(sum(rates) / len(rates), 2),
                                 "aggregate_of_own_times": round(sum(rates), 2),
                                 "note": "each rank's packets over its own step time; `value` uses the max over ranks"}
        print(f"[bench] headline {line['value']} GiB/s", file=sys.stderr, flush=True)
        if cpu is not None:
            line["cpu_baseline"] = cpu
        if world == 1 and not args.no_extra:
            # the other BASELINE configs, timed after the headline in this process (never `value`)
            del arena_alloc, arena, nonces, status
            torch.cuda.empty_cache()
            extra = {}
            # config4_one_gpu last: releasing its 94.5-GB arena halves concurrent H2D + D2H rates for a
            # few seconds (the driver clears released HBM), which would otherwise hit the PCIe legs
            for name, fn in (("config3", lambda: extra_config3(verify=not args.no_verify)),
                             ("config3_host", lambda: extra_config3_host(verify=not args.no_verify)),
                             ("e2e_pinned_host", lambda: extra_e2e(key)),
                             ("config5", lambda: extra_config5(key, args.cpu_threads or host["share"], verify=not args.no_verify)),
                             ("config5_resident", lambda: extra_config5_resident(key, verify=not args.no_verify)),
                             ("two_streams", lambda: extra_two_streams(key)),
                             ("per_packet", extra_per_packet),
                             ("worker_batches", lambda: extra_worker_batches(key)),
                             ("config4_one_gpu", lambda: extra_config4_one_gpu(key))):
                t0 = time.perf_counter()
                try:
                    extra[name] = fn()
                except Exception as e:  # reported, and the run fails below: a broken config is not hidden
                    extra[name] = {"error": f"{type(e).__name__}: {e}"}
                extra[name]["wall_s"] = round(time.perf_counter() - t0, 2)
                print(f"[bench] extra {name}: {extra[name].get('value', extra[name].get('error', ''))} "
                      f"({extra[name]['wall_s']} s)", file=sys.stderr, flush=True)  # progress for long runs
            if cpu is not None and "error" not in extra.get("per_packet", {"error": 1}):
                # the same work on the CPU chain (one packet sealed and opened = one round trip)
                extra["per_packet"]["cpu_chain"] = {
                    "round_trips_per_s_best": cpu["round_trips_per_s_best"], "threads": cpu["cores"],
                    "round_trips_per_s_one_thread": cpu["round_trips_per_s_one_thread"],
                    "cpus_busy": cpu["best_cpus_busy"], "cpu_us_per_pair": cpu["best_cpu_us_per_pair"]}
                pts = {k: v for k, v in extra["per_packet"].items() if isinstance(v, dict) and "cpu_us_per_pair" in v
                       and k != "cpu_chain"}
                if pts:
                    best = min(pts, key=lambda k: pts[k]["cpu_us_per_pair"])
                    extra["per_packet"]["least_host_cpu_per_pair"] = {
                        "point": best, "cpu_us_per_pair": pts[best]["cpu_us_per_pair"],
                        "cpu_chain_cpu_us_per_pair": cpu["best_cpu_us_per_pair"],
                        "below_cpu_chain": pts[best]["cpu_us_per_pair"] < cpu["best_cpu_us_per_pair"]}
            line["extra_configs"] = extra
        print(json.dumps(line), flush=True)
        if any("error" in v for v in line.get("extra_configs", {}).values()):
            sys.exit(1)
        if False in (line.get("sealed_digest_ok"), line.get("opened_digest_ok"), line["status_ok"]):
            sys.exit(1)  # the timed layout's bytes differ from the golden (or an open failed): not a result
    if dist is not None:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
