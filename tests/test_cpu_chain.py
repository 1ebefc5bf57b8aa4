"""BASELINE config 1 harness (oracle/cpu_chain.cpp, bench.py's cpu_baseline): the reference's plugin
chain -- Encryption + Mock over common.Payload, sorted as main.go:50-51, outgoing then incoming
(plugin/plugin_test.go:163-216, worker/outgoing.go:55-80, worker/incoming.go:54-79) -- over the C++
mirror of the Go plugins with OpenSSL's AES-GCM, on the CPU: every payload comes back intact."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_build", "cpu_chain")


def test_cpu_chain_roundtrip_and_rate():
    for threads, L in ((1, 1350), (2, 0), (2, 1433)):
        out = subprocess.run([EXE, str(threads), "500", str(L), "0.2"], capture_output=True, text=True, timeout=60)
        assert out.returncode == 0, out.stderr
        r = json.loads(out.stdout.strip().splitlines()[-1])
        assert r["intact"] is True and r["packets_per_s"] > 0 and r["threads"] == threads


def test_cpu_chain_rejects_oversize():
    out = subprocess.run([EXE, "1", "10", "1441", "0.1"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 2  # 4 + L + 28 must fit common.MaxPacketLength (1472)


def test_cpu_chain_buffered_nonces_and_cpu_accounting():
    """nonces "buffered" (341 per getrandom) vs the reference's one syscall per Encrypt: both intact,
    and the line reports the CPU seconds of the timed part (set-up excluded)."""
    for mode in ("syscall", "buffered"):
        out = subprocess.run([EXE, "2", "300", "1350", "0.2", mode], capture_output=True, text=True, timeout=60)
        assert out.returncode == 0, out.stderr
        r = json.loads(out.stdout.strip().splitlines()[-1])
        assert r["intact"] is True and r["nonces"] == mode
        assert r["user_s"] >= 0 and r["sys_s"] >= 0 and 0 < r["cpus_busy"] <= 2.5


def test_bench_cpu_baseline_sweep():
    """bench.py's cpu_baseline on a 2-thread share: the sweep covers 1 and 2 threads in both nonce modes,
    value is the best faithful point, and the per-thread efficiency follows from the sweep."""
    import sys

    sys.path.insert(0, ROOT)
    import bench

    host = bench.host_cpus()
    key = bytes(range(32))
    cb = bench.cpu_baseline(key, 1350, 2, host, seconds=0.2)
    assert [(p["threads"], p["nonces"], p["pinned"]) for p in cb["sweep"]] == [
        (t, m, pin) for t in (1, 2) for m, pin in (("syscall", False), ("syscall", True), ("buffered", True))]
    faithful = [p for p in cb["sweep"] if p["nonces"] == "syscall"]
    best = max(faithful, key=lambda p: p["GiB_s"])
    one = max(p["packets_per_s"] for p in faithful if p["threads"] == 1)
    assert cb["value"] == best["GiB_s"] and cb["cores"] == best["threads"] and cb["kind"] == "port"
    assert abs(cb["per_thread_efficiency"] - best["packets_per_s"] / (best["threads"] * one)) < 2e-3
    assert cb["intact"] is True and cb["measured_before_gpu_init"] is True
