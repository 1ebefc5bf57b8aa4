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
