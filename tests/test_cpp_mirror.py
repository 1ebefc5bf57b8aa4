"""The C++ host mirror of the reference's Go API (include/quantum.hpp, quantum_amd/csrc/quantum_host.cpp)
through tests/cpp/mirror_test.cpp, a C++ restatement of crypto/crypto_test.go and
plugin/plugin_test.go (built by __graft_entry__.build()).  The device-free tests run on CPU; the
ones that seal/open run on the GPU, all in ONE child process."""
import os
import subprocess

import pytest

from conftest import ROOT

BIN = os.path.join(ROOT, "tests", "cpp", "mirror_test")
CPU_TESTS = ["TestEcdh", "TestSorter", "TestCompression", "TestMock", "TestPayload"]
GPU_TESTS = ["TestAES", "TestEncryption", "TestMulti", "TestEncryptionTamper", "TestMappingAES",
             "TestNewAESSlotsRecycled", "TestMappingAESDeviceSet"]


def run(names, timeout=120, env=None):
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} is missing: build it with __graft_entry__.build()")
    r = subprocess.run([BIN, *names], capture_output=True, text=True, timeout=timeout,
                       env=None if env is None else {**os.environ, **env})
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    for n in names:
        assert f"--- PASS: {n}" in out, out


@pytest.mark.parametrize("name", CPU_TESTS)
def test_cpp_mirror_cpu(name):
    run([name])


def test_cpp_mirror_no_device_set():
    """crypto::NewAES(secret, salt) with an unusable QGCM_DEVICES returns the error (no GPU is touched)."""
    run(["TestNewAESNoDevices"], env={"QGCM_DEVICES": "x"})


@pytest.mark.gpu
def test_cpp_mirror_gpu():
    run(GPU_TESTS)


GO_BIN = os.path.join(ROOT, "tests", "cpp", "go_replay")


def run_go(names, timeout=120):
    """tests/cpp/go_replay.c: the C calls go/crypto/aes_gpu.go makes under crypto_test.go's TestAES and
    go/crypto/aes_gpu_test.go."""
    if not os.path.exists(GO_BIN):
        pytest.fail(f"{GO_BIN} is missing: build it with __graft_entry__.build()")
    r = subprocess.run([GO_BIN, *names], capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    for n in names:
        assert f"--- PASS: {n}" in out, out


def test_go_shim_replay_cpu():
    run_go(["TestCreateError"])


@pytest.mark.gpu
def test_go_shim_replay_gpu():
    run_go(["TestAES", "TestAESEdges", "TestAESConcurrentGoroutines", "TestNewAESAcrossMembers", "TestSlotsRecycled",
            "TestGPUGroupBatch"])
