"""Host code under sanitizers (SURVEY.md §5 "use TSan/ASan on host lib tests"): the snappy codec and
the key math of libqgcm (host-only C++, no HIP) built with g++ -fsanitize=address,undefined and with
-fsanitize=thread, driven by tests/cpp/san_driver.cpp (round trips, malformed streams into
exact-size buffers, the threaded slot codec); the batched TUN and UDP I/O under ASan/UBSan
(tests/cpp/tun_san_driver.cpp, udp_san_driver.cpp).  Any report fails the test."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "quantum_amd", "csrc")
SRCS = [os.path.join(ROOT, "tests", "cpp", "san_driver.cpp"), os.path.join(CSRC, "snappy_codec.cpp"),
        os.path.join(CSRC, "keymath.cpp")]


def build_and_run(tmp_path, flags, args, env_extra):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = tmp_path / "san_driver"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, f"-I{ROOT}/include", *SRCS,
           "-lpthread", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, **env_extra)
    r = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "sanitizer driver ok" in r.stdout, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr


def test_asan_ubsan(tmp_path):
    build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], [],
                  {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0"})


def test_tsan_threaded_slot_codec(tmp_path):
    build_and_run(tmp_path, ["-fsanitize=thread"], ["threads"], {"TSAN_OPTIONS": "halt_on_error=1"})


@pytest.mark.parametrize("mode", ["", "1", "-1"], ids=["preadv2", "io_uring", "poll_read"])
def test_asan_ubsan_tun_reads(tmp_path, mode):
    """quantum_amd/csrc/tun_batch.cpp under ASan/UBSan (tests/cpp/tun_san_driver.cpp): each TUN read form
    (QGCM_TUN_URING unset / 1 / -1) drains 160 routed datagrams in 8-slot batches, every one read once and
    intact, and a written packet reaches a socket.  Skipped where the kernel refuses a TUN device."""
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = tmp_path / "tun_san_driver"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", f"-I{ROOT}/include", os.path.join(ROOT, "tests", "cpp", "tun_san_driver.cpp"),
           os.path.join(CSRC, "tun_batch.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = {k: v for k, v in os.environ.items() if k != "QGCM_TUN_URING"}
    if mode:
        env["QGCM_TUN_URING"] = mode
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0"
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    if r.returncode == 77:
        pytest.skip("TUN device refused")
    assert r.returncode == 0 and "tun driver ok" in r.stdout, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr


def test_asan_ubsan_udp_batches(tmp_path):
    """quantum_amd/csrc/udp_batch.cpp under ASan/UBSan (tests/cpp/udp_san_driver.cpp): 2000 loopback
    datagrams of 1..1472 B through sendmmsg / recvmmsg slot batches, back in order and intact."""
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = tmp_path / "udp_san_driver"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", f"-I{ROOT}/include", os.path.join(ROOT, "tests", "cpp", "udp_san_driver.cpp"),
           os.path.join(CSRC, "udp_batch.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0"))
    assert r.returncode == 0 and "udp driver ok" in r.stdout, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr
