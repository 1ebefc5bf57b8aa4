"""Host code under sanitizers (SURVEY.md §5 "use TSan/ASan on host lib tests"): the snappy codec and
the key math of libqgcm (host-only C++, no HIP) built with g++ -fsanitize=address,undefined and with
-fsanitize=thread, driven by tests/cpp/san_driver.cpp (round trips, malformed streams into
exact-size buffers, the threaded slot codec).  Any report fails the test."""
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
