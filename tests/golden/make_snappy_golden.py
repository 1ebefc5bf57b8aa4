"""Writes tests/golden/snappy.json: for each tests/snappy_inputs.py case, the snappy block encoding
produced by Google's libsnappy 1.1.8 (/opt/conda/lib/libsnappy.so.1, present in this image and on the
GPU boxes) -- the same block algorithm as golang/snappy's Encode (oracle/snappy_oracle.py says why),
which plugin/compression.go:16-19 calls.  Outputs up to 256 B are stored as hex, longer ones as
length + SHA-256.

    python3 tests/golden/make_snappy_golden.py
"""
import ctypes as C
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import snappy_inputs as SI  # noqa: E402


def libsnappy_compress(lib, data: bytes) -> bytes:
    cap = lib.snappy_max_compressed_length(len(data))
    buf = C.create_string_buffer(cap)
    m = C.c_size_t(cap)
    assert lib.snappy_compress(data, len(data), buf, C.byref(m)) == 0
    return buf.raw[:m.value]


def main() -> None:
    lib = C.CDLL("/opt/conda/lib/libsnappy.so.1")
    lib.snappy_compress.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.POINTER(C.c_size_t)]
    lib.snappy_max_compressed_length.argtypes = [C.c_size_t]
    lib.snappy_max_compressed_length.restype = C.c_size_t
    out = {"source": "libsnappy 1.1.8 snappy_compress (Google C++ snappy; same block algorithm as golang/snappy)",
           "cases": []}
    for kind, n in SI.cases():
        data = SI.make(kind, n)
        comp = libsnappy_compress(lib, data)
        e = {"kind": kind, "n": n, "in_sha256": hashlib.sha256(data).hexdigest(), "out_len": len(comp)}
        if len(comp) <= 256:
            e["out_hex"] = comp.hex()
        else:
            e["out_sha256"] = hashlib.sha256(comp).hexdigest()
        out["cases"].append(e)
    with open(os.path.join(HERE, "snappy.json"), "w") as f:
        json.dump(out, f, indent=0)
        f.write("\n")
    print(len(out["cases"]), "cases")


if __name__ == "__main__":
    main()
