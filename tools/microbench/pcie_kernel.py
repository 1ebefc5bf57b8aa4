"""PCIe copies done by a shader (libqgcm's 16-B/lane stream-copy kernel reading or writing pinned
host memory) vs hipMemcpyAsync, one direction and both at once, for 64 MiB chunks over a 1 GiB
pinned host buffer.  Usage: python tools/microbench/pcie_kernel.py
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from quantum_amd import _lib  # noqa: E402
from quantum_amd.crypto import Context  # noqa: E402

TOTAL, CHUNK = 1 << 30, 64 << 20
ctx = Context(device=0, max_keys=1)
lib = _lib.lib()
h_in, h_out = lib.qgcm_host_alloc(TOTAL), lib.qgcm_host_alloc(TOTAL)
d_in = torch.empty(TOTAL, dtype=torch.uint8, device="cuda")
d_out = torch.empty(TOTAL, dtype=torch.uint8, device="cuda")
s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
hip = C.CDLL("libamdhip64.so.7")
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]


def run(h2d: str, d2h: str) -> dict:
    best = None
    for _ in range(3):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        s_in.wait_event(e0)
        s_out.wait_event(e0)
        for o in range(0, TOTAL, CHUNK):
            if h2d == "kernel":
                lib.qgcm_stream_copy(ctx.handle, d_in.data_ptr() + o, h_in + o, CHUNK, s_in.cuda_stream)
            elif h2d == "memcpy":
                hip.hipMemcpyAsync(d_in.data_ptr() + o, h_in + o, CHUNK, 1, s_in.cuda_stream)
            if d2h == "kernel":
                lib.qgcm_stream_copy(ctx.handle, h_out + o, d_out.data_ptr() + o, CHUNK, s_out.cuda_stream)
            elif d2h == "memcpy":
                hip.hipMemcpyAsync(h_out + o, d_out.data_ptr() + o, CHUNK, 2, s_out.cuda_stream)
        torch.cuda.current_stream().wait_stream(s_in)
        torch.cuda.current_stream().wait_stream(s_out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    return {"h2d": h2d, "d2h": d2h, "GB_per_s_each_direction": round(TOTAL / (best * 1e-3) / 1e9, 1)}


if __name__ == "__main__":
    for h2d, d2h in (("memcpy", None), ("kernel", None), (None, "memcpy"), (None, "kernel"),
                     ("memcpy", "memcpy"), ("kernel", "memcpy"), ("memcpy", "kernel"), ("kernel", "kernel")):
        print(json.dumps(run(h2d, d2h)), flush=True)
