"""Stage timing of the resident per-packet kernel (side build with -DQGCM_RES_TRACE): one thread makes
N sequential seal_one/open_one calls; the trace gives, per request, the device clock (100 MHz) at the
dispatcher's bell read, its forward end, the worker's wake-up, packet start / end and the verdict.
Usage: python tools/res_trace.py <lib.so> [n=2000] [payload=1350]"""
import ctypes as C
import statistics
import sys
import time

lib = C.CDLL(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
L = int(sys.argv[3]) if len(sys.argv) > 3 else 1350
vp = C.c_void_p
lib.qgcm_create.restype = vp
lib.qgcm_create.argtypes = [C.c_int, C.c_uint32, C.c_char_p, C.c_int]
lib.qgcm_set_key.argtypes = [vp, C.c_uint32, C.c_char_p]
lib.qgcm_seal_one.argtypes = [vp, C.c_uint32, vp, C.c_long, vp, C.c_uint32, vp]
lib.qgcm_seal_one.restype = C.c_long
lib.qgcm_open_one.argtypes = [vp, C.c_uint32, vp, C.c_long, vp, C.c_uint32]
lib.qgcm_open_one.restype = C.c_long
err = C.create_string_buffer(120)
ctx = lib.qgcm_create(0, 4, err, 120)
assert ctx, err.value
assert lib.qgcm_set_key(ctx, 0, bytes(range(32))) == 0
buf = (C.c_uint8 * (L + 28))()
aad = (C.c_uint8 * 4)(10, 99, 0, 1)
for _ in range(200):
    lib.qgcm_seal_one(ctx, 0, buf, L, aad, 4, None)
    lib.qgcm_open_one(ctx, 0, buf, L + 28, aad, 4)
host = []
for _ in range(n):
    t0 = time.perf_counter()
    assert lib.qgcm_seal_one(ctx, 0, buf, L, aad, 4, None) == L + 28
    t1 = time.perf_counter()
    assert lib.qgcm_open_one(ctx, 0, buf, L + 28, aad, 4) == L
    host += [t1 - t0, time.perf_counter() - t1]
out = (C.c_ulonglong * (8 * 65536))()
m = lib.qgcm_debug_res_trace(out, 65536)
rows = [out[8 * i:8 * i + 8] for i in range(m)][-2 * n:]
def med(f):
    return statistics.median(f(r) for r in rows) / 100.0  # ticks -> us
print(f"{m} traced requests; host call median {statistics.median(host) * 1e6:.1f} us")
print(f"dispatcher forward (bell read -> bells rung)  {med(lambda r: r[1] - r[0]):6.2f} us")
print(f"forward end -> worker awake                   {med(lambda r: r[2] - r[1]):6.2f} us")
print(f"worker awake -> packet start (scan, meta)     {med(lambda r: r[3] - r[2]):6.2f} us")
print(f"packet (stage, compute, write back, drain)    {med(lambda r: r[4] - r[3]):6.2f} us")
print(f"verdict store + trace                         {med(lambda r: r[5] - r[4]):6.2f} us")
print(f"bell read -> verdict                          {med(lambda r: r[5] - r[0]):6.2f} us")
gaps = sorted(rows[i + 1][0] - rows[i][5] for i in range(len(rows) - 1))
print(f"verdict -> next request's bell read (host side + dispatcher poll) median {gaps[len(gaps) // 2] / 100:.2f} us")
