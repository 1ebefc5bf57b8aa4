"""Co-residency experiment: the LDS-bound T-table GCM kernel (libqgcm, one 16-wave workgroup per
CU, 64 VGPRs) and the VALU-bound bitsliced AES-CTR microkernel (libbs.so, one wave per SIMD) on two
streams at once.  If the two use different pipes, the pair finishes in ~max(t1, t2), not t1 + t2.

Run on the GPU box from the repo root:  python tools/microbench/bs/corun.py
"""
import ctypes as C
import os
import sys

os.environ.setdefault("QGCM_VARIANT", "5")
os.environ.setdefault("QGCM_WGS_PER_CU", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from quantum_amd import batch  # noqa: E402
from quantum_amd.crypto import Context  # noqa: E402


def main():
    bs = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libbs.so"))
    bs.bs_launch.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    ctx = Context(device=0, max_keys=4)
    ctx.set_key(0, bytes(range(32)))
    n, L = 1 << 20, 1350
    stride = 1408
    arena = torch.zeros(n * stride + 64, dtype=torch.uint8, device="cuda")[60:60 + n * stride]
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(arena, stride, n, L, 0x0100630a, 1, nonces, 2)
    bs_groups = int(os.environ.get("BS_GROUPS", "43520"))
    bs_grid = int(os.environ.get("BS_GRID", str(torch.cuda.get_device_properties(0).multi_processor_count)))
    bsdata = torch.zeros(bs_groups * 2048 * 16, dtype=torch.uint8, device="cuda")
    rkm = torch.zeros(15 * 128, dtype=torch.int32, device="cuda")
    rkw = torch.zeros(60, dtype=torch.int32, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def table(stream):
        batch.seal_uniform(ctx, arena, stride, n, L, 0, nonces, stream=stream)

    def bsk(stream):
        r = bs.bs_launch(bsdata.data_ptr(), bs_groups, rkm.data_ptr(), rkw.data_ptr(), bs_grid, 1,
                         C.c_void_p(stream.cuda_stream))
        assert r == 0

    def timed(fn, reps=10):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    def both():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        table(s1)
        bsk(s2)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    cur = torch.cuda.current_stream()
    for _ in range(2):
        table(cur)
        bsk(cur)
    t1 = timed(lambda: table(torch.cuda.current_stream()))
    t2 = timed(lambda: bsk(torch.cuda.current_stream()))
    t12 = timed(both)
    blk_t = n * ((L + 15) // 16)
    blk_b = bs_groups * 2048
    print(f"table alone  {t1:.3f} ms ({blk_t / t1 / 1e6:.1f} G blocks/s)")
    print(f"bitsliced    {t2:.3f} ms ({blk_b / t2 / 1e6:.1f} G blocks/s)")
    print(f"together     {t12:.3f} ms (sum {t1 + t2:.3f}, max {max(t1, t2):.3f}); "
          f"combined {(blk_t + blk_b) / t12 / 1e6:.1f} G blocks/s")


if __name__ == "__main__":
    main()
