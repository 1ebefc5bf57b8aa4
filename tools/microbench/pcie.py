"""PCIe copy ceiling on the GPU box: pinned host <-> HBM hipMemcpyAsync rates, one direction at a time
and both directions at once (two streams), for the chunk sizes qgcm_seal_host pipelines with.
The e2e rows of DESIGN.md section 5 are read against these numbers.
Usage: python tools/microbench/pcie.py [--after-free GB]
"""
import json

import torch

TOTAL = 1 << 30  # 1 GiB per direction per measurement


def rate(chunk: int, h2d: bool, d2h: bool, reps: int = 3, stream_host: bool = False, total: int = TOTAL,
         mis: int = 0) -> dict:
    """stream_host: walk a `total`-byte pinned host buffer chunk by chunk (as qgcm_seal_host walks the
    arena) instead of re-copying one chunk-sized buffer.  mis: both ends of every copy start `mis`
    bytes past a 4 KiB boundary (a keyed batch's runs start wherever a record does)."""
    n = total // chunk
    hsz = total if stream_host else chunk
    hs = [torch.empty(hsz + 4096, dtype=torch.uint8, pin_memory=True)[mis:mis + hsz] for _ in range(2)]
    ds = [torch.empty(chunk + 4096, dtype=torch.uint8, device="cuda")[mis:mis + chunk] for _ in range(2)]
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        s_in.wait_event(e0)
        s_out.wait_event(e0)
        for i in range(n):
            o = i * chunk if stream_host else 0
            if h2d:
                with torch.cuda.stream(s_in):
                    ds[0].copy_(hs[0][o:o + chunk], non_blocking=True)
            if d2h:
                with torch.cuda.stream(s_out):
                    hs[1][o:o + chunk].copy_(ds[1], non_blocking=True)
        torch.cuda.current_stream().wait_stream(s_in)
        torch.cuda.current_stream().wait_stream(s_out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    gbs = n * chunk / (best * 1e-3) / 1e9
    return {"chunk_MiB": chunk >> 20, "h2d": h2d, "d2h": d2h, "host_walk_GiB": hsz >> 30, "misalign": mis,
            "GB_per_s_each_direction": round(gbs, 1)}


def after_free(gb: float) -> None:
    """Allocate `gb` GB of HBM through torch, touch it, free it (empty_cache), then rerun a few rows:
    does a huge allocation freed earlier in the process slow later PCIe copies (bench.py runs config 4's
    94.5-GB arena before the pinned-host legs)?"""
    x = torch.empty(int(gb * 1e9), dtype=torch.uint8, device="cuda")
    x.fill_(1)
    torch.cuda.synchronize()
    del x
    torch.cuda.empty_cache()
    import time
    t0 = time.perf_counter()
    for wait in (0, 5, 20, 60):  # does the slowdown wear off (a background clear of the freed HBM)?
        while time.perf_counter() - t0 < wait:
            time.sleep(0.1)
        print(json.dumps({"after_free_GB": gb, "s_after_free": round(time.perf_counter() - t0, 1),
                          **rate(64 << 20, True, True)}), flush=True)


def teardown() -> None:
    """Release every device and pinned-host block torch still caches BEFORE the interpreter exits.

    Under `rocprofv3 --memory-copy-trace` (profiles/r4_s9: SIGSEGV, rc 139, in __cxa_finalize after
    every row had printed) the pinned buffers of rate() -- returned to torch's caching host allocator,
    not freed -- were released by that allocator's static destructor at exit, i.e. a hipHostFree issued
    from __cxa_finalize after the profiler's tool library had already been finalized by its own exit
    handler: the intercepted HIP call jumps into torn-down tracing state.  Freeing the caches here, while
    the runtime and the profiler are both alive, leaves no HIP call for exit time (tools/README.md)."""
    import gc

    torch.cuda.synchronize()
    gc.collect()  # the rate() buffers and streams
    torch.cuda.empty_cache()
    host_empty = getattr(torch._C, "_host_emptyCache", None)
    if host_empty is not None:
        host_empty()  # the caching host (pinned) allocator's free blocks -> hipHostFree now
    torch.cuda.synchronize()


def dump_maps_at_exit(path: str) -> None:
    """Write /proc/self/maps when the interpreter exits (before the C-level finalizers run), so the
    addresses of an exit-time crash report can be resolved to library + offset (tools/resolve_crash.py)."""
    import atexit

    def dump():
        with open(path, "w") as f:
            f.write(open("/proc/self/maps").read())

    atexit.register(dump)


if __name__ == "__main__":
    import os
    import sys
    if os.environ.get("PCIE_MAPS"):
        dump_maps_at_exit(os.environ["PCIE_MAPS"])
    if len(sys.argv) > 1 and sys.argv[1] == "--quick":  # three rows: the exit-time crash reproduction
        for h2d, d2h in ((True, False), (False, True), (True, True)):
            print(json.dumps(rate(64 << 20, h2d, d2h)), flush=True)
        if "--no-teardown" not in sys.argv:
            teardown()
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[1] == "--after-free":
        for h2d, d2h in ((True, False), (False, True), (True, True)):
            print(json.dumps({"after_free_GB": 0, **rate(64 << 20, h2d, d2h)}), flush=True)
        after_free(float(sys.argv[2]))
        teardown()
        sys.exit(0)
    for chunk in (8 << 20, 32 << 20, 128 << 20):
        for h2d, d2h in ((True, False), (False, True), (True, True)):
            print(json.dumps(rate(chunk, h2d, d2h)), flush=True)
    for chunk in (32 << 20, 64 << 20):
        print(json.dumps(rate(chunk, True, True, stream_host=True)), flush=True)
    # a 5 GiB walk (config 3's arena is 4.8 GB): does the rate depend on how much pinned memory a
    # copy stream touches (IOMMU translation reach)?
    for chunk in (64 << 20,):
        print(json.dumps(rate(chunk, True, True, stream_host=True, total=5 << 30)), flush=True)
        print(json.dumps(rate(chunk, True, False, stream_host=True, total=5 << 30)), flush=True)
    # copies whose ends are only 4-B aligned (where a keyed batch's DMA runs start), one way and both
    for mis in (4, 64, 256):
        for h2d, d2h in ((True, False), (False, True), (True, True)):
            print(json.dumps(rate(64 << 20, h2d, d2h, mis=mis)), flush=True)
    teardown()
