"""Smallest reproductions of the exit-time SIGSEGV under `rocprofv3 --memory-copy-trace`
(profiles/r5_s2: a pure-torch script, no libqgcm; resolved frames: librocprofiler-sdk-tool's
__cxa_finalize -> librocprofiler-sdk -> libhsa-runtime64).  Modes:

  copy        one pinned host -> HBM copy and back, then a normal exit
  kernel      a device-only op (no copy), then a normal exit
  copy_reset  as copy, then hipDeviceReset() before the exit (every stream, allocation and HSA queue
              the runtime holds released while the profiler is still alive)
  many        pcie.py's traffic: 64-MiB pinned copies on two side streams, 1 GiB each way x 3
  many_reset  as many, then hipDeviceReset() before the exit

  many_default  as many, all copies on the current (default) stream, no side streams
  ext_streams   as many, on two streams made with hipStreamCreate (torch.cuda.ExternalStream) and
                destroyed with hipStreamDestroy before the exit
  streams_only  two torch.cuda.Stream() side streams, one small copy on each

profiles/r5_s3: copy, kernel and copy_reset exit cleanly under --memory-copy-trace; profiles/r5_s4:
many_reset crashes (hipDeviceReset does not avoid it).

Usage: python3 tools/microbench/crash_min.py <mode>   (run under rocprofv3 ... -- python3 ...)"""
import ctypes
import sys

import torch

mode = sys.argv[1]
hip = ctypes.CDLL("libamdhip64.so")
if mode in ("many_default", "ext_streams", "streams_only"):
    chunk, n = 64 << 20, 16
    hs = [torch.empty(chunk, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    ds = [torch.empty(chunk, dtype=torch.uint8, device="cuda") for _ in range(2)]
    raw = []
    if mode == "ext_streams":
        for _ in range(2):
            h = ctypes.c_void_p()
            assert hip.hipStreamCreateWithFlags(ctypes.byref(h), 1) == 0  # hipStreamNonBlocking
            raw.append(h)
        streams = [torch.cuda.ExternalStream(h.value) for h in raw]
    elif mode == "streams_only":
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        n = 1
    else:
        streams = [torch.cuda.current_stream()] * 2
    for rep in range(3 if mode != "streams_only" else 1):
        for i in range(n):
            with torch.cuda.stream(streams[0]):
                ds[0].copy_(hs[0], non_blocking=True)
            with torch.cuda.stream(streams[1]):
                hs[1].copy_(ds[1], non_blocking=True)
        torch.cuda.synchronize()
    print({"mode": mode, "copies": 2 * n * (3 if mode != "streams_only" else 1)}, flush=True)
    if raw:
        del streams
        torch.cuda.synchronize()
        print({"hipStreamDestroy": [hip.hipStreamDestroy(h) for h in raw]}, flush=True)
    sys.exit(0)
if mode in ("many", "many_reset"):
    chunk, n = 64 << 20, 16
    hs = [torch.empty(chunk, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    ds = [torch.empty(chunk, dtype=torch.uint8, device="cuda") for _ in range(2)]
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
    for rep in range(3):
        e0 = torch.cuda.Event()
        e0.record()
        s_in.wait_event(e0)
        s_out.wait_event(e0)
        for i in range(n):
            with torch.cuda.stream(s_in):
                ds[0].copy_(hs[0], non_blocking=True)
            with torch.cuda.stream(s_out):
                hs[1].copy_(ds[1], non_blocking=True)
        torch.cuda.current_stream().wait_stream(s_in)
        torch.cuda.current_stream().wait_stream(s_out)
        torch.cuda.synchronize()
    print({"mode": mode, "copies": 2 * 3 * n}, flush=True)
    if mode == "many_reset":
        del hs, ds, s_in, s_out
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        torch._C._host_emptyCache()
        print({"hipDeviceReset": hip.hipDeviceReset()}, flush=True)
    sys.exit(0)
if mode in ("copy", "copy_reset"):
    h = torch.ones(1 << 20, dtype=torch.uint8, pin_memory=True)
    d = h.to("cuda", non_blocking=True)
    h2 = d.to("cpu", non_blocking=True).pin_memory()
    torch.cuda.synchronize()
    print({"mode": mode, "ok": bool((h2 == 1).all())}, flush=True)
else:
    x = torch.ones(1 << 20, dtype=torch.uint8, device="cuda") * 2
    torch.cuda.synchronize()
    print({"mode": mode, "ok": True}, flush=True)
if mode == "copy_reset":
    del h, d, h2
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    torch._C._host_emptyCache()
    print({"hipDeviceReset": hip.hipDeviceReset()}, flush=True)
