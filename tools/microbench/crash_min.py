"""Smallest reproductions of the exit-time SIGSEGV under `rocprofv3 --memory-copy-trace`
(profiles/r5_s2: a pure-torch script, no libqgcm; resolved frames: librocprofiler-sdk-tool's
__cxa_finalize -> librocprofiler-sdk -> libhsa-runtime64).  Modes:

  copy        one pinned host -> HBM copy and back, then a normal exit
  kernel      a device-only op (no copy), then a normal exit
  copy_reset  as copy, then hipDeviceReset() before the exit (every stream, allocation and HSA queue
              the runtime holds released while the profiler is still alive)

Usage: python3 tools/microbench/crash_min.py <mode>   (run under rocprofv3 ... -- python3 ...)"""
import ctypes
import sys

import torch

mode = sys.argv[1]
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
    hip = ctypes.CDLL("libamdhip64.so")
    print({"hipDeviceReset": hip.hipDeviceReset()}, flush=True)
