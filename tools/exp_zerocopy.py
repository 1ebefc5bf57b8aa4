"""Experiment: seal/open kernels run directly on a pinned HOST arena (zero-copy: the packet kernels
read and write the slots over PCIe; no hipMemcpy, no staging) vs the pipelined qgcm_seal_host path.
Checks the sealed bytes against the device-resident path.  Usage: python tools/exp_zerocopy.py
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from quantum_amd import _lib, batch  # noqa: E402
from quantum_amd.crypto import Context, derive_key  # noqa: E402

N, L = 1 << 20, 1350
stride = batch.slot_stride(L, align=64)
ctx = Context(device=0, max_keys=4)
ctx.set_key(0, derive_key(b"AES256Key-32Characters1234567890", bytes(range(32))))
lib = _lib.lib()
dev = torch.zeros(N * stride, dtype=torch.uint8, device="cuda")
non_d = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
batch.fill_uniform(dev, stride, N, L, 0x0100630a, 0x5EED0001, non_d, 0x5EED0002)
a_ptr, n_ptr, s_ptr = lib.qgcm_host_alloc(N * stride), lib.qgcm_host_alloc(12 * N), lib.qgcm_host_alloc(N)
host = np.frombuffer((C.c_uint8 * (N * stride)).from_address(a_ptr), np.uint8)
nonces = np.frombuffer((C.c_uint8 * (12 * N)).from_address(n_ptr), np.uint8)
stat = np.frombuffer((C.c_uint8 * N).from_address(s_ptr), np.uint8)
host[:] = dev.cpu().numpy()
nonces[:] = non_d.cpu().numpy()
plain = host.copy()
ref = dev.clone()
batch.seal_uniform(ctx, ref, stride, N, L, 0, non_d)
ref = ref.cpu().numpy()
stream = torch.cuda.current_stream().cuda_stream

res = {}
for it in range(4):
    host[:] = plain
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rc = lib.qgcm_seal_uniform(ctx.handle, a_ptr, stride, N, L, 0, n_ptr, 4, s_ptr, stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    same = bool(np.array_equal(host, ref)) and rc == 0 and int(stat.sum()) == N
    rc2 = lib.qgcm_open_uniform(ctx.handle, a_ptr, stride, N, L + 28, 0, 4, s_ptr, stream)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    back = bool(np.array_equal(host.reshape(N, stride)[:, :4 + L], plain.reshape(N, stride)[:, :4 + L]))
    res = {"exp": "zero-copy kernels on pinned host arena", "seal_s": round(t1 - t0, 4), "open_s": round(t2 - t1, 4),
           "value_GiBps": round(2 * N * L / (t2 - t0) / 2**30, 2),
           "GBps_each_way": round(N * stride / ((t2 - t0) / 2) / 1e9, 2),
           "sealed_equals_device_path": same, "open_ok": back and rc2 == 0 and int(stat.sum()) == N}
    print(json.dumps(res), flush=True)
