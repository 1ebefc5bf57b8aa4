import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from quantum_amd import batch
from quantum_amd.crypto import Context, derive_key
N, L = 1 << 20, 1350
key = derive_key(b"AES256Key-32Characters1234567890", bytes(range(32)))
for stride, off in ((1392, 0), (1408, 60), (1472, 0)):
    arena = torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda")
    base = arena[off:]
    nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(base, stride, N, L, 0x0100630a, 0x5EED0001, nonces, 0x5EED0002)
    for v in (2, 0):
        os.environ["QGCM_VARIANT"] = str(v)
        c = Context(0, 4); c.set_key(0, key)
        for exp in ("0", "1"):
            os.environ["QGCM_EXP"] = exp
            ts = []
            for r in range(6):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(); batch.seal_uniform(c, base, stride, N, L, 0, nonces); e1.record(); torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            os.environ["QGCM_EXP"] = "0"
            print(f"stride {stride} off {off} variant {v} skip_stores={exp}: seal {statistics.median(ts[1:]):.3f} ms", flush=True)
        c.close()
