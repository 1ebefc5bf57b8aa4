"""Runs seal+open of config 2 with one kernel variant (for rocprofv3 PMC passes)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from quantum_amd import batch
from quantum_amd.crypto import Context, derive_key
N, L = 1 << 20, 1350
stride = int(os.environ.get("STRIDE", "1408")); off = int(os.environ.get("OFF", "60"))
key = derive_key(b"AES256Key-32Characters1234567890", bytes(range(32)))
c = Context(0, 4); c.set_key(0, key)
arena = torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda"); base = arena[off:]
nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
batch.fill_uniform(base, stride, N, L, 0x0100630a, 0x5EED0001, nonces, 0x5EED0002)
for _ in range(int(os.environ.get("REPS", "3"))):
    batch.seal_uniform(c, base, stride, N, L, 0, nonces)
    batch.open_uniform(c, base, stride, N, L + 28, 0)
torch.cuda.synchronize()
