import sys, os, time, json
sys.path.insert(0, os.getcwd())
import torch
from quantum_amd import batch
from quantum_amd.crypto import Context, derive_key
N, L = 1 << 20, 1350
stride = batch.slot_stride(L, align=64)
ctx = Context(device=0, max_keys=4)
ctx.set_key(0, derive_key(b"AES256Key-32Characters1234567890", bytes(range(32))))
a = torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda")[60:]
non = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
batch.fill_uniform(a, stride, N, L, 0x0100630a, 1, non, 2)
s = torch.cuda.current_stream()
mode = sys.argv[1] if len(sys.argv) > 1 else "cont"
evs = []
for k in range(400):
    if mode == "sync20" and k % 20 == 0:
        torch.cuda.synchronize()
    if mode == "sleep20" and k % 20 == 0:
        torch.cuda.synchronize()
        time.sleep(0.05)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record(s)
    batch.seal_uniform(ctx, a, stride, N, L, 0, non, stream=s)
    e[1].record(s)
    batch.open_uniform(ctx, a, stride, N, L + 28, 0, stream=s)
    evs.append(e)
torch.cuda.synchronize()
ms = [e[0].elapsed_time(e[1]) for e in evs]
print(mode, [round(sum(ms[i:i+20]) / 20, 3) for i in range(0, 400, 20)])
print(mode, "first 5 after each sync:", [round(sum(ms[i:i+5]) / 5, 3) for i in range(0, 400, 20)][:8])
