"""Config 3 with the slots packed at 4-B alignment (the workload's layout, quantum_amd/workloads.py)
against the same packets with every payload 64-B aligned: the most that realigning the descriptor
kernel's stores could gain (a quad's 64-B store at a 4-B misalignment spans
three 32-B sectors, so config 3 writes 1.65x its algorithmic bytes against config 2's 1.13x).
Same process, same keys, lengths and key mix, interleaved seal+open pairs timed with HIP events.
Usage: python3 tools/exp_config3_align.py [reps=7] [only=both|packed|aligned]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantum_amd import batch, workloads as W  # noqa: E402
from quantum_amd.crypto import Context  # noqa: E402


def aligned_layout(lens):
    """Payload (slot + 4) at a 64-B boundary, slots rounded to 64 B."""
    slot = (4 + lens.astype(np.uint64) + 28 + 63) & ~np.uint64(63)
    offs = np.zeros(len(lens), dtype=np.uint64)
    offs[1:] = np.cumsum(slot)[:-1]
    offs += 60
    used = int(offs[-1] + slot[-1])
    return offs, (used + 64 + W.CHUNK - 1) // W.CHUNK * W.CHUNK


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    only = sys.argv[2] if len(sys.argv) > 2 else "both"
    keys = W.peer_keys()
    ctx = Context(device=0, max_keys=W.NKEYS)
    ctx.set_keys(0, keys)
    lens, kidx = W.lengths(), W.key_indices()
    nonces = torch.from_numpy(W.nonces()).cuda()
    status = torch.zeros(W.N, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    forms = {}
    for name, (offs, size) in (("packed", W.layout(lens)), ("aligned", aligned_layout(lens))):
        if only not in ("both", name):
            continue
        arena = W.device_arena(torch, size, offs, kidx)
        forms[name] = (arena, batch.make_descs(offs, lens, kidx, "cuda"),
                       batch.make_descs(offs, lens.astype(np.int64) + 28, kidx, "cuda"), size)
    times = {k: ([], []) for k in forms}
    ok = True
    for r in range(reps + 1):
        for name, (arena, ds, do, _) in forms.items():
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(stream)
            batch.seal_batch(ctx, arena, ds, W.N, nonces, status=status, stream=stream)
            e[1].record(stream)
            batch.open_batch(ctx, arena, do, W.N, status=status, stream=stream)
            e[2].record(stream)
            torch.cuda.synchronize()
            ok &= int(status.sum()) == W.N
            if r:  # the first pair is warmup
                times[name][0].append(e[0].elapsed_time(e[1]))
                times[name][1].append(e[1].elapsed_time(e[2]))
    payload = int(lens.sum())
    out = {"exp": "config3 layout", "reps": reps, "status_ok": ok}
    for name, (ts, to) in times.items():
        s, o = float(np.median(ts)), float(np.median(to))
        out[name] = {"seal_ms": round(s, 3), "open_ms": round(o, 3),
                     "GiB_s": round(2 * payload / ((s + o) * 1e-3) / 2**30, 1), "arena_bytes": forms[name][3]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
