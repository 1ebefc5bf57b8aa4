"""Where the device snappy encoder's time goes, by data shape: 2^20 slots of 1472 B holding 1350-B
packets that are all random (probes with a growing skip, then one literal), all one repeated HTTP line
(one short literal, then a copy run), config 5's half-and-half, and all zeros (one copy run from the
start).  Each shape: compress timed by HIP events (median of `reps`), the restore copy between reps
outside the timed region; the decoder timed the same way on the compressed slots.

    python3 tools/exp_snappy_mix.py [reps]
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from quantum_amd import batch, workloads as W  # noqa: E402
from quantum_amd.crypto import Context  # noqa: E402

N, L, STRIDE = 1 << 20, 1350, 1472


def shapes() -> dict:
    rng = np.random.default_rng(7)
    line = np.frombuffer(W.C5_LINE, np.uint8)
    rep = np.tile(line, L // len(line) + 1)[:L]
    out = {}
    for name in ("random", "line", "config5", "zeros"):
        host = np.zeros((N, STRIDE), np.uint8)
        if name == "random":
            host[:, 4:4 + L] = rng.integers(0, 256, (N, L), dtype=np.uint8)
        elif name == "line":
            host[:, 4:4 + L] = rep
        elif name == "config5":
            host = W.config5_packets()
        out[name] = host
    return out


def main() -> None:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    ctx = Context(device=0, max_keys=4)  # QGCM_SNAPPY_GROUP etc. as set in the environment
    stream = torch.cuda.current_stream()
    for name, host in shapes().items():
        plain = torch.from_numpy(host.reshape(-1)).cuda()
        arena = plain.clone()
        lens0 = torch.full((N,), L, dtype=torch.int32, device="cuda")
        lens = lens0.clone()
        status = torch.zeros(N, dtype=torch.uint8, device="cuda")
        tc, tu = [], []
        for r in range(reps + 1):
            arena.copy_(plain)
            lens.copy_(lens0)
            torch.cuda.synchronize()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(stream)
            batch.snappy_compress(ctx, arena, STRIDE, N, lens, L, STRIDE - 4 - 28, status=status, stream=stream)
            e[1].record(stream)
            batch.snappy_uncompress(ctx, arena, STRIDE, N, lens, STRIDE - 4, STRIDE - 4, status=status,
                                    stream=stream)
            e[2].record(stream)
            torch.cuda.synchronize()
            if r:
                tc.append(e[0].elapsed_time(e[1]))
                tu.append(e[1].elapsed_time(e[2]))
        ok = bool(torch.equal(arena[:N * STRIDE].view(N, STRIDE)[:, :4 + L], plain.view(N, STRIDE)[:, :4 + L]))
        print(json.dumps({"shape": name, "compress_ms": round(statistics.median(tc), 3),
                          "uncompress_ms": round(statistics.median(tu), 3), "restored": ok}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
