"""Does running the headline's launches on more than one stream help?  Two bench ranks sharing one GPU
(profiles/r6_s5/bench_n2_line.json) sealed and opened 64 M packets at 898 GiB/s together, against
~857 for one process on 2^20, at a LOWER clock (1991 vs 2125 MHz): ~10% fewer cycles per packet, which
points at the single stream's launch tails and gaps.  This times config 2's step (seal all, then open
all; 2^20 x 1350 B, stride 1408, the headline layout) in one process in several stream layouts,
interleaved, `rounds` x `steps` steps each, with the telemetry of bench.py:

  one        bench.py's step: qgcm_seal_uniform(2^20) then qgcm_open_uniform(2^20) on one stream
             (two 2^19-packet launches each, back to back)
  halves     the arena's halves on two streams, each seal then open, no join inside the step
  halvesj    as halves, but both streams join after the seals and after the opens (what a library-side
             split of one call across two streams has to do: the call returns ordered after all its work)
  quarters   four quarters on two streams (q0, q2 on one; q1, q3 on the other), no join
  quarters4  four quarters on four streams, no join

(profiles/r6_s6 also timed a library-side split of each call across a helper stream, joined at the end
of the call, QGCM_UNIFORM_STREAMS=2: 828-829 against 833-836 for one stream; it was removed.)

Every layout ends with the arena's digests checked against tests/golden/rank_digest.json (rank 0's
2^20 prefix = the headline arena) and every status byte 1.

    python3 tools/exp_streams.py [rounds] [steps]      (EXP_MODES="one,halves,...")
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from quantum_amd import batch  # noqa: E402
from quantum_amd.crypto import Context  # noqa: E402


def main() -> None:
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    modes = os.environ.get("EXP_MODES", "one,halves,halvesj,quarters,quarters4").split(",")
    N, L = 1 << 20, 1350
    stride = batch.slot_stride(L, align=64)
    key = bench.derive_key(bench.SECRET, bench.SALT)
    ctx = Context(device=0, max_keys=4)
    ctx.set_key(0, key)
    alloc = torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda")
    arena = alloc[60:]
    nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
    status = torch.zeros(N, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(arena, stride, N, L, int.from_bytes(bench.AAD, "little"), 0x5EED0001, nonces, 0x5EED0002)
    main_s = torch.cuda.current_stream()
    streams = [torch.cuda.Stream() for _ in range(4)]

    def part(k, parts):
        n = N // parts
        return (arena[k * n * stride:(k + 1) * n * stride], nonces[12 * k * n:12 * (k + 1) * n],
                status[k * n:(k + 1) * n], n)

    def pair(s, a, no, st, n):
        batch.seal_uniform(ctx, a, stride, n, L, 0, no, status=None, stream=s)
        batch.open_uniform(ctx, a, stride, n, L + 28, 0, status=st, stream=s)

    def step(mode):
        if mode == "one":
            pair(main_s, arena[:N * stride], nonces, status, N)
        elif mode in ("halves", "quarters", "quarters4"):
            parts = 2 if mode == "halves" else 4
            ns = 4 if mode == "quarters4" else 2
            for k in range(parts):
                pair(streams[k % ns], *part(k, parts))
        elif mode == "halvesj":
            h = [part(0, 2), part(1, 2)]
            for op in ("seal", "open"):
                e = torch.cuda.Event()
                e.record(main_s)
                for i in range(2):
                    streams[i].wait_event(e)
                    a, no, st, n = h[i]
                    if op == "seal":
                        batch.seal_uniform(ctx, a, stride, n, L, 0, no, status=None, stream=streams[i])
                    else:
                        batch.open_uniform(ctx, a, stride, n, L + 28, 0, status=st, stream=streams[i])
                for i in range(2):
                    e2 = torch.cuda.Event()
                    e2.record(streams[i])
                    main_s.wait_event(e2)

    def run(mode, k):
        t0 = time.perf_counter()
        for _ in range(k):
            step(mode)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    gib = 2 * N * L / 2**30
    for r in range(rounds):
        for mode in modes:
            run(mode, 100)  # settle at this layout's load
            tele = bench.GpuTelemetry(0)
            tele.start()
            el = run(mode, steps)
            tele.stop()
            clock = tele.summary()
            tele.close()
            d = bench.rank_digests(ctx, arena, nonces, status, stride, N, L, 0, main_s)
            print(json.dumps({"mode": mode, "round": r, "steps": steps, "GiB_s": round(gib * steps / el, 2),
                              "ms_per_step": round(el * 1e3 / steps, 4), "sclk_mhz_mean": clock["sclk_mhz_mean"],
                              "power_w_mean": clock["power_w_mean"], "ppt_limited_frac": clock.get("ppt_limited_frac"),
                              "mcycles_per_step": (round(el / steps * clock["sclk_mhz_mean"], 3)
                                                   if clock["sclk_mhz_mean"] else None),
                              "status_ok": int(status.sum().item()) == N,
                              "digests_ok": bool(d["sealed_digest_ok"] and d["opened_digest_ok"])}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
