"""Per-workgroup timeline of the uniform kernel (gcm_quad_kernel<*, false>) from a side build with
-DQGCM_QUAD_STATS: where a launch's cycles go at its start and end.  Config 2's step (2^20 x 1350 B,
stride 1408, the headline layout), each launch synchronized and read back on its own.

For each launch: its span (first workgroup start to last workgroup end, device clock), the spread of
workgroup starts (table fill, dispatch), the deciles of workgroup ends, the mean end per XCC, and the
idle fractions of the span: workgroup slots idle after their workgroup ended ("wg_tail"), waves idle
inside a workgroup after their last tile while a sibling still works ("wave_tail"), and CUs idle once
both their workgroups have ended ("cu_idle_frac", with the mean CU end and the tiles done per XCC);
which workgroups share a CU (HW_ID) and how far apart the two end.

    python3 tools/quad_stats.py exp/stats/libqgcm.so [launches]
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from quantum_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
import bench  # noqa: E402
from quantum_amd import batch  # noqa: E402
from quantum_amd.crypto import Context  # noqa: E402


def main() -> None:
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    N, L = 1 << 20, 1350
    stride = batch.slot_stride(L, align=64)
    ctx = Context(device=0, max_keys=4)
    ctx.set_key(0, bench.derive_key(bench.SECRET, bench.SALT))
    alloc = torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda")
    arena = alloc[60:]
    nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
    status = torch.zeros(N, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(arena, stride, N, L, int.from_bytes(bench.AAD, "little"), 0x5EED0001, nonces, 0x5EED0002)
    lib = _lib.lib()
    lib.qgcm_debug_quad_stats.argtypes = [C.c_void_p, C.c_int, C.c_int]
    buf = np.zeros(4096 * 8, dtype=np.uint64)
    tele = bench.GpuTelemetry(0)  # per-XCD clocks over the settle loop (the launches below run one at a time)
    tele.start()
    for _ in range(40):  # settle the clock at this load
        batch.seal_uniform(ctx, arena, stride, N, L, 0, nonces, status=None)
        batch.open_uniform(ctx, arena, stride, N, L + 28, 0, status=status)
    torch.cuda.synchronize()
    tele.stop()
    clocks = tele.summary()
    tele.close()
    rows = []
    for it in range(launches):
        seal = it % 2 == 0
        lib.qgcm_debug_quad_stats(buf.ctypes.data, buf.size, 1)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        if seal:
            batch.seal_uniform(ctx, arena, stride, N, L, 0, nonces, status=None)
        else:
            batch.open_uniform(ctx, arena, stride, N, L + 28, 0, status=status)
        e[1].record()
        torch.cuda.synchronize()
        lib.qgcm_debug_quad_stats(buf.ctypes.data, buf.size, 0)
        st = buf.reshape(-1, 8).astype(np.int64)
        st = st[st[:, 0] > 0]
        start, end, sum_end, tiles, xcc = st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4] & 0xF
        first_end = (1 << 62) - st[:, 6]
        t0, t1 = start.min(), end.max()
        span = float(t1 - t0)
        waves = 16
        wg_tail = float((t1 - end).sum()) / (len(st) * span)
        wave_tail = float((waves * end - sum_end).sum()) / (len(st) * waves * span)
        start_idle = float((start - t0).sum()) / (len(st) * span)
        per_xcc = {int(x): round(float((end[xcc == x] - t0).mean()) / 100, 1) for x in np.unique(xcc)}
        row = {"launch": it, "op": "seal" if seal else "open", "event_ms": round(e[0].elapsed_time(e[1]), 4),
               "wgs": int(len(st)), "span_us": round(span / 100, 1),
               "start_spread_us": round(float(start.max() - t0) / 100, 1),
               "end_deciles_us": [round(float(x) / 100, 1) for x in np.quantile(end - t0, [0, .1, .5, .9, 1])],
               "first_wave_end_deciles_us": [round(float(x) / 100, 1)
                                             for x in np.quantile(first_end - t0, [0, .1, .5, .9, 1])],
               "tiles_per_wg": [int(tiles.min()), int(np.median(tiles)), int(tiles.max())],
               "mean_end_us_per_xcc": per_xcc,
               "start_idle_frac": round(start_idle, 4), "wg_tail_frac": round(wg_tail, 4),
               "wave_tail_frac": round(wave_tail, 4)}
        # co-residency: workgroups on one CU (XCC id, HW_ID bits 8-15: CU, SH, SE)
        wgid = np.nonzero(buf.reshape(-1, 8)[:, 0] > 0)[0]
        cu = (xcc << 8) | ((st[:, 5] >> 8) & 0xFF)
        keys, inv, cnt = np.unique(cu, return_inverse=True, return_counts=True)
        row["cus"] = int(len(keys))
        # a CU is idle once all its workgroups have ended: the launch's CU-level tail, and by XCC
        cend = np.array([end[inv == c].max() for c in range(len(keys))]) - t0
        cx = np.array([xcc[inv == c][0] for c in range(len(keys))])
        row["cu_end_deciles_us"] = [round(float(x) / 100, 1) for x in np.quantile(cend, [0, .1, .5, .9, 1])]
        row["cu_idle_frac"] = round(float((cend.max() - cend).mean() / cend.max()), 4)
        row["mean_cu_end_us_per_xcc"] = {int(x): round(float(cend[cx == x].mean()) / 100, 1) for x in np.unique(cx)}
        row["tiles_per_xcc"] = {int(x): int(tiles[xcc == x].sum()) for x in np.unique(xcc)}
        row["wgs_per_cu"] = {int(k): int(v) for k, v in zip(*np.unique(cnt, return_counts=True))}
        early, late, gaps = [], [], []
        for c in range(len(keys)):
            idx = np.nonzero(inv == c)[0]
            if len(idx) != 2:
                continue
            a, b = idx[np.argsort(end[idx])]
            early.append(int(start[a] <= start[b]))
            late.append(float(end[b] - end[a]) / 100)
            gaps.append(int(wgid[b]) - int(wgid[a]))  # > 0: the lower workgroup index ended first
        if late:
            row["pair_end_gap_us"] = [round(float(x), 1) for x in np.quantile(late, [0, .1, .5, .9, 1])]
            row["pair_early_started_first_frac"] = round(float(np.mean(early)), 3)
            row["pair_lower_index_ended_first_frac"] = round(float(np.mean(np.array(gaps) > 0)), 3)
            gi, gc = np.unique(np.abs(gaps), return_counts=True)
            row["pair_wg_index_gaps"] = {int(g): int(c) for g, c in sorted(zip(gi, gc), key=lambda t: -t[1])[:6]}
        if it < 2:
            np.save(os.path.join(os.environ.get("QS_OUT", "."), f"quad_stats_launch{it}.npy"), buf.reshape(-1, 8).copy())
        rows.append(row)
        print(json.dumps(row), flush=True)
    ok = int(status.sum().item()) == N
    print(json.dumps({"summary": True, "status_ok": ok, "sclk_mhz_mean": clocks.get("sclk_mhz_mean"),
                      "sclk_mhz_mean_per_xcd": clocks.get("sclk_mhz_mean_per_xcd"),
                      "mean_cu_end_us_per_xcc_all": {x: round(float(np.mean([r["mean_cu_end_us_per_xcc"][x] for r in rows])), 1)
                                                     for x in rows[0]["mean_cu_end_us_per_xcc"]},
                      "median_cu_idle_frac": float(np.median([r["cu_idle_frac"] for r in rows])),
                      "median_wg_tail_frac": float(np.median([r["wg_tail_frac"] for r in rows])),
                      "median_wave_tail_frac": float(np.median([r["wave_tail_frac"] for r in rows])),
                      "median_start_idle_frac": float(np.median([r["start_idle_frac"] for r in rows]))}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
