"""Steady-state A/B of whole libqgcm builds in ONE process: config 2's step (seal 2^20 x 1350 B, then
open; stride 1408, the headline layout) run back to back as bench.py's timed loop does, `steps` steps
per build per round after `settle` untimed ones, builds interleaved round by round, with the mean GFX
clock of every timed stretch (bench.GpuTelemetry), so a build's rate and its cycles per step can both be
compared.  tools/ab_libs.py times one synchronized pair per round instead.  Every build's sealed arena
must equal the first build's.

    python3 tools/ab_steady.py lib1.so lib2.so[:ENV=V,ENV2=V2] [...] [--rounds R] [--steps K] [--packets N]

(--packets: batch size, default 2^20; the rank-0 layout and fill at any size.)

A ":ENV=V,..." suffix sets those environment variables around that entry's qgcm_create (the library's
knobs are read there), so one build can be compared with itself under other settings.
"""
import ctypes as C
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def opt(name, dflt):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else dflt


def main() -> None:
    rounds, steps, N = opt("--rounds", 5), opt("--steps", 200), opt("--packets", 1 << 20)
    paths = [a for i, a in enumerate(sys.argv[1:], 1) if not a.startswith("--") and sys.argv[i - 1] not in
             ("--rounds", "--steps", "--packets")]
    L, stride = 1350, 1408
    vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
    libs = {}
    for entry in paths:
        path, _, envs = entry.partition(":")
        env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
        lib = C.CDLL(os.path.abspath(path))
        lib.qgcm_create.restype = vp
        lib.qgcm_create.argtypes = [C.c_int, u32, C.c_char_p, C.c_size_t]
        lib.qgcm_set_key.argtypes = [vp, u32, C.c_char_p]
        lib.qgcm_derive_key.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_char_p]
        lib.qgcm_seal_uniform.argtypes = [vp, vp, u64, u32, u32, u32, vp, u32, vp, vp]
        lib.qgcm_open_uniform.argtypes = [vp, vp, u64, u32, u32, u32, u32, vp, vp]
        lib.qgcm_fill_uniform.argtypes = [vp, u64, u32, u32, u32, u64, vp, u64, vp]
        err = C.create_string_buffer(120)
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        ctx = lib.qgcm_create(0, 4, err, 120)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        assert ctx, err.value
        key = C.create_string_buffer(32)
        assert lib.qgcm_derive_key(bench.SECRET, 32, bench.SALT, 32, key) == 0
        assert lib.qgcm_set_key(ctx, 0, key.raw) == 0
        libs[entry] = (lib, ctx)
    alloc = torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda")
    arena = alloc[60:60 + N * stride]
    nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
    status = torch.zeros(N, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    first = next(iter(libs.values()))[0]
    first.qgcm_fill_uniform(arena.data_ptr(), stride, N, L, int.from_bytes(bench.AAD, "little"), 0x5EED0001,
                            nonces.data_ptr(), 0x5EED0002, stream)
    plain = arena.clone()
    ref = None
    for path, (lib, ctx) in libs.items():
        arena.copy_(plain)
        assert lib.qgcm_seal_uniform(ctx, arena.data_ptr(), stride, N, L, 0, nonces.data_ptr(), 4, None, stream) == 0
        torch.cuda.synchronize()
        ref = arena.clone() if ref is None else ref
        same = bool(torch.equal(arena, ref))
        assert lib.qgcm_open_uniform(ctx, arena.data_ptr(), stride, N, L + 28, 0, 4, status.data_ptr(), stream) == 0
        torch.cuda.synchronize()
        ok = int(status.sum().item()) == N
        print(json.dumps({"lib": path, "sealed_same_as_first": same, "opened_ok": ok}), flush=True)
        assert same and ok

    def run(lib, ctx, k):
        for _ in range(k):
            lib.qgcm_seal_uniform(ctx, arena.data_ptr(), stride, N, L, 0, nonces.data_ptr(), 4, None, stream)
            lib.qgcm_open_uniform(ctx, arena.data_ptr(), stride, N, L + 28, 0, 4, status.data_ptr(), stream)

    res = {p: [] for p in libs}
    gib = 2 * N * L / 2**30
    for r in range(rounds):
        for path, (lib, ctx) in libs.items():
            run(lib, ctx, max(2, 50 * (1 << 20) // N))  # settle at this build's load
            torch.cuda.synchronize()
            tele = bench.GpuTelemetry(0)
            tele.start()
            t0 = time.perf_counter()
            run(lib, ctx, steps)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            tele.stop()
            c = tele.summary()
            tele.close()
            ms = el * 1e3 / steps
            row = {"lib": path, "round": r, "packets": N, "GiB_s": round(gib / (ms * 1e-3), 2), "ms_per_step": round(ms, 4),
                   "sclk_mhz_mean": c["sclk_mhz_mean"], "power_w_mean": c["power_w_mean"],
                   "mcycles_per_step": round(ms * c["sclk_mhz_mean"] / 1e3, 3) if c["sclk_mhz_mean"] else None,
                   "status_ok": int(status.sum().item()) == N}
            res[path].append(row)
            print(json.dumps(row), flush=True)
    for path, rows in res.items():
        print(json.dumps({"lib": path, "median_GiB_s": statistics.median(r["GiB_s"] for r in rows),
                          "median_mcycles_per_step": statistics.median(r["mcycles_per_step"] or 0 for r in rows),
                          "median_sclk": statistics.median(r["sclk_mhz_mean"] or 0 for r in rows)}), flush=True)


if __name__ == "__main__":
    main()
