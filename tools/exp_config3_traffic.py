"""Where config 3's extra read traffic comes from (the segmented kernel reads
1.51x and writes 1.65x its algorithmic bytes, config 2 1.15x / 1.12x).

The same 2^20 packets (quantum_amd/workloads.py lengths, nonces and plaintext) in four forms, each in its
own process so the PMC passes separate them:

  packed          the workload: 1024 peer keys, slots packed at 4-B offsets (payloads at 4 mod 16 or so)
  packed_onekey   the same layout and lengths, every packet under key 0 (one run, one key's tables)
  aligned         1024 keys, every payload 64-B aligned (slots rounded to 64 B, exp_config3_align.py)
  aligned_onekey  aligned and one key

packed - packed_onekey is what 1024 keys' tables cost (the per-packet recombination's reads of the
global comb tables of H^2..H^5 and the length block, and each key run's table fill, fetched by every XCD
whose workgroups work on the key); packed - aligned is what 4-B slot offsets cost (a 64-B granule at a
4-B offset touches an extra line).  Each form: one warmup pair, then 3 seal+open pairs.

  python3 tools/exp_config3_traffic.py run <form>          (under rocprofv3 --pmc ...)
  python3 tools/exp_config3_traffic.py time [reps]         (all four forms in one process, interleaved)
  python3 tools/exp_config3_traffic.py summarize <dir>     (one sub-directory per form x pass)
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

PAIRS = 3
FORMS = ("packed", "packed_onekey", "aligned", "aligned_onekey")


def run(form: str) -> None:
    import torch

    from exp_config3_align import aligned_layout
    from quantum_amd import batch, workloads as W
    from quantum_amd.crypto import Context

    keys = W.peer_keys()
    ctx = Context(device=0, max_keys=W.NKEYS)
    ctx.set_keys(0, keys)
    lens, kidx = W.lengths(), W.key_indices()
    if form.endswith("onekey"):
        kidx = np.zeros_like(kidx)
    offs, size = aligned_layout(lens) if form.startswith("aligned") else W.layout(lens)
    arena = W.device_arena(torch, size, offs, kidx)
    nonces = torch.from_numpy(W.nonces()).cuda()
    status = torch.zeros(W.N, dtype=torch.uint8, device="cuda")
    ds = batch.make_descs(offs, lens, kidx, "cuda")
    do = batch.make_descs(offs, lens.astype(np.int64) + 28, kidx, "cuda")
    ok = True
    for _ in range(PAIRS + 1):
        batch.seal_batch(ctx, arena, ds, W.N, nonces, status=status)
        batch.open_batch(ctx, arena, do, W.N, status=status)
        torch.cuda.synchronize()
        ok &= int(status.sum()) == W.N
    print(json.dumps({"form": form, "status_ok": ok, "payload_bytes": int(lens.sum()), "arena_bytes": size}))
    ctx.close()


def time_forms(reps: int = 7) -> None:
    """Seal+open pairs of the four forms interleaved in one process, HIP events, median GiB/s."""
    import torch

    from exp_config3_align import aligned_layout
    from quantum_amd import batch, workloads as W
    from quantum_amd.crypto import Context

    keys = W.peer_keys()
    ctx = Context(device=0, max_keys=W.NKEYS)
    ctx.set_keys(0, keys)
    lens, kidx0 = W.lengths(), W.key_indices()
    nonces = torch.from_numpy(W.nonces()).cuda()
    status = torch.zeros(W.N, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    forms = {}
    for form in FORMS:
        kidx = np.zeros_like(kidx0) if form.endswith("onekey") else kidx0
        offs, size = aligned_layout(lens) if form.startswith("aligned") else W.layout(lens)
        forms[form] = (W.device_arena(torch, size, offs, kidx), batch.make_descs(offs, lens, kidx, "cuda"),
                       batch.make_descs(offs, lens.astype(np.int64) + 28, kidx, "cuda"))
    times = {f: [] for f in FORMS}
    ok = True
    for r in range(reps + 1):
        for form, (arena, ds, do) in forms.items():
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record(stream)
            batch.seal_batch(ctx, arena, ds, W.N, nonces, status=status, stream=stream)
            batch.open_batch(ctx, arena, do, W.N, status=status, stream=stream)
            e[1].record(stream)
            torch.cuda.synchronize()
            ok &= int(status.sum()) == W.N
            if r:
                times[form].append(e[0].elapsed_time(e[1]))
    payload = int(lens.sum())
    print(json.dumps({"exp": "config3 forms, seal+open pair", "reps": reps, "status_ok": ok,
                      **{f: {"pair_ms": round(float(np.median(t)), 3),
                             "GiB_s": round(2 * payload / (float(np.median(t)) * 1e-3) / 2**30, 1)}
                         for f, t in times.items()}}))
    ctx.close()


def summarize(root: str) -> None:
    """<root>/<form>_<pass>/...counter_collection.csv -> per form and direction: every counter summed
    over the call's packet kernels (gcm_*: the segmented kernel and its per-wave complement), median
    over the calls; FETCH_SIZE x 2 (gfx950), WRITE_SIZE as is, both in bytes, against the algorithmic
    bytes (seal reads L + 16, writes L + 28; open reads L + 32, writes L + 1)."""
    from quantum_amd import workloads as W

    payload = int(W.lengths().sum())
    out = {"payload_bytes": payload, "packets": W.N, "forms": {}}
    for form in FORMS:
        per = collections.defaultdict(lambda: collections.defaultdict(list))  # kind -> counter -> per-call sums
        for f in glob.glob(os.path.join(root, f"{form}_p[0-9]*", "**", "*counter_collection.csv"), recursive=True):
            calls = collections.defaultdict(lambda: collections.defaultdict(float))
            seq = {"seal": -1, "open": -1}
            last = None
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if "gcm_" not in name or ("seg" not in name and "quad" not in name):
                    continue
                kind = "seal" if "<true" in name else "open"
                did = r.get("Dispatch_Id", "")
                if (kind, did) != last and "seg" in name:
                    seq[kind] += 1  # a call = its segmented launch (+ the complement after it)
                last = (kind, did)
                calls[(kind, max(seq[kind], 0))][r["Counter_Name"]] += float(r["Counter_Value"])
            for (kind, _), cnt in calls.items():
                for c, v in cnt.items():
                    per[kind][c].append(v)
        fo = {}
        for kind, cnts in per.items():
            k = {c: statistics.median(v[1:] if len(v) > 1 else v) for c, v in cnts.items()}  # drop the warmup call
            alg_r = payload + W.N * (16 if kind == "seal" else 32)
            alg_w = payload + W.N * (28 if kind == "seal" else 1)
            row = {"calls": max(len(v) for v in cnts.values())}
            if "FETCH_SIZE" in k:
                row["fetch_bytes"] = round(2048.0 * k["FETCH_SIZE"])
                row["fetch_over_algorithmic"] = round(2048.0 * k["FETCH_SIZE"] / alg_r, 3)
            if "WRITE_SIZE" in k:
                row["write_bytes"] = round(1024.0 * k["WRITE_SIZE"])
                row["write_over_algorithmic"] = round(1024.0 * k["WRITE_SIZE"] / alg_w, 3)
            for c in ("TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum", "TCC_REQ_sum"):
                if c in k:
                    row[c] = k[c]
            if "TCC_HIT_sum" in k and "TCC_MISS_sum" in k:
                row["l2_hit_rate"] = round(k["TCC_HIT_sum"] / max(1.0, k["TCC_HIT_sum"] + k["TCC_MISS_sum"]), 4)
            fo[kind] = row
        out["forms"][form] = fo
    for kind in ("seal", "open"):
        try:
            f = {m: out["forms"][m][kind]["fetch_bytes"] for m in FORMS}
        except KeyError:
            continue
        out[f"attribution_{kind}"] = {
            "keys_bytes_per_call": f["packed"] - f["packed_onekey"],
            "keys_bytes_per_packet": round((f["packed"] - f["packed_onekey"]) / W.N, 1),
            "misalignment_bytes_per_call": f["packed"] - f["aligned"],
            "keys_share_of_excess": round((f["packed"] - f["packed_onekey"]) /
                                          max(1, f["packed"] - (payload + W.N * (16 if kind == "seal" else 32))), 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    elif sys.argv[1] == "time":
        time_forms(int(sys.argv[2]) if len(sys.argv) > 2 else 7)
    else:
        summarize(sys.argv[2])
