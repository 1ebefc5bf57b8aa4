"""Config-3 counters per launch of the descriptor packet kernel (tools/profile_config3.sh passes).

HBM traffic from the separate --pmc FETCH_SIZE / WRITE_SIZE runs, corrected as MI355X_MICROARCH.md
"HBM" prescribes (KiB -> bytes; FETCH_SIZE x2 on gfx950 for 16-B/lane streaming reads), against the
algorithmic bytes of the workload (seal reads L + 16, writes L + 28; open reads L + 32,
writes L + 1 per packet), and the LDS-array busy fraction SQ_LDS_IDX_ACTIVE / 256 over
GRBM_GUI_ACTIVE / 8.  Writes <prof>/traffic.json.
Usage: python tools/pmc_config3.py <prof_dir> [kernel_substring=gcm_seg_kernel]
"""
import csv
import glob
import json
import os
import statistics
import sys

PAYLOAD, N = 4751816686, 1 << 20  # quantum_amd/workloads.py (tools/bench_configs.py config3, bench.py extra_configs)
# PMC_PAYLOAD: another workload's payload bytes (tools/ab_libs_desc.py's batch: 4751969452)
PAYLOAD = int(os.environ.get("PMC_PAYLOAD", PAYLOAD))


def per_kernel(prof: str, counter: str, sub: str) -> dict:
    out = {}
    for f in glob.glob(os.path.join(prof, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if r["Counter_Name"] != counter or sub not in name:
                continue
            kind = "seal" if "<true" in name else "open"
            out.setdefault(kind, []).append(float(r["Counter_Value"]))
    return out


def main() -> None:
    prof = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "gcm_seg_kernel"
    fetch, write = per_kernel(prof, "FETCH_SIZE", sub), per_kernel(prof, "WRITE_SIZE", sub)
    lds, gui = per_kernel(prof, "SQ_LDS_IDX_ACTIVE", sub), per_kernel(prof, "GRBM_GUI_ACTIVE", sub)
    res = {"workload": "config3: 2^20 x U{64..9000} B, 1024 keys", "kernel": sub, "payload_bytes": PAYLOAD,
           "source": f"{prof}: rocprofv3 --pmc passes of tools/bench_configs.py config3", "kernels": {}}
    for kind in ("seal", "open"):
        if kind not in fetch or kind not in write:
            continue
        fb, wb = 2048.0 * statistics.median(fetch[kind]), 1024.0 * statistics.median(write[kind])
        alg_r = PAYLOAD + N * (16 if kind == "seal" else 32)
        alg_w = PAYLOAD + N * (28 if kind == "seal" else 1)
        k = {"launches": len(fetch[kind]), "fetch_bytes": round(fb), "write_bytes": round(wb),
             "fetch_over_algorithmic": round(fb / alg_r, 3), "write_over_algorithmic": round(wb / alg_w, 3)}
        if kind in lds and kind in gui:
            k["lds_array_busy"] = round((statistics.median(lds[kind]) / 256) / (statistics.median(gui[kind]) / 8), 3)
            k["gui_active_cycles"] = statistics.median(gui[kind]) / 8
        res["kernels"][kind] = k
    json.dump(res, open(os.path.join(prof, "traffic.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
