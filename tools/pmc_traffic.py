"""HBM traffic per launch of the seal/open packet kernels from rocprofv3 PMC passes.

Reads <prof>/pmc_fetch/*counter_collection.csv and <prof>/pmc_write/*counter_collection.csv (the
separate --pmc FETCH_SIZE and --pmc WRITE_SIZE passes of tools/profile.sh) and writes
<prof>/traffic.json, which bench.py reports as roofline.traffic.  Corrections per
MI355X_MICROARCH.md "HBM": FETCH_SIZE/WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts half the
bytes of 16-B/lane streaming reads (x2); WRITE_SIZE is exact for 16-B/lane stores.
Usage: python tools/pmc_traffic.py <prof_dir> <packets> <payload_len> <stride> [packets_per_launch]
(libqgcm launches a uniform batch in chunks of 2^19 packets: the counters are per launch; hbm_bytes is
scaled to the whole call, per_launch_hbm_bytes keeps the measured value)
"""
import csv
import glob
import json
import os
import statistics
import sys


def per_kernel(prof: str, counter: str) -> dict:
    out = {}
    for f in glob.glob(os.path.join(prof, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if r["Counter_Name"] != counter or "gcm_quad_kernel<" not in name:
                continue
            kind = "seal" if "gcm_quad_kernel<true" in name else "open"
            out.setdefault((kind, name), []).append(float(r["Counter_Value"]) * 1024.0)
    return out


def main() -> None:
    prof, n, L, stride = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    ppl = int(sys.argv[5]) if len(sys.argv) > 5 else n  # packets per launch
    scale = n / ppl
    fetch, write = per_kernel(prof, "FETCH_SIZE"), per_kernel(prof, "WRITE_SIZE")
    # per_kernel scales by 1024 (KiB counters); these two are plain counts
    lds_idx = {k: [x / 1024.0 for x in v] for k, v in per_kernel(prof, "SQ_LDS_IDX_ACTIVE").items()}
    grbm = {k: [x / 1024.0 for x in v] for k, v in per_kernel(prof, "GRBM_GUI_ACTIVE").items()}
    res = {"workload": {"packets": n, "payload_len": L, "slot_stride": stride}, "packets_per_launch": ppl,
           "source": f"{prof}: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes (separate runs) of "
                     "bench.py; FETCH_SIZE x2 (gfx950 16-B/lane read correction), KiB -> bytes; "
                     "lds_array_busy from the SQ_LDS_IDX_ACTIVE / GRBM_GUI_ACTIVE pass",
           "kernels": {}}
    for (kind, name), vals in fetch.items():
        w = write.get((kind, name), [])
        if not w:
            continue
        fb, wb = 2.0 * statistics.median(vals), statistics.median(w)
        alg_r = ppl * (L + 16 if kind == "seal" else L + 32)
        alg_w = ppl * (L + 28 if kind == "seal" else L + 1)
        res["kernels"][kind] = {"name": name, "launches": len(vals), "fetch_bytes": round(fb),
                                "write_bytes": round(wb), "per_launch_hbm_bytes": round(fb + wb),
                                "hbm_bytes": round((fb + wb) * scale),
                                "fetch_over_algorithmic": round(fb / alg_r, 3),
                                "write_over_algorithmic": round(wb / alg_w, 3)}
        # the binding unit: LDS-array busy = SQ_LDS_IDX_ACTIVE per CU over the kernel's
        # cycles per XCD (GRBM_GUI_ACTIVE is summed over the 8 XCDs, SQ_LDS_IDX_ACTIVE over the 256 CUs)
        lds, gui = lds_idx.get((kind, name)), grbm.get((kind, name))
        if lds and gui:
            res["kernels"][kind]["lds_array_busy"] = round((statistics.median(lds) / 256) /
                                                           (statistics.median(gui) / 8), 3)
    json.dump(res, open(os.path.join(prof, "traffic.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
