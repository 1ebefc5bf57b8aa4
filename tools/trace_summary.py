"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py (tools/profile.sh "trace" pass).

Prints, per kernel, calls / mean / min duration (from <prof>/trace/*kernel_stats.csv) and, for the
packet kernels, the mean over the last `timed` launches in <prof>/trace/*kernel_trace.csv (bench.py
runs `warmup` untimed steps first) -- the figure bench.py's HIP-event kernel_ms must agree with.
Usage: python tools/trace_summary.py <prof_dir> [timed=100] > <prof_dir>/kernel_stats_summary.txt
"""
import csv
import glob
import os
import statistics
import sys


def main() -> None:
    prof = sys.argv[1]
    timed = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    stats = glob.glob(os.path.join(prof, "trace", "*kernel_stats.csv"))[0]
    trace = glob.glob(os.path.join(prof, "trace", "*kernel_trace.csv"))[0]
    print(f"rocprofv3 --kernel-trace --stats -- python3 bench.py (tools/profile.sh), {prof}")
    for r in csv.DictReader(open(stats)):
        print(f"{r['Name'][:100]:100s} calls={int(r['Calls']):3d} avg_us={float(r['AverageNs']) / 1e3:9.1f} "
              f"min_us={float(r['MinNs']) / 1e3:9.1f} pct={float(r['Percentage']):6.2f}")
    launches = {}
    for r in csv.DictReader(open(trace)):
        name = r["Kernel_Name"]
        if "gcm_quad_kernel<" not in name:
            continue
        kind = "seal" if "gcm_quad_kernel<true" in name else "open"
        launches.setdefault(kind, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for kind in ("seal", "open"):
        ls = sorted(launches.get(kind, []))[-timed:]
        if ls:
            print(f"{kind}: mean over the {len(ls)} timed launches "
                  f"{statistics.mean(e - s for s, e in ls) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
