"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py (tools/profile.sh "trace" pass).

Prints, per kernel, calls / mean / min duration (from <prof>/trace/*kernel_stats.csv) and, for the
packet kernels, the mean over the last `timed` launches in <prof>/trace/*kernel_trace.csv (bench.py
runs `warmup` untimed steps first) -- the figure bench.py's HIP-event kernel_ms must agree with.
libqgcm launches a uniform batch as back-to-back launches of up to 2^20 packets (kLaunchChunk; 2^19
until round 6), `lpc` per call: the per-call figures group consecutive launches of one kind.
Usage: python tools/trace_summary.py <prof_dir> [timed=100] [lpc=1] > <prof_dir>/kernel_stats_summary.txt
"""
import csv
import glob
import os
import statistics
import sys


def main() -> None:
    prof = sys.argv[1]
    timed = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    lpc = int(sys.argv[3]) if len(sys.argv) > 3 else 1
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
        ls = sorted(launches.get(kind, []))[-timed * lpc:]
        if ls:
            calls = [ls[i:i + lpc] for i in range(0, len(ls) - lpc + 1, lpc)]
            print(f"{kind}: mean over the {len(ls)} timed launches "
                  f"{statistics.mean(e - s for s, e in ls) / 1e3:.1f} us per launch; per call ({lpc} launches) "
                  f"{statistics.mean(sum(e - s for s, e in c) for c in calls) / 1e3:.1f} us of kernel, "
                  f"{statistics.mean(c[-1][1] - c[0][0] for c in calls) / 1e3:.1f} us first start to last end")


if __name__ == "__main__":
    main()
