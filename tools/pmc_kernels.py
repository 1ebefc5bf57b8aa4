"""Per-launch averages of every PMC counter in a rocprofv3 output tree, per kernel whose name contains
one of the given substrings, also divided by a per-launch unit count (e.g. packets).

    python3 tools/pmc_kernels.py <prof_dir> <units_per_launch> <kernel_substring> [...]
"""
import collections
import csv
import glob
import os
import sys


def main() -> None:
    root, units, subs = sys.argv[1], float(sys.argv[2]), sys.argv[3:]
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            hit = next((s for s in subs if s in name), None)
            if hit:
                acc[(hit, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for sub in subs:
        rows = sorted((c, v) for (k, c), v in acc.items() if k == sub)
        if not rows:
            continue
        print(f"{sub} ({root})")
        for c, vals in rows:
            m = sum(vals) / len(vals)
            print(f"   {c:24s} {m:12.4g} per launch {m / units:12.1f} per unit   ({len(vals)} launches)")


if __name__ == "__main__":
    main()
