"""Kernel + copy timeline of a rocprofv3 run (--kernel-trace --memory-copy-trace, csv, -o t): every
dispatch and copy in start order, with its duration and the idle gap before it, for events [first, last).

    python3 tools/kernel_copy_timeline.py <trace dir> <first> <last>

Columns: start (us, from the first event shown), duration (us), gap after the previous event (us),
stream, K kernel name / C copy direction.  profiles/r4_s45 holds the 64-packet host and group pairs.
"""
import csv
import sys


def main() -> None:
    d, first, last = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    ev = []
    for r in csv.DictReader(open(d + "/t_kernel_trace.csv")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:60], r["Stream_Id"]))
    for r in csv.DictReader(open(d + "/t_memory_copy_trace.csv")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   "C " + r["Direction"].replace("MEMORY_COPY_", ""), r["Stream_Id"]))
    ev.sort()
    print(len(ev), "events")
    if not ev[first:last]:
        return
    t0, prev = ev[first][0], None
    for s, e, name, st in ev[first:last]:
        gap = (s - prev) / 1e3 if prev else 0.0
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap{gap:7.1f} s{st} {name}")
        prev = e


if __name__ == "__main__":
    main()
