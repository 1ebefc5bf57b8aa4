"""Summary of a rocprofv3 --memory-copy-trace (+ --kernel-trace) output tree: per copy direction the
count, bytes, busy time and rate while busy; how long both directions were busy at once; and the
wall span from the first to the last copy.  Used to see whether a pipeline's H2D and D2H copies
overlap (the keyed host batch).

    python3 tools/copy_trace_summary.py <prof_dir>
"""
import csv
import glob
import os
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def overlap(x, y):
    i = j = 0
    tot = 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if b > a:
            tot += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main() -> None:
    root = sys.argv[1]
    files = glob.glob(os.path.join(root, "**", "*memory_copy_trace.csv"), recursive=True)
    if not files:
        print("no memory_copy_trace.csv under", root)
        return
    rows = [r for f in files for r in csv.DictReader(open(f))]
    print("columns:", list(rows[0].keys()))
    bykey = {}
    for r in rows:
        d = r.get("Direction") or r.get("Operation") or r.get("Kind") or "?"
        nbytes = 0
        for k in ("Bytes", "Size", "Copy_Bytes"):
            if r.get(k):
                nbytes = int(r[k])
                break
        bykey.setdefault(d, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nbytes))
    iv = {}
    t0 = min(a for v in bykey.values() for a, _, _ in v)
    t1 = max(b for v in bykey.values() for _, b, _ in v)
    for d, v in sorted(bykey.items()):
        u = union([[a, b] for a, b, _ in v])
        busy = sum(b - a for a, b in u)
        nb = sum(n for _, _, n in v)
        iv[d] = u
        rate = nb / busy if busy else 0.0
        print(f"{d:28s} copies {len(v):6d}  bytes {nb / 1e9:9.3f} GB  busy {busy / 1e6:9.2f} ms  "
              f"{rate:7.2f} GB/s while busy  mean {busy / len(v) / 1e3:8.1f} us")
    keys = sorted(iv)
    for i in range(len(keys)):
        for j in range(i + 1, len(keys)):
            print(f"both {keys[i]} and {keys[j]} busy: {overlap(iv[keys[i]], iv[keys[j]]) / 1e6:.2f} ms")
    print(f"span first..last copy: {(t1 - t0) / 1e6:.2f} ms")
    kf = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    kr = [r for f in kf for r in csv.DictReader(open(f))]
    if kr:
        ku = union([[int(r["Start_Timestamp"]), int(r["End_Timestamp"])] for r in kr
                    if t0 <= int(r["Start_Timestamp"]) <= t1])
        print(f"kernels busy within the copy span: {sum(b - a for a, b in ku) / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
