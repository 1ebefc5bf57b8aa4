"""Timeline of one config-5 call from a rocprofv3 kernel + memory-copy trace (tools/trace_config5.sh):
the last seal (or open) call's span, and per stage (H2D copies, D2H copies, worklist kernels, GCM
kernels) the busy time (union of intervals) and the count, so a stage that binds shows as busy ~ span.
Usage: python tools/chain_timeline.py <trace_dir> [seal|open]"""
import csv
import glob
import os
import sys


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    d = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "seal"
    ks = list(csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])))
    cs = list(csv.DictReader(open(glob.glob(os.path.join(d, "*memory_copy_trace.csv"))[0])))
    ev = [("k", r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks]
    ev += [("c", r["Direction"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in cs]
    ev.sort(key=lambda x: x[2])
    # calls = runs of GCM descriptor kernels separated by > 3 ms gaps; seal kernels have "<true"
    gcm = [e for e in ev if e[0] == "k" and ("quad_kernel" in e[1] or "seg_kernel" in e[1])]
    calls, cur = [], []
    for e in gcm:
        if cur and e[2] - cur[-1][3] > 3_000_000:
            calls.append(cur)
            cur = []
        cur.append(e)
    if cur:
        calls.append(cur)
    pick = [c for c in calls if ("<true" in c[0][1]) == (want == "seal")]
    call = pick[-1]
    t0, t1 = call[0][2], call[-1][3]
    # widen to the copies around the call
    win = [e for e in ev if e[3] >= t0 - 2_000_000 and e[2] <= t1 + 2_000_000]
    span0 = min(e[2] for e in win if e[0] == "c")
    span1 = max(e[3] for e in win if e[0] == "c")
    stages = {
        "H2D copies": [e for e in win if e[0] == "c" and "HOST_TO_DEVICE" in e[1]],
        "D2H copies": [e for e in win if e[0] == "c" and "DEVICE_TO_HOST" in e[1]],
        "GCM kernels": [e for e in win if e[0] == "k" and ("quad_kernel" in e[1] or "seg_kernel" in e[1])],
        "other kernels (worklist, copies)": [e for e in win if e[0] == "k" and not ("quad_kernel" in e[1] or "seg_kernel" in e[1])],
    }
    print(f"{want} call: span {(span1 - span0) / 1e6:.2f} ms (first copy start to last copy end)")
    for name, es in stages.items():
        print(f"  {name:34s} n={len(es):5d} busy {union([(e[2], e[3]) for e in es]) / 1e6:7.2f} ms  "
              f"sum {sum(e[3] - e[2] for e in es) / 1e6:7.2f} ms")
    names = {}
    for e in stages["other kernels (worklist, copies)"]:
        k = e[1].split("(")[0][-60:]
        names.setdefault(k, [0, 0])
        names[k][0] += 1
        names[k][1] += e[3] - e[2]
    for k, (n, t) in sorted(names.items(), key=lambda x: -x[1][1])[:8]:
        print(f"     {k:60s} n={n:4d} {t / 1e6:6.2f} ms")


if __name__ == "__main__":
    main()
