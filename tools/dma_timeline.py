"""Per-call timeline of the keyed host batch's DMA-run path from a rocprofv3 kernel + copy trace
(tools/gpu_round.sh tracechunk): for the last seal and open calls, each chunk's copy-in (SDMA, the
member's copy-in stream), descriptor-batch kernels and copy-out (blit kernels on the copy-out stream),
as start offset and duration in ms, and the call's span.

    python3 tools/dma_timeline.py <trace_dir> [calls]
"""
import csv
import glob
import os
import sys


def main() -> None:
    d = sys.argv[1]
    ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    ks = list(csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])))
    cs = list(csv.DictReader(open(glob.glob(os.path.join(d, "*memory_copy_trace.csv"))[0])))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "H2D") for r in cs
          if r["Direction"].endswith("HOST_TO_DEVICE") and r["Stream_Id"] == "1"]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "D2H") for r in ks
           if "copyBuffer" in r["Kernel_Name"] and r["Stream_Id"] == "3"]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "GCM") for r in ks
           if r["Stream_Id"] == "2" and ("gcm_quad" in r["Kernel_Name"] or "gcm_seg" in r["Kernel_Name"])]
    ev.sort()
    # calls: separated by gaps > 5 ms with nothing running
    calls, cur, end = [], [], 0
    for e in ev:
        if cur and e[0] - end > 5_000_000:
            calls.append(cur)
            cur = []
        cur.append(e)
        end = max(end, e[1])
    calls.append(cur)
    for call in calls[-ncalls:]:
        t0 = call[0][0]
        span = (max(e[1] for e in call) - t0) / 1e6
        print(f"call: span {span:.1f} ms")
        for a, b, n in call:
            if (b - a) > 200_000 or n == "GCM":  # skip the side copies
                print(f"   {(a - t0) / 1e6:8.2f} +{(b - a) / 1e6:6.2f}  {n}")


if __name__ == "__main__":
    main()
