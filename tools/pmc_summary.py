import csv, glob, os, sys, collections
root = sys.argv[1]
res = collections.defaultdict(dict)
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    tag = f.split(os.sep)[len(root.split(os.sep))]
    v = tag.split("_")[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "gcm_" not in r["Kernel_Name"] or "kernel<" not in r["Kernel_Name"]: continue
        kind = "seal" if "<true" in r["Kernel_Name"] else "open"
        acc[(kind, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (kind, c), vals in acc.items():
        res[(v, kind)][c] = sum(vals) / len(vals)
for (v, kind), d in sorted(res.items()):
    print(f"== {v} {kind}")
    for c in sorted(d): print(f"   {c:28s} {d[c]:.4g}")
