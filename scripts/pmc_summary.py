"""Summarise rocprofv3 --pmc CSVs (per kernel, averaged per dispatch)."""
import collections, csv, glob, sys
root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"].split("(")[0][-40:]
        agg[kn][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
for kn, d in agg.items():
    if not any(s in kn for s in ("assign", "stats", "rerank", "fullscan", "fused")):
        continue
    out = {}
    for c, vals in d.items():
        per = collections.defaultdict(float)
        for disp, v in vals:
            per[disp] += v
        out[c] = sum(per.values()) / len(per)
    print(kn)
    for c in sorted(out):
        print(f"   {c:32s} {out[c]:.4g}")
