"""profiles/traffic.json: per-launch HBM bytes of a config's dominant kernel from
separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes, with the gfx950 corrections
of MI355X_MICROARCH.md (FETCH_SIZE is KB and counts half of wide streaming
reads; WRITE_SIZE is exact for 16-B streaming stores).  One entry per config;
bench.py reads the entry of the config it runs.

    python scripts/make_traffic.py ROOT CONFIG "kernel substring" ALG_BYTES [profiles/traffic.json]
"""
import collections
import csv
import json
import os
import sys

root, cfg, kname, alg = sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4])
out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic.json")


def per_launch(path, counter):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if kname in r["Kernel_Name"] and r["Counter_Name"] == counter:
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    vals = sorted(per.values())
    big = [v for v in vals if v >= 0.01 * vals[-1]]  # gated no-op dispatches left out
    return sum(big) / len(big), len(big)


f_kb, nf = per_launch(f"{root}/pmc_fetch/run_counter_collection.csv", "FETCH_SIZE")
w_kb, nw = per_launch(f"{root}/pmc_write/run_counter_collection.csv", "WRITE_SIZE")
try:
    db = json.load(open(out))
except (OSError, ValueError):
    db = {}
if "config" in db:  # round-2 single-entry layout
    db = {db["config"]: db}
db[cfg] = {
    "config": cfg, "kernel_name": kname,
    "fetch_size_kb": f_kb, "write_size_kb": w_kb, "launches_fetch": nf, "launches_write": nw,
    "bytes_per_launch": f_kb * 1024 * 2 + w_kb * 1024,
    "algorithmic_bytes_per_launch": alg,
    "correction": "FETCH_SIZE (KB) x1024 x2: gfx950 reports half the bytes of wide streaming reads "
                  "(MI355X_MICROARCH.md, HBM); WRITE_SIZE x1024",
    "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, python3 bench.py --config {cfg} "
              "--steps 3 --warmup 1 --no-cpu-baseline (1 x MI355X)",
}
if os.environ.get("ROUND"):
    db[cfg]["round"] = int(os.environ["ROUND"])
json.dump(db, open(out, "w"), indent=1)
print(json.dumps(db[cfg], indent=1))
