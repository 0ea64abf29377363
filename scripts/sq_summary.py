"""profiles/rN_*_sq_*.json from an SQ counter pass of scripts/gpu_sq.sh.

usage: python scripts/sq_summary.py gpurun_out/TAG OUT.json ["kernel name substring"] [config]
Per dispatch of the kernel: duration from the pass's own timestamps, clock =
GRBM_GUI_ACTIVE / 8 XCDs / duration, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
1024 SIMDs / per-XCD GRBM cycles, SQ_* as fractions of SQ_WAVE_CYCLES."""
import collections
import csv
import json
import sys

root, out = sys.argv[1], sys.argv[2]
kname = sys.argv[3] if len(sys.argv) > 3 else "k_fused<4, 8, true, 0, false>"
cfg = sys.argv[4] if len(sys.argv) > 4 else "c3"
per = collections.defaultdict(lambda: {"raw": collections.defaultdict(float)})
for r in csv.DictReader(open(f"{root}/pmc_sq/run_counter_collection.csv")):
    if kname not in r["Kernel_Name"]:
        continue
    d = per[int(r["Dispatch_Id"])]
    d["raw"][r["Counter_Name"]] += float(r["Counter_Value"])
    d["duration_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
rows = []
for disp in sorted(per):
    d = per[disp]
    raw = d["raw"]
    grbm = raw["GRBM_GUI_ACTIVE"] / 8.0
    wc = raw.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    row = {"dispatch": disp, "duration_ms": d["duration_ms"], "clock_ghz": grbm / (d["duration_ms"] * 1e6)}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in raw:
        row["mfma_busy_per_simd"] = raw["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024.0 / grbm
    # SQ_* cycle counters as fractions of SQ_WAVE_CYCLES (quad-cycle units
    # cancel); LDS-array cycles per CU cycle (256 CUs)
    for name in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_LDS",
                 "SQ_ACTIVE_INST_LDS", "SQ_BUSY_CYCLES"):
        if name in raw:
            row[name.lower()[3:]] = raw[name] / wc
    # instruction counts per launch (SQ_INSTS_*)
    for name in raw:
        if name.startswith("SQ_INSTS_"):
            row[name.lower()[3:] + "_per_launch"] = raw[name]
    if "SQ_LDS_IDX_ACTIVE" in raw:
        row["lds_active_per_cu_cycle"] = raw["SQ_LDS_IDX_ACTIVE"] / 256.0 / grbm
    if "SQ_LDS_BANK_CONFLICT" in raw and "SQ_LDS_IDX_ACTIVE" in raw:
        row["lds_conflict_frac"] = raw["SQ_LDS_BANK_CONFLICT"] / max(raw["SQ_LDS_IDX_ACTIVE"], 1.0)
    row["raw"] = dict(raw)
    rows.append(row)
# gated no-op dispatches (a stopped batch's later launches) are left out, as
# in scripts/trace_summary.py: shorter than 1% of the longest dispatch
longest = max(r["duration_ms"] for r in rows)
rows = [r for r in rows if r["duration_ms"] >= 0.01 * longest]
mean = {k: sum(r[k] for r in rows) / len(rows) for k in rows[0] if k not in ("dispatch", "raw")}
ctrs = sorted(rows[0]["raw"]) if rows else []
json.dump({"kernel": f"{kname} ({cfg})",
           "source": f"rocprofv3 --pmc {' '.join(ctrs)} -- python3 bench.py --config {cfg} --warmup 1 "
                     "--no-cpu-baseline (scripts/gpu_sq.sh)",
           "notes": "clock = GRBM_GUI_ACTIVE/8 XCDs / dispatch duration; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / "
                    "1024 SIMDs / per-XCD GRBM cycles; SQ_* fractions of SQ_WAVE_CYCLES (quad-cycle units cancel)",
           "mean": mean, "dispatches": rows}, open(out, "w"), indent=1)
print(json.dumps(mean, indent=1))
