"""profiles/rN_c3_sq_counters.json from the SQ counter pass of scripts/gpu_final2.sh.

usage: python scripts/sq_summary.py gpurun_out/TAG OUT.json ["kernel name substring"]
Per dispatch of the kernel: duration from the pass's own timestamps, clock =
GRBM_GUI_ACTIVE / 8 XCDs / duration, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
1024 SIMDs / per-XCD GRBM cycles, SQ_* as fractions of SQ_WAVE_CYCLES."""
import collections
import csv
import json
import sys

root, out = sys.argv[1], sys.argv[2]
kname = sys.argv[3] if len(sys.argv) > 3 else "k_fused<4, 8, true, 0, false>"
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
    wc = raw["SQ_WAVE_CYCLES"]
    rows.append({"dispatch": disp, "duration_ms": d["duration_ms"],
                 "clock_ghz": grbm / (d["duration_ms"] * 1e6),
                 "mfma_busy_per_simd": raw["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024.0 / grbm,
                 "active_inst_any": raw["SQ_ACTIVE_INST_ANY"] / wc, "active_inst_valu": raw["SQ_ACTIVE_INST_VALU"] / wc,
                 "wait_inst_any": raw["SQ_WAIT_INST_ANY"] / wc, "wait_any": raw["SQ_WAIT_ANY"] / wc,
                 "raw": dict(raw)})
# gated no-op dispatches (a stopped batch's later launches) are left out, as
# in scripts/trace_summary.py: shorter than 1% of the longest dispatch
longest = max(r["duration_ms"] for r in rows)
rows = [r for r in rows if r["duration_ms"] >= 0.01 * longest]
mean = {k: sum(r[k] for r in rows) / len(rows) for k in rows[0] if k not in ("dispatch", "raw")}
json.dump({"kernel": f"{kname} (c3)",
           "source": "rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY "
                     "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -- python3 bench.py "
                     "--steps 3 --warmup 1 --no-cpu-baseline (scripts/gpu_final2.sh)",
           "notes": "clock = GRBM_GUI_ACTIVE/8 XCDs / dispatch duration; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / "
                    "1024 SIMDs / per-XCD GRBM cycles; SQ_* fractions of SQ_WAVE_CYCLES (quad-cycle units cancel)",
           "mean": mean, "dispatches": rows}, open(out, "w"), indent=1)
print(json.dumps(mean, indent=1))
