"""Per-kernel summary of a rocprofv3 kernel trace (run_kernel_trace.csv) with
gated no-op dispatches left out.

A stopped batch (convergence, empties, NaN) turns its remaining launches into
no-ops that return after reading the gate word (a few microseconds).  rocprofv3's
own --stats averages them in; this summary drops every dispatch shorter than
1% of that kernel's longest dispatch, and prints both the raw and the kept
counts, so that a roofline fraction can be recomputed from profiles/ alone.

    python scripts/trace_summary.py run_kernel_trace.csv [--json out.json]
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict


def summarise(path: str, cut: float = 0.01):
    rows = list(csv.DictReader(open(path)))
    durs = defaultdict(list)
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
        t0 = int(r.get("Start_Timestamp") or r.get("BeginNs"))
        t1 = int(r.get("End_Timestamp") or r.get("EndNs"))
        durs[name].append(t1 - t0)
    out = []
    for name, ds in durs.items():
        mx = max(ds)
        kept = [d for d in ds if d >= cut * mx]
        out.append({
            "kernel": name, "calls": len(ds), "kept": len(kept),
            "avg_us_kept": sum(kept) / len(kept) / 1e3, "min_us_kept": min(kept) / 1e3,
            "max_us": mx / 1e3, "total_ms_kept": sum(kept) / 1e6,
            "avg_us_raw": sum(ds) / len(ds) / 1e3,
        })
    out.sort(key=lambda e: -e["total_ms_kept"])
    return out


def main():
    path = sys.argv[1]
    res = summarise(path)
    print(f"{'calls':>6} {'kept':>5} {'avg_us(kept)':>13} {'min_us':>10} {'max_us':>10} {'total_ms':>10} {'avg_us(raw)':>12}  kernel")
    for e in res:
        print(f"{e['calls']:6d} {e['kept']:5d} {e['avg_us_kept']:13.1f} {e['min_us_kept']:10.1f} {e['max_us']:10.1f} "
              f"{e['total_ms_kept']:10.2f} {e['avg_us_raw']:12.1f}  {e['kernel'][:90]}")
    if "--json" in sys.argv:
        json.dump(res, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
