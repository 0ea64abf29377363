"""Per-dispatch durations, in launch order, of the kernels whose names contain
any of the given substrings, from a rocprofv3 --kernel-trace csv directory:
    python3 scripts/trace_seq.py gpurun_out/X k_s1 k_fused16 k_s1_delta
"""
import csv
import glob
import sys


def main():
    root, subs = sys.argv[1], sys.argv[2:]
    files = glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "")
                if any(s in name for s in subs):
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    for i, (a, b, name) in enumerate(rows):
        print(f"{i:4d} {(b - a) / 1e6:10.3f} ms  {name[:70]}")


if __name__ == "__main__":
    main()
