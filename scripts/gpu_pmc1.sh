# one PMC pass over bench.py (c3_small) for a given KM_ABLATE; prints per-kernel counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc1}; mkdir -p $OUT
for A in ${ABL_LIST:-0}; do
  KM_ABLATE=$A timeout -k 5 120 rocprofv3 --pmc ${PMC:-GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY} --kernel-trace --output-format csv -d $OUT/a$A -o run -- python3 bench.py --config ${CFG:-c3_small} --steps 3 --warmup 1 --no-cpu-baseline > $OUT/a$A.log 2>&1 || { echo "pmc $A failed"; tail -3 $OUT/a$A.log; exit 1; }
  python3 - <<PY
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.defaultdict(set)
for r in csv.DictReader(open('$OUT/a$A/run_counter_collection.csv')):
    if 'fused' not in r['Kernel_Name'] and 'assign' not in r['Kernel_Name']: continue
    agg[r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
dur = []
for r in csv.DictReader(open('$OUT/a$A/run_kernel_trace.csv')):
    if 'fused' in r['Kernel_Name'] or 'assign' in r['Kernel_Name']: dur.append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
print('ablate=$A', 'avg dur us', round(sum(dur)/len(dur)/1e3, 1) if dur else None)
for c, d in sorted(agg.items()): print('   ', c, '%.4g' % (sum(d.values()) / len(d)))
PY
done
