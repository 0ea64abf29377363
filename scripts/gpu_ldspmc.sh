#!/bin/bash
# LDS / stall counter pass over the fused kernels (one --pmc pass per screen)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ldspmc}; mkdir -p $OUT
for m in ${SCREENS:-0 2}; do
  timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/s$m -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --screen $m > $OUT/s$m.log 2>&1 || { echo "pass $m failed"; tail -5 $OUT/s$m.log; exit 1; }
  python3 - $OUT/s$m/run_counter_collection.csv <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if 'fused' not in r['Kernel_Name']: continue
    agg[(r['Kernel_Name'][:40], r['Dispatch_Id'])][r['Counter_Name']] += float(r['Counter_Value'])
for (k, dsp), v in list(agg.items())[-2:]:
    w = v['SQ_WAVE_CYCLES']
    print(k, dsp, {c: (round(x / w, 3) if c.startswith('SQ_WAIT') or c == 'SQ_ACTIVE_INST_ANY' else x) for c, x in v.items()})
PY
done
