# fused-kernel ablations (KM_ABLATE=0..4) on c3; kernel time from rocprofv3 stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abl}; mkdir -p $OUT
for A in ${ABL_LIST:-0 1 2 3 4}; do
  KM_ABLATE=$A timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/a$A -o run -- python3 bench.py --config ${CFG:-c3} --steps 4 --warmup 1 --no-cpu-baseline > $OUT/a$A.json 2> $OUT/a$A.err || { echo "abl $A failed"; tail -3 $OUT/a$A.err; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/a$A/run_kernel_stats.csv')):
    if 'fused' in r['Name'] or 'assign' in r['Name']: print('ablate=$A', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e6,3),'ms')
"
done
