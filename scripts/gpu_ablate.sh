set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/abl; mkdir -p $OUT
for A in 0 1 2; do
  KM_MFMA_WAVES=12 KM_ABLATE=$A timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/a$A -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/a$A.json 2> $OUT/a$A.err || { echo "abl $A failed"; tail -3 $OUT/a$A.err; exit 1; }
  echo "ablate=$A"; grep -E "k_assign_mfma" $OUT/a$A/run_kernel_trace.csv | awk -F, '{print $0}' | python3 -c "
import sys,csv
rows=list(csv.reader(sys.stdin))
import collections
d=collections.defaultdict(list)
for r in rows:
    name=[x for x in r if 'k_assign_mfma' in x][0]
    st=int(r[-2]) if r[-2].isdigit() else None
    d[name[:60]].append(r)
print({k:len(v) for k,v in d.items()})
"
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/a$A/run_kernel_stats.csv')):
    if 'assign' in r['Name']: print('   ', r['Name'][:45], r['Calls'], round(float(r['AverageNs'])/1e6,3),'ms')
"
done
