# GPU parity tests, then rocprofv3 kernel stats of the bench for each config in CFGS
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ks}; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
for C in ${CFGS:-c3}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$C -o run -- python3 bench.py --config $C --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > $OUT/$C.json 2> $OUT/$C.err || { echo "$C failed"; tail -5 $OUT/$C.err; exit 1; }
  python3 -c "
import csv,json
d=json.load(open('$OUT/$C.json')); print('$C', round(d['value'],2), 'it/s', round(d['ms_per_step'],3), 'ms/step', d['resolve'])
for r in csv.DictReader(open('$OUT/$C/run_kernel_stats.csv')):
    if int(r['Calls'])>=${STEPS:-10}: print('  ', r['Calls'].rjust(4), ('%.1f'%(float(r['AverageNs'])/1e3)).rjust(9),'us', r['Name'][:50])
"
done
