# c5 poor-seed checks: repair / empty tests (incl. the 50M full-size one) and
# the c5 / c5_poor benches (step with 4093 empties repaired on the device)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c5poor}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "poor or repair or empty" -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -12 $OUT/t.log
[ $rc -ne 0 ] && exit 1
for spec in "c5p1 c5_poor 1 0" "c5p3 c5_poor 3 0" "c5 c5 3 1"; do
  set -- $spec
  timeout -k 10 300 python -u bench.py --config $2 --steps $3 --warmup $4 --no-cpu-baseline > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$1.json'));print('$1', round(d['value'],3), round(d['ms_per_step'],2), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d.get('empty_repairs_on_device'))"
done
