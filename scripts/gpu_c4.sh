# c4 (1B x 32, k=1024) on one GPU: steady-state steps and device repairs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c4}; mkdir -p $OUT
timeout -k 10 500 python -u bench.py --config c4 --steps ${STEPS:-6} --warmup ${WARM:-3} --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || { tail -5 $OUT/c4.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c4.json'));print('c4', round(d['value'],3), round(d['ms_per_step'],2), round(d['roofline']['frac'],3), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['resolve'], 'repairs', d['empty_repairs_on_device'])"
