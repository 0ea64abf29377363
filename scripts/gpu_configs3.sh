#!/bin/bash
# bench lines of the non-headline configs (one process each)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-cfg3}; mkdir -p $OUT
for C in ${CFGS:-c5 c5_poor w784 c3_shard8}; do
  timeout -k 10 400 python3 bench.py --config $C --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > $OUT/$C.json 2> $OUT/$C.err || { echo "$C failed"; tail -3 $OUT/$C.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$C.json'));print('$C', round(d['value'],2), round(d['ms_per_step'],2), round(d['roofline']['frac'],3), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['resolve'])"
done
