#!/bin/bash
# k_fullscan entries per wave (KM_FS_G) and workgroups per CU (KM_FS_WG) on c5, diagnostic library
cd "${GRAFT_REPO_ROOT:-/root/repo}"
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/fsg; mkdir -p $OUT
cp $P/libkmeans_amd.so $OUT/prod.so
cp $P/libkmeans_amd_diag.so $P/libkmeans_amd.so
for V in "2 1" "4 1" "2 2" "4 2"; do
  set -- $V
  KM_FS_G=$1 KM_FS_WG=$2 timeout -k 10 300 python3 bench.py --config ${CFG:-c5} --steps 4 --warmup 2 --no-cpu-baseline > $OUT/g$1w$2.json 2> $OUT/g$1w$2.err || { tail -3 $OUT/g$1w$2.err; cp $OUT/prod.so $P/libkmeans_amd.so; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/g$1w$2.json'));print('G=$1 WG=$2', round(d['value'],3), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()})"
done
cp $OUT/prod.so $P/libkmeans_amd.so
