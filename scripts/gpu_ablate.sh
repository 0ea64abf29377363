#!/bin/bash
# fused-kernel ablations on c3 with the diagnostic library (KM_ABLATE=0..8,
# results wrong by design for 1..6): assign-kernel time from bench's HIP events
cd "${GRAFT_REPO_ROOT:-/root/repo}"
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/${TAG:-abl}; mkdir -p $OUT
cp $P/libkmeans_amd.so $OUT/prod.so
cp $P/libkmeans_amd_diag.so $P/libkmeans_amd.so
for A in ${ABL_LIST:-0 1 2 3 4 5}; do
  KM_ABLATE=$A timeout -k 10 300 python3 bench.py --config ${CFG:-c3} --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --screen 0 > $OUT/a$A.json 2> $OUT/a$A.err || { echo "abl $A failed"; tail -3 $OUT/a$A.err; cp $OUT/prod.so $P/libkmeans_amd.so; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/a$A.json'));print('ablate=$A', round(d['value'],2), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()})"
done
cp $OUT/prod.so $P/libkmeans_amd.so
