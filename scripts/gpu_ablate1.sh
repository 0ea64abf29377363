#!/bin/bash
# first-iteration ablations of k_fused on c3 (identical takeSample centroids for
# every variant, screen forced to fp16x3): assign time of that one iteration
cd "${GRAFT_REPO_ROOT:-/root/repo}"
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/${TAG:-abl1}; mkdir -p $OUT
cp $P/libkmeans_amd.so $OUT/prod.so
cp $P/libkmeans_amd_diag.so $P/libkmeans_amd.so
for A in ${ABL_LIST:-0 3 0 3}; do
  KM_ABLATE=$A timeout -k 10 300 python3 bench.py --config ${CFG:-c3} --steps 1 --warmup 0 --no-cpu-baseline --screen 0 > $OUT/a$A.json 2> $OUT/a$A.err || { echo "abl $A failed"; tail -3 $OUT/a$A.err; cp $OUT/prod.so $P/libkmeans_amd.so; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/a$A.json'));print('ablate=$A', {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['resolve'])"
done
cp $OUT/prod.so $P/libkmeans_amd.so
