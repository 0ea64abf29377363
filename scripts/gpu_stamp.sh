# k_fusedp phase stamps (diagnostic library, KM_ABLATE=9) and an SQ counter
# pass of the product kernel at c3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/${TAG:-stamp}; mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --screen 0 > $OUT/pmc_sq.log 2>&1 || { echo sq pass failed; tail -5 $OUT/pmc_sq.log; exit 1; }
python3 scripts/sq_summary.py $OUT $OUT/sq.json "k_fusedp<4, 8, false" | head -12
cp $P/libkmeans_amd.so $OUT/prod.so
cp $P/libkmeans_amd_diag.so $P/libkmeans_amd.so
for A in 9 0; do
  KM_ABLATE=$A timeout -k 10 300 python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --screen 0 > $OUT/a$A.json 2> $OUT/a$A.err || { echo "abl $A failed"; tail -3 $OUT/a$A.err; cp $OUT/prod.so $P/libkmeans_amd.so; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/a$A.json'));print('ablate=$A', {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['resolve'])"
  grep "km stamps" $OUT/a$A.err | tail -4
done
cp $OUT/prod.so $P/libkmeans_amd.so
