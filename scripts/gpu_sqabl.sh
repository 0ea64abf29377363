# SQ counter passes (clock, MFMA busy) of the c3 fused kernel ablations and
# fast screens in the diagnostic library: where the power goes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/${TAG:-sqabl}; mkdir -p $OUT
cp $P/libkmeans_amd.so $OUT/prod.so
cp $P/libkmeans_amd_diag.so $P/libkmeans_amd.so
CTRS="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
run() {  # name screen kernel-substring [env...]
  local name=$1 scr=$2 kn=$3; shift 3
  mkdir -p $OUT/$name
  ( for e in "$@"; do export "$e"; done
    timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/$name/pmc_sq -o run -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --screen $scr > $OUT/$name/log 2>&1 ) || { echo "$name failed"; tail -5 $OUT/$name/log; cp $OUT/prod.so $P/libkmeans_amd.so; exit 1; }
  python3 scripts/sq_summary.py $OUT/$name $OUT/$name.json "$kn" > /dev/null
  python3 -c "
import json; d=json.load(open('$OUT/$name.json'))
for r in d['dispatches']:
  if r['duration_ms'] > 0.1: print('$name', round(r['duration_ms'],3), 'ms', round(r['clock_ghz'],3), 'GHz mfma', round(r['mfma_busy_per_simd'],3), 'valu', round(r['active_inst_valu'],3), 'winst', round(r['wait_inst_any'],3), 'wany', round(r['wait_any'],3))"
}
run base 0 "k_fused<4, 8, true, 0"
run abl1 0 "k_fused<4, 8, true, 1" KM_ABLATE=1
run abl2 0 "k_fused<4, 8, true, 2" KM_ABLATE=2
run abl3 0 "k_fused<4, 8, true, 3" KM_ABLATE=3
run abl5 0 "k_fused<4, 8, true, 5" KM_ABLATE=5
run fast1 2 "k_fused1<4, 8, 1"
run fast2 3 "k_fused1<4, 8, 2"
cp $OUT/prod.so $P/libkmeans_amd.so
