# SQ counter passes (clock, MFMA busy, VALU / wait fractions) of the c3 assign
# kernel in several builds / settings, one rocprofv3 pass each:
#   product lib (k_fusedp), k_fused build, diagnostic lib with KM_FUSED=0
#   (k_assign_mfma, 12 waves, top-2 chains)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/${TAG:-sqcmp}; mkdir -p $OUT
cp $P/libkmeans_amd.so $OUT/prod.so
CTRS="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
run() {  # name lib kernel-substring [env...]
  local name=$1 lib=$2 kn=$3; shift 3
  cp $P/libkmeans_amd_$lib.so $P/libkmeans_amd.so
  mkdir -p $OUT/$name
  ( for e in "$@"; do export "$e"; done
    timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/$name/pmc_sq -o run -- python3 bench.py --config ${CFG:-c3} --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$name/log 2>&1 ) || { echo "$name failed"; tail -5 $OUT/$name/log; cp $OUT/prod.so $P/libkmeans_amd.so; exit 1; }
  python3 scripts/sq_summary.py $OUT/$name $OUT/$name.json "$kn" | python3 -c "import json,sys; d=json.load(sys.stdin); print('$name', {k: round(v,3) for k,v in d.items()})"
}
cp $P/libkmeans_amd.so $P/libkmeans_amd_prod.so
run fusedp prod "k_fusedp<4, 8, false"
run fused fused "k_fused<4, 8, true, 0, false"
run mfma diag "k_assign_mfma<4, 12" KM_FUSED=0 KM_TOP2=1 KM_MFMA_WAVES=12
cp $OUT/prod.so $P/libkmeans_amd.so
rm -f $P/libkmeans_amd_prod.so
