# SQ counter pass (clock, MFMA busy, VALU / wait fractions) of one kernel per
# arm, one rocprofv3 --pmc pass per arm (counters never split over passes):
#   SQARMS="shape16|libkmeans_amd.so|k_fused16<2, 8;shape32|libkmeans_amd_f32.so|k_fused<4, 8" \
#     CFG=c3 TAG=r4_sq bash scripts/gpu_sq.sh
# arms are separated by ';', an arm is name|library|kernel-substring[|ENV=V ENV=V];
# the library is chosen through KM_LIB (nothing is copied over the product library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/${TAG:-sq}; mkdir -p $OUT
CTRS=${CTRS:-"GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"}
echo "$SQARMS" | tr ';' '\n' | while IFS='|' read -r name lib kn envs; do
  [ -z "$name" ] && continue
  mkdir -p $OUT/$name
  ( export KM_LIB=$PWD/$P/$lib; for e in $envs; do export "$e"; done
    timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/$name/pmc_sq -o run -- python3 bench.py --config ${CFG:-c3} --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > $OUT/$name/log 2>&1 ) || { echo "$name failed"; tail -5 $OUT/$name/log; exit 1; }
  python3 scripts/sq_summary.py $OUT/$name $OUT/$name.json "$kn" ${CFG:-c3} | python3 -c "import json,sys; d=json.load(sys.stdin); print('$name', {k: round(v,3) for k,v in d.items()})" || exit 1
done
