# HBM traffic of each config's dominant kernel: FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes -> profiles/traffic.json (scripts/make_traffic.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-traffic}; mkdir -p $OUT
pass() {  # cfg counter
  timeout -s KILL ${PT:-300} rocprofv3 --pmc $2 --output-format csv -d $OUT/$1/pmc_$3 -o run -- python3 bench.py --config $1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$1_$3.log 2>&1 || { echo "$1 $2 failed"; tail -5 $OUT/$1_$3.log; exit 1; }
}
# SPECS: "config|kernel name substring|algorithmic bytes" entries separated by ';'
IFS=';' read -ra SPEC_LIST <<< "${SPECS:-c2|k_assign_small<16|680000000;c3|k_fused16<2, 8, true|25600000000}"
for spec in "${SPEC_LIST[@]}"; do
  C=${spec%%|*}; rest=${spec#*|}; K=${rest%%|*}; A=${rest#*|}
  pass $C FETCH_SIZE fetch && pass $C WRITE_SIZE write || exit 1
  python3 scripts/make_traffic.py $OUT/$C $C "$K" $A $OUT/traffic.json | grep -E "bytes_per_launch|algorithmic" 
done
