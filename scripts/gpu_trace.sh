set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-trace}; CFG=${CFG:-c3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --config $CFG --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo failed; tail -5 $OUT/bench.err; exit 1; }
python3 - <<'PY'
import csv,os
out=os.environ.get('OUT','')
PY
cut -d, -f1-4 $OUT/run_kernel_stats.csv | head -14
