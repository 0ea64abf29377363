# full check: GPU parity tests, smoke, bench (c3 default), rocprofv3 stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gpu_tests.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 8 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || { echo prof failed; tail -5 $OUT/prof.err; exit 1; }
cut -d, -f1-6 $OUT/prof/run_kernel_stats.csv | head -14
