# Round 6: the delta fall-back (ABI 7) -- the k_s1 / multi-rank GPU tests,
# then c5 / c5_poor / c4 bench lines with it.  Output: gpurun_out/$TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6n}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_gpu_s1.py tests/test_gpu_multirank.py} \
  -x -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for CFG in ${CFGS:-c5_poor c5 c4}; do
  timeout -k 10 500 python -u bench.py --config $CFG --steps 10 --no-cpu-baseline > $OUT/bench_$CFG.json 2> $OUT/bench_$CFG.err || { echo bench $CFG failed; tail -20 $OUT/bench_$CFG.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$CFG.json'));print('$CFG', round(d['value'],2), round(d['ms_per_step'],3), d['kernel_avg_ms'], d['resolve'], d['first_iter'])"
done
