# GPU tests + default bench + c2 bench (round-2 checks)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo bench failed; tail -20 $OUT/bench_c3.err; exit 1; }
cat $OUT/bench_c3.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernel_avg_ms'])"
timeout -k 10 300 python -u bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo bench c2 failed; tail -20 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernel_avg_ms'])"
