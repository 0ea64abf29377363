# round-2 artefacts: GPU tests, smoke, default bench (with CPU baseline),
# rocprofv3 kernel stats of the same bench, separate FETCH_SIZE / WRITE_SIZE
# and SQ counter passes, and the c2 bench with its own kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-final2r}; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo tests failed; tail -20 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
fi
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
echo bench ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err || { echo trace failed; tail -5 $OUT/trace.err; exit 1; }
echo trace ok
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1 || { echo fetch pass failed; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1 || { echo write pass failed; exit 1; }
echo pmc ok
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_sq.log 2>&1 || { echo sq pass failed; exit 1; }
echo sq ok
timeout -k 10 300 python -u bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo c2 bench failed; tail -5 $OUT/bench_c2.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c2 -o run -- python3 bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/trace_bench_c2.json 2> $OUT/trace_c2.err || { echo c2 trace failed; tail -5 $OUT/trace_c2.err; exit 1; }
echo c2 ok
