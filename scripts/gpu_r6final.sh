# Round-6 artefacts on one box per phase (PHASE=tests | benches | counters).
#   tests:    the whole GPU suite and smoke()
#   benches:  bench lines of every BASELINE config (c3 with the CPU baseline
#             and first_iter, c5 / c5_poor with the predict leg), rocprofv3
#             kernel traces of c3 / c4 / c5 (summaries: trace_summary.py), the
#             two-rank gloo rehearsal
#   counters: SQ pass of the product k_s1 at c3, FETCH / WRITE passes of c3,
#             c4, c5's dominant kernels (traffic.json entries)
# Output: gpurun_out/$TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6final}; mkdir -p $OUT
case ${PHASE:-tests} in
tests)
  timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
  tail -2 $OUT/smoke.log
  ;;
benches)
  timeout -k 10 500 python -u bench.py --config c3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo bench c3 failed; tail -20 $OUT/bench_c3.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_c3.json'));print('c3', round(d['value'],2), round(d['ms_per_step'],3), d['kernel_avg_ms'], d['first_iter'], d['cpu_baseline']['value'])"
  SPECS="c2| c4| c5|--predict,3 c5_poor|--predict,3 c3_shard8|" TAG=$TAG bash scripts/gpu_benches.sh || exit 1
  for CFG in c3 c4 c5; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$CFG -o run -- python3 bench.py --config $CFG --no-cpu-baseline --no-first-iter > $OUT/trace_bench_$CFG.json 2> $OUT/trace_$CFG.err || { echo trace $CFG failed; tail -5 $OUT/trace_$CFG.err; exit 1; }
    python3 scripts/trace_summary.py $(ls $OUT/trace_$CFG/*kernel_trace.csv | head -1) > $OUT/trace_summary_$CFG.txt && head -6 $OUT/trace_summary_$CFG.txt
  done
  ;;
counters)
  SQARMS="product|libkmeans_amd.so|k_s1<2, 8, 1" CFG=c3 TAG=$TAG/sq bash scripts/gpu_sq.sh || exit 1
  ROUND=6 SPECS="c3|k_s1<2, 8, 1|25600000000;c5|k_assign_mfma16<|25600000000;c4|k_s1<1, 32, 1|128000000000" TAG=$TAG/traffic bash scripts/gpu_traffic.sh || exit 1
  ;;
esac
