# Round 6: the full scans' fp32 prefilter -- its parity tests, then c5 /
# c5_poor bench lines and a c5 kernel trace.  Output: gpurun_out/$TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6s}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_s1.py::test_full_scan_prefilter_equidistant_groups \
  tests/test_gpu_s1.py::test_one_mfma_unfused_screen_predict_vs_oracle tests/test_gpu_parity.py \
  tests/test_gpu_contraction.py -x -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
TAG=$TAG SKIP_TESTS=1 CFGS="${CFGS:-c5 c5_poor}" BENCH_ARGS="--steps 10 --no-first-iter" bash scripts/gpu_round.sh
