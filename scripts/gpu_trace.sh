# rocprofv3 kernel trace + stats of one bench run, and the per-dispatch
# sequence of the named kernels:
#   CFG=c3 STEPS=20 KERNELS="k_s1 k_fused16" TAG=r5_trace bash scripts/gpu_trace.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-trace}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --config ${CFG:-c3} --steps ${STEPS:-20} --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo "trace failed"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
python3 scripts/trace_seq.py $OUT/prof ${KERNELS:-k_s1} > $OUT/seq.txt && cat $OUT/seq.txt
