# Round bench lines on one box: every BASELINE config (c3 default settings,
# c5 / c5_poor with the predict leg), then the two-rank torchrun rehearsal
# over gloo on the one GPU (allreduce timing).  TAG names gpurun_out/<TAG>.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-benches}; mkdir -p $OUT
for spec in ${SPECS:-"c2|" "c4|" "c5|--predict 3" "c5_poor|--predict 3"}; do
  CFG=${spec%%|*}; ARGS=${spec#*|}; ARGS=${ARGS//,/ }  # SPECS from the environment: commas for spaces
  timeout -k 10 400 python -u bench.py --config $CFG --no-cpu-baseline $ARGS > $OUT/bench_$CFG.json 2> $OUT/bench_$CFG.err || { echo "bench $CFG failed"; tail -5 $OUT/bench_$CFG.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$CFG.json'));print('$CFG', round(d['value'],3), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['roofline']['kernel'][:40], (d.get('predict') or {}).get('kernel_ms'))"
done
if [ -z "${SKIP_TORCHRUN:-}" ]; then
  KM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --config c3_small --steps 10 --warmup 2 > $OUT/torchrun2_c3_small.json 2> $OUT/torchrun2.err || { echo "torchrun failed"; tail -20 $OUT/torchrun2.err; exit 1; }
  cat $OUT/torchrun2_c3_small.json
fi
