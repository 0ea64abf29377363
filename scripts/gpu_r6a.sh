# Round-6 first box: the delta-statistics tests (long fit, full size,
# unfused geometries, uneven shards), the two-rank rehearsal of the k_s1 path
# and of the fp16x3 path with per-call host timers, and the c3 bench line
# (first_iter, cpu_baseline).  Output: gpurun_out/r6a.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6a}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_s1.py tests/test_gpu_multirank.py \
  "tests/test_gpu_fullsize.py::test_full_size_c3_delta_fit_through_lloyd_runner" \
  -x -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for SCR in -1 1; do
  KM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29600 + SCR + 1)) bench.py --gpus 2 --config c3_small --steps 10 \
    --warmup 2 --screen $SCR > $OUT/tr2_screen$SCR.json 2> $OUT/tr2_screen$SCR.err || { echo "torchrun $SCR failed"; tail -5 $OUT/tr2_screen$SCR.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/tr2_screen$SCR.json').read().strip().splitlines()[-1]);print('screen $SCR', round(d['ms_per_step'],3), d['kernel_avg_ms'], d['host_ms_per_step'])"
done
timeout -k 10 400 python -u bench.py --config c3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench failed"; tail -5 $OUT/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_c3.json'));print('c3', round(d['value'],2), round(d['ms_per_step'],3), d['kernel_avg_ms'], d['first_iter'], d['cpu_baseline']['value'])"
