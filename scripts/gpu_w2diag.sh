# Two-rank rehearsal on the one GPU: default screen and the fp16x3 screen
# (full statistics every iteration), and the single-rank c3_small line, to
# locate the phase that grows with two processes.  Output: gpurun_out/$TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-w2diag}; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --config c3_small --steps 10 --warmup 2 --no-cpu-baseline > $OUT/w1.json 2> $OUT/w1.err || { echo w1 failed; tail -5 $OUT/w1.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/w1.json'));print('w1', round(d['ms_per_step'],3), d['kernel_avg_ms'], d['first_iter']['iter1_ms'])"
for SCR in -1 1; do
  KM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29640 + SCR + 1)) bench.py --gpus 2 --config c3_small --steps 10 \
    --warmup 2 --screen $SCR > $OUT/w2_$SCR.json 2> $OUT/w2_$SCR.err || { echo "w2 $SCR failed"; tail -5 $OUT/w2_$SCR.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/w2_$SCR.json').read().strip().splitlines()[-1]);print('w2 $SCR', round(d['ms_per_step'],3), d['kernel_avg_ms'], d['host_ms_per_step'], d['first_iter']['iter1_ms'])"
done
