set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 8 > gpurun_out/r1_bench.json 2> gpurun_out/r1_bench.err; echo "bench rc=$?"
tail -c 3000 gpurun_out/r1_bench.json
