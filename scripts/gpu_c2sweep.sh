set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "32 4" "16 8" "8 8" "8 16" "4 16" "16 12"; do
  set -- $cfg
  KM_SMALL_R=$1 KM_SMALL_BPC=$2 timeout -k 10 200 python -u bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/c2_$1_$2.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/c2_$1_$2.json'));print('R=$1 bpc=$2', round(d['value'],1),'it/s', round(d['kernel_avg_ms']['assign']*1000,1),'us', round(d['roofline']['achieved']))"
done
