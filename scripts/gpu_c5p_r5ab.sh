# c5_poor and c3_shard8 on one box, alternating: the round-5 library and package against
# the current one (profiles/r6_c5_poor_r5_ab.json, r6_c3_shard8_r5_ab.json); gpurun_ab_r5/
# staged as for scripts/gpu_c2_r5ab.sh.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r6_c5p_r5ab; mkdir -p $OUT
for spec in c5_poor:1 c5_poor:2 c3_shard8:1 c3_shard8:2; do
  C=${spec%%:*}; R=${spec##*:}
  (cd gpurun_ab_r5 && timeout -k 10 400 python -u bench.py --config $C --steps 10 --no-cpu-baseline > ../$OUT/$C.r5.$R.json 2> ../$OUT/$C.r5.$R.err) || { echo r5 $C failed; tail -5 $OUT/$C.r5.$R.err; exit 1; }
  timeout -k 10 400 python -u bench.py --config $C --steps 10 --no-cpu-baseline --no-first-iter > $OUT/$C.r6.$R.json 2> $OUT/$C.r6.$R.err || { echo r6 $C failed; tail -5 $OUT/$C.r6.$R.err; exit 1; }
  python3 -c "
import json
for t in ['r5','r6']:
    d=json.loads(open('$OUT/$C.'+t+'.$R.json').read().strip().splitlines()[-1]); print('$C', t, $R, round(d['value'],2), {k:round(v,2) for k,v in d['kernel_avg_ms'].items()})"
done
