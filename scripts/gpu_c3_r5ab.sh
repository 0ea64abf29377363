# c3 on one box, alternating: the round-5 library and package against the
# current one (profiles/r6_c3_r5_ab.json).  gpurun_ab_r5/ is staged before the
# call from commit 19c48c3 (git worktree add; make in its csrc; copy the
# package, bench.py, kmeans_amd.py and oracle/) and deleted afterwards.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r6_c3_r5ab; mkdir -p $OUT
for R in 1 2; do
  (cd gpurun_ab_r5 && timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > ../$OUT/r5.$R.json 2> ../$OUT/r5.$R.err) || { echo r5 failed; tail -5 $OUT/r5.$R.err; exit 1; }
  timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline --no-first-iter > $OUT/r6.$R.json 2> $OUT/r6.$R.err || { echo r6 failed; tail -5 $OUT/r6.$R.err; exit 1; }
  python3 -c "
import json
for t in ['r5','r6']:
    d=json.loads(open('$OUT/'+t+'.$R.json').read().strip().splitlines()[-1]); print(t, $R, round(d['value'],1), d['kernel_avg_ms'])"
done
