set -o pipefail
cd $GRAFT_REPO_ROOT
for F in 1 0; do
  KM_FUSED=$F timeout -k 10 120 python -u scripts/debug_ties.py ${ARGS:-20000 64 128} || exit 1
done
