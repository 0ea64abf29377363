# SQ counters of k_s1 (c3) and the bench line, one rocprofv3 --pmc pass
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-s1sq}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_small_fold.py -q --timeout 120 --timeout-method thread > $OUT/fold.log 2>&1; echo "fold tests rc=$?"; tail -2 $OUT/fold.log
SQARMS="s1|libkmeans_amd.so|k_s1<2, 8, 1>;f16|libkmeans_amd.so|k_fused16<2, 8, true, true>" CFG=c3 STEPS=6 TAG=${TAG:-s1sq} bash scripts/gpu_sq.sh
