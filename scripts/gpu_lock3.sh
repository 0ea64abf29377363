# lockstep (select form) in the product: full parity file, then c3 / c5 A/B
# against the per-entry chunk pass (libkmeans_amd_head.so), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contraction.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lock3_parity.log 2>&1 || { echo parity failed; grep -E "FAILED" gpurun_out/lock3_parity.log | head; tail -5 gpurun_out/lock3_parity.log; exit 1; }
tail -1 gpurun_out/lock3_parity.log
TAG=lock3 LIBS="lock head" CFGS="c3 c5" ROUNDS=2 STEPS=10 bash scripts/gpu_abn.sh
