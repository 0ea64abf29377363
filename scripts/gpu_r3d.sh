# small-path parity (product lib: quad kernel at dp 16) + c2 A/B of the
# dp-16 kernels in the diagnostic library (KM_SMALL_QUAD = 0 / 2 / 4 / 8)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3d
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contraction.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3d/parity.log 2>&1 || { echo parity failed; grep -E "FAILED|Error" gpurun_out/r3d/parity.log | head; tail -30 gpurun_out/r3d/parity.log; exit 1; }
tail -1 gpurun_out/r3d/parity.log
TAG=r3d/c2 CFG=c2 STEPS=50 RUNS="KM_SMALL_QUAD=0 KM_SMALL_QUAD=2 KM_SMALL_QUAD=4 KM_SMALL_QUAD=8 KM_SMALL_QUAD=0 KM_SMALL_QUAD=4" bash scripts/gpu_envab.sh
