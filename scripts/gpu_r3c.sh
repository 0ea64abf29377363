# parity file + diagnostic-library experiments: c2 rows per thread (KM_SMALL_U)
# and the k_assign_mfma path at c3 (KM_FUSED=0, waves, top-2 chains, ablations)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3c/parity.log 2>&1 || { echo parity failed; grep -E "FAILED|Error" gpurun_out/r3c/parity.log | head; tail -20 gpurun_out/r3c/parity.log; exit 1; }
tail -1 gpurun_out/r3c/parity.log
TAG=r3c/c2 CFG=c2 STEPS=50 RUNS="KM_SMALL_U=1 KM_SMALL_U=2 KM_SMALL_U=1 KM_SMALL_U=2" bash scripts/gpu_envab.sh || exit 1
TAG=r3c/c3 CFG=c3 RUNS="KM_FUSED=1 KM_FUSED=0,KM_TOP2=1,KM_MFMA_WAVES=12 KM_FUSED=0,KM_TOP2=1,KM_MFMA_WAVES=8 KM_FUSED=0,KM_TOP2=0,KM_MFMA_WAVES=12 KM_FUSED=0,KM_TOP2=0,KM_MFMA_WAVES=12,KM_ABLATE=1" bash scripts/gpu_envab.sh
