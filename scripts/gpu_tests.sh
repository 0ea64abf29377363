set -o pipefail
cd $GRAFT_REPO_ROOT
rocminfo | grep -E "gfx|Compute Unit" | head -4 > gpurun_out/r1_rocminfo.txt 2>&1 || true
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1 && echo SMOKE_OK
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1_gpu_tests.log 2>&1; echo "pytest rc=$?"
