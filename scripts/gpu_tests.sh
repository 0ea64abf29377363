#!/bin/bash
# the full -m gpu suite, one process, per-test timeouts
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
grep -E "FAILED|ERROR" gpurun_out/gpu_tests.log | head -20
exit $rc
