#!/bin/bash
# parity tests of the MFMA path, then an A/B/A of two library builds on c5
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/c5ab; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -v --timeout 300 --timeout-method thread -k "${TESTK:-one_step or near_ties or c5 or fullsize}" > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log; grep -E "FAILED|ERROR" $OUT/tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
CFG=${CFG:-c5} STEPS=${STEPS:-6} bash scripts/gpu_ablib.sh
