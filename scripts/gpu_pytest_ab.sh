# one pytest selection under several values of an env knob:
#   VAR=KM_FS_VEC VALS="0 1" SEL="tests/test_gpu_parity.py -k near_ties" bash scripts/gpu_pytest_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
for V in ${VALS}; do
  env $VAR=$V timeout -k 10 300 python -u -m pytest ${SEL} -q --timeout 120 --timeout-method thread > gpurun_out/pab_$V.log 2>&1
  echo "$VAR=$V rc=$?"; tail -1 gpurun_out/pab_$V.log
done
