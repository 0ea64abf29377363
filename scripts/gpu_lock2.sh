# lockstep forensics: the helper probe, then the c3-shape one-step test on the
# HEAD library (per-entry chunk pass) and on the lockstep library, 3x each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
timeout -k 10 120 python3 scripts/probes/np_pw2_probe.py || exit 1
cp $P/libkmeans_amd.so /tmp/lock.so
for V in head lock head lock; do
  if [ $V = head ]; then cp $P/libkmeans_amd_head.so $P/libkmeans_amd.so; else cp /tmp/lock.so $P/libkmeans_amd.so; fi
  timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q --timeout 150 --timeout-method thread -k "one_step_vs_oracle and 50000-64-256" > gpurun_out/lock2_$V.log 2>&1
  echo "$V rc=$?"; tail -1 gpurun_out/lock2_$V.log
done
cp /tmp/lock.so $P/libkmeans_amd.so
