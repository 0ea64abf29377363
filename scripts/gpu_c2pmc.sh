# c2 small path characterisation: SQ issue/wait counters and HBM bytes of k_assign_small
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/c2pmc; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/pmc_sq -o run -- python3 scripts/small_probe.py c2 > $OUT/pmc_sq.log 2>&1 || { echo sq pass failed; tail -5 $OUT/pmc_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 scripts/small_probe.py c2 > $OUT/pmc_fetch.log 2>&1 || { echo fetch pass failed; tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/small_probe.py c2 > $OUT/trace.log 2>&1 || { echo trace failed; tail -5 $OUT/trace.log; exit 1; }
python3 scripts/pmc_summary.py $OUT
