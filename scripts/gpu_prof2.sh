# SQ / LDS counter passes over scripts/small_probe.py (fit + predict launches
# of one config), each pass its own bounded run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-prof2}
CFG=${CFG:-c3_small}
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for P in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD" ; do
  i=$((i+1))
  timeout -k 5 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- python3 scripts/small_probe.py $CFG > $OUT/pmc$i.log 2>&1 || { echo "pmc$i failed"; tail -3 $OUT/pmc$i.log; exit 1; }
done
echo done
