# rocprofv3: kernel-trace stats + PMC passes (each pass its own run, bounded)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-prof}
CFG=${CFG:-c3_small}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1 || { echo trace failed; tail -5 $OUT/trace.log; exit 1; }
echo trace ok
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD" \
         "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH" \
         "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -k 5 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc$i.log 2>&1 || { echo "pmc$i failed"; tail -3 $OUT/pmc$i.log; }
done
echo done
