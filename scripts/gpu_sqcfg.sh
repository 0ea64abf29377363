# SQ counter passes of the dominant MFMA kernel per config (default c5 and c4):
# pass 1 clock, MFMA busy, VALU, waits; pass 2 LDS and co-execution counters
#   SPECS="c5|k_assign_mfma<8" bash scripts/gpu_sqcfg.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sqcfg}; mkdir -p $OUT
CTRS="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
CTRS2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_VALU_MFMA_COEXEC_CYCLES"
for spec in ${SPECS:-"c5|k_assign_mfma<8" "c4|k_assign_mfma<2"}; do
  C=${spec%%|*}; K=${spec#*|}
  mkdir -p $OUT/$C $OUT/$C/p2
  timeout -s KILL 300 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/$C/pmc_sq -o run -- python3 bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$C/log 2>&1 || { echo "$C failed"; tail -5 $OUT/$C/log; exit 1; }
  python3 scripts/sq_summary.py $OUT/$C $OUT/$C.json "$K" > /dev/null
  python3 -c "
import json; d=json.load(open('$OUT/$C.json'))
for r in d['dispatches']:
  if r['duration_ms'] > 1: print('$C', round(r['duration_ms'],2), 'ms', round(r['clock_ghz'],3), 'GHz mfma', round(r['mfma_busy_per_simd'],3), 'x clock', round(r['mfma_busy_per_simd']*r['clock_ghz'],3), 'valu', round(r['active_inst_valu'],3))"
  if [ -n "${PASS2:-1}" ]; then
    timeout -s KILL 300 rocprofv3 --pmc $CTRS2 --output-format csv -d $OUT/$C/p2/pmc_sq -o run -- python3 bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$C/log2 2>&1 || { echo "$C pass 2 failed"; tail -5 $OUT/$C/log2; exit 1; }
    python3 scripts/sq_summary.py $OUT/$C/p2 $OUT/$C.p2.json "$K" > /dev/null
    python3 -c "
import json; d=json.load(open('$OUT/$C.p2.json'))
for r in d['dispatches']:
  if r['duration_ms'] > 1: print('$C', round(r['duration_ms'],2), 'ms', {k: v for k, v in r['raw'].items()})"
  fi
done
