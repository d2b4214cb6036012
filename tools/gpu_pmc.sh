#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only; never combined with sys/runtime traces).
# usage: tools/gpu_pmc.sh <outdir> <program args...>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$1"; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${PMC_HBM_ONLY:-0}" = 1 ]; then PMC_SETS=("FETCH_SIZE" "WRITE_SIZE"); else PMC_SETS=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_COUNT"
 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
 "FETCH_SIZE"
 "WRITE_SIZE"
); fi
i=0
for G in "${PMC_SETS[@]}"; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $G -d "$OUT/p$i" -o pmc --output-format csv -- "$@" > "$OUT/p$i.log" 2>&1) || { echo "pmc pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  i=$((i+1))
done
echo "pmc done"
