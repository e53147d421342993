#!/bin/bash
# One PMC pass over the exact_counts step (tools/exact_ab.py): how busy each
# CU's LDS is (SQ_LDS_IDX_ACTIVE / SQ_BUSY_CU_CYCLES) per kernel
set -u
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-ldsu}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC \
  SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc1" -o run \
  -- python3 "$R/tools/exact_ab.py" P > "$OUT/pmc1.log" 2>&1 || exit $?
cd "$R" && python3 tools/pmc_summary.py "$OUT" "$OUT/sum" > /dev/null 2>&1
echo done
