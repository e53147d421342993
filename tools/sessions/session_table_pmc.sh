#!/bin/bash
# PMC passes over the exact_counts step (tools/exact_ab.py, config-2 input):
# issue, LDS and memory counters of the grouped-table kernels (one counter set
# per rocprofv3 run), summarised per kernel
set -u
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-tpmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc$i" -o run -- python3 "$R/tools/exact_ab.py" P > "$OUT/pmc$i.log" 2>&1 || exit $?
done
cd "$R" && python3 tools/pmc_summary.py "$OUT" "$OUT/sum" > /dev/null 2>&1
echo done
