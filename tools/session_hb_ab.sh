#!/bin/bash
# k_xgroup with 2048-slot LDS tables (NK_XG_HB=11: half the neurons per pass,
# 4 or 5 workgroups per CU by NK_XG_WPE) vs 4096 (12, three per CU): the
# grouped-table tests under 11, then interleaved exact_counts step timings
set -u
OUT=gpurun_out/${TAG:-hb}
mkdir -p "$OUT"
NK_XG_HB=11 timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py -x -q --timeout 120 \
  --timeout-method thread > "$OUT/pytest_hb11.log" 2>&1 || { tail -20 "$OUT/pytest_hb11.log"; exit 1; }
tail -1 "$OUT/pytest_hb11.log"
for i in 1 2 3; do
  for v in "NK_XG_HB=12" "NK_XG_HB=11 NK_XG_WPE=4" "NK_XG_HB=11 NK_XG_WPE=5"; do
    env $v timeout -k 10 150 python -u tools/exact_ab.py "$v" >> "$OUT/ab.log" 2>&1 || exit $?
  done
done
grep exact_ms "$OUT/ab.log"
