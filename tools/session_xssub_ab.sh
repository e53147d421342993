#!/bin/bash
# k_xscatter at one workgroup per CU: 4096-record sub-tiles + LDS padding (the
# default) vs 8192-record sub-tiles (NK_XS_SUB=8192) vs three per CU
# (NK_XS_LDS_PAD=0): grouped-table tests under 8192, then interleaved timings
# of the exact_counts step (tools/exact_ab.py)
set -u
OUT=gpurun_out/${TAG:-xssub}
mkdir -p "$OUT"
NK_XS_SUB=8192 timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py -x -q --timeout 120 \
  --timeout-method thread > "$OUT/pytest_sub8192.log" 2>&1 || { tail -20 "$OUT/pytest_sub8192.log"; exit 1; }
tail -1 "$OUT/pytest_sub8192.log"
for i in 1 2 3; do
  for v in "NK_XS_LDS_PAD=0" "NK_XS_SUB=4096" "NK_XS_SUB=8192"; do
    env $v timeout -k 10 150 python -u tools/exact_ab.py "$v" >> "$OUT/ab.log" 2>&1 || exit $?
  done
done
grep exact_ms "$OUT/ab.log"
