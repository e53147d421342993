#!/bin/bash
# K1a<KEYS> bucket size (NK_XBIN_BITS 13/14/15: 245/123/62 buckets at P = 2M,
# 1/2/4 k_xgroup passes per group): the grouped-table tests under 14 and 15,
# then interleaved timings of the exact_counts step (tools/exact_ab.py)
set -u
OUT=gpurun_out/${TAG:-xbin}
mkdir -p "$OUT"
for v in 14 15; do
  f="$OUT/pytest_xbin$v.log"
  NK_XBIN_BITS=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py -x -q --timeout 120 \
    --timeout-method thread > "$f" 2>&1 || { tail -20 "$f"; exit 1; }
  tail -1 "$f"
done
for i in 1 2 3; do
  for v in 13 14 15; do
    NK_XBIN_BITS=$v timeout -k 10 150 python -u tools/exact_ab.py "NK_XBIN_BITS=$v" >> "$OUT/ab.log" 2>&1 || exit $?
  done
done
grep exact_ms "$OUT/ab.log"
