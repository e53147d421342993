#!/bin/bash
# k_xgroup variants (NK_XG_BLOCK / NK_XG_DIRECT / NK_XG_GPW): the grouped-table
# tests under two of them, then interleaved timings of the exact_counts step
# (tools/exact_ab.py) for each
set -u
OUT=gpurun_out/${TAG:-xg}
mkdir -p "$OUT"
for v in "NK_XG_BLOCK=512 NK_XG_DIRECT=1 NK_XG_GPW=4" "NK_XG_DIRECT=1 NK_XG_GPW=4"; do
  f="$OUT/pytest_$(echo $v | tr ' =' '__').log"
  env $v timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py -x -q --timeout 120 --timeout-method thread \
    > "$f" 2>&1 || { tail -20 "$f"; exit 1; }
  tail -1 "$f"
done
for i in 1 2 3; do
  for v in "NK_XG_BLOCK=256" "NK_XG_DIRECT=1" "NK_XG_DIRECT=1 NK_XG_GPW=4" "NK_XG_BLOCK=512 NK_XG_DIRECT=1" \
           "NK_XG_BLOCK=512 NK_XG_DIRECT=1 NK_XG_GPW=4" "NK_XG_BLOCK=512 NK_XG_DIRECT=1 NK_XG_GPW=2"; do
    env $v timeout -k 10 150 python -u tools/exact_ab.py "$v" >> "$OUT/ab.log" 2>&1 || exit $?
  done
done
grep exact_ms "$OUT/ab.log"
