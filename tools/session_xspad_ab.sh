#!/bin/bash
# k_xscatter workgroups per CU (NK_XS_LDS_PAD: 0 -> 3, 30000 -> 2, 80000 -> 1):
# interleaved timings of the exact_counts step (tools/exact_ab.py), then the
# grouped-table tests under the padded launch
set -u
OUT=gpurun_out/${TAG:-xspad}
mkdir -p "$OUT"
for i in 1 2 3; do
  for v in 0 30000 80000; do
    NK_XS_LDS_PAD=$v timeout -k 10 150 python -u tools/exact_ab.py "NK_XS_LDS_PAD=$v" >> "$OUT/ab.log" 2>&1 || exit $?
  done
done
grep exact_ms "$OUT/ab.log"
NK_XS_LDS_PAD=30000 timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py -x -q --timeout 120 \
  --timeout-method thread > "$OUT/pytest_pad.log" 2>&1 || { tail -20 "$OUT/pytest_pad.log"; exit 1; }
tail -1 "$OUT/pytest_pad.log"
