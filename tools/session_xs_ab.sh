#!/bin/bash
# k_xscatter direct-store variant (NK_XS_DIRECT=1) with the k_xgroup settings
# in $XG: the grouped-table tests under it, then interleaved timings of the
# exact_counts step (tools/exact_ab.py) against the LDS-staged scatter
set -u
OUT=gpurun_out/${TAG:-xs}
XG=${XG:-}
mkdir -p "$OUT"
f="$OUT/pytest_xs_direct.log"
env $XG NK_XS_DIRECT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py -x -q --timeout 120 \
  --timeout-method thread > "$f" 2>&1 || { tail -20 "$f"; exit 1; }
tail -1 "$f"
for i in 1 2 3 4; do
  for v in "NK_XS_DIRECT=0" "NK_XS_DIRECT=1"; do
    env $XG $v timeout -k 10 150 python -u tools/exact_ab.py "$XG $v" >> "$OUT/ab.log" 2>&1 || exit $?
  done
done
grep exact_ms "$OUT/ab.log"
