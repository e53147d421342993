#!/bin/bash
# k_xgroup parallel-probe insert (NK_XG_PAR=1, the default) vs one probe chain
# per record at a time (0): the grouped-table tests, then interleaved timings
# of the exact_counts step (tools/exact_ab.py)
set -u
OUT=gpurun_out/${TAG:-par}
mkdir -p "$OUT"
f="$OUT/pytest_table.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py -x -q --timeout 120 --timeout-method thread \
  > "$f" 2>&1 || { tail -20 "$f"; exit 1; }
tail -1 "$f"
for i in 1 2 3 4; do
  for v in "NK_XG_PAR=0" "NK_XG_PAR=1"; do
    env $v ${XS:-} timeout -k 10 150 python -u tools/exact_ab.py "$v ${XS:-}" >> "$OUT/ab.log" 2>&1 || exit $?
  done
done
grep exact_ms "$OUT/ab.log"
