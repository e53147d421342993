#!/bin/bash
# round 5, session r: kernel trace of the default bench (3 batches in flight):
# the count stream's cycle and what the finishes cost it
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_r}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr3" -o run \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras > "$OUT/tr3.log" 2>&1) || { tail "$OUT/tr3.log"; exit 1; }
grep '^{' "$OUT/tr3.log" | cut -c1-330
python3 tools/timeline_inflight.py "$OUT/tr3" 60 > $OUT/timeline3.txt; tail -25 $OUT/timeline3.txt
