#!/bin/bash
# round 5, session v: kernel trace of the 1-rank sliced rehearsal with three
# batches in flight (0.69 vs 0.565 ms with two, profiles/r05_u)
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_v}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/tr" -o run \
  -- python3 "$R/bench.py" --no-extras --no-cpu-baseline --steps 20 --force-dist --inflight 3 > "$OUT/b.log" 2>&1) || { tail "$OUT/b.log"; exit 1; }
grep '^{' "$OUT/b.log" | cut -c1-200
