#!/bin/bash
# rocprofv3 kernel trace + stats of a short side-line run (no parity legs):
#   bash tools/sessions/trace_side.sh <tag> config4|config5 [extra bench args]
set -u
TAG=$1; W=$2; shift 2
R=$(pwd)
OUT=$R/gpurun_out/$TAG/trace_$W
mkdir -p "$OUT"
export TMPDIR=/tmp
EXTRA=""
[ "$W" = config4 ] && EXTRA="--shard-of 8"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run \
  -- python3 "$R/bench.py" --workload "$W" --steps 3 --warmup 1 --settle 0 --no-side-parity $EXTRA "$@" \
  > "$OUT/bench.log" 2>&1
