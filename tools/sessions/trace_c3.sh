#!/bin/bash
# kernel + memory-copy trace of the config-3 streaming step (no parity legs)
set -u
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out/$TAG/trace_config3
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT" -o run \
  -- python3 "$R/bench.py" --workload config3 --steps 2 --no-side-parity > "$OUT/bench.log" 2>&1
