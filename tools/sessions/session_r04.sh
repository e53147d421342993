#!/bin/bash
# headline bench (driver form) + side lines with PMC (configs given)
set -u
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-300
bash tools/sessions/session_side.sh "$TAG" "$@"
