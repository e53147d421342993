#!/bin/bash
# A/B: config-5 coarse partition width (NK_WIDE_BITS 20 = default 245 coarse
# buckets at P = 256 M, 21 = 123 buckets: half the reservation atomics per K1g
# tile, K1s splits 64 ways), interleaved, at 115 Mbases and 12.5 Gbases
set -u
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
for i in 1 2; do
  for wb in 20 21; do
    NK_WIDE_BITS=$wb timeout -k 10 300 python3 -u bench.py --workload config5 --bases 115000000 --steps 20 --warmup 2 \
      --no-side-parity --no-cpu-baseline > "$OUT/c5s_wb${wb}_$i.log" 2>&1 || exit $?
    NK_WIDE_BITS=$wb timeout -k 10 300 python3 -u bench.py --workload config5 --steps 3 --warmup 1 \
      --no-side-parity --no-cpu-baseline > "$OUT/c5_wb${wb}_$i.log" 2>&1 || exit $?
  done
done
for f in "$OUT"/c5*.log; do
  python3 - "$f" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[1].split("/")[-1], d["ms_per_step"], d["stage_ms_event_steps"].get("count"), d["roofline"]["avg_launch_ms"])
PY
done
