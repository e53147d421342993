#!/bin/bash
# 1-rank rehearsal of the multi-GPU step (in-library RCCL communicator, world 1)
# interleaved with the plain one-GPU step.  Variants (name=flags), default:
# the plain finish and the pool-sliced finish at bench.py's default in-flight
# count; extra "name=flags" arguments replace them.
set -u
TAG=$1
shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
COMMON="--steps 50 --warmup 3 --no-cpu-baseline --no-extras"
if [ $# -eq 0 ]; then
  set -- "dist_plain=--force-dist --finish plain" "dist_sliced=--force-dist --finish sliced"
fi
for i in 1 2 3; do
  timeout -k 10 200 python3 -u bench.py $COMMON > "$OUT/plain_$i.log" 2>&1 || exit $?
  for v in "$@"; do
    name=${v%%=*}
    flags=${v#*=}
    timeout -k 10 200 python3 -u bench.py $COMMON $flags > "$OUT/${name}_$i.log" 2>&1 || exit $?
  done
done
for f in "$OUT"/*.log; do
  python3 - "$f" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[1].split("/")[-1], d["ms_per_step"], d["ms_per_step_one_in_flight"], d["inflight"], d.get("parity_ranks", {}).get("all_equal"))
PY
done
