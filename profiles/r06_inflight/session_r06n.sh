#!/bin/bash
# round 6, session n: three vs four batches in flight (interleaved pairs)
set -u
mkdir -p gpurun_out/r06n
export TMPDIR=/tmp
for round in 1 2 3 4 5; do
  for m in 3 4; do
    log=gpurun_out/r06n/bench_m${m}_$round.log
    timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras --inflight $m > $log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); r=d['roofline']; print('m$m', $round, d['value'], d['ms_per_step'], d['ms_per_step_one_in_flight'], r['avg_launch_ms'])"
  done
done
