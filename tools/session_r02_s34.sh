#!/bin/bash
# Round 2, session 34: 3 vs 4 batches in flight on one count stream (A/B, two runs each).
set -u
mkdir -p gpurun_out/s34
export TMPDIR=/tmp
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), d['roofline']['avg_launch_ms'], d.get('inflight_handles_same_results'))"; }
for r in 1 2; do
  for m in 3 4; do
    timeout -k 10 300 python -u bench.py --inflight $m --no-cpu-baseline --no-extras > gpurun_out/s34/m${m}_${r}.log 2>&1 || exit $?
    summ gpurun_out/s34/m${m}_${r}.log
  done
done
