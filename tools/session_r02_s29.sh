#!/bin/bash
# Round 2, session 29: the side workloads through the overlapped bench loop
# (config 5: k=63, 128-bit keys, pool 256 M; config 4: strong-scaling input
# on one GPU), one and two batches in flight.
set -u
mkdir -p gpurun_out/s29
export TMPDIR=/tmp
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), d['total_spikes'], d.get('inflight_handles_same_results'))"; }
for w in config5 config4; do
  for m in 1 2; do
    timeout -k 10 400 python -u bench.py --workload $w --steps 10 --no-cpu-baseline --inflight $m > gpurun_out/s29/${w}_$m.log 2>&1 || { tail -30 gpurun_out/s29/${w}_$m.log; exit 1; }
    summ gpurun_out/s29/${w}_$m.log
  done
done
