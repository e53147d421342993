#!/bin/bash
# round 6, session zp: the count-stamp readout moved after the one-at-a-time
# run -- that run's K1a and step back to their values before the readout existed?
set -u
O=gpurun_out/r06zp; mkdir -p $O
for round in 1 2; do
  timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_$round.log 2>&1 || { tail -20 $O/bench_$round.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_$round.log') if l.startswith('{')][-1]); k=d['k1a_ms_steps']; print($round, d['ms_per_step'], d['ms_per_step_one_in_flight'], round(sum(k)/len(k),4), d['roofline']['frac'], d['count_stream_device_clock'])"
done
