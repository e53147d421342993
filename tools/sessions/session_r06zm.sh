#!/bin/bash
# round 6, session zm: the count stream on the device clock (K1a stamps of
# every handle merged) in the driver's bench command, without a profiler
set -u
O=gpurun_out/r06zm; mkdir -p $O
for round in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_$round.log 2>&1 || { tail -20 $O/bench_$round.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_$round.log') if l.startswith('{')][-1]); print($round, d['ms_per_step'], d['count_stream_device_clock'], d['k1a_ms_steps_overlapped'])"
done
timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-extras > $O/bench_50.log 2>&1 || exit 1
python3 -c "import json; d=json.loads([l for l in open('$O/bench_50.log') if l.startswith('{')][-1]); print(50, d['ms_per_step'], d['count_stream_device_clock'])"
