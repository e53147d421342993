#!/bin/bash
# Round 2, session 23: batches in flight 1 / 2 / 3 on one GPU (50 steps, two
# rounds), and a kernel trace of the 3-in-flight run.
set -u
mkdir -p gpurun_out/s23
export TMPDIR=/tmp
R=$(pwd)
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); h=d['step_ms_host']; print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), 'steady', round(sorted(h)[len(h)//2],4), d['roofline']['avg_launch_ms'], d['total_spikes'], d.get('inflight_handles_same_results'))"; }
for round in 1 2; do
  for m in 1 2 3; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --inflight $m > gpurun_out/s23/b${m}_$round.log 2>&1 || { tail -30 gpurun_out/s23/b${m}_$round.log; exit 1; }
    summ gpurun_out/s23/b${m}_$round.log
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s23/trace -o run -- python3 $R/bench.py --steps 20 --warmup 1 --settle 0.1 --no-cpu-baseline --no-extras --inflight 3 > $R/gpurun_out/s23/trace.log 2>&1 || exit $?
echo done
