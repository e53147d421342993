#!/bin/bash
# Round 2, session 26: batches in flight with the count streams CU-masked
# (--free-cus F leaves F CUs to the finishes), F = 0 / 8 / 16 / 32, two rounds.
set -u
mkdir -p gpurun_out/s26
export TMPDIR=/tmp
R=$(pwd)
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); h=d['step_ms_host']; print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), 'steady', round(sorted(h)[len(h)//2],4), d['roofline']['avg_launch_ms'], 'k1a_ovl', round(sum(d['k1a_ms_steps_overlapped'])/max(1,len(d['k1a_ms_steps_overlapped'])),4), d['total_spikes'], d.get('inflight_handles_same_results'))"; }
for round in 1 2; do
  for f in 0 8 16 32; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --free-cus $f > gpurun_out/s26/f${f}_$round.log 2>&1 || { tail -30 gpurun_out/s26/f${f}_$round.log; exit 1; }
    summ gpurun_out/s26/f${f}_$round.log
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s26/trace -o run -- python3 $R/bench.py --steps 20 --warmup 1 --settle 0.1 --no-cpu-baseline --no-extras --free-cus 16 > $R/gpurun_out/s26/trace.log 2>&1 || exit $?
echo done
