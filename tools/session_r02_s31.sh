#!/bin/bash
# Round 2, session 31: batches in flight with all counts on ONE stream
# (NK_BENCH_SHARED_COUNT_STREAM=1) vs a stream per handle, m = 2 / 3, two rounds.
set -u
mkdir -p gpurun_out/s31
export TMPDIR=/tmp
R=$(pwd)
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); h=d['step_ms_host']; print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), 'steady', round(sorted(h)[len(h)//2],4), d['total_spikes'], d.get('inflight_handles_same_results'))"; }
for round in 1 2; do
  for m in 2 3; do
    for sh in 0 1; do
      NK_BENCH_SHARED_COUNT_STREAM=$sh timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --inflight $m > gpurun_out/s31/m${m}_sh${sh}_$round.log 2>&1 || { tail -30 gpurun_out/s31/m${m}_sh${sh}_$round.log; exit 1; }
      summ gpurun_out/s31/m${m}_sh${sh}_$round.log
    done
  done
done
cd /tmp && NK_BENCH_SHARED_COUNT_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/s31/trace -o run -- python3 $R/bench.py --steps 20 --warmup 1 --settle 0.05 --no-cpu-baseline --no-extras --inflight 3 > $R/gpurun_out/s31/trace.log 2>&1 || exit $?
echo done
