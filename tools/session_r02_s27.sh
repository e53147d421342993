#!/bin/bash
# Round 2, session 27: CU-masked count streams with the freed CUs spread over
# the mask (NK_CU_MASK_SPREAD=1), F = 8 / 16, against F = 0.
set -u
mkdir -p gpurun_out/s27
export TMPDIR=/tmp
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); h=d['step_ms_host']; print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), 'steady', round(sorted(h)[len(h)//2],4), d['roofline']['avg_launch_ms'], 'k1a_ovl', round(sum(d['k1a_ms_steps_overlapped'])/max(1,len(d['k1a_ms_steps_overlapped'])),4), d['total_spikes'], d.get('inflight_handles_same_results'))"; }
for round in 1 2; do
  for f in 0 8 16; do
    NK_CU_MASK_SPREAD=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --free-cus $f > gpurun_out/s27/f${f}_$round.log 2>&1 || { tail -30 gpurun_out/s27/f${f}_$round.log; exit 1; }
    summ gpurun_out/s27/f${f}_$round.log
  done
done
