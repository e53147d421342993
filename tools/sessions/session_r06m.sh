#!/bin/bash
# round 6, session m: the prep of each count on its handle's own stream
# (NK_PREP_AHEAD=1: beside the previous batch's count kernel) against inline,
# interleaved pairs, plus one rocprof trace of it
set -u
mkdir -p gpurun_out/r06m
export TMPDIR=/tmp
for round in 1 2 3 4; do
  for t in A P; do
    e=X=1; [ $t = P ] && e=NK_PREP_AHEAD=1
    log=gpurun_out/r06m/bench_${t}_$round.log
    env $e timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras > $log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); r=d['roofline']; print('$t', $round, d['value'], d['ms_per_step'], d['ms_per_step_one_in_flight'], r['avg_launch_ms'])"
  done
done
NK_PREP_AHEAD=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r06m/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/r06m/prof.log 2>&1 || exit $?
