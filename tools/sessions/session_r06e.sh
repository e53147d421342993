#!/bin/bash
# round 6, session e: count chain (K1a of batch i+1 beside K1b of batch i,
# batches alternating between two count streams) against the one count stream
set -u
mkdir -p gpurun_out/r06e
export TMPDIR=/tmp
run() {  # tag env args...
  local tag=$1 envs=$2; shift 2
  local log=gpurun_out/r06e/bench_$tag.log
  env $envs timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras --defer-hist off "$@" > $log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], d['ms_per_step_one_in_flight'], r['avg_launch_ms'], d['k1a_ms_steps_overlapped'][:3])"
}
for round in 1 2 3; do
  run A_$round "X=1"
  run chain_$round "NK_COUNT_CHAIN=1" --count-streams 2
  run s2_$round "X=1" --count-streams 2
done
NK_COUNT_CHAIN=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r06e/prof_chain -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras --defer-hist off --count-streams 2 > gpurun_out/r06e/prof_chain.log 2>&1 || exit $?
