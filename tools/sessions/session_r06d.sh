#!/bin/bash
# round 6, session d: deferred histogram with 4 batches in flight; K1a's
# offsets as plain stores (K1b reading them from the MALL) against nontemporal
set -u
mkdir -p gpurun_out/r06d
export TMPDIR=/tmp
run() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  local log=gpurun_out/r06d/bench_$tag.log
  NK_AB_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras "$@" > $log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], d['ms_per_step_one_in_flight'], r['avg_launch_ms'], r.get('k1a_alone_ms'))"
}
for round in 1 2; do
  run off4_$round "" --inflight 4 --defer-hist off
  run on4_$round "" --inflight 4 --defer-hist on
  run A_$round "" --defer-hist off
  run offplain_$round tools/bin/ab/offplain/libneurokmer.so --defer-hist off
done
NK_AB_LIB=tools/bin/ab/offplain/libneurokmer.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r06d/prof_offplain -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras --defer-hist off --inflight 1 > gpurun_out/r06d/prof_offplain.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r06d/prof_on4 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras --inflight 4 --defer-hist on > gpurun_out/r06d/prof_on4.log 2>&1 || exit $?
