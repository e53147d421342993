#!/bin/bash
# Round 3, session 15: K1a as a persistent grid (NK_K1A_PERSIST workgroups):
# parity, then interleaved steps one GPU (3 in flight) and the 1-rank RCCL
# rehearsal with 1..3 batches in flight.
set -u
mkdir -p gpurun_out/r03_s15
export TMPDIR=/tmp
NK_K1A_PERSIST=720 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "mixed or config2 or pool" > gpurun_out/r03_s15/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_s15/tests.log; [ $rc -ne 0 ] && exit $rc
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['ms_per_step_one_in_flight'], d['roofline']['avg_launch_ms'])"; }
B="--steps 30 --warmup 5 --no-cpu-baseline --no-extras"
for rep in 1 2; do
for v in "p3:0:--inflight 3" "p3x720:720:--inflight 3" "p3x744:744:--inflight 3" "d1:0:--force-dist --inflight 1" "d2x720:720:--force-dist --inflight 2" "d3x720:720:--force-dist --inflight 3"; do
  name=${v%%:*}_$rep; rest=${v#*:}; per=${rest%%:*}; flags=${rest#*:}
  NK_K1A_PERSIST=$per timeout -k 10 200 python -u bench.py $B $flags > gpurun_out/r03_s15/$name.log 2>&1 || exit $?
  summ gpurun_out/r03_s15/$name.log
done
done
