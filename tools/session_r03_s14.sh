#!/bin/bash
# Round 3, session 14: the merge + gather as one kernel (k_merge_gather); the bench's
# N > 1 control group on gloo (the library's RCCL communicator carries the data).
set -u
mkdir -p gpurun_out/r03_s14
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_rccl.py tests/test_gpu_dist.py tests/test_gpu_slices.py tests/test_gpu_inflight.py \
  > gpurun_out/r03_s14/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_s14/tests.log; [ $rc -ne 0 ] && exit $rc
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['ms_per_step_one_in_flight'], d['roofline']['avg_launch_ms'], d['config']['collectives'])"; }
B="--steps 30 --warmup 5 --no-cpu-baseline --no-extras --inflight 1"
for rep in 1 2 3; do
for v in "plain:" "lib:--force-dist" "libnomg:--force-dist"; do
  name=${v%%:*}_$rep; flags=${v#*:}
  if [ "${name%%_*}" = libnomg ]; then export NK_NO_MERGE_GATHER=1; else unset NK_NO_MERGE_GATHER; fi
  timeout -k 10 200 python -u bench.py $B $flags > gpurun_out/r03_s14/$name.log 2>&1 || exit $?
  summ gpurun_out/r03_s14/$name.log
done
done
