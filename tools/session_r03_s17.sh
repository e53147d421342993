#!/bin/bash
# Round 3, session 17: the whole -m gpu suite + smoke on the current tree, the
# driver-form bench, and the N > 1 launch path rehearsed (1 rank: gloo control
# group on loopback + the library's RCCL communicator; 1 and 2 in flight).
set -u
mkdir -p gpurun_out/r03_s17
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
  > gpurun_out/r03_s17/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r03_s17/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > gpurun_out/r03_s17/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r03_s17/smoke.log
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['ms_per_step_one_in_flight'], d['roofline']['avg_launch_ms'], d['config']['collectives'])"; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_s17/bench.log 2>&1 || exit $?
summ gpurun_out/r03_s17/bench.log
B="--steps 30 --warmup 5 --no-cpu-baseline --no-extras"
timeout -k 10 200 python -u bench.py $B --force-dist > gpurun_out/r03_s17/d1.log 2>&1 || exit $?
summ gpurun_out/r03_s17/d1.log
timeout -k 10 200 python -u bench.py $B --force-dist --inflight 2 > gpurun_out/r03_s17/d2.log 2>&1 || exit $?
summ gpurun_out/r03_s17/d2.log
timeout -k 10 200 python -u bench.py $B --inflight 1 > gpurun_out/r03_s17/p1.log 2>&1 || exit $?
summ gpurun_out/r03_s17/p1.log
