#!/bin/bash
# Round 3, session 8: the whole -m gpu suite + smoke after the config-5 work,
# then the driver-form bench.
set -u
mkdir -p gpurun_out/r03_s8
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
  > gpurun_out/r03_s8/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/r03_s8/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > gpurun_out/r03_s8/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r03_s8/smoke.log
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), d['roofline']['avg_launch_ms'])"; }
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_s8/bench.log 2>&1 || exit $?
summ gpurun_out/r03_s8/bench.log
