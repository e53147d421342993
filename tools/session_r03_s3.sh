#!/bin/bash
# Round 3, session 3: the derived neuron state (no v / r / spike-count writes
# after a LIF from the reset state): the whole -m gpu suite, then benches.
set -u
mkdir -p gpurun_out/r03_s3
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
  > gpurun_out/r03_s3/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/r03_s3/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), d['roofline']['avg_launch_ms'])"; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/r03_s3/bench.log 2>&1 || exit $?
summ gpurun_out/r03_s3/bench.log
timeout -k 10 300 python -u bench.py --workload config5 --steps 10 --no-cpu-baseline --no-extras > gpurun_out/r03_s3/c5.log 2>&1 || exit $?
summ gpurun_out/r03_s3/c5.log
