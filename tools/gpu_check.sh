#!/bin/bash
# One GPU session: parity tests, then a short bench.  Stops at the first
# fault / abort / timeout (exit codes other than 0 and 1 from pytest).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=20 ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"
tail -5 gpurun_out/bench.log
exit $rc
