#!/bin/bash
# Round 2, session 3: state check after the container was re-created —
# the GPU test suite, smoke and the default bench.
set -u
mkdir -p gpurun_out/s3
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s3/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/s3/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/s3/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/s3/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s3/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/s3/bench_default.log | cut -c1-700
