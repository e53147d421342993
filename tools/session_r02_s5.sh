#!/bin/bash
# Round 2, session 5: the whole GPU suite after the boundary changes + default bench.
set -u
mkdir -p gpurun_out/s5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s5/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s5/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/s5/pytest_gpu.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s5/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/s5/bench_default.log | cut -c1-400
