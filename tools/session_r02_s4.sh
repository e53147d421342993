#!/bin/bash
# Round 2, session 4: boundary gaps closed (rows past top_n, table on demand,
# 128-bit exact table, process_sequence without exact_counts) + the default bench.
set -u
mkdir -p gpurun_out/s4
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/s4/pytest_boundary.log 2>&1 || { tail -40 gpurun_out/s4/pytest_boundary.log; exit 1; }
tail -3 gpurun_out/s4/pytest_boundary.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s4/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/s4/bench_default.log | cut -c1-400
