#!/bin/bash
# Round 2, session 9: associative memory on the device vs the oracle.
set -u
mkdir -p gpurun_out/s9
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_assoc.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/s9/pytest_assoc.log 2>&1 || { tail -60 gpurun_out/s9/pytest_assoc.log; exit 1; }
tail -15 gpurun_out/s9/pytest_assoc.log
