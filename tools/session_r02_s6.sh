#!/bin/bash
# Round 2, session 6: pool-sliced multi-rank finish + warm-up shards (2 ranks on
# the one GPU over gloo), the existing multi-rank tests.
set -u
mkdir -p gpurun_out/s6
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_slices.py tests/test_gpu_dist.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/s6/pytest_slices.log 2>&1 || { tail -60 gpurun_out/s6/pytest_slices.log; exit 1; }
tail -15 gpurun_out/s6/pytest_slices.log
