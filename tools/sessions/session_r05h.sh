#!/bin/bash
# round 5, session h: the whole -m gpu suite, then config 3 and config 5 lines with parity
set -u
OUT=gpurun_out/${1:-r05_h}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python3 -u bench.py --workload config3 > $OUT/bench_config3.log 2>&1 || { echo "c3 failed"; tail $OUT/bench_config3.log; exit 1; }
tail -1 $OUT/bench_config3.log | cut -c1-400
timeout -k 10 600 python3 -u bench.py --workload config5 > $OUT/bench_config5.log 2>&1 || { echo "c5 failed"; tail $OUT/bench_config5.log; exit 1; }
tail -1 $OUT/bench_config5.log | cut -c1-400
