#!/bin/bash
# Round 2, session 30: why a third batch in flight does not start its count
# right after the previous count — kernel trace + HIP API trace of the
# overlapped run (m = 3), short.
set -u
mkdir -p gpurun_out/s30
export TMPDIR=/tmp
R=$(pwd)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $R/gpurun_out/s30/trace -o run -- python3 $R/bench.py --steps 12 --warmup 1 --settle 0.05 --no-cpu-baseline --no-extras --inflight 3 > $R/gpurun_out/s30/trace.log 2>&1 || exit $?
ls -la $R/gpurun_out/s30/trace
