#!/bin/bash
# Round 2, session 16: timed steps with no events at all (stage_timing 3, A)
# vs events at both ends of a call (stage_timing 2).
set -u
mkdir -p gpurun_out/s16
export TMPDIR=/tmp
timeout -k 10 600 bash tools/ab_run.sh env:NK_BENCH_TIMED_LEVEL=2 > gpurun_out/s16/ab.log 2>&1 || { cat gpurun_out/s16/ab.log; exit 1; }
cat gpurun_out/s16/ab.log
