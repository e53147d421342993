#!/bin/bash
# Round 2, session 13: K1b pad records spread over 64 spill bins (A/B + trace).
set -u
mkdir -p gpurun_out/s13
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 bash tools/ab_run.sh spreadpad > gpurun_out/s13/ab.log 2>&1 || { cat gpurun_out/s13/ab.log; exit 1; }
cat gpurun_out/s13/ab.log
cd /tmp && NK_AB_LIB=$R/tools/bin/ab/spreadpad/libneurokmer.so timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s13/trace -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > $R/gpurun_out/s13/trace.log 2>&1 || exit $?
cd $R && python tools/trace_gaps.py gpurun_out/s13/trace/run_kernel_trace.csv --steps 2 > gpurun_out/s13/timeline.txt 2>&1; tail -9 gpurun_out/s13/timeline.txt
