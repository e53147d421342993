#!/bin/bash
# Round 2, session 11: A/B — prep without the currents memset (experiment:
# does the 4.5 us gap before K1a go with it?), with kernel traces of both.
set -u
mkdir -p gpurun_out/s11
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 bash tools/ab_run.sh nocz > gpurun_out/s11/ab.log 2>&1 || { cat gpurun_out/s11/ab.log; exit 1; }
cat gpurun_out/s11/ab.log
cd /tmp && NK_AB_LIB=$R/tools/bin/ab/nocz/libneurokmer.so timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s11/trace_nocz -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > $R/gpurun_out/s11/trace_nocz.log 2>&1 || exit $?
cd $R && python tools/trace_gaps.py gpurun_out/s11/trace_nocz/run_kernel_trace.csv --steps 2 > gpurun_out/s11/timeline_nocz.txt 2>&1; tail -9 gpurun_out/s11/timeline_nocz.txt
