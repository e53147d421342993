#!/bin/bash
# Round 2, session 15b: K1a span stamped by the first and the last-dispatched workgroups only (A = new, prev = every workgroup stamps)
# in-kernel span stamps (global atomics)?  A/B without them + a trace.
set -u
mkdir -p gpurun_out/s15b
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 bash tools/ab_run.sh prev > gpurun_out/s15b/ab.log 2>&1 || { cat gpurun_out/s15b/ab.log; exit 1; }
cat gpurun_out/s15b/ab.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s15b/trace -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > $R/gpurun_out/s15b/trace.log 2>&1 || exit $?
cd $R && python tools/trace_gaps.py gpurun_out/s15b/trace/run_kernel_trace.csv --steps 2 > gpurun_out/s15b/timeline.txt 2>&1; tail -9 gpurun_out/s15b/timeline.txt
