#!/bin/bash
# Round 2, session 18: the multi-rank step's overhead on one GPU (1-rank RCCL
# rehearsal) with the round's changes, and its kernel timeline.
set -u
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 bash tools/dist_rehearsal.sh > gpurun_out/reh.log 2>&1 || { tail -20 gpurun_out/reh.log; exit 1; }
cat gpurun_out/reh.log
python tools/trace_gaps.py gpurun_out/prof_reh/trace/run_kernel_trace.csv --steps 2 > gpurun_out/prof_reh/timeline.txt 2>&1; tail -16 gpurun_out/prof_reh/timeline.txt
