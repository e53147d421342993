#!/bin/bash
# parity tests + bench, an A/B of the in-tree library against the given
# variants, then a kernel trace of the bench and its per-step timeline
set -u
bash tools/gpu_check.sh || exit $?
bash tools/ab_run.sh "$@" || exit $?
bash tools/profile.sh ${TAG:-s4} trace || exit $?
python3 tools/trace_gaps.py gpurun_out/prof_${TAG:-s4}/trace/run_kernel_trace.csv --steps 3 | tee gpurun_out/step_timeline_${TAG:-s4}.txt
