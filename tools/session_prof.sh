#!/bin/bash
# Refresh the committed evidence: bench (default steps), rocprofv3 kernel trace
# of the bench, PMC passes for K1 (HBM bytes, VALU instructions, busy cycles).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-s5}
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c1-160
bash tools/profile.sh $TAG trace || exit $?
bash tools/profile.sh $TAG pmc FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES"
