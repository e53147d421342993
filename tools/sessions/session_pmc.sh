#!/bin/bash
# bench at the default and a short step count, then PMC passes (one counter set
# per rocprofv3 run) over the bench: HBM bytes and VALU activity per kernel
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench5.log 2>&1 || exit $?
bash tools/profile.sh ${TAG:-s4} pmc FETCH_SIZE WRITE_SIZE "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" VALUBusy
