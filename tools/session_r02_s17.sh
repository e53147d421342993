#!/bin/bash
# Round 2, session 17: the round's evidence — full GPU suite, smoke, default
# bench (full CPU baseline + parity), kernel trace, K1a PMC passes.
set -u
mkdir -p gpurun_out/s17
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/s17/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s17/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s17/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s17/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/s17/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s17/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/s17/bench_default.log | cut -c1-300
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s17/trace -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > $R/gpurun_out/s17/trace.log 2>&1 || exit $?
cd $R && python tools/trace_gaps.py gpurun_out/s17/trace/run_kernel_trace.csv --steps 3 > gpurun_out/s17/timeline.txt 2>&1; tail -9 gpurun_out/s17/timeline.txt
TAG=r02f timeout -k 10 600 bash tools/profile.sh r02f pmc FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" || exit $?
ls gpurun_out/prof_r02f
