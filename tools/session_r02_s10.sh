#!/bin/bash
# Round 2, session 10: pruned final top-N selection — parity tests, then A/B vs
# the previous commit (tools/bin/ab/prev), and a kernel trace.
set -u
mkdir -p gpurun_out/s10
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py tests/test_gpu_configs.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/s10/pytest.log 2>&1 || { tail -40 gpurun_out/s10/pytest.log; exit 1; }
tail -2 gpurun_out/s10/pytest.log
timeout -k 10 600 bash tools/ab_run.sh prev > gpurun_out/s10/ab.log 2>&1 || { cat gpurun_out/s10/ab.log; exit 1; }
cat gpurun_out/s10/ab.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s10/trace_c2 -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > $R/gpurun_out/s10/trace_c2.log 2>&1 || exit $?
cd $R && python tools/trace_gaps.py gpurun_out/s10/trace_c2/run_kernel_trace.csv --steps 2 > gpurun_out/s10/timeline_c2.txt 2>&1; tail -9 gpurun_out/s10/timeline_c2.txt
