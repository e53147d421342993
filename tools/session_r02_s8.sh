#!/bin/bash
# Round 2, session 8: top-N pass fusion (rows above T emitted in the count pass,
# emit only for blocks short of `need`, LDS-staged tie scan) and bin-0
# aggregation of the LIF spike histogram: GPU tests + config-5 / config-2 timings.
set -u
mkdir -p gpurun_out/s8
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/s8/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s8/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s8/pytest_gpu.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-extras > gpurun_out/s8/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/s8/bench_c2.log | cut -c1-300
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s8/trace_c5 -o run -- python3 $R/bench.py --workload config5 --steps 3 --warmup 1 --settle 0 --no-cpu-baseline --no-extras > $R/gpurun_out/s8/trace_c5.log 2>&1 || exit $?
cd $R && python tools/trace_gaps.py gpurun_out/s8/trace_c5/run_kernel_trace.csv --steps 1 > gpurun_out/s8/timeline_c5.txt 2>&1; tail -20 gpurun_out/s8/timeline_c5.txt
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s8/trace_c2 -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > $R/gpurun_out/s8/trace_c2.log 2>&1 || exit $?
cd $R && python tools/trace_gaps.py gpurun_out/s8/trace_c2/run_kernel_trace.csv --steps 2 > gpurun_out/s8/timeline_c2.txt 2>&1; tail -10 gpurun_out/s8/timeline_c2.txt
