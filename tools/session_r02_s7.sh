#!/bin/bash
# Round 2, session 7: config-5 shape on one GPU (k=63, 128-bit keys, pool 256M):
# plain step, the 1-rank pool-sliced rehearsal, and a kernel trace of the plain step.
set -u
mkdir -p gpurun_out/s7
export TMPDIR=/tmp
R=$(pwd)
#timeout -k 10 400 python -u bench.py --workload config5 --steps 5 --no-cpu-baseline --no-extras > gpurun_out/s7/bench_c5.log 2>&1 || exit $?
#tail -1 gpurun_out/s7/bench_c5.log | cut -c1-500
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --workload config5 --steps 5 --force-dist --dist-backend nccl --no-cpu-baseline --no-extras > gpurun_out/s7/bench_c5_sliced1.log 2>&1 || exit $?
tail -1 gpurun_out/s7/bench_c5_sliced1.log | cut -c1-500
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s7/trace_c5 -o run -- python3 $R/bench.py --workload config5 --steps 3 --warmup 1 --settle 0 --no-cpu-baseline --no-extras > $R/gpurun_out/s7/trace_c5.log 2>&1 || exit $?
cd $R && python tools/trace_gaps.py gpurun_out/s7/trace_c5/run_kernel_trace.csv --steps 1 > gpurun_out/s7/timeline_c5.txt 2>&1; cat gpurun_out/s7/timeline_c5.txt | tail -30
