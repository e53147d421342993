#!/bin/bash
# Overhead of the multi-rank step on one GPU: bench.py --force-dist in a
# 1-rank RCCL process group (all-reduce, key all-gather and merge run; no
# xGMI traffic), next to the plain N=1 step, plus a kernel trace of the
# rehearsal.  Not the metric.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517
ROOT=$(pwd)
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/reh_plain.log 2>&1 || exit $?
tail -1 gpurun_out/reh_plain.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --force-dist > gpurun_out/reh_dist.log 2>&1 || exit $?
tail -1 gpurun_out/reh_dist.log | cut -c1-400
mkdir -p $ROOT/gpurun_out/prof_reh
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_reh/trace -o run -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --force-dist > $ROOT/gpurun_out/prof_reh/trace.log 2>&1
