#!/bin/bash
# round 6, session a: baseline on this box + the headline with 8192-neuron Part
# buckets (245 buckets, NK_PART_MIN_BITS=13) against 32768 (62): K1a and K1b cost
set -u
mkdir -p gpurun_out/r06a
export TMPDIR=/tmp
bash tools/ab_run.sh pbits13 || exit $?
for v in A pbits13; do
  lib=""; [ $v = A ] || lib=tools/bin/ab/$v/libneurokmer.so
  NK_AB_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r06a/prof_$v -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras --inflight 1 > gpurun_out/r06a/bench_$v.log 2>&1 || exit $?
done
