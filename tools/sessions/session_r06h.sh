#!/bin/bash
# round 6, session h: config 3's resident count through the Part path and the
# wide two-level path (coarse buckets of 2^17 / 2^18 neurons), with kernel stats
set -u
mkdir -p gpurun_out/r06h
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c3_paths.py 31600000 part,17,18 > gpurun_out/r06h/paths.log 2>&1 || { tail -20 gpurun_out/r06h/paths.log; exit 1; }
cat gpurun_out/r06h/paths.log
for m in part 17; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06h/prof_$m -o run --output-format csv -- python3 -u tools/c3_paths.py 31600000 $m > gpurun_out/r06h/prof_$m.log 2>&1 || exit $?
done
