#!/bin/bash
# round 6, session zl: kernel trace of the one-rank RCCL rehearsal (the N > 1
# bench path: sliced finish, two batches in flight)
set -u
O=gpurun_out/r06zl
R=$(pwd)
mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --force-dist > $R/$O/bench.log 2>&1) || exit $?
grep '^{' $O/bench.log | cut -c1-200
