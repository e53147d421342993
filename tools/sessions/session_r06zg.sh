#!/bin/bash
# round 6, session zg: the loopback suite with the quiescent-after-merge build
# and the previous build, twice each (a world-3 refine case failed once)
set -u
O=gpurun_out/r06zg
mkdir -p $O
export TMPDIR=/tmp
for round in 1 2; do
  NK_AB_LIB=tools/bin/ab/prevq/libneurokmer.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_loopback.py > $O/old_$round.log 2>&1; echo "old $round rc=$?"; tail -1 $O/old_$round.log
  timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_loopback.py > $O/new_$round.log 2>&1; echo "new $round rc=$?"; tail -1 $O/new_$round.log
done
