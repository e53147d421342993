#!/bin/bash
# round 6, session q: the wave sort through DPP / swizzle exchanges, declined groups listed,
# against the hash table (NK_XG_HASH=1); kernel trace of the wave sort
set -u
O=gpurun_out/r06q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_table.py > $O/pytest_table.log 2>&1 || { tail -40 $O/pytest_table.log; exit 1; }
tail -1 $O/pytest_table.log
for round in 1 2 3; do
  NK_XG_HASH=1 timeout -k 10 180 python -u tools/exact_ab.py hash >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 180 python -u tools/exact_ab.py ws >> $O/ab.log 2>&1 || exit 1
  NK_XG_WS1=1 timeout -k 10 180 python -u tools/exact_ab.py ws1 >> $O/ab.log 2>&1 || exit 1
done
grep exact_ms $O/ab.log
R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_ws -o run --output-format csv -- python3 -u $R/tools/exact_ab.py ws > $R/$O/prof_ws.log 2>&1 || exit $?
