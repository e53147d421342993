#!/bin/bash
# round 6, session o: the exact table's per-neuron wave sort (k_xgroup_ws):
# table parity, interleaved A/B against the hash table alone (NK_XG_HASH=1),
# kernel trace of both; the big-pool parity cases with <= 64 coarse buckets
set -u
O=gpurun_out/r06o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_table.py > $O/pytest_table.log 2>&1 || { tail -40 $O/pytest_table.log; exit 1; }
tail -2 $O/pytest_table.log
for round in 1 2 3; do
  NK_XG_HASH=1 timeout -k 10 180 python -u tools/exact_ab.py hash >> $O/ab.log 2>&1 || exit 1
  timeout -k 10 180 python -u tools/exact_ab.py ws >> $O/ab.log 2>&1 || exit 1
  NK_XG_WS1=1 timeout -k 10 180 python -u tools/exact_ab.py ws1 >> $O/ab.log 2>&1 || exit 1
done
grep exact_ms $O/ab.log
R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_ws -o run --output-format csv -- python3 -u $R/tools/exact_ab.py ws > $R/$O/prof_ws.log 2>&1 || exit $?
NK_XG_HASH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_hash -o run --output-format csv -- python3 -u $R/tools/exact_ab.py hash > $R/$O/prof_hash.log 2>&1 || exit $?
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "pools or wide or skewed or (config3 and not 1gb)" > $O/pytest_pools.log 2>&1 || { tail -40 $O/pytest_pools.log; exit 1; }
tail -2 $O/pytest_pools.log
