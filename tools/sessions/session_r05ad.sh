#!/bin/bash
# round 5, session ad: host time of a count's enqueue (tools/host_overhead.py)
set -u
OUT=gpurun_out/${1:-r05_ad}; mkdir -p $OUT
timeout -k 10 300 python3 -u tools/host_overhead.py 400 > $OUT/host.log 2>&1 || { tail $OUT/host.log; exit 1; }
tail -2 $OUT/host.log
