#!/bin/bash
# round 5, session af: the driver's bench command with the lean CPU baseline beside the port
set -u
OUT=gpurun_out/${1:-r05_af}; mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
python3 -c "import json; d=[json.loads(l) for l in open('$OUT/bench.log') if l.startswith('{')][-1]; print(d['ms_per_step'], d['cpu_baseline'])"
