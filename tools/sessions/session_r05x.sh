#!/bin/bash
# round 5, session x: config 5 with more, smaller k_gen_split launches (each
# launch's records then fit the 256 MB Infinity Cache when the next launch's
# workgroups split them): 32 (default), 128, 256, 512 launches
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_x}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="$R/bench.py --workload config5 --steps 3 --warmup 1 --settle 0 --no-side-parity --no-cpu-baseline --no-extras"
for round in 1 2; do
  for n in 32 128 256 512; do
    NK_SPLIT_LAUNCHES=$n timeout -k 10 300 python3 $B > "$OUT/c5_${n}_$round.log" 2>&1 || { tail "$OUT/c5_${n}_$round.log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c5_${n}_$round.log').read().strip().splitlines()[-1]); print('$n', $round, d['ms_per_step'], d.get('stage_ms_event_steps'))"
  done
done
