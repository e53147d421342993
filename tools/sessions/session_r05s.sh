#!/bin/bash
# round 5, session s: config 5 with the split in persistent workgroups
# (NK_GS_SPLIT_WGS = n: the first n workgroups of each k_gen_split launch split
# every item of the previous launch's records, the rest hash), against the
# fused form (0)
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_s}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="$R/bench.py --workload config5 --steps 3 --warmup 1 --settle 0 --no-side-parity --no-cpu-baseline --no-extras"
for round in 1 2; do
  for n in 0 256 512 768; do
    NK_GS_SPLIT_WGS=$n timeout -k 10 300 python3 $B > "$OUT/c5_${n}_$round.log" 2>&1 || { tail "$OUT/c5_${n}_$round.log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c5_${n}_$round.log').read().strip().splitlines()[-1]); print('$n', $round, d['ms_per_step'], d.get('stage_ms_event_steps'))"
  done
done
(cd /tmp && NK_GS_SPLIT_WGS=512 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
   -d "$OUT/tr_512" -o run -- python3 $B > "$OUT/tr_512.log" 2>&1) || { tail "$OUT/tr_512.log"; exit 1; }
python3 $R/tools/trace_gs.py "$OUT/tr_512" p512 | head -6
