#!/bin/bash
# round 5, session ac: config 5's K1g with a fill counter and a region eighth
# per (coarse bucket, XCD) -- a timing-only ablation build (xcdfill) -- against
# the in-tree one, one k_part_gen launch (NK_SPLIT_LAUNCHES=1), twice each
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_ac}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="$R/bench.py --workload config5 --steps 3 --warmup 1 --settle 0 --no-side-parity --no-cpu-baseline --no-extras"
for round in 1 2; do
  for tag in A xcdfill; do
    lib=""; [ $tag != A ] && lib=$R/tools/bin/ab/$tag/libneurokmer.so
    (cd /tmp && NK_AB_LIB=$lib NK_SPLIT_LAUNCHES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
       -d "$OUT/tr_${tag}_$round" -o run -- python3 $B > "$OUT/tr_${tag}_$round.log" 2>&1) || { tail "$OUT/tr_${tag}_$round.log"; exit 1; }
    python3 - "$OUT/tr_${tag}_$round/run_kernel_stats.csv" $tag $round <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'part_gen' in r['Name'] or 'k_split' in r['Name']:
        print(sys.argv[2], sys.argv[3], r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e6,3), 'ms')
PY
  done
done
