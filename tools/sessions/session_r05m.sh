#!/bin/bash
# round 5, session m: what K1g's time is (config 5, one k_part_gen launch over
# the whole input, NK_SPLIT_LAUNCHES=1): the in-tree library (pool modulo as a
# template argument), the previous branchy form, and ablations of it (no sort
# + store, no staging, no LDS rank atomic); then the pipelined count both ways
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_m}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="$R/bench.py --workload config5 --steps 3 --warmup 1 --settle 0 --no-side-parity --no-cpu-baseline --no-extras"
for tag in A g_branchy g_nosort g_nostage_nosort g_all; do
  lib=""; [ $tag != A ] && lib=$R/tools/bin/ab/$tag/libneurokmer.so
  (cd /tmp && NK_AB_LIB=$lib NK_SPLIT_LAUNCHES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$OUT/tr_$tag" -o run -- python3 $B > "$OUT/tr_$tag.log" 2>&1) || { tail "$OUT/tr_$tag.log"; exit 1; }
  python3 - "$OUT/tr_$tag/run_kernel_stats.csv" $tag <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'part_gen' in r['Name'] or 'k_split' in r['Name']:
        print(sys.argv[2], r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e6,3), 'ms')
PY
done
for round in 1 2; do
  for tag in A g_branchy; do
    lib=""; [ $tag != A ] && lib=$R/tools/bin/ab/$tag/libneurokmer.so
    NK_AB_LIB=$lib timeout -k 10 300 python3 $B > "$OUT/pipe_${tag}_$round.log" 2>&1 || { tail "$OUT/pipe_${tag}_$round.log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/pipe_${tag}_$round.log').read().strip().splitlines()[-1]); print('$tag', $round, d['ms_per_step'], d.get('count_ms'), d.get('stage_ms'))"
  done
done
