#!/bin/bash
# round 5, session aa: config 3's resident count (pmc_side.py run: counts only)
# with and without the per-XCD sub-regions: K1a time (kernel trace) and WRITE_SIZE
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_aa}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in "sub:X=1" "flat:NK_NO_XCD_REGIONS=1"; do
  tag=${v%%:*}; envs=${v#*:}
  (cd /tmp && env $envs timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_$tag" -o run \
    -- python3 "$R/tools/pmc_side.py" run --workload config3 > "$OUT/tr_$tag.log" 2>&1) || { tail "$OUT/tr_$tag.log"; exit 1; }
  (cd /tmp && env $envs timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_$tag/pmc1" -o run \
    -- python3 "$R/tools/pmc_side.py" run --workload config3 > "$OUT/pmc_$tag.log" 2>&1) || { tail "$OUT/pmc_$tag.log"; exit 1; }
  python3 - "$OUT" $tag <<'PY'
import csv, sys
from collections import defaultdict
o, t = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(f"{o}/tr_{t}/run_kernel_stats.csv")):
    if 'k_part<' in r['Name'] or 'k_bucket_hist' in r['Name']:
        print(t, r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us', round(float(r['TotalDurationNs'])/1e6, 2), 'ms total')
w = defaultdict(float); n = defaultdict(int)
for r in csv.DictReader(open(f"{o}/pmc_{t}/pmc1/run_counter_collection.csv")):
    if 'k_part<' in r['Kernel_Name']:
        w['k_part'] += float(r['Counter_Value']); n['k_part'] += 1
print(t, 'k_part WRITE_SIZE total GB', round(w['k_part'] * 1024 / 1e9, 2), 'dispatch-rows', n['k_part'])
PY
done
