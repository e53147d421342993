#!/bin/bash
# Interleaved A/B in the driver's form (bench.py --steps 20 --warmup 5), R
# rounds of every variant in turn; variants: A (in-tree library), a tag of
# tools/bin/ab/<tag>/libneurokmer.so, or "env:NAME=VAL[,NAME=VAL]" (in-tree
# library with that environment).  Prints one line per run, then medians.
#   R=5 bash tools/ab5.sh OUTDIR A tagB env:NK_X=1
set -u
OUT=$1; shift
R=${R:-5}
mkdir -p "$OUT"
export TMPDIR=/tmp
for round in $(seq 1 $R); do
  for tag in "$@"; do
    lib=""; envs=""
    case $tag in
      A) ;;
      env:*) envs=$(echo "${tag#env:}" | tr ',' ' ') ;;
      *) lib=tools/bin/ab/$tag/libneurokmer.so ;;
    esac
    log=$OUT/$(echo "$tag" | tr ':=,' '___')_$round.log
    env NK_AB_LIB=$lib $envs timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras \
      > "$log" 2>&1 || exit $?
    python3 - "$log" "$tag" "$round" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], d.get("ms_per_step_one_in_flight"),
      r["avg_launch_ms"], r["valu"].get("hash_only_ms"), flush=True)
PY
  done
done
python3 - "$OUT" "$@" <<'PY'
import glob, json, statistics, sys
out = sys.argv[1]
print("variant  ms_per_step(med)  one_in_flight(med)  k1a_ms(med)  hash_only(med)  n")
for tag in sys.argv[2:]:
    rows = []
    for f in sorted(glob.glob(f"{out}/{tag.replace(':','_').replace('=','_').replace(',','_')}_*.log")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        rows.append((d["ms_per_step"], d.get("ms_per_step_one_in_flight"), d["roofline"]["avg_launch_ms"],
                     d["roofline"]["valu"].get("hash_only_ms") or 0))
    if rows:
        med = [statistics.median(x[i] for x in rows) for i in range(4)]
        print(f"{tag:30s} {med[0]:.4f} {med[1]:.4f} {med[2]:.4f} {med[3]:.4f} {len(rows)}")
PY
