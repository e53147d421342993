#!/bin/bash
# round 5, session p: the XCD of each workgroup (tools/xccmap.hip), then K1a
# at pool 16 M: flat regions, and sub-regions per XCD by tile & 7 or by
# HW_REG_XCC_ID, with nontemporal or plain record stores (time + WRITE_SIZE)
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_p}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 5 60 tools/bin/xccmap | tee $OUT/xccmap.txt || exit 1
for v in "flat:NK_NO_XCD_REGIONS=1" "blk_nt:X=1" "blk_plain:NK_SUB_STORES=plain" "hw_nt:NK_SUB_MAP=hw" "hw_plain:NK_SUB_MAP=hw NK_SUB_STORES=plain"; do
  mode=${v%%:*}; envs=${v#*:}
  (cd /tmp && env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_$mode" -o run \
    -- python3 "$R/bench.py" --pool 16000000 --steps 20 --warmup 5 --inflight 1 --no-cpu-baseline --no-extras \
    > "$OUT/tr_$mode.log" 2>&1) || { tail "$OUT/tr_$mode.log"; exit 1; }
  (cd /tmp && env $envs timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_$mode/pmc1" -o run \
    -- python3 "$R/bench.py" --pool 16000000 --steps 5 --warmup 2 --no-cpu-baseline --no-extras --settle 0 \
    > "$OUT/pmc_$mode.log" 2>&1) || { tail "$OUT/pmc_$mode.log"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc_$mode" "$OUT/pmc_$mode" > /dev/null 2>&1 || true
  python3 - "$OUT" $mode <<'PY'
import csv, json, sys
o, m = sys.argv[1], sys.argv[2]
t = {r['Name'][:24]: float(r['AverageNs']) / 1e3 for r in csv.DictReader(open(f"{o}/tr_{m}/run_kernel_stats.csv"))}
w = {k[:24]: v['WRITE_SIZE'] * 1024 / 1e6 for k, v in json.load(open(f"{o}/pmc_{m}/pmc_per_kernel_mean.json")).items()}
k1a = [k for k in t if k.startswith('void nk::k_part<')][0]
k1b = [k for k in t if k.startswith('void nk::k_bucket_hist')][0]
print(m, 'K1a %.1f us' % t[k1a], 'write %.0f MB' % w.get(k1a, -1), '| K1b %.1f us' % t[k1b],
      '| uniq %.1f us' % t.get('void nk::k_uniq_scan<tru', -1))
PY
done
