#!/bin/bash
# round 5, session t: the key-gather diagnostic (test + the bench's extras under
# a kernel trace: K1a<KEYS> and the table kernels beside it)
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_t}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_diag.py -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_diag.log 2>&1 || { tail -30 $OUT/pytest_diag.log; exit 1; }
tail -1 $OUT/pytest_diag.log
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr" -o run \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench.log" 2>&1) || { tail "$OUT/bench.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, json, sys
o = sys.argv[1]
d = json.loads([l for l in open(o + "/bench.log") if l.startswith('{"metric')][-1])
print("exact_counts_step", d["exact_counts_step"], "key_gather", d["key_gather"])
for r in csv.DictReader(open(o + "/tr/run_kernel_stats.csv")):
    n = r["Name"]
    if any(x in n for x in ("k_part<", "k_x", "key_gather", "k_bucket_hist")):
        print(n[:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
