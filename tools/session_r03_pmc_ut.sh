#!/bin/bash
# PMC counters of the config-5 step (k_uniq_tiles diagnosis)
set -u
mkdir -p gpurun_out/r03_pmc_ut
export TMPDIR=/tmp
ROOT=$(pwd)
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d $ROOT/gpurun_out/r03_pmc_ut/p1 -o run -- python3 $ROOT/bench.py --workload config5 --steps 1 --warmup 0 --settle 0 --no-cpu-baseline --no-extras > $ROOT/gpurun_out/r03_pmc_ut/p1.log 2>&1 || exit $?
cd $ROOT
f=$(find gpurun_out/r03_pmc_ut/p1 -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r['Kernel_Name'][:40]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    cnt[(k, r['Counter_Name'])] += 1
for k, d in agg.items():
    if 'uniq' in k or 'bucket' in k or 'part_gen' in k:
        n = max(cnt[(k, c)] for c in d)
        print(k, {c: round(v / n) for c, v in d.items()})
PY
