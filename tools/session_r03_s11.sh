#!/bin/bash
# Round 3, session 11: which communicator slows K1a (profiles/r03_s10: +20 %
# with torch's RCCL group and the library's communicator both set up).
set -u
mkdir -p gpurun_out/r03_s11
export TMPDIR=/tmp
ROOT=$(pwd)
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['roofline']['avg_launch_ms'])"; }
B="--steps 20 --warmup 5 --no-cpu-baseline --no-extras --inflight 1"
for v in plain "torchonly:--force-dist --dist-init-only --dist-python" "nkonly:--force-dist --dist-init-only --dist-backend gloo --nk-comm" "both:--force-dist --dist-init-only" "glooonly:--force-dist --dist-init-only --dist-backend gloo"; do
  name=${v%%:*}; flags=""; [ "$name" != "$v" ] && flags=${v#*:}
  timeout -k 10 200 python -u bench.py $B $flags > gpurun_out/r03_s11/$name.log 2>&1 || exit $?
  summ gpurun_out/r03_s11/$name.log
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/r03_s11/prof_both -o run -- python3 $ROOT/bench.py --force-dist --dist-init-only --steps 6 --warmup 1 --settle 0.1 --no-cpu-baseline --no-extras --inflight 1 > $ROOT/gpurun_out/r03_s11/prof_both.log 2>&1 || exit $?
cd $ROOT
f=$(find gpurun_out/r03_s11/prof_both -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
c = collections.Counter(r['Kernel_Name'][:60] for r in rows)
for k, v in c.most_common(): print(v, k)
PY
