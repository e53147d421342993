#!/bin/bash
# round 5, session y: the grouped exact table for k > 32 (K1g<KEYS>) -- the
# table tests, then the exact-table step at k = 45 grouped vs the sorted build
set -u
OUT=gpurun_out/${1:-r05_y}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
[ "${SKIP_PT:-0}" = 1 ] || timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_table.py tests/test_gpu_boundary.py > $OUT/pt.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
for v in "grouped:X=1" "sorted:NK_EXACT_SORT=1"; do  # (k = 45: no key-gather diagnostic)
  tag=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python3 -u bench.py --k 45 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/k45_$tag.log 2>&1 || { tail $OUT/k45_$tag.log; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$OUT/k45_$tag.log') if l.startswith('{')][-1]; print('$tag', d['ms_per_step'], d['exact_counts_step'])"
done
