#!/bin/bash
# round 6, session zj (= zf without its tests): the quiescent handle after nk_merge_export (no
# cross-stream wait before the next count) in the one-rank RCCL rehearsal,
# against the previous build; the multi-rank tests
set -u
O=gpurun_out/r06zj
mkdir -p $O
export TMPDIR=/tmp
# (the multi-rank tests: session r06zi)

for round in 1 2 3 4; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --force-dist > $O/new_$round.log 2>&1 || exit 1
  NK_AB_LIB=tools/bin/ab/prevq/libneurokmer.so timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --force-dist > $O/old_$round.log 2>&1 || exit 1
  for v in new old; do
    python3 -c "import json; d=json.loads([l for l in open('$O/${v}_$round.log').read().splitlines() if l.startswith('{')][-1]); print('$v', $round, d['ms_per_step'], d['inflight'])"
  done
done
