#!/bin/bash
# round 6, session ze: the N > 1 rehearsal on the final tree -- bench.py in a
# one-rank RCCL group (in-library sliced finish, two batches in flight) against
# the plain one-GPU step, three interleaved pairs
set -u
O=gpurun_out/r06ze
mkdir -p $O
export TMPDIR=/tmp
for round in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/plain_$round.log 2>&1 || exit 1
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --force-dist > $O/dist1_$round.log 2>&1 || exit 1
  for v in plain dist1; do
    python3 -c "import json; d=json.loads([l for l in open('$O/${v}_$round.log').read().splitlines() if l.startswith('{')][-1]); print('$v', $round, d['ms_per_step'], d['inflight'], d['config']['parallelism'][:40])"
  done
done
