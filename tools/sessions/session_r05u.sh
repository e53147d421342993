#!/bin/bash
# round 5, session u: the 1-rank sliced rehearsal (in-library RCCL
# communicator) with two and three batches in flight, interleaved
set -u
OUT=gpurun_out/${1:-r05_u}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  for m in 2 3; do
    timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --steps 50 --force-dist --inflight $m \
      > $OUT/dist_if${m}_$i.log 2>&1 || { echo "failed"; tail $OUT/dist_if${m}_$i.log; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$OUT/dist_if${m}_$i.log') if l.startswith('{')][-1]; print('if$m', $i, d['ms_per_step'], d['inflight'], d.get('parity_ranks'))"
  done
done
timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --steps 50 > $OUT/plain3.log 2>&1 || exit 1
python3 -c "import json; d=[json.loads(l) for l in open('$OUT/plain3.log') if l.startswith('{')][-1]; print('plain3', d['ms_per_step'])"
