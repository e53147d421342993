#!/bin/bash
# round 5, session w: the sliced finish in two calls (nk_finalize_sliced_dist_
# begin / _end) with the count after next gated on an event -- tests, then the
# 1-rank rehearsal with two (host-enqueued) and three (gated) batches in flight
set -u
OUT=gpurun_out/${1:-r05_w}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_rccl.py tests/test_gpu_loopback.py > $OUT/pt.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
for i in 1 2 3; do
  for m in 2 3; do
    timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --steps 50 --force-dist --inflight $m \
      > $OUT/dist_if${m}_$i.log 2>&1 || { echo "failed"; tail $OUT/dist_if${m}_$i.log; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$OUT/dist_if${m}_$i.log') if l.startswith('{')][-1]; print('if$m', $i, d['ms_per_step'], d['inflight'], d.get('parity_ranks'), d.get('step_ms_host', [])[:3])"
  done
done
