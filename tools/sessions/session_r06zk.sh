#!/bin/bash
# round 6, session zk: the multi-rank, multi-stream and ingest tests five times
# over (after the null-stream zeroing race), stopping at the first failure
set -u
O=gpurun_out/r06zk
mkdir -p $O
export TMPDIR=/tmp
for round in 1 2 3 4 5; do
  timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_loopback.py tests/test_gpu_dist.py tests/test_gpu_slices.py tests/test_gpu_inflight.py tests/test_gpu_fused.py tests/test_gpu_rccl.py tests/test_gpu_table.py > $O/pytest_$round.log 2>&1
  rc=$?
  echo "round $round rc=$rc $(tail -1 $O/pytest_$round.log)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
