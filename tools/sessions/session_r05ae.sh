#!/bin/bash
# round 5, session ae: the whole -m gpu suite and smoke() once more on the
# final tree (stability check before the round ends)
set -u
OUT=gpurun_out/${1:-r05_ae}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
