#!/bin/bash
# Parity tests of one A/B variant library (VARIANT=<tag>), then the A/B timing
# of the in-tree library against the given tags (tools/ab_run.sh).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${VARIANT:-}" ]; then
  NK_AB_LIB=tools/bin/ab/$VARIANT/libneurokmer.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$VARIANT.log 2>&1
  rc=$?
  echo "pytest($VARIANT) rc=$rc"; tail -5 gpurun_out/pytest_gpu_$VARIANT.log
  [ $rc -ne 0 ] && exit $rc
fi
bash tools/ab_run.sh "$@"
