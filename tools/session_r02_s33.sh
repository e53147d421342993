#!/bin/bash
# Round 2, session 33 (final): pytest -m gpu on the current tree, then the
# session-32 sequence (smoke, default bench with extras, a second default
# bench, config 4, a kernel trace of the default bench).
set -u
mkdir -p gpurun_out/s33
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/s33/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/s33/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
bash tools/session_r02_s32.sh
