#!/bin/bash
# Round 3, session 2: parity of the new SipHash tail + K16 (quick GPU tests),
# then an interleaved A/B: in-tree vs round-2 code vs K1a at 2 workgroups/CU.
set -u
mkdir -p gpurun_out/r03_s2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py > gpurun_out/r03_s2/parity.log 2>&1
rc=$?; tail -3 gpurun_out/r03_s2/parity.log; [ $rc -ne 0 ] && exit $rc
R=5 bash tools/ab5.sh gpurun_out/r03_s2/ab A r2code env:NK_K1A_DYN_LDS=20000
